// bwd5.hip -- launchers of the round-5 attention backward kernels (bwd5.h), a translation unit of
// their own (VGPR-form MFMA accumulators, like capi.hip); capi.hip dispatches to them.
#include <hip/hip_runtime.h>

#include "attn_kernels.h"
#include "bwd2.h"
#include "bwd5.h"

namespace sae {

template <int NW, int MINW, int SCHED>
static hipError_t dkdv5_run(hipStream_t st, const AttnArgs& a) {
  const long long grid = (long long)((a.Nk + 32 * NW - 1) / (32 * NW)) * a.H * a.B;
  if (grid > 0x7fffffffLL) return hipErrorInvalidConfiguration;
  const size_t lds = 2 * (2 * (size_t)F2<64>::TILE + 512);
  hipLaunchKernelGGL((attn_bwd5_dkdv_kernel<NW, MINW, SCHED>), dim3((unsigned)grid), dim3(64 * NW), lds, st, a);
  return hipGetLastError();
}

template <int PRIO>
static hipError_t dkdv6_run(hipStream_t st, const AttnArgs& a) {
  const long long grid = (long long)((a.Nk + 127) / 128) * a.H * a.B;
  if (grid > 0x7fffffffLL) return hipErrorInvalidConfiguration;
  const size_t lds = 65536;   // 3-deep tile ring (3 x 16.9 KB) / the final partial-sum image (64 KB)
  hipError_t e = hipFuncSetAttribute((const void*)attn_bwd6_dkdv_kernel<PRIO>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((attn_bwd6_dkdv_kernel<PRIO>), dim3((unsigned)grid), dim3(512), lds, st, a);
  return hipGetLastError();
}

template <int PRIO>
static hipError_t dq6_run(hipStream_t st, const AttnArgs& a) {
  const long long grid = (long long)((a.Nq + 127) / 128) * a.H * a.B;
  if (grid > 0x7fffffffLL) return hipErrorInvalidConfiguration;
  const size_t lds = 49152;   // 3-deep K / V ring (3 x 16 KB); the final partial-sum image (32 KB)
  hipLaunchKernelGGL((attn_bwd6_dq_kernel<PRIO>), dim3((unsigned)grid), dim3(512), lds, st, a);
  return hipGetLastError();
}

// the dQ pass of the ping-pong form (publishes delta into a.delta for the dK / dV pass)
hipError_t bwd6_dq_launch(hipStream_t st, const AttnArgs& a, int prio) {
  return prio ? dq6_run<1>(st, a) : dq6_run<0>(st, a);
}

template <int MINW>
static hipError_t dkdv7_run(hipStream_t st, const AttnArgs& a) {
  const long long grid = (long long)((a.Nk + 127) / 128) * a.H * a.B;
  if (grid > 0x7fffffffLL) return hipErrorInvalidConfiguration;
  const size_t lds = 3 * (2 * (size_t)F2<64>::TILE + 512);
  hipLaunchKernelGGL((attn_bwd7_dkdv_kernel<MINW>), dim3((unsigned)grid), dim3(256), lds, st, a);
  return hipGetLastError();
}

// the LDS-DMA staged pair: dQ pass publishing -delta and lse log2 e (PUB2), then bwd7 dK / dV
hipError_t bwd7_launch(hipStream_t st, const AttnArgs& a, int variant) {
  {
    const long long grid = (long long)((a.Nq + 127) / 128) * a.H * a.B;
    if (grid > 0x7fffffffLL) return hipErrorInvalidConfiguration;
    const size_t lds = 4 * (size_t)F2<64>::TILE;
    hipLaunchKernelGGL((attn_bwd2_dq_kernel<64, 4, 2, false, false, true>), dim3((unsigned)grid), dim3(256), lds, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return variant == 1 ? dkdv7_run<1>(st, a) : dkdv7_run<2>(st, a);
}

// the dK / dV pass (the dQ pass that precedes it publishes delta into a.delta)
hipError_t bwd5_dkdv_launch(hipStream_t st, const AttnArgs& a, int variant) {
  switch (variant) {
    case 1: return dkdv5_run<4, 1, 1>(st, a);
    case 2: return dkdv5_run<4, 2, 0>(st, a);
    case 3: return dkdv5_run<4, 1, 0>(st, a);
    case 17: return dkdv5_run<4, 2, 2>(st, a);   // hand body + two register stages
    case 18: return dkdv5_run<4, 1, 2>(st, a);
    case 7: return dkdv6_run<0>(st, a);
    case 8: return dkdv6_run<1>(st, a);
#ifdef SAE_DEV_KNOBS
    case 4: return dkdv5_run<4, 2, 11>(st, a);   // timing probes (wrong results)
    case 5: return dkdv5_run<4, 2, 12>(st, a);
    case 6: return dkdv5_run<4, 2, 13>(st, a);
    case 11: return dkdv5_run<4, 2, 14>(st, a);
    case 12: return dkdv5_run<4, 2, 15>(st, a);
    case 13: return dkdv5_run<4, 2, 16>(st, a);
    case 14: return dkdv5_run<4, 2, 17>(st, a);
#endif
    default: return dkdv5_run<4, 2, 1>(st, a);
  }
}

}  // namespace sae
