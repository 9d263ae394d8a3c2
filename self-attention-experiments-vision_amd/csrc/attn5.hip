// attn5.hip -- launchers of the round-5 attention kernels (fwd5.h), in a translation unit of their
// own so that they build in seconds (capi.hip holds every other kernel).  capi.hip dispatches to
// these; they report launch errors as hipError_t.
#include <hip/hip_runtime.h>

#include "attn_kernels.h"
#include "fwd5.h"

namespace sae {

template <int NW, int MINW, bool LSUM, int NSU>
static hipError_t fwd5_run(hipStream_t st, const AttnArgs& a) {
  const long long grid = (long long)((a.Nq + 32 * NW - 1) / (32 * NW)) * a.H * a.B;
  if (grid > 0x7fffffffLL) return hipErrorInvalidConfiguration;
  const size_t lds = 4 * (size_t)F2<64>::TILE;
  hipLaunchKernelGGL((attn_fwd5_kernel<NW, MINW, LSUM, NSU>), dim3((unsigned)grid), dim3(64 * NW), lds, st, a);
  return hipGetLastError();
}

template <int PRIO>
static hipError_t fwd6_run(hipStream_t st, const AttnArgs& a) {
  const long long grid = (long long)((a.Nq + 127) / 128) * a.H * a.B;
  if (grid > 0x7fffffffLL) return hipErrorInvalidConfiguration;
  const size_t lds = 49152;   // 3-deep K / V ring; the final merge image (32 KB + 2 KB)
  hipLaunchKernelGGL((attn_fwd6_kernel<PRIO>), dim3((unsigned)grid), dim3(512), lds, st, a);
  return hipGetLastError();
}

// variant: 0 = default; others select schedule / occupancy forms (dev builds, SAE_FWD_VARIANT)
hipError_t fwd5_launch(hipStream_t st, const AttnArgs& a, int variant) {
  const bool d48 = a.D <= 48;
  switch (variant) {
    case 1: return d48 ? fwd5_run<4, 2, true, 3>(st, a) : fwd5_run<4, 2, true, 4>(st, a);
    case 2: return d48 ? fwd5_run<4, 3, false, 3>(st, a) : fwd5_run<4, 3, false, 4>(st, a);
    case 3: return d48 ? fwd5_run<8, 1, false, 3>(st, a) : fwd5_run<8, 1, false, 4>(st, a);
    case 4: return fwd6_run<0>(st, a);
    case 5: return fwd6_run<1>(st, a);
    default: return d48 ? fwd5_run<4, 2, false, 3>(st, a) : fwd5_run<4, 2, false, 4>(st, a);
  }
}

}  // namespace sae
