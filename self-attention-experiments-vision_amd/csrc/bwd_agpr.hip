// bwd_agpr.hip -- attention kernels built for ONE wave per SIMD with the MFMA accumulators in the
// accumulator register file (AGPRs): this translation unit is compiled WITHOUT
// -amdgpu-mfma-vgpr-form (build.py), so a kernel can use the whole 512-register file (256 VGPRs
// for operands and softmax state + AGPRs for dK / dV) instead of the 256 VGPRs of the rest of the
// library.  Launchers only; the kernels live in the shared headers.
#include <hip/hip_runtime.h>

#include "attn_kernels.h"
#include "bwd2.h"

namespace sae {

// dK / dV pass of the two-pass backward (bwd2.h) at one wave per SIMD; PIPE = both query halves'
// S / dP chains issued back to back (see attn_bwd2_dkdv_kernel)
template <int DP, bool PIPE>
hipError_t dkdv_agpr_launch(hipStream_t st, const AttnArgs& a) {
  constexpr int NW = 4;
  const long long grid = (long long)((a.Nk + 32 * NW - 1) / (32 * NW)) * a.H * a.B;
  const size_t lds = 2 * (2 * (size_t)F2<DP>::TILE + 512);
  hipLaunchKernelGGL((attn_bwd2_dkdv_kernel<DP, NW, 1, false, false, PIPE>), dim3((unsigned)grid), dim3(64 * NW), lds,
                     st, a);
  return hipGetLastError();
}

hipError_t bwd2_dkdv_agpr(hipStream_t st, const AttnArgs& a, int dp, bool pipe) {
  if (dp == 32) return pipe ? dkdv_agpr_launch<32, true>(st, a) : dkdv_agpr_launch<32, false>(st, a);
  if (dp == 64) return pipe ? dkdv_agpr_launch<64, true>(st, a) : dkdv_agpr_launch<64, false>(st, a);
  return hipErrorInvalidValue;
}

// both passes of the two-pass backward (bwd2.h) with the accumulators in AGPRs: dQ pass at MQ waves
// per SIMD, dK / dV pass at MK (the head_dim 128 instances: BoTNet)
template <int DP, int MQ, int MK, bool REL>
hipError_t bwd2_agpr_launch(hipStream_t st, const AttnArgs& a) {
  {
    const long long grid = (long long)((a.Nq + 127) / 128) * a.H * a.B;
    const size_t lds = 4 * (size_t)F2<DP>::TILE + (REL ? 2 * kRelImg : 0);
    const void* fn = (const void*)attn_bwd2_dq_kernel<DP, 4, MQ, false, REL>;
    if (lds > 64 * 1024) {
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((attn_bwd2_dq_kernel<DP, 4, MQ, false, REL>), dim3((unsigned)grid), dim3(256), lds, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const long long grid = (long long)((a.Nk + 127) / 128) * a.H * a.B;
  const size_t lds = 2 * (2 * (size_t)F2<DP>::TILE + 512 + (REL ? kRelImg : 0));
  const void* fn = (const void*)attn_bwd2_dkdv_kernel<DP, 4, MK, false, REL>;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((attn_bwd2_dkdv_kernel<DP, 4, MK, false, REL>), dim3((unsigned)grid), dim3(256), lds, st, a);
  return hipGetLastError();
}

hipError_t bwd2_agpr128(hipStream_t st, const AttnArgs& a, bool rel, int variant) {
  if (variant == 0) return rel ? bwd2_agpr_launch<128, 1, 1, true>(st, a) : bwd2_agpr_launch<128, 1, 1, false>(st, a);
  return rel ? bwd2_agpr_launch<128, 2, 1, true>(st, a) : bwd2_agpr_launch<128, 2, 1, false>(st, a);
}

}  // namespace sae
