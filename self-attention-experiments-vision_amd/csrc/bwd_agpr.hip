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

}  // namespace sae
