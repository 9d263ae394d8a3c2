// capi.hip -- the C ABI (include/sae_attn.h): descriptor validation, template dispatch and
// stream-ordered launches.  No allocation, no host synchronisation, no global mutable state
// besides the thread-local error string.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <stdarg.h>
#include <initializer_list>
#include <string>
#include <algorithm>
#include <type_traits>
#include <mutex>

#include "../../include/sae_attn.h"
#include "attn_kernels.h"
#include "th_kernels.h"
#include "th2.h"
#include "variants.h"
#include "fwd2.h"
#include "bwd2.h"
#include "bwd3.h"
#include "cls.h"
#include "gemm_dw.h"
#include "gemm_nt.h"
#include "gemm8.h"
#include "gemm_f32.h"
#include "gemm_dw8.h"
#include "loss.h"
#include "tokens.h"
#include "patch.h"
#include "ln.h"
#include "adamw.h"

using namespace sae;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int ok() {
  g_err.clear();
  return SAE_OK;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(SAE_EHIP, "%s: launch failed: %s", what, hipGetErrorString(e));
  return ok();
}

int elem_size(int dtype) { return dtype == SAE_DTYPE_BF16 ? 2 : 4; }

bool aligned16(const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; }

int pick_dp(int D) { return D <= 32 ? 32 : (D <= 64 ? 64 : (D <= 128 ? 128 : 0)); }

int validate(const sae_attn_desc* d, bool bwd) {
  if (!d) return fail(SAE_EINVAL, "desc is NULL");
  if (d->batch < 1 || d->heads < 1 || d->seq_q < 1 || d->seq_k < 1 || d->head_dim < 1)
    return fail(SAE_EINVAL, "batch/heads/seq_q/seq_k/head_dim must be >= 1 (got %d/%d/%d/%d/%d)", d->batch,
                d->heads, d->seq_q, d->seq_k, d->head_dim);
  if (d->dtype != SAE_DTYPE_BF16 && d->dtype != SAE_DTYPE_F32)
    return fail(SAE_EINVAL, "dtype %d is not SAE_DTYPE_F32 or SAE_DTYPE_BF16", d->dtype);
  if (!pick_dp(d->head_dim)) return fail(SAE_EUNSUPPORTED, "head_dim %d > 128 is not supported", d->head_dim);
  if ((d->flags & ~SAE_FLAG_RELPOS) != 0) return fail(SAE_EINVAL, "unknown flags 0x%x", d->flags);
  if (d->flags & SAE_FLAG_RELPOS) {
    if (d->rel_h < 1 || d->rel_w < 1 || d->rel_h * d->rel_w != d->seq_k)
      return fail(SAE_EINVAL, "relpos grid %dx%d does not match seq_k %d", d->rel_h, d->rel_w, d->seq_k);
    if (d->rel_w > 64 || d->rel_h > 64 || d->seq_k > 4096)
      return fail(SAE_EUNSUPPORTED, "relpos grid %dx%d exceeds 64x64", d->rel_h, d->rel_w);
  }
  if (d->seq_q > (1 << 24) || d->seq_k > (1 << 24)) return fail(SAE_EUNSUPPORTED, "sequence too long");
  if (!(d->scale > 0.f)) return fail(SAE_EINVAL, "scale must be > 0 (got %g)", (double)d->scale);
  {  // per-(batch, head) row ranges are addressed through 32-bit buffer descriptors
    const int es = d->dtype == SAE_DTYPE_BF16 ? 2 : 4;
    const int64_t* st[8] = {d->q_stride, d->k_stride, d->v_stride, d->o_stride,
                            d->do_stride, d->dq_stride, d->dk_stride, d->dv_stride};
    const char* nm[8] = {"q", "k", "v", "o", "dout", "dq", "dk", "dv"};
    for (int i = 0; i < (bwd ? 8 : 4); ++i) {
      const int64_t n = (i == 1 || i == 2 || i == 6 || i == 7) ? d->seq_k : d->seq_q;
      if (st[i][1] < d->head_dim)
        return fail(SAE_EINVAL, "%s token stride %lld < head_dim %d", nm[i], (long long)st[i][1], d->head_dim);
      if (n * st[i][1] * es >= ((int64_t)1 << 31))
        return fail(SAE_EUNSUPPORTED, "%s: %lld tokens x stride %lld exceed 32-bit row addressing", nm[i],
                    (long long)n, (long long)st[i][1]);
    }
  }
  (void)bwd;
  return SAE_OK;
}

bool strides_vec(const int64_t* s, int epc) { return s[0] % epc == 0 && s[1] % epc == 0 && s[2] % epc == 0; }

void fill_args(AttnArgs& a, const sae_attn_desc* d) {
  memset(&a, 0, sizeof a);
  a.B = d->batch;
  a.H = d->heads;
  a.Nq = d->seq_q;
  a.Nk = d->seq_k;
  a.D = d->head_dim;
  for (int i = 0; i < 3; ++i) {
    a.qs[i] = d->q_stride[i];
    a.ks[i] = d->k_stride[i];
    a.vs[i] = d->v_stride[i];
    a.os[i] = d->o_stride[i];
    a.dos[i] = d->do_stride[i];
    a.dqs[i] = d->dq_stride[i];
    a.dks[i] = d->dk_stride[i];
    a.dvs[i] = d->dv_stride[i];
  }
  a.scale = d->scale;
  if (d->flags & SAE_FLAG_RELPOS) {
    a.rel_h = d->rel_h;
    a.rel_w = d->rel_w;
    a.rel_magic = div_magic(d->rel_w);
  }
}

// ---------------------------------------------------------------- template dispatch helpers
template <template <typename, int, bool, bool> class L, typename... Args>
int dispatch(int dtype, int dp, bool vec, bool rel, Args&&... args) {
#define SAE_CASE(T, DPV)                                                            \
  if (dp == DPV) {                                                                  \
    if (vec) return rel ? L<T, DPV, true, true>::run(args...) : L<T, DPV, true, false>::run(args...); \
    return rel ? L<T, DPV, false, true>::run(args...) : L<T, DPV, false, false>::run(args...);        \
  }
  if (dtype == SAE_DTYPE_BF16) {
    SAE_CASE(__bf16, 32) SAE_CASE(__bf16, 64) SAE_CASE(__bf16, 128)
  } else {
    SAE_CASE(float, 32) SAE_CASE(float, 64) SAE_CASE(float, 128)
  }
#undef SAE_CASE
  return fail(SAE_EUNSUPPORTED, "no kernel instance for dtype %d dp %d", dtype, dp);
}

// Kernels asking for more than 64 KiB of dynamic LDS raise their limit once (up to the 160 KiB
// of a gfx950 CU); failure is reported, never silently ignored.
int lds_attr(const void* fn, size_t bytes) {
  if (bytes > 160 * 1024) return fail(SAE_EUNSUPPORTED, "kernel needs %zu bytes of LDS (> 160 KiB)", bytes);
  if (bytes <= 64 * 1024) return SAE_OK;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) return fail(SAE_EHIP, "hipFuncSetAttribute(%zu B LDS): %s", bytes, hipGetErrorString(e));
  return SAE_OK;
}

int rel_lds_floats(const AttnArgs& a) { return a.rel_h ? 32 * (a.rel_h + a.rel_w + 1) : 0; }

template <typename T, int DP, bool VEC, bool REL> struct FwdL {
  static int run(hipStream_t st, const AttnArgs& a) {
    const int nqb = (a.Nq + kBQ - 1) / kBQ;
    const long long grid = (long long)nqb * a.H * a.B;
    if (grid > 0x7fffffffLL) return fail(SAE_EUNSUPPORTED, "grid too large");
    size_t lds = nbuf<T, DP>() * 2 * Img<T, DP>::bytes(kBK) + (REL ? 4 * rel_lds_floats(a) * sizeof(float) : 0);
    if (int rc = lds_attr((const void*)attn_fwd_kernel<T, DP, VEC, REL>, lds)) return rc;
    hipLaunchKernelGGL((attn_fwd_kernel<T, DP, VEC, REL>), dim3((unsigned)grid), dim3(256), lds, st, a);
    return check_launch("attn_fwd");
  }
};

// lean bf16 forward (fwd2.h): NW waves x 32 query rows per workgroup
template <int DP, int NW, int MINW, bool LSUM, bool ROT = false, int NSU = DP / 16, bool REL = false,
          bool FIX = false, bool PSC = false>
int fwd2_run(hipStream_t st, const AttnArgs& a) {
  const int nqb = (a.Nq + 32 * NW - 1) / (32 * NW);
  const long long grid = (long long)nqb * a.H * a.B;
  if (grid > 0x7fffffffLL) return fail(SAE_EUNSUPPORTED, "grid too large");
  const size_t lds = 4 * (size_t)F2<DP>::TILE + (REL ? 2 * kRelImg : 0);
  if (int rc = lds_attr((const void*)attn_fwd2_kernel<DP, NW, MINW, LSUM, ROT, NSU, REL, FIX, PSC>, lds)) return rc;
  hipLaunchKernelGGL((attn_fwd2_kernel<DP, NW, MINW, LSUM, ROT, NSU, REL, FIX, PSC>), dim3((unsigned)grid),
                     dim3(64 * NW), lds, st, a);
  return check_launch("attn_fwd2");
}

// BoTNet relative logits on the lean bf16 kernels: the table columns (Hs + Ws) fit the two extra
// score k-steps; larger grids (up to 64 x 64) and fp32 take the v1 kernels
static bool rel_lean(const AttnArgs& a) { return a.rel_h + a.rel_w <= kRelCols; }

// single query row (CaiT class attention, CeiT LCA): the K/V stream kernels of cls.h
constexpr int kClsMaxKeys = 1 << 20;
static bool cls_ok(const sae_attn_desc* d) {
  return d->seq_q == 1 && d->seq_k <= kClsMaxKeys && d->head_dim <= 128 && d->dtype == SAE_DTYPE_BF16 &&
         !(d->flags & SAE_FLAG_RELPOS);
}
template <bool BWD> int cls_run(hipStream_t st, const AttnArgs& a) {
  const long long grid = (long long)a.B * a.H;
  if (grid > 0x7fffffffLL) return fail(SAE_EUNSUPPORTED, "grid too large");
  const bool two = a.D > 64;
  const size_t lds = two ? cls_lds_bytes<2>() : cls_lds_bytes<1>();
  const void* fn = BWD ? (two ? (const void*)attn_cls_bwd_kernel<2> : (const void*)attn_cls_bwd_kernel<1>)
                       : (two ? (const void*)attn_cls_fwd_kernel<2> : (const void*)attn_cls_fwd_kernel<1>);
  if (int rc = lds_attr(fn, lds)) return rc;
  if (BWD) {
    if (two) hipLaunchKernelGGL(attn_cls_bwd_kernel<2>, dim3((unsigned)grid), dim3(256), lds, st, a);
    else hipLaunchKernelGGL(attn_cls_bwd_kernel<1>, dim3((unsigned)grid), dim3(256), lds, st, a);
    return check_launch("attn_cls_bwd");
  }
  if (two) hipLaunchKernelGGL(attn_cls_fwd_kernel<2>, dim3((unsigned)grid), dim3(256), lds, st, a);
  else hipLaunchKernelGGL(attn_cls_fwd_kernel<1>, dim3((unsigned)grid), dim3(256), lds, st, a);
  return check_launch("attn_cls_fwd");
}

// Development A/B knobs (schedule variants picked by environment variable) exist only in the
// debug build (build.py --dev defines SAE_DEV_KNOBS); the release library takes the fixed
// dispatch below and never reads the environment on a launch path.
#ifdef SAE_DEV_KNOBS
int dev_knob(const char* name) {
  const char* e = getenv(name);
  if (!e || !*e) return 0;
  return atoi(e[0] == 'v' ? e + 1 : e);
}
#else
constexpr int dev_knob(const char*) { return 0; }
#endif

template <int DP, bool ROT = false> int fwd2_dispatch(hipStream_t st, const AttnArgs& a, int var) {
#ifdef SAE_DEV_KNOBS
  if (!ROT) switch (var) {
    case 2: return fwd2_run<DP, 8, 2, true>(st, a);
    case 4: return fwd2_run<DP, 4, 2, true>(st, a);
    case 5: return fwd2_run<DP, 4, 3, true>(st, a);
    case 6: return fwd2_run<DP, 4, 3, false>(st, a);
    case 7: return fwd2_run<DP, 4, 3, true, false, DP / 16, false, true>(st, a);
    case 8: return fwd2_run<DP, 4, 2, true, false, DP / 16, false, true>(st, a);
    case 9: return fwd2_run<DP, 4, 3, false, false, DP / 16, false, true>(st, a);
    default: break;
  }
  if constexpr (DP <= 64) {
    if (!ROT && var == 40) return fwd2_run<DP, 4, 3, false, false, DP / 16, false, true, true>(st, a);   // prescaled q
    if (!ROT && var == 41) return fwd2_run<DP, 4, 3, true, false, DP / 16, false, true, true>(st, a);    // + MFMA row sum
    if (!ROT && var == 42) return fwd2_run<DP, 4, 2, false, false, DP / 16, false, true, true>(st, a);
  }
#endif
  // D <= 64 without rotary: three waves per SIMD, row sum on the VALU, running max fixed by the
  // first tile (FIX, with the tracking sweep as the in-kernel fallback): 23.2 vs 24.6 us at
  // DeiT-S, 95.4 vs 96.5 us at ViT-B@384 (profiles/r03b_fwdvar.txt, bitwise-equal outputs)
  // (the rotary instances take the same variant: the fused-rotary forward stays bit-equal to the
  // standalone rotary pass + this forward, tests/test_gpu_rotary.py)
  if constexpr (DP <= 64) {
    if (!ROT && DP == 64 && a.D <= 48) return fwd2_run<DP, 4, 3, false, false, 3, false, true>(st, a);
    return fwd2_run<DP, 4, 3, false, ROT, DP / 16, false, true>(st, a);
  }
  // long key ranges at D <= 64: three waves per SIMD, row sum on the VALU is 2.5 % faster at
  // N = 577 and equal at N = 197 (profiles/r01_attn_fwd_f0_vs_f6_interleaved_v13.txt); at
  // D = 128 it is 2x slower
  if constexpr (DP <= 64)
    if (a.Nk >= 512) return fwd2_run<DP, 4, 3, false, ROT>(st, a);
  (void)var;
  // head_dim 48 (CaiT) in 64-wide tiles: QK^T skips the all-zero fourth k-step
  if constexpr (DP == 64 && !ROT)
    if (a.D <= 48) return fwd2_run<DP, 4, 2, true, false, 3>(st, a);
  return fwd2_run<DP, 4, 2, true, ROT>(st, a);
}

// lean bf16 backward (bwd2.h): dQ pass (publishes delta) then dK/dV pass
template <int DP, int NWQ, int MQ, int NWK, int MK, bool ROT = false, bool REL = false>
int bwd2_run(hipStream_t st, const AttnArgs& a) {
  {
    const long long grid = (long long)((a.Nq + 32 * NWQ - 1) / (32 * NWQ)) * a.H * a.B;
    if (grid > 0x7fffffffLL) return fail(SAE_EUNSUPPORTED, "grid too large");
    const size_t lds = 4 * (size_t)F2<DP>::TILE + (REL ? 2 * kRelImg : 0);
    if (int rc = lds_attr((const void*)attn_bwd2_dq_kernel<DP, NWQ, MQ, ROT, REL>, lds)) return rc;
    hipLaunchKernelGGL((attn_bwd2_dq_kernel<DP, NWQ, MQ, ROT, REL>), dim3((unsigned)grid), dim3(64 * NWQ), lds, st,
                       a);
    if (int rc = check_launch("attn_bwd2_dq")) return rc;
  }
  const long long grid = (long long)((a.Nk + 32 * NWK - 1) / (32 * NWK)) * a.H * a.B;
  if (grid > 0x7fffffffLL) return fail(SAE_EUNSUPPORTED, "grid too large");
  const size_t lds = 2 * (2 * (size_t)F2<DP>::TILE + 512 + (REL ? kRelImg : 0));
  if (int rc = lds_attr((const void*)attn_bwd2_dkdv_kernel<DP, NWK, MK, ROT, REL>, lds)) return rc;
  hipLaunchKernelGGL((attn_bwd2_dkdv_kernel<DP, NWK, MK, ROT, REL>), dim3((unsigned)grid), dim3(64 * NWK), lds, st,
                     a);
  return check_launch("attn_bwd2_dkdv");
}

template <int DP, bool ROT = false> int bwd2_run_default(hipStream_t st, const AttnArgs& a) {
  return bwd2_run<DP, 4, 2, 4, 2, ROT>(st, a);
}

}  // namespace
namespace sae {
hipError_t bwd2_dkdv_agpr(hipStream_t st, const AttnArgs& a, int dp, bool pipe);   // bwd_agpr.hip
hipError_t bwd2_agpr128(hipStream_t st, const AttnArgs& a, bool rel, int variant);  // bwd_agpr.hip
}
namespace {

// two-pass backward with the dK / dV pass from bwd_agpr.hip (one wave per SIMD, AGPR accumulators)
template <int DP> int bwd2_run_agpr(hipStream_t st, const AttnArgs& a, bool pipe) {
  {
    const long long grid = (long long)((a.Nq + 127) / 128) * a.H * a.B;
    if (grid > 0x7fffffffLL) return fail(SAE_EUNSUPPORTED, "grid too large");
    const size_t lds = 4 * (size_t)F2<DP>::TILE;
    hipLaunchKernelGGL((attn_bwd2_dq_kernel<DP, 4, 2>), dim3((unsigned)grid), dim3(256), lds, st, a);
    if (int rc = check_launch("attn_bwd2_dq")) return rc;
  }
  const hipError_t e = bwd2_dkdv_agpr(st, a, DP, pipe);
  if (e != hipSuccess) return fail(SAE_EHIP, "attn_bwd2_dkdv (agpr): %s", hipGetErrorString(e));
  return ok();
}

// single-pass bf16 backward (bwd3.h): one workgroup per (batch, head) holding all Nk <= 256 keys
// (8 waves x 32 keys, two waves per SIMD); longer key ranges take the two-pass bwd2
constexpr int kB3Keys = 256;

template <int DP, int NW, int KPW, bool ROT = false, int NSU = DP / 16, bool STAG = false, bool PRIO = false>
int bwd3_run(hipStream_t st, const AttnArgs& a) {
  using C = B3<DP, NW, KPW>;
  static_assert(C::BK == kB3Keys, "bwd3 dispatch assumes 256-key blocks");
  const long long grid = (long long)a.H * a.B;
  if (a.Nk > C::BK) return fail(SAE_EINVAL, "bwd3: %d keys > %d", a.Nk, C::BK);
  if (grid > 0x7fffffffLL) return fail(SAE_EUNSUPPORTED, "grid too large");
  if (int rc = lds_attr((const void*)attn_bwd3_kernel<DP, NW, KPW, ROT, NSU, STAG, PRIO>, C::LDS)) return rc;
  hipLaunchKernelGGL((attn_bwd3_kernel<DP, NW, KPW, ROT, NSU, STAG, PRIO>), dim3((unsigned)grid), dim3(64 * NW),
                     C::LDS, st, a);
  return check_launch("attn_bwd3");
}

template <typename T, int DP, bool VEC, bool REL> struct BwdL {
  static int run(hipStream_t st, const AttnArgs& a) {
    {  // dQ (+ delta) first: it publishes delta for the dK/dV pass
      const int nqb = (a.Nq + kBQ - 1) / kBQ;
      const long long grid = (long long)nqb * a.H * a.B;
      size_t lds = nbuf<T, DP>() * 2 * Img<T, DP>::bytes(kBK) + (REL ? 8 * rel_lds_floats(a) * sizeof(float) : 0);
      if (int rc = lds_attr((const void*)attn_bwd_dq_kernel<T, DP, VEC, REL>, lds)) return rc;
      hipLaunchKernelGGL((attn_bwd_dq_kernel<T, DP, VEC, REL>), dim3((unsigned)grid), dim3(256), lds, st, a);
      int rc = check_launch("attn_bwd_dq");
      if (rc) return rc;
    }
    {
      const int nkb = (a.Nk + kBKV - 1) / kBKV;
      const long long grid = (long long)nkb * a.H * a.B;
      size_t lds = nbuf<T, DP>() * (2 * Img<T, DP>::bytes(kBQT) + 2 * kBQT * sizeof(float) +
                        (REL ? (size_t)kBQT * (a.rel_h + a.rel_w + 1) * sizeof(float) : 0));
      if (int rc = lds_attr((const void*)attn_bwd_dkdv_kernel<T, DP, VEC, REL>, lds)) return rc;
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<T, DP, VEC, REL>), dim3((unsigned)grid), dim3(256), lds, st, a);
      return check_launch("attn_bwd_dkdv");
    }
  }
};

}  // namespace

// ------------------------------------------------------------------ talking-heads launchers
namespace {
void fill_th(ThArgs& a, const sae_attn_desc* d) {
  memset(&a, 0, sizeof a);
  a.B = d->batch;
  a.H = d->heads;
  a.Nq = d->seq_q;
  a.Nk = d->seq_k;
  a.D = d->head_dim;
  for (int i = 0; i < 3; ++i) {
    a.qs[i] = d->q_stride[i];
    a.ks[i] = d->k_stride[i];
    a.vs[i] = d->v_stride[i];
    a.os[i] = d->o_stride[i];
    a.dos[i] = d->do_stride[i];
    a.dqs[i] = d->dq_stride[i];
    a.dks[i] = d->dk_stride[i];
    a.dvs[i] = d->dv_stride[i];
  }
  a.scale = d->scale;
}

bool th_vec(const sae_attn_desc* d, std::initializer_list<const void*> ptrs, bool bwd) {
  const int epc = 16 / elem_size(d->dtype);
  bool v = d->head_dim % epc == 0 && strides_vec(d->q_stride, epc) && strides_vec(d->k_stride, epc) &&
           strides_vec(d->v_stride, epc) && strides_vec(d->o_stride, epc);
  if (bwd)
    v = v && strides_vec(d->do_stride, epc) && strides_vec(d->dq_stride, epc) && strides_vec(d->dk_stride, epc) &&
        strides_vec(d->dv_stride, epc);
  for (const void* p : ptrs) v = v && aligned16(p);
  return v;
}

template <typename T, int DP, bool VEC> int th_fwd_run(hipStream_t st, const ThArgs& a) {
  const int nqb = (a.Nq + 31) / 32;
  size_t lds = kTabBytes + 2 * (size_t)a.H * 4096 + (sizeof(T) == 2 ? (size_t)a.H * Img<T, DP>::bytes(32) : 0);
  if (int rc = lds_attr((const void*)th_fwd_kernel<T, DP, VEC>, lds)) return rc;
  hipLaunchKernelGGL((th_fwd_kernel<T, DP, VEC>), dim3(nqb * a.B), dim3(64 * a.H), lds, st, a);
  return check_launch("th_fwd");
}

template <typename T, int DP, bool VEC> int th_bwd_run(hipStream_t st, ThArgs a) {
  const int nqb = (a.Nq + 31) / 32, nkb = (a.Nk + 31) / 32;
  a.nblk = nqb * a.B;
  size_t lds_q = kTabBytes + 2 * (size_t)a.H * 4096 + (size_t)a.H * 2 * a.H * 64 * sizeof(float) +
                 (sizeof(T) == 2 ? (size_t)a.H * Img<T, DP>::bytes(32) : 0);
  if (int rc = lds_attr((const void*)th_bwd_q_kernel<T, DP, VEC>, lds_q)) return rc;
  hipLaunchKernelGGL((th_bwd_q_kernel<T, DP, VEC>), dim3(nqb * a.B), dim3(64 * a.H), lds_q, st, a);
  if (int rc = check_launch("th_bwd_q")) return rc;
  size_t lds_kv = kTabBytes + 2 * (size_t)a.H * 4096 + (size_t)a.H * 64 * sizeof(float) +
                  (sizeof(T) == 2 ? (size_t)a.H * 2 * Img<T, DP>::bytes(32) : 0);
  if (int rc = lds_attr((const void*)th_bwd_kv_kernel<T, DP, VEC>, lds_kv)) return rc;
  hipLaunchKernelGGL((th_bwd_kv_kernel<T, DP, VEC>), dim3(nkb * a.B), dim3(64 * a.H), lds_kv, st, a);
  if (int rc = check_launch("th_bwd_kv")) return rc;
  hipLaunchKernelGGL(th_reduce_kernel, dim3(2 * a.H * a.H), dim3(256), 0, st, a);
  return check_launch("th_reduce");
}

// bf16 with the head mixes on the MFMA (th2.h).  H <= 8: one wave per head (NWMAX 8).  9..16 heads:
// two heads per wave (eight waves of <= 256 registers; sixteen waves of 128 spilled heavily).
template <int DP, int NWMAX, bool ROT, int HPW, bool LEAN = false, int NSU = DP / 16>
int th2_fwd_run(hipStream_t st, const ThArgs& a) {
  const int nqb = (a.Nq + 31) / 32, nw = (a.H + HPW - 1) / HPW;
  const size_t lds = th2_lds_bytes<DP, NWMAX * HPW <= 8>(a.H, 1, LEAN);
  if (int rc = lds_attr((const void*)th2_fwd_kernel<DP, NWMAX, ROT, HPW, LEAN, NSU>, lds)) return rc;
  hipLaunchKernelGGL((th2_fwd_kernel<DP, NWMAX, ROT, HPW, LEAN, NSU>), dim3(nqb * a.B), dim3(64 * nw), lds, st, a);
  return check_launch("th2_fwd");
}

// LEAN: the query pass at two workgroups per CU (the key pass LEAN -- K / V / Q / dO re-read per
// query tile, 13 spilled registers -- measured 306 vs 230 us: profiles/r06t_th_kv_lean_rejected.txt)
template <int DP, int NWMAX, bool ROT, int HPW, bool LEAN = false, int NSU = DP / 16>
int th2_bwd_run(hipStream_t st, ThArgs a) {
  constexpr bool KST = NWMAX * HPW <= 8;
  const int nqb = (a.Nq + 31) / 32, nkb = (a.Nk + 31) / 32, nw = (a.H + HPW - 1) / HPW;
  a.nblk = nqb * a.B;
  const size_t lds = th2_lds_bytes<DP, KST>(a.H, LEAN ? 2 : HPW);
  const size_t lds_kv = th2_kv_lds_bytes<DP, KST>(a.H, KST && HPW == 1);
  if (int rc = lds_attr((const void*)th2_bwd_q_kernel<DP, NWMAX, ROT, HPW, LEAN, NSU>, lds)) return rc;
  if (int rc = lds_attr((const void*)th2_bwd_kv_kernel<DP, NWMAX, ROT, HPW>, lds_kv)) return rc;
  hipLaunchKernelGGL((th2_bwd_q_kernel<DP, NWMAX, ROT, HPW, LEAN, NSU>), dim3(nqb * a.B), dim3(64 * nw), lds, st, a);
  if (int rc = check_launch("th2_bwd_q")) return rc;
  hipLaunchKernelGGL((th2_bwd_kv_kernel<DP, NWMAX, ROT, HPW>), dim3(nkb * a.B), dim3(64 * nw), lds_kv, st, a);
  if (int rc = check_launch("th2_bwd_kv")) return rc;
  hipLaunchKernelGGL(th_reduce_kernel, dim3(2 * a.H * a.H), dim3(256), 0, st, a);
  return check_launch("th_reduce");
}

// <= 8 heads: the forward at <= 128 VGPRs, two workgroups per CU (CaiT-S24 207 -> 184 us,
// profiles/r05v_th_lean_ab.txt)
// round 6, DP 64 at D <= 48 (every CaiT width): three head-dim k-steps (NSU 3) -- the forward fits
// 128 VGPRs without spills (its scratch traffic was 1.4x the algorithmic bytes: 172 -> 160 us at
// CaiT-S24, 1.05x; profiles/r06s_th_lean_ab.txt)
template <int DP> int th2_fwd_dispatch(hipStream_t st, const ThArgs& a) {
  if constexpr (DP == 64)
    if (a.H <= 8 && a.D <= 48)
      return a.rope.sin ? th2_fwd_run<64, 8, true, 1, true, 3>(st, a) : th2_fwd_run<64, 8, false, 1, true, 3>(st, a);
  if (a.rope.sin) return a.H <= 8 ? th2_fwd_run<DP, 8, true, 1, true>(st, a) : th2_fwd_run<DP, 8, true, 2>(st, a);
  return a.H <= 8 ? th2_fwd_run<DP, 8, false, 1, true>(st, a) : th2_fwd_run<DP, 8, false, 2>(st, a);
}
// round 6: the query pass LEAN (two workgroups per CU) at <= 8 heads without rotary (CaiT-S24
// backward 540 -> 474 us; profiles/r06s_th_lean_ab.txt)
template <int DP> int th2_bwd_dispatch(hipStream_t st, const ThArgs& a) {
  if constexpr (DP == 64)
    if (a.H <= 8 && !dev_knob("SAE_TH_BWDQ_WIDE")) {
      if (a.rope.sin) {
        // (rotary at D <= 48: fwd + bwd 886 -> 785 us at CaiT-S24 shape; the query pass at one
        // workgroup per CU, 210 VGPRs, 614 vs 572 us backward -- profiles/r06w_th_rotary_ab.txt)
        if (a.D <= 48) return th2_bwd_run<64, 8, true, 1, true, 3>(st, a);
      } else {
        return a.D <= 48 ? th2_bwd_run<64, 8, false, 1, true, 3>(st, a) : th2_bwd_run<64, 8, false, 1, true>(st, a);
      }
    }
  if (a.rope.sin) return a.H <= 8 ? th2_bwd_run<DP, 8, true, 1>(st, a) : th2_bwd_run<DP, 8, true, 2>(st, a);
  return a.H <= 8 ? th2_bwd_run<DP, 8, false, 1>(st, a) : th2_bwd_run<DP, 8, false, 2>(st, a);
}

}  // namespace

int th_fwd(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v, const float* th1,
           const float* th2, void* o, float* lse, const RopeTab* rope) {
  ThArgs a;
  fill_th(a, d);
  if (rope) a.rope = *rope;
  a.q = q;
  a.k = k;
  a.v = v;
  a.o = o;
  a.lse = lse;
  a.th1 = th1;
  a.th2 = th2;
  const bool vec = th_vec(d, {q, k, v, o}, false);
  hipStream_t st = (hipStream_t)stream;
  const int dp = pick_dp(d->head_dim);
  if (d->dtype == SAE_DTYPE_BF16 && vec) {   // head mixes on the matrix pipe
    if (dp == 32) return th2_fwd_dispatch<32>(st, a);
    if (dp == 64) return th2_fwd_dispatch<64>(st, a);
  }
  if (rope) return fail(SAE_EUNSUPPORTED, "rotary: fused only on the bf16 talking-heads path (aligned strides)");
  if (d->heads > kThMaxH) return fail(SAE_EUNSUPPORTED, "talking heads: %d heads > %d on the fp32 / unaligned path",
                                      d->heads, kThMaxH);
#define TH_F(T, DPV) \
  if (dp == DPV) return vec ? th_fwd_run<T, DPV, true>(st, a) : th_fwd_run<T, DPV, false>(st, a);
  if (d->dtype == SAE_DTYPE_BF16) {
    TH_F(__bf16, 32) TH_F(__bf16, 64)
  } else {
    TH_F(float, 32) TH_F(float, 64)
  }
#undef TH_F
  return fail(SAE_EUNSUPPORTED, "talking heads: no kernel for dtype %d head_dim %d", d->dtype, d->head_dim);
}

size_t th_bwd_workspace_bytes(const sae_attn_desc* d) {
  const size_t delta = (((size_t)d->batch * d->heads * d->seq_q * sizeof(float)) + 255) & ~(size_t)255;
  const size_t nblk = (size_t)((d->seq_q + 31) / 32) * d->batch;
  return delta + ((nblk * 2 * d->heads * d->heads * sizeof(float) + 255) & ~(size_t)255);
}

int th_bwd(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v, const float* th1,
           const float* th2, const float* lse, const void* dout, void* dq, void* dk, void* dv, float* dth1,
           float* dth2, void* workspace, const RopeTab* rope) {
  ThArgs a;
  fill_th(a, d);
  if (rope) a.rope = *rope;
  a.q = q;
  a.k = k;
  a.v = v;
  a.lse = const_cast<float*>(lse);
  a.dout = dout;
  a.dq = dq;
  a.dk = dk;
  a.dv = dv;
  a.th1 = th1;
  a.th2 = th2;
  a.dth1 = dth1;
  a.dth2 = dth2;
  a.delta = reinterpret_cast<float*>(workspace);
  a.part = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) +
                                    ((((size_t)d->batch * d->heads * d->seq_q * sizeof(float)) + 255) & ~(size_t)255));
  const bool vec = th_vec(d, {q, k, v, dout, dq, dk, dv}, true);
  hipStream_t st = (hipStream_t)stream;
  const int dp = pick_dp(d->head_dim);
  if (d->dtype == SAE_DTYPE_BF16 && vec) {
    if (dp == 32) return th2_bwd_dispatch<32>(st, a);
    if (dp == 64) return th2_bwd_dispatch<64>(st, a);
  }
  if (rope) return fail(SAE_EUNSUPPORTED, "rotary: fused only on the bf16 talking-heads path (aligned strides)");
  if (d->heads > kThMaxH) return fail(SAE_EUNSUPPORTED, "talking heads: %d heads > %d on the fp32 / unaligned path",
                                      d->heads, kThMaxH);
#define TH_B(T, DPV) \
  if (dp == DPV) return vec ? th_bwd_run<T, DPV, true>(st, a) : th_bwd_run<T, DPV, false>(st, a);
  if (d->dtype == SAE_DTYPE_BF16) {
    TH_B(__bf16, 32) TH_B(__bf16, 64)
  } else {
    TH_B(float, 32) TH_B(float, 64)
  }
#undef TH_B
  return fail(SAE_EUNSUPPORTED, "talking heads: no kernel for dtype %d head_dim %d", d->dtype, d->head_dim);
}

// ==================================================================================== C ABI
// one gemm_dw launch (with or without the bias column sums), NG wave groups per workgroup
template <class XL, class YL, int NG>
static int dw_launch(const DwArgs& a, bool bias, long long grid, size_t lds, hipStream_t st) {
  const void* fn = bias ? (const void*)gemm_dw_kernel<true, XL, YL, NG> : (const void*)gemm_dw_kernel<false, XL, YL, NG>;
  if (int rc = lds_attr(fn, lds)) return rc;
  if (bias)
    hipLaunchKernelGGL((gemm_dw_kernel<true, XL, YL, NG>), dim3((unsigned)grid), dim3(256 * NG), lds, st, a);
  else
    hipLaunchKernelGGL((gemm_dw_kernel<false, XL, YL, NG>), dim3((unsigned)grid), dim3(256 * NG), lds, st, a);
  return 0;
}

// the LDS-DMA form of the plain weight-gradient kernel (gemm_dw8.h)
template <int NG, int NS = kDw8NS, int STAG = 0>
static int dw8_launch(const DwArgs& a, bool bias, long long grid, hipStream_t st) {
  constexpr int lds = dw8_lds_bytes<NG, NS>();
  const void* fn = bias ? (const void*)gemm_dw8_kernel<true, NG, NS, STAG> : (const void*)gemm_dw8_kernel<false, NG, NS, STAG>;
  if (int rc = lds_attr(fn, lds)) return rc;
  if (bias)
    hipLaunchKernelGGL((gemm_dw8_kernel<true, NG, NS, STAG>), dim3((unsigned)grid), dim3(256 * NG), lds, st, a);
  else
    hipLaunchKernelGGL((gemm_dw8_kernel<false, NG, NS, STAG>), dim3((unsigned)grid), dim3(256 * NG), lds, st, a);
  return 0;
}

// one sae_gemm_nt launch: TM x 128 tiles, two LDS stage buffers of BK-deep A and B images
template <int EPI, class AL>
static int nt_launch(const NtArgs& g, long long grid, hipStream_t st) {
  size_t lds = 2 * (NtRows<AL>::value + kNtT) * NtDepth<AL>::value * 2;
  if constexpr (NtIsDma<AL>::value) lds = (size_t)AL::kNB * 2 * kNtT * 32 * 2;
  if (int rc = lds_attr((const void*)gemm_nt_kernel<EPI, AL>, lds)) return rc;
  hipLaunchKernelGGL((gemm_nt_kernel<EPI, AL>), dim3((unsigned)grid), dim3(256), lds, st, g);
  return 0;
}

// compute units of the current device (persistent grids), cached per device
static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

// tile height of a gemm8 / gemm8x launch: 224 where 256-row tiles quantize worse onto the CUs --
// cost = rounds of tiles over the CUs x rows per tile (M = 25,216 into 384 features: 198 tiles of
// 256 rows, one round on 256 CUs with 58 idle, vs 226 of 224 rows; M = 18,464 into 768: 219 vs 249)
static int g8_pick_bm(int M, int N, int BN) {
#ifdef SAE_DEV_KNOBS
  if (dev_knob("SAE_NT_BM256")) return 256;
#endif
  const long long G = device_cus(), tn = (N + BN - 1) / BN;
  auto cost = [&](int bm) { return ((((long long)M + bm - 1) / bm * tn + G - 1) / G) * bm; };
  return cost(224) < cost(256) ? 224 : 256;
}

// Work-stealing counters of the persistent gemm8 launches (gemm8.h, DYN; dev builds): 8 group tickets
// and a done word per slot, each on a 128-byte line of its own; a slot belongs to one stream (launches on one
// stream are ordered, so a slot is never used by two running launches; the last workgroup of a
// launch resets it).  A graph captured on a stream keeps that stream's slot in its kernel nodes.
#ifdef SAE_DEV_KNOBS
constexpr int kG8Slots = 64, kG8SlotWords = 288;   // 8 group tickets + done, 128 bytes apart
__device__ unsigned g_g8_ctr[kG8Slots * kG8SlotWords];

static unsigned* g8_slot(hipStream_t st) {
  static std::mutex mu;
  static hipStream_t owner[64][kG8Slots];
  static int used[64] = {0};
  static unsigned* base[64] = {nullptr};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (!base[dev]) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_g8_ctr)) != hipSuccess) return nullptr;
    base[dev] = reinterpret_cast<unsigned*>(p);
  }
  for (int i = 0; i < used[dev]; ++i)
    if (owner[dev][i] == st) return base[dev] + kG8SlotWords * i;
  if (used[dev] == kG8Slots) return nullptr;   // more streams than slots: the static walk
  owner[dev][used[dev]] = st;
  return base[dev] + kG8SlotWords * used[dev]++;
}
#endif

// one persistent gemm8 launch (BM x BN tiles, one 8-wave workgroup per CU).  The work-stealing walk
// (DYN, dev builds: SAE_G8_DYN=1) measured 3 % slower on the DeiT-S step and no better under the
// one-GPU RCCL contention emulation (profiles/r06c_g8_dyn_ab.txt), so the release walk is static.
template <int EPI, int BN, int BK, int NS, int BM, int WGM = 2, bool XW = false>
static int g8_launch_bm(const NtArgs& g0, hipStream_t st) {
  constexpr int lds = g8_lds_bytes<BN, BK, NS, WGM>() + kG8TickBytes;
  const long long tiles = (long long)((g0.M + BM - 1) / BM) * ((g0.N + BN - 1) / BN);
  const long long grid = std::min<long long>(tiles, device_cus());
  NtArgs g = g0;
  // epilogue stores non-temporal except for the gelu' multiply on 2 x 4 waves (whose 96-byte row segments then
  // left L2 unmerged: 77 -> 102 MB written); DeiT-S step 8.02 -> 7.96 ms with every epilogue
  // non-temporal, the plain / GELU launches faster and the multiply slower (profiles/r06z_g8_nts_ab.txt).
  // The multiply's aux (gelu'(h)) tile loaded non-temporal: level in isolation, DeiT-S step
  // 8.01 -> 7.85 ms (profiles/r06z4_g8_aux_nt_ab.txt)
  g.nts = ((EPI != kEpiDGelu || WGM == 4) && !dev_knob("SAE_G8_NO_NTS") ? 1 : 0) | (!dev_knob("SAE_G8_NO_AUX_NT") ? 2 : 0);
#ifdef SAE_DEV_KNOBS
  g.ctr = (NS == 2 && tiles > grid && grid >= 8 && dev_knob("SAE_G8_DYN")) ? g8_slot(st) : nullptr;
  if (g.ctr) {
    if constexpr (NS == 2) {
      if (int rc = lds_attr((const void*)gemm8_nt_kernel<EPI, BN, BK, NS, 0, BM, true>, lds)) return rc;
      hipLaunchKernelGGL((gemm8_nt_kernel<EPI, BN, BK, NS, 0, BM, true>), dim3((unsigned)grid), dim3(512), lds, st, g);
      return 0;
    }
  }
#endif
  if (int rc = lds_attr((const void*)gemm8_nt_kernel<EPI, BN, BK, NS, 0, BM, false, WGM, XW>, lds)) return rc;
  hipLaunchKernelGGL((gemm8_nt_kernel<EPI, BN, BK, NS, 0, BM, false, WGM, XW>), dim3((unsigned)grid), dim3(512), lds, st, g);
  return 0;
}
template <int EPI, int BN, int BK, int NS>
static int g8_launch(const NtArgs& g, hipStream_t st) {
#ifdef SAE_DEV_KNOBS
  if constexpr (BK == 64 && NS == 2) {   // dev A/B: 32-deep stages, 4-deep ring (three stages in flight)
    if (dev_knob("SAE_G8_DEPTH") == 1)
      return g8_pick_bm(g.M, g.N, BN) == 224 ? g8_launch_bm<EPI, BN, 32, 4, 224>(g, st)
                                             : g8_launch_bm<EPI, BN, 32, 4, 256>(g, st);
  }
#endif
  // plain 192-wide tiles: whole-row epilogue stores through the shared row image (XW): QKV forward
  // 32.9 -> 31.4 us, DeiT-S step -0.13 % (profiles/r06xw_g8_xw_ab.txt)
  if constexpr (EPI == kEpiNone && BN == 192)
    if (!dev_knob("SAE_G8_NO_XW"))
      return g8_pick_bm(g.M, g.N, BN) == 224 ? g8_launch_bm<EPI, BN, BK, NS, 224, 2, true>(g, st)
                                             : g8_launch_bm<EPI, BN, BK, NS, 256, 2, true>(g, st);
  return g8_pick_bm(g.M, g.N, BN) == 224 ? g8_launch_bm<EPI, BN, BK, NS, 224>(g, st)
                                         : g8_launch_bm<EPI, BN, BK, NS, 256>(g, st);
}

// GELU forward at K < 768 (the epilogue's VALU work, which scales with the outputs, outweighs the
// reduction): 256 x 128 tiles when they put fewer outputs on the busiest CU than 224 / 256 x 192 --
// DeiT-S / CaiT-S FF Dense_0 (M 25,216 / 25,088 into 1,536): 5 rounds of 32 K outputs against 4 of
// 43 K, 68.0 -> 63.8 us same box (profiles/r05ai_g8_bn128_ab.txt; the GELU' input gradient measured
// level, so it keeps the 192-wide tiles)
static bool g8_gelu_bn128(int M, int N, int K) {
  if (K >= 768 || N % 128 || dev_knob("SAE_G8_NO_BN128")) return false;
  const long long G = device_cus();
  const int bm = g8_pick_bm(M, N, 192);
  const long long c192 = (((long long)(M + bm - 1) / bm * ((N + 191) / 192) + G - 1) / G) * bm * 192;
  const long long c128 = (((long long)(M + 255) / 256 * (N / 128) + G - 1) / G) * 256 * 128;
  return c128 < c192;
}

// one gemm8x launch (BM x BN tiles, ping-pong wave groups, one tile per workgroup)
template <int EPI, int BN, int BM>
static int g8x_launch_bm(const NtArgs& g, hipStream_t st) {
  constexpr int lds = g8x_lds_bytes<BN, BM>();
  if (int rc = lds_attr((const void*)gemm8x_nt_kernel<EPI, BN, true, BM>, lds)) return rc;
  const long long tiles = (long long)((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm8x_nt_kernel<EPI, BN, true, BM>), dim3((unsigned)tiles), dim3(512), lds, st, g);
  return 0;
}
template <int EPI, int BN>
static int g8x_launch(const NtArgs& g, hipStream_t st) {
  return g8_pick_bm(g.M, g.N, BN) == 224 ? g8x_launch_bm<EPI, BN, 224>(g, st) : g8x_launch_bm<EPI, BN, 256>(g, st);
}

// Kernel choice for sae_gemm_nt (round 5: a rule on tile fill and reduction depth instead of the
// BASELINE shape whitelist; every width in create_model.py:6-215 routes to one of these):
//   gemm8x  (ping-pong 256 x 256 tiles): reductions K >= 768 into outputs that fill 256-wide tiles
//           but not 192-wide ones (N % 256 == 0 and N % 192 != 0: ViT-L 1024 / 4096, CvT-W24 1024),
//           plus the 768-feature outputs (ViT-B / CaiT-M output projection, QKV / Dense_0 input
//           gradients, Dense_1 forward; 0.90-0.98 of the library, profiles/r04i_g8probe.txt);
//   gemm8   (persistent 224/256 x 192 tiles): outputs that fill 192-wide tiles (N % 192 == 0) at
//           K >= 384 -- every DeiT-S / CaiT-S projection, the ViT-B wide K = 768 forwards;
//   128-row sae_gemm_nt: the rest -- small M (classifier heads, CLS rows), K < 384 (DeiT-Ti, the
//           C = 192 widths), K not a multiple of 64 (KT instances: CaiT-XXS / XS 288, CvT 368, TNT
//           inner 24 / 40 and their FF widths), the GELU' epilogue beyond K = 384 (its 256-token
//           tile), N not a multiple of 192 or 256.
// Both persistent kernels need M >= 4096 (enough tiles to fill the CUs) and K % 64 == 0.
static bool g8x_route(int M, int N, int K, int epilogue) {
  if (epilogue == SAE_EPI_DGELU || K < 768 || K % 64 || M < 4096 || N % 256) return false;
  return N == 768 || N % 192 != 0;
}

// gemm8 (gemm8.h) or the 128-row sae_gemm_nt: tools/probe/gemm8_probe.py, profiles/r04c_g8probe.txt --
// gemm8 wins on the 384-feature outputs at every depth (DeiT-S / CaiT output projection, QKV and
// FF Dense_0 input gradients, Dense_1 forward: 412-692 -> 497-849 TF/s) and on the wide K = 768
// ViT-B forwards (QKV 2304 features 750 -> 850-900, FF Dense_0 + GELU 673-700 -> 715-729: level with
// the library's 830-960); the 128-row kernel stays on the DeiT-S wide K = 384 outputs (a tie) and
// the GELU' epilogue (gemm8 has none)
// Round 4 (224-row tiles, g8_pick_bm): also the DeiT-S / CaiT wide K = 384 outputs -- QKV forward
// 593 -> 647 TF/s, FF Dense_0 + GELU 546 -> 563, Dense_1 input gradient with GELU' 497 -> 509
// (profiles/r04k_g8probe.txt, v53 vs rel)
// Round 5: with the saved-gelu' multiply epilogue (SAE_EPI_MUL_AUX, `gp`) the GELU' epilogue no
// longer bounds the deeper ViT-B input gradient either, so gemm8 takes it at every K.
static bool g8_route(int M, int N, int K, int epilogue, bool gp = false) {
  if (N % 192 || K % 64 || K < 384 || M < 4096) return false;
  return epilogue != SAE_EPI_DGELU || K == 384 || (gp && !dev_knob("SAE_G8_NO_MUL"));
}

extern "C" {

void sae_attn_desc_init(sae_attn_desc* d, int32_t batch, int32_t heads, int32_t seq_q, int32_t seq_k,
                        int32_t head_dim, int32_t dtype, float scale) {
  memset(d, 0, sizeof *d);
  d->batch = batch;
  d->heads = heads;
  d->seq_q = seq_q;
  d->seq_k = seq_k;
  d->head_dim = head_dim;
  d->dtype = dtype;
  d->scale = scale;
  const int64_t hq[3] = {(int64_t)seq_q * heads * head_dim, (int64_t)heads * head_dim, head_dim};
  const int64_t hk[3] = {(int64_t)seq_k * heads * head_dim, (int64_t)heads * head_dim, head_dim};
  for (int i = 0; i < 3; ++i) {
    d->q_stride[i] = d->o_stride[i] = d->do_stride[i] = d->dq_stride[i] = hq[i];
    d->k_stride[i] = d->v_stride[i] = d->dk_stride[i] = d->dv_stride[i] = hk[i];
  }
}

// rotary tables of the _rotary entry points: fp32 [max(seq_q, seq_k)][head_dim / 2]
static int rope_check(const sae_attn_desc* d, const float* sin_tab, const float* cos_tab) {
  if (!sin_tab || !cos_tab) return fail(SAE_EINVAL, "rotary: sin_tab / cos_tab must be non-NULL");
  if (!aligned16(sin_tab) || !aligned16(cos_tab)) return fail(SAE_EINVAL, "rotary: tables must be 16-byte aligned");
  if (d->head_dim % 8 || d->head_dim > 64)
    return fail(SAE_EUNSUPPORTED, "rotary: fused rotary needs head_dim %% 8 == 0 and <= 64 (got %d)", d->head_dim);
  return SAE_OK;
}
static RopeTab make_rope(const sae_attn_desc* d, const float* sin_tab, const float* cos_tab) {
  RopeTab t;
  t.sin = sin_tab;
  t.cos = cos_tab;
  t.P = d->head_dim / 2;
  t.n = std::max(d->seq_q, d->seq_k);
  return t;
}

static int attn_fwd_impl(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                         const float* bias_h, const float* bias_w, void* o, float* lse, const RopeTab* rope);

int sae_attn_fwd(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                 const float* bias_h, const float* bias_w, void* o, float* lse) {
  return attn_fwd_impl(stream, d, q, k, v, bias_h, bias_w, o, lse, nullptr);
}

int sae_attn_fwd_rotary(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                        const float* sin_tab, const float* cos_tab, void* o, float* lse) {
  if (!d) return fail(SAE_EINVAL, "NULL descriptor");
  if (int rc = rope_check(d, sin_tab, cos_tab)) return rc;
  const RopeTab t = make_rope(d, sin_tab, cos_tab);
  return attn_fwd_impl(stream, d, q, k, v, nullptr, nullptr, o, lse, &t);
}

static int attn_fwd_impl(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                         const float* bias_h, const float* bias_w, void* o, float* lse, const RopeTab* rope) {
  int rc = validate(d, false);
  if (rc) return rc;
  if (!q || !k || !v || !o) return fail(SAE_EINVAL, "q/k/v/o must be non-NULL");
  const bool rel = d->flags & SAE_FLAG_RELPOS;
  if (rel && (!bias_h || !bias_w)) return fail(SAE_EINVAL, "SAE_FLAG_RELPOS needs bias_h and bias_w");
  AttnArgs a;
  fill_args(a, d);
  a.q = q;
  a.k = k;
  a.v = v;
  a.out = o;
  a.lse = lse;
  a.bias_h = bias_h;
  a.bias_w = bias_w;
  const int epc = 16 / elem_size(d->dtype);
  const bool vec = d->head_dim % epc == 0 && strides_vec(d->q_stride, epc) && strides_vec(d->k_stride, epc) &&
                   strides_vec(d->v_stride, epc) && strides_vec(d->o_stride, epc) && aligned16(q) &&
                   aligned16(k) && aligned16(v) && aligned16(o);
  const int var = dev_knob("SAE_FWD_VARIANT");
  if (rope) {   // rotary rides on the lean bf16 kernels only, in the envelope of sae_attn_bwd_rotary
    const int dp = pick_dp(d->head_dim);
    if (d->dtype != SAE_DTYPE_BF16 || !vec || rel || d->flags || dp > 64)
      return fail(SAE_EUNSUPPORTED, "rotary: fused only on the bf16 path with head_dim <= 64 (16-byte aligned "
                  "strides, no flags)");
    a.rope = *rope;
    if (dp == 32) return fwd2_dispatch<32, true>((hipStream_t)stream, a, 0);
    return fwd2_dispatch<64, true>((hipStream_t)stream, a, 0);
  }
  if (var != 1 && vec && cls_ok(d)) return cls_run<false>((hipStream_t)stream, a);
  if (var != 1 && d->dtype == SAE_DTYPE_BF16 && vec && !rel) {
    const int dp = pick_dp(d->head_dim);
    if (dp == 32) return fwd2_dispatch<32>((hipStream_t)stream, a, var);
    if (dp == 64) return fwd2_dispatch<64>((hipStream_t)stream, a, var);
    if (dp == 128) return fwd2_dispatch<128>((hipStream_t)stream, a, var);
  }
  if (var != 1 && d->dtype == SAE_DTYPE_BF16 && vec && rel && rel_lean(a)) {   // BoTNet
    const int dp = pick_dp(d->head_dim);
    hipStream_t st = (hipStream_t)stream;
    if (dp == 32) return fwd2_run<32, 4, 2, true, false, 2, true>(st, a);
    if (dp == 64) return fwd2_run<64, 4, 2, true, false, 4, true>(st, a);
    return fwd2_run<128, 4, 2, true, false, 8, true>(st, a);
  }
  return dispatch<FwdL>(d->dtype, pick_dp(d->head_dim), vec, rel, (hipStream_t)stream, a);
}

static size_t delta_bytes(const sae_attn_desc* d) {
  return (((size_t)d->batch * d->heads * d->seq_q * sizeof(float)) + 255) & ~(size_t)255;
}

size_t sae_attn_bwd_workspace_bytes(const sae_attn_desc* d) {
  if (!d) return 0;
  return delta_bytes(d);   // delta [B, H, Nq]
}

static int attn_bwd_impl(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                         const void* o, const float* lse, const void* dout, const float* bias_h,
                         const float* bias_w, void* dq, void* dk, void* dv, float* dbias_h, float* dbias_w,
                         void* workspace, const RopeTab* rope);

int sae_attn_bwd(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                 const void* o, const float* lse, const void* dout, const float* bias_h, const float* bias_w,
                 void* dq, void* dk, void* dv, float* dbias_h, float* dbias_w, void* workspace) {
  return attn_bwd_impl(stream, d, q, k, v, o, lse, dout, bias_h, bias_w, dq, dk, dv, dbias_h, dbias_w, workspace,
                       nullptr);
}

int sae_attn_bwd_rotary(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                        const void* o, const float* lse, const void* dout, const float* sin_tab,
                        const float* cos_tab, void* dq, void* dk, void* dv, void* workspace) {
  if (!d) return fail(SAE_EINVAL, "NULL descriptor");
  if (int rc = rope_check(d, sin_tab, cos_tab)) return rc;
  const RopeTab t = make_rope(d, sin_tab, cos_tab);
  return attn_bwd_impl(stream, d, q, k, v, o, lse, dout, nullptr, nullptr, dq, dk, dv, nullptr, nullptr, workspace,
                       &t);
}

static int attn_bwd_impl(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                         const void* o, const float* lse, const void* dout, const float* bias_h,
                         const float* bias_w, void* dq, void* dk, void* dv, float* dbias_h, float* dbias_w,
                         void* workspace, const RopeTab* rope) {
  int rc = validate(d, true);
  if (rc) return rc;
  if (!q || !k || !v || !o || !lse || !dout || !dq || !dk || !dv || !workspace)
    return fail(SAE_EINVAL, "q/k/v/o/lse/dout/dq/dk/dv/workspace must be non-NULL");
  const bool rel = d->flags & SAE_FLAG_RELPOS;
  if (rel && (!bias_h || !bias_w || !dbias_h || !dbias_w))
    return fail(SAE_EINVAL, "SAE_FLAG_RELPOS needs bias_h, bias_w, dbias_h, dbias_w");
  AttnArgs a;
  fill_args(a, d);
  a.q = q;
  a.k = k;
  a.v = v;
  a.o = o;
  a.lse = const_cast<float*>(lse);
  a.dout = dout;
  a.dq = dq;
  a.dk = dk;
  a.dv = dv;
  a.delta = reinterpret_cast<float*>(workspace);
  a.bias_h = bias_h;
  a.bias_w = bias_w;
  a.dbias_h = dbias_h;
  a.dbias_w = dbias_w;
  const int epc = 16 / elem_size(d->dtype);
  const bool vec = d->head_dim % epc == 0 && strides_vec(d->q_stride, epc) && strides_vec(d->k_stride, epc) &&
                   strides_vec(d->v_stride, epc) && strides_vec(d->o_stride, epc) &&
                   strides_vec(d->do_stride, epc) && strides_vec(d->dq_stride, epc) &&
                   strides_vec(d->dk_stride, epc) && strides_vec(d->dv_stride, epc) && aligned16(q) &&
                   aligned16(k) && aligned16(v) && aligned16(o) && aligned16(dout) && aligned16(dq) &&
                   aligned16(dk) && aligned16(dv);
  const int var = dev_knob("SAE_BWD_VARIANT");
  if (rope) {   // rotary rides on the lean bf16 kernels only
    const int dp = pick_dp(d->head_dim);
    if (d->dtype != SAE_DTYPE_BF16 || !vec || rel || d->flags || dp > 64)
      return fail(SAE_EUNSUPPORTED, "rotary: fused only on the bf16 path with head_dim <= 64 (16-byte aligned "
                  "strides, no flags)");
    a.rope = *rope;
    hipStream_t st = (hipStream_t)stream;
    if (a.Nk <= kB3Keys)
      return dp == 32 ? bwd3_run<32, 8, 1, true, 2, true>(st, a) : bwd3_run<64, 8, 1, true, 4, true>(st, a);
    return dp == 32 ? bwd2_run_default<32, true>(st, a) : bwd2_run_default<64, true>(st, a);
  }
  if (var != 1 && vec && cls_ok(d)) return cls_run<true>((hipStream_t)stream, a);
  if (var != 1 && d->dtype == SAE_DTYPE_BF16 && vec && !rel) {
    const int dp = pick_dp(d->head_dim);
    hipStream_t st = (hipStream_t)stream;
    if (a.Nk <= kB3Keys && var != 2 && var < 10 && dp <= 64) {
#ifdef SAE_DEV_KNOBS
      if (var == 3) {   // four waves x two 32-key sub-blocks (one wave per SIMD): measured slower
        if (dp == 32) return bwd3_run<32, 4, 2>(st, a);
        if (dp == 64) return bwd3_run<64, 4, 2>(st, a);
      }
      if (var >= 5 && var <= 7 && dp == 64) {   // no stagger / stagger + priority / priority only
        const bool d48 = d->head_dim <= 48;
        if (var == 5) return d48 ? bwd3_run<64, 8, 1, false, 3>(st, a) : bwd3_run<64, 8, 1, false, 4>(st, a);
        if (var == 6) return d48 ? bwd3_run<64, 8, 1, false, 3, true, true>(st, a) : bwd3_run<64, 8, 1, false, 4, true, true>(st, a);
        return d48 ? bwd3_run<64, 8, 1, false, 3, false, true>(st, a) : bwd3_run<64, 8, 1, false, 4, false, true>(st, a);
      }
#endif
      // waves 4-7 staggered (the previous tile's dQ first): DeiT-S 53.6 -> 53.2 us, CaiT-S24
      // 130.7 -> 128.3 us (profiles/r06g_bwd3_stagger_ab.txt; same sums, bit-identical results)
      if (dp == 32) return bwd3_run<32, 8, 1, false, 2, true>(st, a);
      if (dp == 64 && d->head_dim <= 48) return bwd3_run<64, 8, 1, false, 3, true>(st, a);   // CaiT head_dim 48
      if (dp == 64) return bwd3_run<64, 8, 1, false, 4, true>(st, a);
    }
#ifdef SAE_DEV_KNOBS
    if (dp == 64 && (var == 10 || var == 11)) return bwd2_run_agpr<64>(st, a, var == 11);
#endif
    if (dp == 32) return bwd2_run_default<32>(st, a);
    if (dp == 64) return bwd2_run_default<64>(st, a);
#ifdef SAE_DEV_KNOBS
    if (var == 30) {
      const hipError_t e = bwd2_agpr128(st, a, false, 0);
      return e == hipSuccess ? ok() : fail(SAE_EHIP, "bwd2 agpr: %s", hipGetErrorString(e));
    }
    if (var == 32) return bwd2_run<128, 4, 1, 4, 1>(st, a);
#endif
    // head_dim 128 (BoTNet): the dK / dV pass at one wave per SIMD (the dK / dV accumulators of 32
    // keys x 128 columns plus the K / V fragments need more than half the register file), built in
    // the AGPR translation unit (bwd_agpr.hip: accumulators in AGPRs, no spills; bot14 bwd
    // 222 -> 216 us, bot7 49 -> 47 us same box, profiles/r03f_bot_agpr_ab.txt)
    {
      const hipError_t e = bwd2_agpr128(st, a, false, 1);
      return e == hipSuccess ? ok() : fail(SAE_EHIP, "attn_bwd2 (head_dim 128): %s", hipGetErrorString(e));
    }
  }
  if (var != 1 && d->dtype == SAE_DTYPE_BF16 && vec && rel && rel_lean(a)) {   // BoTNet relative logits
    const int dp = pick_dp(d->head_dim);
    hipStream_t st = (hipStream_t)stream;
    if (dp == 32) return bwd2_run<32, 4, 2, 4, 2, false, true>(st, a);
    if (dp == 64) return bwd2_run<64, 4, 2, 4, 1, false, true>(st, a);
    // head_dim 128 with relative logits: at 14 x 14 both passes at one wave per SIMD in the AGPR
    // unit (the dQ pass's relative-logit state spills 75 VGPRs at two waves per SIMD): bot14+rel
    // bwd 315 -> 298 us; the 7 x 7 grid keeps the two-wave dQ pass (59 vs 67 us)
    if (a.Nk >= 128) {
      const hipError_t e = bwd2_agpr128(st, a, true, 0);
      return e == hipSuccess ? ok() : fail(SAE_EHIP, "attn_bwd2 (relpos, head_dim 128): %s", hipGetErrorString(e));
    }
    return bwd2_run<128, 4, 2, 4, 1, false, true>(st, a);
  }
  return dispatch<BwdL>(d->dtype, pick_dp(d->head_dim), vec, rel, (hipStream_t)stream, a);
}

// ------------------------------------------------------------------------- relative logits
static int rel_validate(int B, int H, int Hs, int Ws, int D, int dtype) {
  if (B < 1 || H < 1 || Hs < 1 || Ws < 1 || D < 1) return fail(SAE_EINVAL, "relpos sizes must be >= 1");
  if (dtype != SAE_DTYPE_BF16 && dtype != SAE_DTYPE_F32) return fail(SAE_EINVAL, "bad dtype %d", dtype);
  if (Hs > 64 || Ws > 64) return fail(SAE_EUNSUPPORTED, "relpos grid %dx%d exceeds 64x64", Hs, Ws);
  return SAE_OK;
}

int sae_relpos_bias_fwd(void* stream, int32_t B, int32_t H, int32_t Hs, int32_t Ws, int32_t D, int32_t dtype,
                        const void* qhat, const int64_t qs[3], const float* eh, const float* ew, float* bias_h,
                        float* bias_w) {
  int rc = rel_validate(B, H, Hs, Ws, D, dtype);
  if (rc) return rc;
  if (!qhat || !qs || !eh || !ew || !bias_h || !bias_w) return fail(SAE_EINVAL, "NULL argument");
  RelArgs a;
  memset(&a, 0, sizeof a);
  a.qhat = qhat;
  for (int i = 0; i < 3; ++i) a.qs[i] = qs[i];
  a.eh = eh;
  a.ew = ew;
  a.bias_h = bias_h;
  a.bias_w = bias_w;
  a.B = B;
  a.H = H;
  a.Hs = Hs;
  a.Ws = Ws;
  a.D = D;
  const long long n = (long long)B * H * Hs * Ws * (Hs + Ws);
  const dim3 g((unsigned)((n + 255) / 256));
  if (dtype == SAE_DTYPE_BF16)
    hipLaunchKernelGGL(relpos_bias_fwd_kernel<__bf16>, g, dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(relpos_bias_fwd_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("relpos_bias_fwd");
}

size_t sae_relpos_bias_bwd_workspace_bytes(int32_t B, int32_t Hs, int32_t Ws, int32_t D) {
  if (B < 1 || Hs < 1 || Ws < 1 || D < 1) return 0;
  return (((size_t)B * ((2 * Hs - 1) + (2 * Ws - 1)) * D * sizeof(float)) + 255) & ~(size_t)255;
}

int sae_relpos_bias_bwd(void* stream, int32_t B, int32_t H, int32_t Hs, int32_t Ws, int32_t D, int32_t dtype,
                        const void* qhat, const int64_t qs[3], const float* eh, const float* ew,
                        const float* dbias_h, const float* dbias_w, const void* dq_in, void* dq_out,
                        const int64_t dqs[3], float* demb_h, float* demb_w, void* workspace) {
  int rc = rel_validate(B, H, Hs, Ws, D, dtype);
  if (rc) return rc;
  if (!qhat || !qs || !eh || !ew || !dbias_h || !dbias_w || !dq_out || !dqs || !demb_h || !demb_w || !workspace)
    return fail(SAE_EINVAL, "NULL argument");
  RelArgs a;
  memset(&a, 0, sizeof a);
  a.qhat = qhat;
  for (int i = 0; i < 3; ++i) {
    a.qs[i] = qs[i];
    a.dqs[i] = dqs[i];
  }
  a.eh = eh;
  a.ew = ew;
  a.dbias_h = dbias_h;
  a.dbias_w = dbias_w;
  a.dq_in = dq_in;
  a.dq_out = dq_out;
  a.demb_h = demb_h;
  a.demb_w = demb_w;
  a.part = reinterpret_cast<float*>(workspace);
  a.B = B;
  a.H = H;
  a.Hs = Hs;
  a.Ws = Ws;
  a.D = D;
  hipStream_t st = (hipStream_t)stream;
  const long long n1 = (long long)B * Hs * Ws * H * D;
  const long long n2 = (long long)B * ((2 * Hs - 1) + (2 * Ws - 1)) * D;
  const int n3 = ((2 * Hs - 1) + (2 * Ws - 1)) * D;
  if (dtype == SAE_DTYPE_BF16) {
    hipLaunchKernelGGL(relpos_bias_bwd_dq_kernel<__bf16>, dim3((unsigned)((n1 + 255) / 256)), dim3(256), 0, st, a);
    hipLaunchKernelGGL(relpos_bias_bwd_emb_partial_kernel<__bf16>, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0,
                       st, a);
  } else {
    hipLaunchKernelGGL(relpos_bias_bwd_dq_kernel<float>, dim3((unsigned)((n1 + 255) / 256)), dim3(256), 0, st, a);
    hipLaunchKernelGGL(relpos_bias_bwd_emb_partial_kernel<float>, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0,
                       st, a);
  }
  hipLaunchKernelGGL(relpos_bias_bwd_emb_reduce_kernel, dim3((unsigned)((n3 + 255) / 256)), dim3(256), 0, st, a);
  return check_launch("relpos_bias_bwd");
}

// ---------------------------------------------------------------------------------- rotary
int sae_rotary(void* stream, int32_t B, int32_t N, int32_t H, int32_t D, int32_t dtype, const void* x,
               const int64_t xs[3], void* y, const int64_t ys[3], const float* sin_t, const float* cos_t,
               int32_t inverse) {
  if (B < 1 || N < 1 || H < 1 || D < 2 || (D & 1)) return fail(SAE_EINVAL, "rotary needs sizes >= 1 and even D");
  if (dtype != SAE_DTYPE_BF16 && dtype != SAE_DTYPE_F32) return fail(SAE_EINVAL, "bad dtype %d", dtype);
  if (!x || !xs || !y || !ys || !sin_t || !cos_t) return fail(SAE_EINVAL, "NULL argument");
  RotArgs a;
  memset(&a, 0, sizeof a);
  a.x = x;
  a.y = y;
  for (int i = 0; i < 3; ++i) {
    a.xs[i] = xs[i];
    a.ys[i] = ys[i];
  }
  a.sin_t = sin_t;
  a.cos_t = cos_t;
  a.B = B;
  a.N = N;
  a.H = H;
  a.D = D;
  a.sgn = inverse ? -1.f : 1.f;
  const long long n = (long long)B * N * H * (D / 2);
  const dim3 g((unsigned)((n + 255) / 256));
  if (dtype == SAE_DTYPE_BF16)
    hipLaunchKernelGGL(rotary_kernel<__bf16>, g, dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(rotary_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("rotary");
}

// --------------------------------------------------------------------------- talking heads
int sae_th_attn_fwd(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                    const float* th1, const float* th2, void* o, float* lse) {
  int rc = validate(d, false);
  if (rc) return rc;
  if (d->flags) return fail(SAE_EINVAL, "talking heads takes no flags");
  if (!q || !k || !v || !th1 || !th2 || !o || !lse) return fail(SAE_EINVAL, "NULL argument");
  if (d->heads > SAE_TH_MAX_HEADS || d->head_dim > SAE_TH_MAX_HEAD_DIM)
    return fail(SAE_EUNSUPPORTED, "talking heads needs heads <= %d and head_dim <= %d", SAE_TH_MAX_HEADS,
                SAE_TH_MAX_HEAD_DIM);
  if (int rc = th_fwd(stream, d, q, k, v, th1, th2, o, lse)) return rc;
  return ok();
}

size_t sae_th_attn_bwd_workspace_bytes(const sae_attn_desc* d) {
  if (!d) return 0;
  return th_bwd_workspace_bytes(d);
}

int sae_th_attn_bwd(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                    const float* th1, const float* th2, const float* lse, const void* dout, void* dq, void* dk,
                    void* dv, float* dth1, float* dth2, void* workspace) {
  int rc = validate(d, true);
  if (rc) return rc;
  if (d->flags) return fail(SAE_EINVAL, "talking heads takes no flags");
  if (!q || !k || !v || !th1 || !th2 || !lse || !dout || !dq || !dk || !dv || !dth1 || !dth2 || !workspace)
    return fail(SAE_EINVAL, "NULL argument");
  if (d->heads > SAE_TH_MAX_HEADS || d->head_dim > SAE_TH_MAX_HEAD_DIM)
    return fail(SAE_EUNSUPPORTED, "talking heads needs heads <= %d and head_dim <= %d", SAE_TH_MAX_HEADS,
                SAE_TH_MAX_HEAD_DIM);
  if (int rc = th_bwd(stream, d, q, k, v, th1, th2, lse, dout, dq, dk, dv, dth1, dth2, workspace)) return rc;
  return ok();
}

int sae_th_attn_fwd_rotary(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                           const float* th1, const float* th2, const float* sin_tab, const float* cos_tab, void* o,
                           float* lse) {
  int rc = validate(d, false);
  if (rc) return rc;
  if (d->flags) return fail(SAE_EINVAL, "talking heads takes no flags");
  if (!q || !k || !v || !th1 || !th2 || !o || !lse) return fail(SAE_EINVAL, "NULL argument");
  if (d->heads > SAE_TH_MAX_HEADS || d->head_dim > SAE_TH_MAX_HEAD_DIM)
    return fail(SAE_EUNSUPPORTED, "talking heads needs heads <= %d and head_dim <= %d", SAE_TH_MAX_HEADS,
                SAE_TH_MAX_HEAD_DIM);
  if (int rc2 = rope_check(d, sin_tab, cos_tab)) return rc2;
  const RopeTab t = make_rope(d, sin_tab, cos_tab);
  if (int rc2 = th_fwd(stream, d, q, k, v, th1, th2, o, lse, &t)) return rc2;
  return ok();
}

int sae_th_attn_bwd_rotary(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v,
                           const float* th1, const float* th2, const float* lse, const void* dout,
                           const float* sin_tab, const float* cos_tab, void* dq, void* dk, void* dv, float* dth1,
                           float* dth2, void* workspace) {
  int rc = validate(d, true);
  if (rc) return rc;
  if (d->flags) return fail(SAE_EINVAL, "talking heads takes no flags");
  if (!q || !k || !v || !th1 || !th2 || !lse || !dout || !dq || !dk || !dv || !dth1 || !dth2 || !workspace)
    return fail(SAE_EINVAL, "NULL argument");
  if (d->heads > SAE_TH_MAX_HEADS || d->head_dim > SAE_TH_MAX_HEAD_DIM)
    return fail(SAE_EUNSUPPORTED, "talking heads needs heads <= %d and head_dim <= %d", SAE_TH_MAX_HEADS,
                SAE_TH_MAX_HEAD_DIM);
  if (int rc2 = rope_check(d, sin_tab, cos_tab)) return rc2;
  const RopeTab t = make_rope(d, sin_tab, cos_tab);
  if (int rc2 = th_bwd(stream, d, q, k, v, th1, th2, lse, dout, dq, dk, dv, dth1, dth2, workspace, &t)) return rc2;
  return ok();
}

// ------------------------------------------------------------------ projection gradients
static void dw_plan(int M, int I, int J, int* S, int* chunk, int slots = 512) {
  // at most `slots` workgroups = one resident round (512: 2 per CU x 256 CUs; 256 for the 8-wave
  // two-group kernel): a 513th would run alone in a second round (the old ceil() rule launched
  // 513 / 540 / 513 for the DeiT-S QKV / FF / output projections).  A smaller slot count gives
  // fewer splits, so the 512-slot plan's workspace bounds every plan's.
  const int tiles = ((I + kDwT - 1) / kDwT) * ((J + kDwT - 1) / kDwT);
  int s = slots / tiles;
  s = std::max(1, std::min(s, (M + 255) / 256));
  int c = (M + s - 1) / s;
  c = (c + kDwK - 1) / kDwK * kDwK;
  *chunk = c;
  *S = (M + c - 1) / c;
}

size_t sae_gemm_dw_workspace_bytes(int32_t M, int32_t I, int32_t J) {
  if (M < 1 || I < 1 || J < 1) return 0;
  int S, chunk;
  dw_plan(M, I, J, &S, &chunk);
  return (((size_t)S * I * J * 4 + 255) & ~(size_t)255) + (((size_t)S * J * 4 + 255) & ~(size_t)255);
}

static int gemm_dw_impl(void* stream, int32_t M, int32_t I, int32_t J, const void* x, int64_t ldx, const void* dy,
                        int64_t ldy, float* dw, int64_t ldw, float* db, int32_t accumulate, void* workspace,
                        int32_t jblock);

int sae_gemm_dw(void* stream, int32_t M, int32_t I, int32_t J, const void* x, int64_t ldx, const void* dy,
                int64_t ldy, float* dw, int64_t ldw, float* db, int32_t accumulate, void* workspace) {
  return gemm_dw_impl(stream, M, I, J, x, ldx, dy, ldy, dw, ldw, db, accumulate, workspace, 0);
}

int sae_gemm_dw_blocked(void* stream, int32_t M, int32_t I, int32_t J, int32_t jblock, const void* x, int64_t ldx,
                        const void* dy, int64_t ldy, float* dw, float* db, int32_t accumulate, void* workspace) {
  if (jblock < 4 || jblock % 4 || J % jblock)
    return fail(SAE_EINVAL, "gemm_dw_blocked: jblock (%d) must be a multiple of 4 dividing J (%d)", jblock, J);
  return gemm_dw_impl(stream, M, I, J, x, ldx, dy, ldy, dw, J, db, accumulate, workspace, jblock);
}

static int gemm_dw_impl(void* stream, int32_t M, int32_t I, int32_t J, const void* x, int64_t ldx, const void* dy,
                        int64_t ldy, float* dw, int64_t ldw, float* db, int32_t accumulate, void* workspace,
                        int32_t jblock) {
  if (M < 1 || I < 1 || J < 1) return fail(SAE_EINVAL, "gemm_dw: M/I/J must be >= 1 (got %d/%d/%d)", M, I, J);
  if (I % 8 || J % 8) return fail(SAE_EUNSUPPORTED, "gemm_dw: I (%d) and J (%d) must be multiples of 8", I, J);
  if (ldx < I || ldy < J || ldw < J || ldx % 8 || ldy % 8 || ldw % 4)
    return fail(SAE_EINVAL, "gemm_dw: bad leading dimensions ldx %lld ldy %lld ldw %lld", (long long)ldx,
                (long long)ldy, (long long)ldw);
  if (!x || !dy || !dw || !workspace) return fail(SAE_EINVAL, "gemm_dw: x/dy/dw/workspace must be non-NULL");
  if (!aligned16(x) || !aligned16(dy) || !aligned16(dw) || !aligned16(workspace))
    return fail(SAE_EINVAL, "gemm_dw: x, dy, dw and workspace must be 16-byte aligned");
  DwArgs a;
  memset(&a, 0, sizeof a);
  a.x = reinterpret_cast<const __bf16*>(x);
  a.dy = reinterpret_cast<const __bf16*>(dy);
  a.M = M;
  a.I = I;
  a.J = J;
  // wave groups per workgroup (gemm_dw.h): two for small outputs (<= 64 tiles of 128 x 128: every
  // DeiT-S / CaiT projection), where half the splits still fill the chip and halve the fp32
  // partial traffic (output projection dW + reduce 34.8 -> 30.6 us); one for the larger ViT-B
  // outputs, where halving the splits would leave CUs idle (FF 139 -> 205 us)
  const int tiles = ((I + kDwT - 1) / kDwT) * ((J + kDwT - 1) / kDwT);
  int NG = tiles <= 64 ? 2 : 1;
  int dw8v = 0;   // dev A/B: 1 = one 4-wave group with an 8-deep ring (one workgroup per CU)
#ifdef SAE_DEV_KNOBS
  dw8v = dev_knob("SAE_DW8_VARIANT");
  if (dw8v == 1) NG = 1;
#endif
  dw_plan(M, I, J, &a.S, &a.chunk, dw8v == 1 ? 256 : 512 / NG);
  if ((long long)(a.chunk + 4 * NG * kDwK) * std::max(ldx, ldy) * 2 >= (1LL << 31))
    return fail(SAE_EUNSUPPORTED, "gemm_dw: token chunk exceeds 32-bit buffer addressing");
  a.part = reinterpret_cast<float*>(workspace);
  a.bpart = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) +
                                     (((size_t)a.S * I * J * 4 + 255) & ~(size_t)255));
  a.dw = dw;
  a.db = db;
  a.ldx = ldx;
  a.ldy = ldy;
  a.ldw = ldw;
  a.accumulate = accumulate;
  a.jblock = jblock;
  hipStream_t st = (hipStream_t)stream;
  const long long grid = (long long)a.S * ((I + kDwT - 1) / kDwT) * ((J + kDwT - 1) / kDwT);
  const size_t lds = NG * 4 * kDwK * 256;
  typedef DwRow<false> XR;
  typedef DwRow<true> YR;
  bool dma = true;
#ifdef SAE_DEV_KNOBS
  dma = !dev_knob("SAE_DW_OLD");
#endif
  if (dma && dw8v == 1) {
    if (int rc = dw8_launch<1, 8>(a, db != nullptr, grid, st)) return rc;
#ifdef SAE_DEV_KNOBS
  } else if (dma && NG == 2 && (dw8v == 2 || dw8v == 3)) {   // wave-group offset A/B: none / a whole stage
    if (int rc = dw8v == 2 ? dw8_launch<2, kDw8NS, 0>(a, db != nullptr, grid, st)
                           : dw8_launch<2, kDw8NS, 1>(a, db != nullptr, grid, st))
      return rc;
#endif
  } else if (dma) {
    // two wave groups half a stage apart (STAG 2): DeiT-S step 8.148 -> 8.056 ms same box
    // (profiles/r06h_dw8_stagger_ab.txt); a whole stage apart measured level
    if (int rc = NG == 2 ? dw8_launch<2, kDw8NS, 2>(a, db != nullptr, grid, st) : dw8_launch<1>(a, db != nullptr, grid, st))
      return rc;
  } else if (NG == 2) {
    if (int rc = dw_launch<XR, YR, 2>(a, db != nullptr, grid, lds, st)) return rc;
  } else {
    if (int rc = dw_launch<XR, YR, 1>(a, db != nullptr, grid, lds, st)) return rc;
  }
  if (int rc = check_launch("gemm_dw")) return rc;
  const long long n4 = (long long)I * J / 4;
  const unsigned rb = (unsigned)std::min<long long>((n4 + kDwRedCols - 1) / kDwRedCols, 4096);
  hipLaunchKernelGGL(gemm_dw_reduce_kernel, dim3(rb, db ? 2 : 1), dim3(256), 0, st, a);
  return check_launch("gemm_dw_reduce");
}

// ------------------------------------------------------------------ fp32 projections
// split-K plan: more splits only while the output tiles leave the chip idle and each split keeps
// >= 1,024 of depth (the weight gradients: K = the token count); independent of `colsum` so the
// workspace bound holds for both
static void f32_plan(int M, int N, int K, int* S, int* kchunk) {
  const int tiles = ((M + kF32T - 1) / kF32T) * ((N + kF32T - 1) / kF32T);
  int s = 1;
  if (tiles < 256 && K >= 2048) s = std::min((512 + tiles - 1) / tiles, K / 1024);
  s = std::max(1, std::min(s, 64));
  int c = (K + s - 1) / s;
  c = (c + kF32K - 1) / kF32K * kF32K;
  *kchunk = c;
  *S = (K + c - 1) / c;
}

size_t sae_gemm_f32_workspace_bytes(int32_t M, int32_t N, int32_t K) {
  if (M < 1 || N < 1 || K < 1) return 0;
  int S, c;
  f32_plan(M, N, K, &S, &c);
  return S > 1 ? (size_t)S * (M + 1) * N * 4 : 0;
}

int sae_gemm_f32(void* stream, int32_t M, int32_t N, int32_t K, const float* a, int64_t sam, int64_t sak,
                 const float* b, int64_t sbk, int64_t sbn, const float* bias, float* c, int64_t ldc,
                 float* colsum, int32_t accumulate, void* workspace) {
  if (M < 1 || N < 1 || K < 1) return fail(SAE_EINVAL, "gemm_f32: M/N/K must be >= 1 (got %d/%d/%d)", M, N, K);
  if (!a || !b || !c) return fail(SAE_EINVAL, "gemm_f32: a, b and c must be non-NULL");
  const bool ak = sak == 1, bk = sbk == 1;
  if (ak ? (sam < K || sam % 4 || K % 4) : (sam != 1 || sak < M || sak % 4 || M % 4))
    return fail(SAE_EUNSUPPORTED, "gemm_f32: A needs unit stride along k (sam >= K, K and sam multiples of 4) "
                "or along m (sak >= M, M and sak multiples of 4); got sam %lld sak %lld", (long long)sam,
                (long long)sak);
  if (bk ? (sbn < K || sbn % 4 || K % 4) : (sbn != 1 || sbk < N || sbk % 4 || N % 4))
    return fail(SAE_EUNSUPPORTED, "gemm_f32: B needs unit stride along k (sbn >= K, K and sbn multiples of 4) "
                "or along n (sbk >= N, N and sbk multiples of 4); got sbk %lld sbn %lld", (long long)sbk,
                (long long)sbn);
  if (ldc < N) return fail(SAE_EINVAL, "gemm_f32: ldc (%lld) < N (%d)", (long long)ldc, N);
  if (!aligned16(a) || !aligned16(b)) return fail(SAE_EINVAL, "gemm_f32: a and b must be 16-byte aligned");
  F32Args g;
  memset(&g, 0, sizeof g);
  g.a = a;
  g.b = b;
  g.bias = bias;
  g.c = c;
  g.colsum = colsum;
  g.sam = sam;
  g.sak = sak;
  g.sbk = sbk;
  g.sbn = sbn;
  g.ldc = ldc;
  g.M = M;
  g.N = N;
  g.K = K;
  g.accumulate = accumulate;
  f32_plan(M, N, K, &g.S, &g.kchunk);
  if (g.S > 1) {
    if (!workspace || !aligned16(workspace))
      return fail(SAE_EINVAL, "gemm_f32: this shape splits K: pass sae_gemm_f32_workspace_bytes() of 16-byte "
                  "aligned workspace");
    g.part = reinterpret_cast<float*>(workspace);
  }
  const int Mx = M + (colsum ? 1 : 0);
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((Mx + kF32T - 1) / kF32T, (N + kF32T - 1) / kF32T, g.S);
  if (ak && bk) hipLaunchKernelGGL((gemm_f32_kernel<true, true>), grid, dim3(256), 0, st, g);
  else if (ak) hipLaunchKernelGGL((gemm_f32_kernel<true, false>), grid, dim3(256), 0, st, g);
  else if (bk) hipLaunchKernelGGL((gemm_f32_kernel<false, true>), grid, dim3(256), 0, st, g);
  else hipLaunchKernelGGL((gemm_f32_kernel<false, false>), grid, dim3(256), 0, st, g);
  if (int rc = check_launch("gemm_f32")) return rc;
  if (g.S > 1) {
    const long long n = (long long)Mx * N;
    const unsigned rb = (unsigned)std::min<long long>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(gemm_f32_reduce_kernel, dim3(rb), dim3(256), 0, st, g);
    return check_launch("gemm_f32_reduce");
  }
  return 0;
}

// ------------------------------------------------------------ forward / input-gradient GEMMs
// bench.py --emulate-rccl: workgroups that hold their CU's slots (waves, LDS) for `ticks` of the
// 100 MHz real-time counter while sleeping -- the CU footprint of an RCCL ring channel
__global__ void occupy_cus_kernel(long long ticks) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) lds[0] = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

int sae_occupy_cus(void* stream, int32_t workgroups, int32_t threads, int32_t lds_bytes, float usec) {
  if (workgroups < 1 || threads < 64 || threads > 1024 || lds_bytes < 0 || lds_bytes > 160 * 1024 || !(usec >= 0.f))
    return fail(SAE_EINVAL, "occupy_cus: bad arguments (%d workgroups, %d threads, %d B LDS, %g us)", workgroups,
                threads, lds_bytes, (double)usec);
  if (int rc = lds_attr((const void*)occupy_cus_kernel, (size_t)lds_bytes)) return rc;
  hipLaunchKernelGGL(occupy_cus_kernel, dim3((unsigned)workgroups), dim3((unsigned)threads), (size_t)lds_bytes,
                     (hipStream_t)stream, (long long)(usec * 100.f));
  return check_launch("occupy_cus");
}

__global__ void flag_bump_kernel(unsigned* flag) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int sae_flag_bump(void* stream, uint32_t* flags, int32_t index) {
  if (!flags || index < 0) return fail(SAE_EINVAL, "flag_bump: flags must be non-NULL and index >= 0");
  hipLaunchKernelGGL(flag_bump_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (unsigned*)flags + index);
  return check_launch("flag_bump");
}

int sae_stream_wait_flag(void* stream, const uint32_t* flag, uint32_t value) {
  if (!flag || ((uintptr_t)flag & 3)) return fail(SAE_EINVAL, "stream_wait_flag: flag must be a non-NULL 4-byte-aligned pointer");
  const hipError_t e = hipStreamWaitValue32((hipStream_t)stream, const_cast<uint32_t*>(flag), value,
                                            hipStreamWaitValueGte, 0xffffffffu);
  if (e != hipSuccess) return fail(SAE_EHIP, "hipStreamWaitValue32: %s", hipGetErrorString(e));
  return ok();
}

int sae_gemm_nt_route(int32_t M, int32_t N, int32_t K, int32_t epilogue) {
  if (M < 1 || N < 1 || K < 1 || K % 8 || N % 8 || epilogue < SAE_EPI_NONE || epilogue > SAE_EPI_MUL_AUX)
    return SAE_NT_ROUTE_NONE;
  const bool gp = epilogue >= SAE_EPI_GELU_GRAD;
  if (gp) epilogue -= 2;   // the gelu' forms run on the GELU / GELU' kernels
  if (g8x_route(M, N, K, epilogue)) return SAE_NT_ROUTE_GEMM8X;
  if (g8_route(M, N, K, epilogue, gp)) return SAE_NT_ROUTE_GEMM8;
  return K % kNtK ? SAE_NT_ROUTE_TILE128_KTAIL : SAE_NT_ROUTE_TILE128;
}

int sae_gemm_nt(void* stream, int32_t M, int32_t N, int32_t K, const void* a, int64_t lda, const void* bt,
                int64_t ldb, const float* bias, void* c, int64_t ldc, int32_t epilogue, const void* aux,
                int64_t ldaux, void* c2) {
  if (M < 1 || N < 1 || K < 1) return fail(SAE_EINVAL, "gemm_nt: M/N/K must be >= 1 (got %d/%d/%d)", M, N, K);
  if (K % 8 || N % 8) return fail(SAE_EUNSUPPORTED, "gemm_nt: K (%d) and N (%d) must be multiples of 8", K, N);
  if (lda < K || ldb < K || ldc < N || lda % 8 || ldb % 8 || ldc % 8)
    return fail(SAE_EINVAL, "gemm_nt: bad leading dimensions lda %lld ldb %lld ldc %lld", (long long)lda,
                (long long)ldb, (long long)ldc);
  if (!a || !bt || !c) return fail(SAE_EINVAL, "gemm_nt: a/bt/c must be non-NULL");
  if (epilogue < SAE_EPI_NONE || epilogue > SAE_EPI_MUL_AUX)
    return fail(SAE_EINVAL, "gemm_nt: unknown epilogue %d", epilogue);
  // SAE_EPI_GELU_GRAD / SAE_EPI_MUL_AUX: the GELU / GELU' kernels with the saved operand gelu'(h)
  const bool gp = epilogue >= SAE_EPI_GELU_GRAD;
  if (gp) epilogue -= 2;
  if (epilogue == SAE_EPI_GELU && !c2) return fail(SAE_EINVAL, "gemm_nt: the GELU epilogue needs c2 (pre-activation out)");
  if (epilogue == SAE_EPI_DGELU && (!aux || ldaux < N || ldaux % 8 || bias))
    return fail(SAE_EINVAL, "gemm_nt: the GELU-derivative epilogue needs aux (ldaux >= N, multiple of 8) and no bias");
  if (!aligned16(a) || !aligned16(bt) || !aligned16(c) || !aligned16(c2) || !aligned16(aux) || !aligned16(bias))
    return fail(SAE_EINVAL, "gemm_nt: a, bt, c, c2, aux and bias must be 16-byte aligned");
  if (256LL * std::max(lda, ldb) * 2 >= (1LL << 31))
    return fail(SAE_EUNSUPPORTED, "gemm_nt: a 256-row block exceeds 32-bit buffer addressing");
  NtArgs g;
  memset(&g, 0, sizeof g);
  g.a = reinterpret_cast<const __bf16*>(a);
  g.bt = reinterpret_cast<const __bf16*>(bt);
  g.bias = bias;
  g.aux = reinterpret_cast<const __bf16*>(aux);
  g.gp = gp ? 1 : 0;
  g.c = reinterpret_cast<__bf16*>(c);
  g.c2 = reinterpret_cast<__bf16*>(c2);
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.ldaux = ldaux;
  hipStream_t st = (hipStream_t)stream;
  if (g8x_route(M, N, K, epilogue)
#ifdef SAE_DEV_KNOBS
      && !dev_knob("SAE_NT_NO_G8")
#endif
  ) {
    const int rc = epilogue == SAE_EPI_NONE ? g8x_launch<kEpiNone, 256>(g, st) : g8x_launch<kEpiGelu, 256>(g, st);
    if (rc) return rc;
    return check_launch("gemm8x_nt");
  }
  if (g8_route(M, N, K, epilogue, gp)
#ifdef SAE_DEV_KNOBS
      && !dev_knob("SAE_NT_NO_G8")
#endif
  ) {
    if (epilogue == SAE_EPI_GELU && g8_gelu_bn128(M, N, K)) {
      // 4 x 2 waves (64 x 64 wave tiles): whole 128-byte output lines per wave row segment --
      // writes 172 -> 155 MB (= algorithmic), 57.1 -> 54.8 us at DeiT-S (profiles/r06w4_g8_wgm4_ab.txt)
      if (int rc = dev_knob("SAE_G8_WGM2") ? g8_launch_bm<kEpiGelu, 128, 64, 2, 256>(g, st)
                                           : g8_launch_bm<kEpiGelu, 128, 64, 2, 256, 4>(g, st)) return rc;
      return check_launch("gemm8_nt");
    }
    // the gelu' multiply on the same 256 x 128 tiles and 4 x 2 waves (whole-line stores, now also
    // non-temporal): 59.5 -> 53.8 us at DeiT-S, reads 128 -> 111 MB (profiles/r06m128_g8_mul_ab.txt)
    if (epilogue == SAE_EPI_DGELU && !dev_knob("SAE_G8_MUL192") && g8_gelu_bn128(M, N, K)) {
      if (int rc = g8_launch_bm<kEpiDGelu, 128, 64, 2, 256, 4>(g, st)) return rc;
      return check_launch("gemm8_nt");
    }
    const int rc = epilogue == SAE_EPI_NONE   ? g8_launch<kEpiNone, 192, 64, 2>(g, st)
                   : epilogue == SAE_EPI_GELU ? g8_launch<kEpiGelu, 192, 64, 2>(g, st)
                                              : g8_launch<kEpiDGelu, 192, 64, 2>(g, st);
    if (rc) return rc;
    return check_launch("gemm8_nt");
  }
  // tile height: 256 tokens for the GELU / GELU' epilogue GEMMs at K >= 768 (the ViT-B FF block:
  // the epilogue's VALU work per output is amortised over twice the MFMA work per tile;
  // tools/nt_probe.py at M 36928 K 768 N 3072: GELU 512 -> 634, GELU' 548 -> 609 TF/s) when that
  // still gives >= 2 tiles per CU; 128 otherwise (plain GEMMs: no gain, profiles/r03n_nt_probe.txt)
  const long long tn = (N + kNtT - 1) / kNtT;
  const long long grid128 = (long long)((M + kNtT - 1) / kNtT) * tn;
  // every launch below uses 128-row tiles (grid128) or taller ones (fewer workgroups)
  if (grid128 >= (1LL << 31)) return fail(SAE_EUNSUPPORTED, "gemm_nt: grid too large");
  bool tall = epilogue != SAE_EPI_NONE && K >= 768 && (long long)((M + 255) / 256) * tn >= 512;
#ifdef SAE_DEV_KNOBS
  const int ntv = dev_knob("SAE_NT_VARIANT");
  if (ntv) tall = ntv == 2;
  if ((ntv == 3 || ntv == 4) && K % kNtK == 0) {   // LDS-DMA staging, 3 / 4 stage buffers (no K tail)
    int rc;
    if (ntv == 3)
      rc = epilogue == SAE_EPI_NONE ? nt_launch<kEpiNone, NtDmaA<3>>(g, grid128, st)
           : epilogue == SAE_EPI_GELU ? nt_launch<kEpiGelu, NtDmaA<3>>(g, grid128, st)
                                      : nt_launch<kEpiDGelu, NtDmaA<3>>(g, grid128, st);
    else
      rc = epilogue == SAE_EPI_NONE ? nt_launch<kEpiNone, NtDmaA<4>>(g, grid128, st)
           : epilogue == SAE_EPI_GELU ? nt_launch<kEpiGelu, NtDmaA<4>>(g, grid128, st)
                                      : nt_launch<kEpiDGelu, NtDmaA<4>>(g, grid128, st);
    if (rc) return rc;
    return check_launch("gemm_nt");
  }
#endif
  const int TM = tall ? 256 : kNtT;
  const long long grid = (long long)((M + TM - 1) / TM) * tn;
  // stage depth: the GELU / GELU' epilogue GEMMs at reduction depth <= 384 (DeiT-S / CaiT FF
  // block) run 32-deep stages (32 KiB of LDS: 3-4 workgroups per CU, so one tile's epilogue VALU
  // overlaps other tiles' MFMAs; same-box step A/B 9.19 -> 9.10 ms); deeper reductions (ViT-B,
  // K 768) and the plain GEMM keep 64-deep stages (2 workgroups per CU), which are faster there
  const bool shallow = K <= 384;
  if (K % kNtK) {   // K-tail instances (K % 8 == 0): 64-deep stages, the last one partial
    int rc = epilogue == SAE_EPI_NONE   ? nt_launch<kEpiNone, NtRowAT<64, 128, true>>(g, grid128, st)
             : epilogue == SAE_EPI_GELU ? nt_launch<kEpiGelu, NtRowAT<64, 128, true>>(g, grid128, st)
                                        : nt_launch<kEpiDGelu, NtRowAT<64, 128, true>>(g, grid128, st);
    if (rc) return rc;
    return check_launch("gemm_nt");
  }
  if (tall) {
    const int rc = epilogue == SAE_EPI_NONE ? nt_launch<kEpiNone, NtRowAT<32, 256>>(g, grid, st)
                   : epilogue == SAE_EPI_GELU ? nt_launch<kEpiGelu, NtRowAT<32, 256>>(g, grid, st)
                                              : nt_launch<kEpiDGelu, NtRowAT<32, 256>>(g, grid, st);
    if (rc) return rc;
    return check_launch("gemm_nt");
  }
  switch (epilogue) {
    case SAE_EPI_NONE:
      if (int rc = nt_launch<kEpiNone, NtRowAT<64>>(g, grid, st)) return rc;
      break;
    case SAE_EPI_GELU:
      if (int rc = shallow ? nt_launch<kEpiGelu, NtRowAT<32>>(g, grid, st) : nt_launch<kEpiGelu, NtRowAT<64>>(g, grid, st))
        return rc;
      break;
    default:
      if (int rc = shallow ? nt_launch<kEpiDGelu, NtRowAT<32>>(g, grid, st) : nt_launch<kEpiDGelu, NtRowAT<64>>(g, grid, st))
        return rc;
      break;
  }
  return check_launch("gemm_nt");
}

// ------------------------------------------------------------------------ patch embedding
static int patch_geom(const sae_patch_desc* d, PatchGeom* g, int* M, int* K) {
  if (!d) return fail(SAE_EINVAL, "patch_embed: NULL descriptor");
  if (d->batch < 1 || d->height < 1 || d->width < 1 || d->channels < 1 || d->patch_h < 1 || d->patch_w < 1 ||
      d->embed < 1)
    return fail(SAE_EINVAL, "patch_embed: sizes must be >= 1");
  if (d->layout != SAE_LAYOUT_NHWC && d->layout != SAE_LAYOUT_HWCN)
    return fail(SAE_EINVAL, "patch_embed: unknown layout %d", d->layout);
  if (d->dtype != SAE_DTYPE_BF16 && d->dtype != SAE_DTYPE_F32)
    return fail(SAE_EINVAL, "patch_embed: unknown image dtype %d", d->dtype);
  if (d->height % d->patch_h || d->width % d->patch_w)
    return fail(SAE_EINVAL, "patch_embed: image %dx%d is not a whole number of %dx%d patches", d->height, d->width,
                d->patch_h, d->patch_w);
  const long long k = (long long)d->patch_h * d->patch_w * d->channels;
  const long long elems = (long long)d->batch * d->height * d->width * d->channels;
  const long long L = (long long)(d->height / d->patch_h) * (d->width / d->patch_w);
  if (k % kNtK || (d->patch_w * d->channels) % 8 || d->embed % 8)
    return fail(SAE_EUNSUPPORTED, "patch_embed: needs ph*pw*C %% 64 == 0, pw*C %% 8 == 0, embed %% 8 == 0 "
                "(got K %lld, pw*C %d, embed %d)", k, d->patch_w * d->channels, d->embed);
  if (d->layout == SAE_LAYOUT_HWCN && d->batch % 8)
    return fail(SAE_EUNSUPPORTED, "patch_embed: the HWCN layout needs batch %% 8 == 0 (got %d)", d->batch);
  if (elems >= (1LL << 31) || L * d->batch >= (1LL << 31))
    return fail(SAE_EUNSUPPORTED, "patch_embed: more than 2^31 image elements or tokens");
  memset(g, 0, sizeof *g);
  g->Nb = d->batch;
  g->Himg = d->height;
  g->Wimg = d->width;
  g->C = d->channels;
  g->Ph = d->patch_h;
  g->Pw = d->patch_w;
  g->gw = d->width / d->patch_w;
  g->L = (int)L;
  g->PwC = d->patch_w * d->channels;
  g->WC = d->width * d->channels;
  g->dL = FDiv::make((unsigned)L);
  g->dNb = FDiv::make((unsigned)d->batch);
  g->dgw = FDiv::make((unsigned)g->gw);
  g->dPwC = FDiv::make((unsigned)g->PwC);
  *M = (int)(L * d->batch);
  *K = (int)k;
  return 0;
}

extern "C++" {
template <bool HWCN, bool F32>
static int patch_fwd_launch(hipStream_t st, const NtArgs& g, long long grid) {
  const size_t lds = 4 * kNtT * kNtK * 2;
  const void* fn = (const void*)gemm_nt_kernel<kEpiNone, NtPatchA<HWCN, F32>>;
  if (int rc = lds_attr(fn, lds)) return rc;
  hipLaunchKernelGGL((gemm_nt_kernel<kEpiNone, NtPatchA<HWCN, F32>>), dim3((unsigned)grid), dim3(256), lds, st, g);
  return check_launch("patch_embed_fwd");
}
}  // extern "C++"

int sae_patch_embed_fwd(void* stream, const sae_patch_desc* d, const void* images, const void* wt, const float* bias,
                        void* out) {
  NtArgs g;
  memset(&g, 0, sizeof g);
  int M, K;
  if (int rc = patch_geom(d, &g.pg, &M, &K)) return rc;
  if (!images || !wt || !out) return fail(SAE_EINVAL, "patch_embed: images/wt/out must be non-NULL");
  if (!aligned16(images) || !aligned16(wt) || !aligned16(out) || !aligned16(bias))
    return fail(SAE_EINVAL, "patch_embed: images, wt, out and bias must be 16-byte aligned");
  g.pg.x = images;
  g.bt = reinterpret_cast<const __bf16*>(wt);
  g.bias = bias;
  g.c = reinterpret_cast<__bf16*>(out);
  g.M = M;
  g.N = d->embed;
  g.K = K;
  g.ldb = K;
  g.ldc = d->embed;
  const long long grid = (long long)((M + kNtT - 1) / kNtT) * ((d->embed + kNtT - 1) / kNtT);
  hipStream_t st = (hipStream_t)stream;
  const bool hwcn = d->layout == SAE_LAYOUT_HWCN, f32 = d->dtype == SAE_DTYPE_F32;
  int rc = hwcn ? (f32 ? patch_fwd_launch<true, true>(st, g, grid) : patch_fwd_launch<true, false>(st, g, grid))
                : (f32 ? patch_fwd_launch<false, true>(st, g, grid) : patch_fwd_launch<false, false>(st, g, grid));
  return rc ? rc : ok();
}

int sae_patch_gather(void* stream, const sae_patch_desc* d, const void* images, void* patches) {
  PatchGeom g;
  int M, K;
  if (int rc = patch_geom(d, &g, &M, &K)) return rc;
  if (d->layout != SAE_LAYOUT_HWCN) return fail(SAE_EUNSUPPORTED, "patch_gather: HWCN images only");
  if (!images || !patches) return fail(SAE_EINVAL, "patch_gather: images / patches must be non-NULL");
  if (!aligned16(images) || !aligned16(patches))
    return fail(SAE_EINVAL, "patch_gather: images and patches must be 16-byte aligned");
  g.x = images;
  const dim3 grid((unsigned)g.L, (unsigned)((g.Nb + 63) / 64), (unsigned)((K / 8 + 3) / 4));
  if (d->dtype == SAE_DTYPE_F32)
    hipLaunchKernelGGL(patch_gather_hwcn_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, g,
                       reinterpret_cast<__bf16*>(patches), K);
  else
    hipLaunchKernelGGL(patch_gather_hwcn_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, g,
                       reinterpret_cast<__bf16*>(patches), K);
  return check_launch("patch_gather");
}

size_t sae_patch_embed_bwd_workspace_bytes(const sae_patch_desc* d) {
  PatchGeom g;
  int M, K;
  if (patch_geom(d, &g, &M, &K)) return 0;
  return sae_gemm_dw_workspace_bytes(M, K, d->embed);
}

extern "C++" {
template <bool HWCN, bool F32>
static int patch_dw_launch(hipStream_t st, const DwArgs& a, long long grid) {
  using YL = typename std::conditional<HWCN, DwPermY, DwRow<true>>::type;
  const size_t lds = 4 * kDwK * 256;
  const void* fb = (const void*)gemm_dw_kernel<true, DwPatchX<HWCN, F32>, YL>;
  const void* fn = (const void*)gemm_dw_kernel<false, DwPatchX<HWCN, F32>, YL>;
  if (int rc = lds_attr(fb, lds)) return rc;
  if (int rc = lds_attr(fn, lds)) return rc;
  if (a.db)
    hipLaunchKernelGGL((gemm_dw_kernel<true, DwPatchX<HWCN, F32>, YL>), dim3((unsigned)grid), dim3(256), lds, st, a);
  else
    hipLaunchKernelGGL((gemm_dw_kernel<false, DwPatchX<HWCN, F32>, YL>), dim3((unsigned)grid), dim3(256), lds, st, a);
  return check_launch("patch_embed_dw");
}
}  // extern "C++"

int sae_patch_embed_bwd(void* stream, const sae_patch_desc* d, const void* images, const void* dout, float* dw,
                        float* db, int32_t accumulate, void* workspace) {
  DwArgs a;
  memset(&a, 0, sizeof a);
  int M, K;
  if (int rc = patch_geom(d, &a.pg, &M, &K)) return rc;
  if (!images || !dout || !dw || !workspace)
    return fail(SAE_EINVAL, "patch_embed_bwd: images/dout/dw/workspace must be non-NULL");
  if (!aligned16(images) || !aligned16(dout) || !aligned16(dw) || !aligned16(db) || !aligned16(workspace))
    return fail(SAE_EINVAL, "patch_embed_bwd: images, dout, dw, db and workspace must be 16-byte aligned");
  const int J = d->embed;
  a.pg.x = images;
  a.dy = reinterpret_cast<const __bf16*>(dout);
  a.M = M;
  a.I = K;
  a.J = J;
  dw_plan(M, K, J, &a.S, &a.chunk);
  if ((long long)a.chunk * J * 2 >= (1LL << 31))
    return fail(SAE_EUNSUPPORTED, "patch_embed_bwd: token chunk exceeds 32-bit buffer addressing");
  a.part = reinterpret_cast<float*>(workspace);
  a.bpart = reinterpret_cast<float*>(reinterpret_cast<char*>(workspace) + (((size_t)a.S * K * J * 4 + 255) & ~(size_t)255));
  a.dw = dw;
  a.db = db;
  a.ldy = J;
  a.ldw = J;
  a.accumulate = accumulate;
  hipStream_t st = (hipStream_t)stream;
  const long long grid = (long long)a.S * ((K + kDwT - 1) / kDwT) * ((J + kDwT - 1) / kDwT);
  const bool hwcn = d->layout == SAE_LAYOUT_HWCN, f32 = d->dtype == SAE_DTYPE_F32;
  int rc = hwcn ? (f32 ? patch_dw_launch<true, true>(st, a, grid) : patch_dw_launch<true, false>(st, a, grid))
                : (f32 ? patch_dw_launch<false, true>(st, a, grid) : patch_dw_launch<false, false>(st, a, grid));
  if (rc) return rc;
  const long long n4 = (long long)K * J / 4;
  const unsigned rb = (unsigned)std::min<long long>((n4 + kDwRedCols - 1) / kDwRedCols, 4096);
  hipLaunchKernelGGL(gemm_dw_reduce_kernel, dim3(rb, db ? 2 : 1), dim3(256), 0, st, a);
  if (int rc2 = check_launch("patch_embed_dw_reduce")) return rc2;
  return ok();
}

int sae_weight_cast(void* stream, int32_t K, int32_t N, const float* w, void* w16, void* wt16) {
  if (K < 1 || N < 1) return fail(SAE_EINVAL, "weight_cast: K/N must be >= 1 (got %d/%d)", K, N);
  if (!w || (!w16 && !wt16)) return fail(SAE_EINVAL, "weight_cast: w and at least one output must be non-NULL");
  hipLaunchKernelGGL(weight_cast_kernel, dim3((N + 31) / 32, (K + 31) / 32), dim3(256), 0, (hipStream_t)stream, w,
                     reinterpret_cast<__bf16*>(w16), reinterpret_cast<__bf16*>(wt16), K, N);
  return check_launch("weight_cast");
}

int sae_weight_cast_multi(void* stream, int32_t n, const sae_weight_cast_item* items) {
  if (n < 0 || (n > 0 && !items)) return fail(SAE_EINVAL, "weight_cast_multi: bad item list");
  hipStream_t st = (hipStream_t)stream;
  for (int base = 0; base < n; base += kCastMax) {
    CastList L;
    memset(&L, 0, sizeof L);
    L.n = std::min(kCastMax, n - base);
    long long tiles = 0;
    for (int j = 0; j < L.n; ++j) {
      const sae_weight_cast_item& s = items[base + j];
      if (!s.w || s.K < 1 || s.N < 1 || (!s.w16 && !s.wt16) || s.col0 < 0 ||
          (s.w16 && s.ld16 < s.col0 + s.N) || (s.wt16 && s.ldT < s.K))
        return fail(SAE_EINVAL, "weight_cast_multi: item %d invalid (K %d N %d ld16 %d ldT %d col0 %d)", base + j,
                    s.K, s.N, s.ld16, s.ldT, s.col0);
      CastItem& c = L.it[j];
      c.w = s.w;
      c.w16 = reinterpret_cast<__bf16*>(s.w16);
      c.wt16 = reinterpret_cast<__bf16*>(s.wt16);
      c.K = s.K;
      c.N = s.N;
      c.ld16 = s.ld16;
      c.ldT = s.ldT;
      c.col0 = s.col0;
      const auto a8 = [](const void* p) { return ((uintptr_t)p & 7) == 0; };
      c.vec = s.K % 4 == 0 && s.N % 4 == 0 && s.col0 % 4 == 0 && aligned16(s.w) &&
              (!s.w16 || (s.ld16 % 4 == 0 && a8(s.w16))) && (!s.wt16 || (s.ldT % 4 == 0 && a8(s.wt16)));
      c.tiles = c.vec ? ((s.K + 63) / 64) * ((s.N + 63) / 64) : ((s.K + 31) / 32) * ((s.N + 31) / 32);
      tiles += c.tiles;
    }
    if (tiles >= (1LL << 31)) return fail(SAE_EUNSUPPORTED, "weight_cast_multi: too many tiles");
    hipLaunchKernelGGL(weight_cast_multi_kernel, dim3((unsigned)tiles), dim3(256), 0, st, L);
    if (int rc = check_launch("weight_cast_multi")) return rc;
  }
  return ok();
}

// ------------------------------------------------------------ residual add + LayerNorm
// rows per wave: with the rows software-pipelined (ln.h) fewer, longer-lived waves win -- 2048 / 1024
// -> 1024 / 512 workgroups: DeiT-S step 8.220 -> 8.174 ms same box (profiles/r05ac_ln_grid_ab.txt;
// before the pipelining, 512 backward workgroups were slower: too few rows in flight)
static int ln_fwd_blocks(int M) { return std::max(1, std::min((M + 3) / 4, 1024)); }
static int ln_bwd_blocks(int M) { return std::max(1, std::min((M + 3) / 4, 512)); }

static int ln_check(int32_t M, int32_t C) {
  if (M < 1 || C < 4) return fail(SAE_EINVAL, "layernorm: M (%d) and C (%d) must be >= 1 / >= 4", M, C);
  if (C % 4 || C > 4 * 64 * kLnMaxV)
    return fail(SAE_EUNSUPPORTED, "layernorm: C (%d) must be a multiple of 4 and <= %d", C, 4 * 64 * kLnMaxV);
  return SAE_OK;
}

static int ln_fwd_impl(void* stream, int32_t M, int32_t C, const float* x, const void* delta, float* xout,
                       const float* gamma, const float* beta, void* y, float* mean, float* rstd, float eps,
                       const float* lsc, const float* rsc, int32_t rpb);

int sae_layernorm_fwd(void* stream, int32_t M, int32_t C, const float* x, const void* delta, float* xout,
                      const float* gamma, const float* beta, void* y, float* mean, float* rstd, float eps) {
  return ln_fwd_impl(stream, M, C, x, delta, xout, gamma, beta, y, mean, rstd, eps, nullptr, nullptr, 1);
}

int sae_layernorm_fwd_scaled(void* stream, int32_t M, int32_t C, const float* x, const void* delta, float* xout,
                             const float* gamma, const float* beta, void* y, float* mean, float* rstd, float eps,
                             const float* layerscale, const float* rowscale, int32_t rows_per_sample) {
  if (!delta || !layerscale) return fail(SAE_EINVAL, "layernorm_fwd_scaled: delta and layerscale are required");
  if (rowscale && (rows_per_sample < 1 || M % rows_per_sample))
    return fail(SAE_EINVAL, "layernorm_fwd_scaled: rows_per_sample (%d) must divide M (%d)", rows_per_sample, M);
  if (!aligned16(layerscale)) return fail(SAE_EINVAL, "layernorm_fwd_scaled: layerscale needs 16-byte alignment");
  return ln_fwd_impl(stream, M, C, x, delta, xout, gamma, beta, y, mean, rstd, eps, layerscale, rowscale,
                     rows_per_sample);
}

static int ln_fwd_impl(void* stream, int32_t M, int32_t C, const float* x, const void* delta, float* xout,
                       const float* gamma, const float* beta, void* y, float* mean, float* rstd, float eps,
                       const float* lsc, const float* rsc, int32_t rpb) {
  if (int rc = ln_check(M, C)) return rc;
  if (!x || !gamma || !beta || !y || !mean || !rstd) return fail(SAE_EINVAL, "layernorm_fwd: NULL argument");
  if ((delta == nullptr) != (xout == nullptr))
    return fail(SAE_EINVAL, "layernorm_fwd: delta and xout must both be given or both be NULL");
  if (!aligned16(x) || !aligned16(xout) || !aligned16(gamma) || !aligned16(beta) || ((uintptr_t)delta & 7) ||
      ((uintptr_t)y & 7))
    return fail(SAE_EINVAL, "layernorm_fwd: x/xout/gamma/beta need 16-byte, delta/y 8-byte alignment");
  LnArgs a;
  memset(&a, 0, sizeof a);
  a.x = x;
  a.delta = reinterpret_cast<const __bf16*>(delta);
  a.xout = xout;
  a.gamma = gamma;
  a.beta = beta;
  a.y = reinterpret_cast<__bf16*>(y);
  a.mean = mean;
  a.rstd = rstd;
  a.M = M;
  a.C = C;
  a.eps = eps;
  a.lsc = lsc;
  a.rsc = rsc;
  a.rpb = rpb > 0 ? rpb : 1;
  const int nv = (C / 4 + 63) / 64;
  int lnb = ln_fwd_blocks(M);
#ifdef SAE_DEV_KNOBS
  if (int v = dev_knob("SAE_LN_FWD_BLOCKS")) lnb = std::max(1, std::min((M + 3) / 4, v));
#endif
  const dim3 g(lnb), b(256);
  hipStream_t st = (hipStream_t)stream;
  switch (nv) {
    case 1: hipLaunchKernelGGL(ln_fwd_kernel<1>, g, b, 0, st, a); break;
    case 2: hipLaunchKernelGGL(ln_fwd_kernel<2>, g, b, 0, st, a); break;
    case 3: hipLaunchKernelGGL(ln_fwd_kernel<3>, g, b, 0, st, a); break;
    default: hipLaunchKernelGGL(ln_fwd_kernel<4>, g, b, 0, st, a); break;
  }
  return check_launch("layernorm_fwd");
}

size_t sae_layernorm_bwd_workspace_bytes(int32_t M, int32_t C) {
  if (M < 1 || C < 1) return 0;
  return (size_t)ln_bwd_blocks(M) * 3 * C * sizeof(float);   // room for the scaled form
}

// ------------------------------------------------------------------ encoder input tokens
static int tokens_check(int32_t B, int32_t L, int32_t E) {
  if (B < 1 || L < 1 || E < 4 || E % 4 || E > 4096)
    return fail(SAE_EINVAL, "tokens: B %d, L %d, E %d (E a multiple of 4, <= 4096)", B, L, E);
  return 0;
}

int sae_tokens_fwd(void* stream, int32_t B, int32_t L, int32_t E, const void* tokens, const float* cls,
                   const float* pos, float* x) {
  if (int rc = tokens_check(B, L, E)) return rc;
  if (!tokens || !cls || !pos || !x) return fail(SAE_EINVAL, "tokens_fwd: NULL argument");
  if (!aligned16(cls) || !aligned16(pos) || !aligned16(x) || ((uintptr_t)tokens & 7))
    return fail(SAE_EINVAL, "tokens_fwd: cls / pos / x need 16-byte, tokens 8-byte alignment");
  const long long total = (long long)B * (L + 1) * (E / 4);
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(tokens_fwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const __bf16*>(tokens), cls, pos, x, B, L, E);
  return check_launch("tokens_fwd");
}

int sae_tokens_bwd(void* stream, int32_t B, int32_t L, int32_t E, const float* dx, void* dtokens, float* dcls,
                   float* dpos) {
  if (int rc = tokens_check(B, L, E)) return rc;
  if (!dx || !dtokens || !dpos) return fail(SAE_EINVAL, "tokens_bwd: NULL argument");
  if (!aligned16(dx) || !aligned16(dpos) || (dcls && !aligned16(dcls)) || ((uintptr_t)dtokens & 7))
    return fail(SAE_EINVAL, "tokens_bwd: dx / dcls / dpos need 16-byte, dtokens 8-byte alignment");
  const int E4 = E / 4;
  const int G = std::max(1, std::min(B, 512 / E4));
  const size_t lds = (size_t)G * E4 * 16;
  if (int rc = lds_attr((const void*)tokens_bwd_kernel, lds)) return rc;
  hipLaunchKernelGGL(tokens_bwd_kernel, dim3((unsigned)(L + 1)), dim3((unsigned)(G * E4)), lds, (hipStream_t)stream,
                     dx, reinterpret_cast<__bf16*>(dtokens), dcls, dpos, B, L, E);
  return check_launch("tokens_bwd");
}

// ------------------------------------------------------------------ training loss
static int ce_check(int32_t rows, int32_t classes, const void* logits, int64_t ld, int32_t dtype,
                    const int64_t* labels) {
  if (rows < 1 || rows > SAE_CE_MAX_ROWS || classes < 1 || ld < classes)
    return fail(SAE_EINVAL, "smoothed_ce: rows %d (1..%d), classes %d, ld %lld", rows, SAE_CE_MAX_ROWS, classes,
                (long long)ld);
  if (dtype != SAE_DTYPE_BF16 && dtype != SAE_DTYPE_F32) return fail(SAE_EINVAL, "smoothed_ce: bad dtype %d", dtype);
  if (!logits || !labels) return fail(SAE_EINVAL, "smoothed_ce: NULL logits / labels");
  return 0;
}

int sae_smoothed_ce_fwd(void* stream, int32_t rows, int32_t classes, const void* logits, int64_t ld,
                        int32_t dtype, const int64_t* labels, float alpha, float* lse, float* row_loss, float* loss) {
  if (int rc = ce_check(rows, classes, logits, ld, dtype, labels)) return rc;
  if (!lse || !row_loss || !loss) return fail(SAE_EINVAL, "smoothed_ce_fwd: NULL lse / row_loss / loss");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SAE_DTYPE_BF16)
    hipLaunchKernelGGL(smoothed_ce_fwd_kernel<__bf16>, dim3(rows), dim3(256), 0, st,
                       reinterpret_cast<const __bf16*>(logits), (long long)ld, labels, classes, alpha, lse, row_loss);
  else
    hipLaunchKernelGGL(smoothed_ce_fwd_kernel<float>, dim3(rows), dim3(256), 0, st,
                       reinterpret_cast<const float*>(logits), (long long)ld, labels, classes, alpha, lse, row_loss);
  if (int rc = check_launch("smoothed_ce_fwd")) return rc;
  hipLaunchKernelGGL(smoothed_ce_mean_kernel, dim3(1), dim3(256), 0, st, row_loss, rows, loss);
  return check_launch("smoothed_ce_mean");
}

int sae_smoothed_ce_bwd(void* stream, int32_t rows, int32_t classes, const void* logits, int64_t ld,
                        int32_t dtype, const int64_t* labels, float alpha, const float* lse,
                        const float* grad_loss, void* dlogits, int64_t ldd) {
  if (int rc = ce_check(rows, classes, logits, ld, dtype, labels)) return rc;
  if (!lse || !grad_loss || !dlogits || ldd < classes)
    return fail(SAE_EINVAL, "smoothed_ce_bwd: NULL lse / grad_loss / dlogits or ldd < classes");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SAE_DTYPE_BF16)
    hipLaunchKernelGGL(smoothed_ce_bwd_kernel<__bf16>, dim3(rows), dim3(256), 0, st,
                       reinterpret_cast<const __bf16*>(logits), (long long)ld, labels, rows, classes, alpha, lse,
                       grad_loss, reinterpret_cast<__bf16*>(dlogits), (long long)ldd);
  else
    hipLaunchKernelGGL(smoothed_ce_bwd_kernel<float>, dim3(rows), dim3(256), 0, st,
                       reinterpret_cast<const float*>(logits), (long long)ld, labels, rows, classes, alpha, lse,
                       grad_loss, reinterpret_cast<float*>(dlogits), (long long)ldd);
  return check_launch("smoothed_ce_bwd");
}

static int ln_bwd_impl(void* stream, int32_t M, int32_t C, const float* x, const float* mean, const float* rstd,
                       const float* gamma, const void* dy, const float* dxin, float* dx, void* ddelta,
                       float* dgamma, float* dbeta, void* workspace, const void* delta, const float* lsc,
                       const float* rsc, int32_t rpb, float* dlsc);

int sae_layernorm_bwd(void* stream, int32_t M, int32_t C, const float* x, const float* mean, const float* rstd,
                      const float* gamma, const void* dy, const float* dxin, float* dx, void* ddelta, float* dgamma,
                      float* dbeta, void* workspace) {
  return ln_bwd_impl(stream, M, C, x, mean, rstd, gamma, dy, dxin, dx, ddelta, dgamma, dbeta, workspace, nullptr,
                     nullptr, nullptr, 1, nullptr);
}

int sae_layernorm_bwd_scaled(void* stream, int32_t M, int32_t C, const float* x, const float* mean,
                             const float* rstd, const float* gamma, const void* dy, const float* dxin, float* dx,
                             void* ddelta, float* dgamma, float* dbeta, void* workspace, const void* delta,
                             const float* layerscale, const float* rowscale, int32_t rows_per_sample,
                             float* dlayerscale) {
  if (!delta || !layerscale || !dlayerscale)
    return fail(SAE_EINVAL, "layernorm_bwd_scaled: delta, layerscale and dlayerscale are required");
  if (rowscale && (rows_per_sample < 1 || M % rows_per_sample))
    return fail(SAE_EINVAL, "layernorm_bwd_scaled: rows_per_sample (%d) must divide M (%d)", rows_per_sample, M);
  if (!aligned16(layerscale) || ((uintptr_t)delta & 7))
    return fail(SAE_EINVAL, "layernorm_bwd_scaled: layerscale needs 16-byte, delta 8-byte alignment");
  return ln_bwd_impl(stream, M, C, x, mean, rstd, gamma, dy, dxin, dx, ddelta, dgamma, dbeta, workspace, delta,
                     layerscale, rowscale, rows_per_sample, dlayerscale);
}

// ---------------------------------------------------------------------------------- AdamW
static_assert(sizeof(sae_adamw_chunk) == sizeof(AdamwChunk) && SAE_ADAMW_CHUNK == kAdamwChunk,
              "sae_adamw_chunk mirrors AdamwChunk");

int sae_adamw_plan(int32_t n_items, float* const* p, const float* const* g, float* const* m, float* const* v,
                   const int64_t* n, sae_adamw_chunk* chunks, int64_t max_chunks, int64_t* n_chunks) {
  if (n_items < 0 || !n_chunks || (n_items > 0 && (!p || !g || !m || !v || !n)))
    return fail(SAE_EINVAL, "adamw_plan: bad arguments");
  int64_t k = 0;
  for (int32_t i = 0; i < n_items; ++i) {
    if (n[i] < 0 || (n[i] > 0 && (!p[i] || !g[i] || !m[i] || !v[i])))
      return fail(SAE_EINVAL, "adamw_plan: item %d invalid", i);
    for (int64_t off = 0; off < n[i]; off += SAE_ADAMW_CHUNK, ++k) {
      if (k < max_chunks && chunks) {
        sae_adamw_chunk& c = chunks[k];
        c.p = p[i] + off;
        c.g = g[i] + off;
        c.m = m[i] + off;
        c.v = v[i] + off;
        c.n = (int32_t)std::min<int64_t>(SAE_ADAMW_CHUNK, n[i] - off);
        c.vec = c.n == SAE_ADAMW_CHUNK && aligned16(c.p) && aligned16(c.g) && aligned16(c.m) && aligned16(c.v);
      }
    }
  }
  *n_chunks = k;
  if (k > max_chunks) return fail(SAE_EINVAL, "adamw_plan: %lld chunks > capacity %lld", (long long)k,
                                  (long long)max_chunks);
  return ok();
}

int sae_adamw_step(void* stream, int64_t n_chunks, const sae_adamw_chunk* chunks, int32_t* step, float lr,
                   float beta1, float beta2, float eps, float weight_decay) {
  if (n_chunks < 0 || n_chunks >= (1LL << 31) || (n_chunks > 0 && !chunks) || !step)
    return fail(SAE_EINVAL, "adamw_step: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adamw_tick_kernel, dim3(1), dim3(64), 0, st, step);
  if (int rc = check_launch("adamw_tick")) return rc;
  if (n_chunks == 0) return ok();
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)n_chunks), dim3(256), 0, st,
                     reinterpret_cast<const AdamwChunk*>(chunks), step, lr, beta1, beta2, eps, weight_decay);
  return check_launch("adamw");
}

static_assert(sizeof(sae_adamw_cast_tile) == sizeof(AdamwCastTile), "sae_adamw_cast_tile mirrors AdamwCastTile");

int sae_adamw_cast_plan(int32_t n_items, float* const* p, const float* const* g, float* const* m,
                        float* const* v, const int32_t* K, const int32_t* N, void* const* w16, const int32_t* ld16,
                        void* const* wt16, const int32_t* ldT, const int32_t* col0, sae_adamw_cast_tile* tiles,
                        int64_t max_tiles, int64_t* n_tiles) {
  if (n_items < 0 || !n_tiles || (n_items > 0 && (!p || !g || !m || !v || !K || !N || !col0)))
    return fail(SAE_EINVAL, "adamw_cast_plan: bad arguments");
  const auto a8 = [](const void* q) { return ((uintptr_t)q & 7) == 0; };
  int64_t k = 0;
  for (int32_t i = 0; i < n_items; ++i) {
    void* o16 = w16 ? w16[i] : nullptr;
    void* oT = wt16 ? wt16[i] : nullptr;
    const int32_t l16 = ld16 ? ld16[i] : 0, lT = ldT ? ldT[i] : 0;
    if (!p[i] || !g[i] || !m[i] || !v[i] || K[i] < 1 || N[i] < 1 || col0[i] < 0 || (!o16 && !oT) ||
        (o16 && l16 < col0[i] + N[i]) || (oT && lT < K[i]))
      return fail(SAE_EINVAL, "adamw_cast_plan: item %d invalid (K %d N %d col0 %d ld16 %d ldT %d)", i, K[i], N[i],
                  col0[i], l16, lT);
    if (K[i] % 4 || N[i] % 4 || col0[i] % 4 || !aligned16(p[i]) || !aligned16(g[i]) || !aligned16(m[i]) ||
        !aligned16(v[i]) || (o16 && (l16 % 4 || !a8(o16))) || (oT && (lT % 4 || !a8(oT))))
      return fail(SAE_EUNSUPPORTED, "adamw_cast_plan: item %d needs K/N/col0/ld multiples of 4 and aligned buffers",
                  i);
    for (int32_t k0 = 0; k0 < K[i]; k0 += 64)
      for (int32_t n0 = 0; n0 < N[i]; n0 += 64, ++k) {
        if (k < max_tiles && tiles) {
          sae_adamw_cast_tile& t = tiles[k];
          t.p = p[i];
          t.g = g[i];
          t.m = m[i];
          t.v = v[i];
          t.w16 = o16;
          t.wt16 = oT;
          t.K = K[i];
          t.N = N[i];
          t.ld16 = l16;
          t.ldT = lT;
          t.col0 = col0[i];
          t.k0 = k0;
          t.n0 = n0;
          t.pad = 0;
        }
      }
  }
  *n_tiles = k;
  if (k > max_tiles)
    return fail(SAE_EINVAL, "adamw_cast_plan: %lld tiles > capacity %lld", (long long)k, (long long)max_tiles);
  return ok();
}

int sae_adamw_step_cast(void* stream, int64_t n_chunks, const sae_adamw_chunk* chunks, int64_t n_tiles,
                        const sae_adamw_cast_tile* tiles, int32_t* step, float lr, float beta1, float beta2, float eps,
                        float weight_decay) {
  if (n_chunks < 0 || n_tiles < 0 || n_chunks + n_tiles >= (1LL << 31) || (n_chunks > 0 && !chunks) ||
      (n_tiles > 0 && !tiles) || !step)
    return fail(SAE_EINVAL, "adamw_step_cast: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(adamw_tick_kernel, dim3(1), dim3(64), 0, st, step);
  if (int rc = check_launch("adamw_tick")) return rc;
  if (n_chunks + n_tiles == 0) return ok();
  hipLaunchKernelGGL(adamw_cast_kernel, dim3((unsigned)(n_chunks + n_tiles)), dim3(256), 0, st,
                     reinterpret_cast<const AdamwChunk*>(chunks), (int)n_chunks,
                     reinterpret_cast<const AdamwCastTile*>(tiles), step, lr, beta1, beta2, eps, weight_decay);
  return check_launch("adamw_cast");
}

static int ln_bwd_impl(void* stream, int32_t M, int32_t C, const float* x, const float* mean, const float* rstd,
                       const float* gamma, const void* dy, const float* dxin, float* dx, void* ddelta,
                       float* dgamma, float* dbeta, void* workspace, const void* delta, const float* lsc,
                       const float* rsc, int32_t rpb, float* dlsc) {
  if (int rc = ln_check(M, C)) return rc;
  if (!x || !mean || !rstd || !gamma || !dy || !dx || !dgamma || !dbeta || !workspace)
    return fail(SAE_EINVAL, "layernorm_bwd: NULL argument");
  if (!aligned16(x) || !aligned16(dxin) || !aligned16(dx) || !aligned16(gamma) || !aligned16(workspace) ||
      ((uintptr_t)dy & 7) || ((uintptr_t)ddelta & 7))
    return fail(SAE_EINVAL, "layernorm_bwd: x/dxin/dx/gamma/workspace need 16-byte, dy/ddelta 8-byte alignment");
  LnArgs a;
  memset(&a, 0, sizeof a);
  a.x = x;
  a.mean = const_cast<float*>(mean);
  a.rstd = const_cast<float*>(rstd);
  a.gamma = gamma;
  a.dy = reinterpret_cast<const __bf16*>(dy);
  a.dxin = dxin;
  a.dx = dx;
  a.ddelta = reinterpret_cast<__bf16*>(ddelta);
  a.part = reinterpret_cast<float*>(workspace);
  a.dgamma = dgamma;
  a.dbeta = dbeta;
  a.M = M;
  a.C = C;
  a.nblk = ln_bwd_blocks(M);
#ifdef SAE_DEV_KNOBS
  if (int v = dev_knob("SAE_LN_BWD_BLOCKS")) a.nblk = std::max(1, std::min(a.nblk, v));   // (workspace: <= default)
#endif
  a.delta = reinterpret_cast<const __bf16*>(delta);
  a.lsc = lsc;
  a.rsc = rsc;
  a.rpb = rpb > 0 ? rpb : 1;
  a.dlsc = dlsc;
  const int nv = (C / 4 + 63) / 64;
  const dim3 g(a.nblk), b(256);
  hipStream_t st = (hipStream_t)stream;
  const bool sc = lsc != nullptr;
  const int np = sc ? 3 : 2;
#define LNB(NV)                                                                \
  if (sc) hipLaunchKernelGGL((ln_bwd_kernel<NV, 3>), g, b, 0, st, a);          \
  else hipLaunchKernelGGL((ln_bwd_kernel<NV, 2>), g, b, 0, st, a);
  switch (nv) {
    case 1: LNB(1) break;
    case 2: LNB(2) break;
    case 3: LNB(3) break;
    default: LNB(4) break;
  }
#undef LNB
  if (int rc = check_launch("layernorm_bwd")) return rc;
  const dim3 rg((np * (C / 4) + kLnRedCols - 1) / kLnRedCols);
  if (sc) hipLaunchKernelGGL(ln_bwd_reduce_kernel<3>, rg, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(ln_bwd_reduce_kernel<2>, rg, dim3(256), 0, st, a);
  return check_launch("layernorm_bwd_reduce");
}

const char* sae_last_error(void) { return g_err.c_str(); }

int32_t sae_abi_version(void) { return SAE_ABI_VERSION; }

const char* sae_build_info(void) { return "sae_attn gfx950 (" __DATE__ " " __TIME__ ")"; }

#ifdef SAE_STAMPS
// diagnostic build only (not declared in sae_attn.h): copy / clear the in-kernel stamp table
int sae_dev_stamps(void* dst, size_t bytes, int clear) {
  if (bytes > sizeof(unsigned long long) * (size_t)kStampRecs) return fail(SAE_EINVAL, "stamps: %zu bytes", bytes);
  hipError_t e;
  e = hipDeviceSynchronize();   // every stream: no kernel may be writing stamps meanwhile
  if (e == hipSuccess && clear) {
    void* p = nullptr;
    e = hipGetSymbolAddress(&p, HIP_SYMBOL(g_sae_stamps));
    if (e == hipSuccess) e = hipMemset(p, 0, sizeof(unsigned long long) * (size_t)kStampRecs);
    if (e == hipSuccess) e = hipDeviceSynchronize();
  } else if (e == hipSuccess) {
    e = hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_sae_stamps), bytes, 0, hipMemcpyDeviceToHost);
  }
  if (e != hipSuccess) return fail(SAE_EHIP, "stamps: %s", hipGetErrorString(e));
  return ok();
}
#endif

}  // extern "C"
