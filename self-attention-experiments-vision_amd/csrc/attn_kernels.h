// attn_kernels.h -- fused flash-style attention forward / backward for gfx950.
//
// Replaces the XLA chain of models/layers/attentions/attention.py:39-58 (q/sqrt(D), QK^T
// einsum, softmax, AV einsum) and its autodiff backward.  Layout is the reference's
// token-major [B, N, H, D]; the scores never touch HBM.
//
// Forward (attn_fwd): one 256-thread workgroup = 4 waves = 128 query rows of one (b, h);
// each wave owns 32 query rows with the query on the MFMA lane ("swapped" QK^T: S^T = K Q^T),
// so the online-softmax state (m, l) and the O^T rescale are per-lane scalars.  K/V tiles of
// 64 keys are staged global -> registers -> LDS (loads for tile t+1 in flight during tile t);
// P^T feeds O^T = V^T P^T straight from the accumulator registers, V^T read with
// ds_read_b64_tr_b16.
//
// Backward = two deterministic passes (no HBM atomics), in this order:
//   attn_bwd_dq  : query on the lane; delta = rowsum(dO o O) from the fragments in registers
//                  (published for the next pass), S^T and dP^T recomputed with -lse/scale and
//                  -delta as the initial accumulators, dQ^T += K^T dS^T (+ the BoTNet
//                  relative-logit gradient reduced in LDS).
//   attn_bwd_dkdv: key on the lane; a workgroup owns 128 keys and sweeps all query tiles,
//                  S = Q K^T, dP = dO V^T (same accumulator init), dV^T += dO^T P,
//                  dK^T += Q^T dS.
#pragma once
#include "common.h"

namespace sae {

struct AttnArgs {
  const void* q;
  const void* k;
  const void* v;
  const void* o;
  void* out;        // fwd: o; bwd unused
  float* lse;       // fwd output / bwd input
  const void* dout;
  void* dq;
  void* dk;
  void* dv;
  float* delta;     // bwd workspace [B, H, Nq]
  const float* bias_h;
  const float* bias_w;
  float* dbias_h;
  float* dbias_w;
  int B, H, Nq, Nk, D;
  long long qs[3], ks[3], vs[3], os[3], dos[3], dqs[3], dks[3], dvs[3];
  float scale;
  int rel_h, rel_w, rel_magic;
  RopeTab rope;     // rotary tables (the ROT kernel instances), rope.sin == nullptr otherwise
};

constexpr int kBQ = 128;   // query rows per forward / dq workgroup (4 waves x 32)
constexpr int kBK = 64;    // keys per staged K/V tile
constexpr int kBKV = 128;  // keys per dkdv workgroup (4 waves x 32)
constexpr int kBQT = 64;   // query rows per staged tile in dkdv

// K/V (or Q/dO) tiles are double-buffered (one barrier per tile) except fp32 at head_dim 128,
// whose tiles are too large for two buffers plus the BoTNet tables in 160 KiB of LDS.
template <typename T, int DP> constexpr int nbuf() { return (sizeof(T) == 4 && DP == 128) ? 1 : 2; }

template <typename T, int DP, bool REL>
constexpr int fwd_lds_bytes_static() {
  return 2 * Img<T, DP>::bytes(kBK);
}

// ================================================================================ forward
// Lazy rescale (cdna_hip_programming.md T13): the running max m is only moved when some row's
// tile max exceeds it by more than THR (log2 units), so P <= 2^THR.  bf16: THR = 8 (P is fed to
// the MFMA in bf16, whose relative precision does not depend on magnitude); f32: THR = 0 (exact
// textbook online softmax).  The decision is wave-uniform and taken before any P of the tile is
// exponentiated (T13 safe order).
template <typename T> struct LazyThr { static constexpr float v = sizeof(T) == 2 ? 8.f : 0.f; };

template <typename T, int DP, bool REL, bool MASK>
__device__ __forceinline__ void fwd_tile(const char* ldsK, const char* ldsV, const typename MF<T>::frag* qf,
                                         f32x16* acco, float& m, float& l, int key0, int Nk, float sl2,
                                         const float* wbrow, int rel_h, int rel_w, int rel_magic, int h, int r32,
                                         int lane) {
  using M = MF<T>;
  using I = Img<T, DP>;
  constexpr int NS = DP / M::KSTEP, NP = 32 / M::KSTEP, NT = DP / 32;
  // masked tail: the second 32-key half is skipped when it holds no valid key
  const bool two = !MASK || key0 + 32 < Nk;
  f32x16 sacc[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    sacc[u] = zero16();
    if (u == 1 && !two) continue;
#pragma unroll
    for (int s = 0; s < NS; ++s) sacc[u] = M::mma(I::rowfrag(ldsK, 32 * u + r32, s, h), qf[s], sacc[u]);
  }
  // scores: REL -> x = s*sl2 + bias (log2 domain); otherwise keep raw s and fold sl2 into the exp FMA
  float mx = -kInf;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (u == 1 && !two) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = key0 + 32 * u + row_of(r, h);
      float x = sacc[u][r];
      if constexpr (REL) {
        const int kk = min(key, Nk - 1);
        const int kx = (kk * rel_magic) >> 20;
        const int ky = kk - kx * rel_w;
        x = x * sl2 + wbrow[kx] + wbrow[rel_h + ky];
      }
      if constexpr (MASK) x = key < Nk ? x : -kInf;
      sacc[u][r] = x;
      mx = fmaxf(mx, x);
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  if constexpr (!REL) mx *= sl2;                  // scale > 0 (validated)
  if (!__all(mx - m <= LazyThr<T>::v)) {
    const float mn = fmaxf(m, mx);
    const float alpha = ex2(m - mn);
    m = mn;
    l *= alpha;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acco[t][r] *= alpha;
  }
  float ls = 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (u == 1 && !two) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = REL ? ex2(sacc[u][r] - m) : ex2(__builtin_fmaf(sacc[u][r], sl2, -m));
      sacc[u][r] = p;
      ls += p;
    }
  }
  l += ls;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (u == 1 && !two) continue;
#pragma unroll
    for (int s2 = 0; s2 < NP; ++s2) {
      const typename M::frag pf = acc_frag<T>(sacc[u], s2);
#pragma unroll
      for (int t = 0; t < NT; ++t) acco[t] = M::mma(I::colfrag(ldsV, 32 * u, s2, 32 * t, lane), pf, acco[t]);
    }
  }
}

template <typename T, int DP, bool VEC, bool REL>
__global__ __launch_bounds__(256, DP >= 128 ? 1 : ((DP == 64 && sizeof(T) == 2 && !REL && VEC) ? 3 : 2)) void attn_fwd_kernel(AttnArgs a) {
  using M = MF<T>;
  using I = Img<T, DP>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // double-buffered K/V tiles: [buf][K | V], one barrier per key tile
  constexpr int TB = 2 * I::bytes(kBK);
  float* ldsB = reinterpret_cast<float*>(smem + nbuf<T, DP>() * TB);   // REL: [4][32][RW]

  const int nqb = (a.Nq + kBQ - 1) / kBQ;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb;
  bid /= nqb;
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q = qb * kBQ + w * 32 + r32;
  const bool active = qb * kBQ + __builtin_amdgcn_readfirstlane(w) * 32 < a.Nq;

  const T* Q = reinterpret_cast<const T*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const T* K = reinterpret_cast<const T*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const T* V = reinterpret_cast<const T*>(a.v) + b * a.vs[0] + hh * a.vs[2];

  constexpr int NS = DP / M::KSTEP;        // k-steps over the head dim
  constexpr int NT = DP / 32;              // 32-wide head-dim tiles of O^T

  typename M::frag qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) qf[s] = gfrag<T, VEC>(Q, q, a.Nq, a.qs[1], a.D, s, h);

  const int RW = a.rel_h + a.rel_w + 1;
  if constexpr (REL) {
    // stage this wave's 32 rows of bias_h | bias_w (pre-multiplied by log2 e)
    float* wb = ldsB + w * 32 * RW;
    const size_t rowoff = ((size_t)b * a.H + hh) * a.Nq;
    for (int i = lane; i < 32 * (RW - 1); i += 64) {
      const int rr = i / (RW - 1), cc = i % (RW - 1);
      const int qq = qb * kBQ + w * 32 + rr;
      float val = 0.f;
      if (qq < a.Nq)
        val = cc < a.rel_h ? a.bias_h[(rowoff + qq) * a.rel_h + cc]
                           : a.bias_w[(rowoff + qq) * a.rel_w + (cc - a.rel_h)];
      wb[rr * RW + cc] = val * kLog2e;
    }
  }
  const float* wbrow = ldsB + (w * 32 + r32) * RW;

  f32x16 acco[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acco[t] = zero16();
  float m = -kInf, l = 0.f;
  const float sl2 = a.scale * kLog2e;
  const int nkt = (a.Nk + kBK - 1) / kBK;
  const int nfull = a.Nk / kBK;

  Stage<T, DP, kBK, VEC> kst, vst;
  const __amdgpu_buffer_rsrc_t rk = row_rsrc(K, a.Nk, a.ks[1]);
  const __amdgpu_buffer_rsrc_t rv = row_rsrc(V, a.Nk, a.vs[1]);
  if constexpr (VEC) {
    kst.load_buf(rk, 0, a.ks[1], a.D, tid);
    vst.load_buf(rv, 0, a.vs[1], a.D, tid);
  } else {
    kst.load(K, 0, a.Nk, a.ks[1], a.D, tid);
    vst.load(V, 0, a.Nk, a.vs[1], a.D, tid);
  }

  kst.write(smem, tid);
  vst.write(smem + I::bytes(kBK), tid);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const char* ldsK = smem + (nbuf<T, DP>() == 2 ? (kt & 1) : 0) * TB;
    const char* ldsV = ldsK + I::bytes(kBK);
    const bool more = kt + 1 < nkt;
    if (more) {                               // next tile global -> registers, in flight during compute
      if constexpr (VEC) {
        kst.load_buf(rk, (kt + 1) * kBK, a.ks[1], a.D, tid);
        vst.load_buf(rv, (kt + 1) * kBK, a.vs[1], a.D, tid);
      } else {
        kst.load(K, (kt + 1) * kBK, a.Nk, a.ks[1], a.D, tid);
        vst.load(V, (kt + 1) * kBK, a.Nk, a.vs[1], a.D, tid);
      }
    }
    if (active) {                              // waves with no valid query row only stage + sync
      if (kt < nfull)
        fwd_tile<T, DP, REL, false>(ldsK, ldsV, qf, acco, m, l, kt * kBK, a.Nk, sl2, wbrow, a.rel_h, a.rel_w,
                                    a.rel_magic, h, r32, lane);
      else
        fwd_tile<T, DP, REL, true>(ldsK, ldsV, qf, acco, m, l, kt * kBK, a.Nk, sl2, wbrow, a.rel_h, a.rel_w,
                                   a.rel_magic, h, r32, lane);
    }
    if (more) {                               // the other buffer was last read before the previous barrier
      if (nbuf<T, DP>() == 1) __syncthreads();
      char* nk = smem + (nbuf<T, DP>() == 2 ? ((kt + 1) & 1) : 0) * TB;
      kst.write(nk, tid);
      vst.write(nk + I::bytes(kBK), tid);
    }
    __syncthreads();
  }

  l += __shfl_xor(l, 32);
  const float inv = 1.f / l;
  if (q < a.Nq) {
    T* O = reinterpret_cast<T*>(a.out) + b * a.os[0] + hh * a.os[2] + (long long)q * a.os[1];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4<T, VEC>(O, 32 * t + 8 * g + 4 * h, a.D, acco[t][4 * g] * inv, acco[t][4 * g + 1] * inv,
                       acco[t][4 * g + 2] * inv, acco[t][4 * g + 3] * inv);
    if (h == 0 && a.lse) a.lse[((size_t)b * a.H + hh) * a.Nq + q] = (m + lg2(l)) * kLn2;
  }
}

// ===================================================================== backward: dK, dV
template <typename T, int DP, bool VEC, bool REL>
__global__ __launch_bounds__(256, DP >= 128 ? 1 : 2) void attn_bwd_dkdv_kernel(AttnArgs a) {
  using M = MF<T>;
  using I = Img<T, DP>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // double-buffered query tile: [buf][Q img | dO img | -lse/scale [64] | -delta [64] | REL bias [64][RW]]
  const int RW = a.rel_h + a.rel_w + 1;
  const int TB = 2 * I::bytes(kBQT) + 2 * kBQT * 4 + (REL ? kBQT * RW * 4 : 0);

  const int nkb = (a.Nk + kBKV - 1) / kBKV;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = bid % nkb;
  bid /= nkb;
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int key = kb * kBKV + w * 32 + r32;
  const bool active = kb * kBKV + __builtin_amdgcn_readfirstlane(w) * 32 < a.Nk;

  const T* Q = reinterpret_cast<const T*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const T* K = reinterpret_cast<const T*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const T* V = reinterpret_cast<const T*>(a.v) + b * a.vs[0] + hh * a.vs[2];
  const T* G = reinterpret_cast<const T*>(a.dout) + b * a.dos[0] + hh * a.dos[2];
  const size_t rowoff = ((size_t)b * a.H + hh) * a.Nq;

  constexpr int NS = DP / M::KSTEP;
  constexpr int NP = 32 / M::KSTEP;
  constexpr int NT = DP / 32;

  typename M::frag kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    kf[s] = gfrag<T, VEC>(K, key, a.Nk, a.ks[1], a.D, s, h);
    vf[s] = gfrag<T, VEC>(V, key, a.Nk, a.vs[1], a.D, s, h);
  }
  f32x16 adk[NT], adv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) { adk[t] = zero16(); adv[t] = zero16(); }

  const float sl2 = a.scale * kLog2e;
  int kx = 0, ky = 0;
  if constexpr (REL) {
    const int kk = min(key, a.Nk - 1);
    kx = (kk * a.rel_magic) >> 20;
    ky = kk - kx * a.rel_w;
  }
  const int nqt = (a.Nq + kBQT - 1) / kBQT;

  Stage<T, DP, kBQT, VEC> qst, gst;
  const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
  const __amdgpu_buffer_rsrc_t rg = row_rsrc(G, a.Nq, a.dos[1]);
  if constexpr (VEC) {
    qst.load_buf(rq, 0, a.qs[1], a.D, tid);
    gst.load_buf(rg, 0, a.dos[1], a.D, tid);
  } else {
    qst.load(Q, 0, a.Nq, a.qs[1], a.D, tid);
    gst.load(G, 0, a.Nq, a.dos[1], a.D, tid);
  }

  // this tile's row constants (-lse/scale, -delta) are fetched into registers together with
  // the Q / dO tile (issue early, write late) -- never a dependent global load inside the loop
  float rc_l = 0.f, rc_d = 0.f;
  auto fetch_rc = [&](int qt) {
    if (tid < kBQT) {
      const int qq = qt * kBQT + tid;
      rc_l = qq < a.Nq ? a.lse[rowoff + qq] : kInf;
      rc_d = qq < a.Nq ? a.delta[rowoff + qq] : 0.f;
    }
  };
  fetch_rc(0);
  // writes the staged Q / dO registers and this tile's row constants into buffer `buf`
  auto put = [&](char* buf, int qt) {
    qst.write(buf, tid);
    gst.write(buf + I::bytes(kBQT), tid);
    float* L = reinterpret_cast<float*>(buf + 2 * I::bytes(kBQT));
    float* Dl = L + kBQT;
    if (tid < kBQT) {
      L[tid] = -rc_l / a.scale;
      Dl[tid] = -rc_d;
    }
    if constexpr (REL) {
      float* Bb = Dl + kBQT;
      for (int i = tid; i < kBQT * (RW - 1); i += 256) {
        const int rr = i / (RW - 1), cc = i % (RW - 1);
        const int qq = qt * kBQT + rr;
        float val = 0.f;
        if (qq < a.Nq)
          val = cc < a.rel_h ? a.bias_h[(rowoff + qq) * a.rel_h + cc]
                             : a.bias_w[(rowoff + qq) * a.rel_w + (cc - a.rel_h)];
        Bb[rr * RW + cc] = val * kLog2e;
      }
    }
  };
  put(smem, 0);
  __syncthreads();

  for (int qt = 0; qt < nqt; ++qt) {
    const char* ldsQ = smem + (nbuf<T, DP>() == 2 ? (qt & 1) : 0) * TB;
    const char* ldsG = ldsQ + I::bytes(kBQT);
    const float* ldsL = reinterpret_cast<const float*>(ldsQ + 2 * I::bytes(kBQT));
    const float* ldsD = ldsL + kBQT;
    const float* ldsB = ldsD + kBQT;
    const bool more = qt + 1 < nqt;
    if (more) {
      fetch_rc(qt + 1);
      if constexpr (VEC) {
        qst.load_buf(rq, (qt + 1) * kBQT, a.qs[1], a.D, tid);
        gst.load_buf(rg, (qt + 1) * kBQT, a.dos[1], a.D, tid);
      } else {
        qst.load(Q, (qt + 1) * kBQT, a.Nq, a.qs[1], a.D, tid);
        gst.load(G, (qt + 1) * kBQT, a.Nq, a.dos[1], a.D, tid);
      }
    }
    const int nu = !active ? 0 : (qt * kBQT + 32 < a.Nq ? 2 : 1);   // skip padding halves / idle waves
#pragma unroll 1
    for (int u = 0; u < nu; ++u) {
      // row constants as the initial accumulators: S - lse/scale and dP - delta
      f32x16 sp, dp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(ldsL + 32 * u + 8 * g + 4 * h);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(ldsD + 32 * u + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sp[4 * g + j] = l4[j];
          dp[4 * g + j] = d4[j];
        }
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sp = M::mma(I::rowfrag(ldsQ, 32 * u + r32, s, h), kf[s], sp);
        dp = M::mma(I::rowfrag(ldsG, 32 * u + r32, s, h), vf[s], dp);
      }
      // sp: S[q = 32u + row_of(r,h)][key = lane] - lse/scale; dp: dP - delta
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float x = sp[r] * sl2;
        if constexpr (REL) {
          const int ql = 32 * u + row_of(r, h);
          x += ldsB[ql * RW + kx] + ldsB[ql * RW + a.rel_h + ky];
        }
        const float p = ex2(x);
        sp[r] = p;
        dp[r] = p * dp[r];
      }
#pragma unroll
      for (int s2 = 0; s2 < NP; ++s2) {
        const typename M::frag pf = acc_frag<T>(sp, s2);
        const typename M::frag sf = acc_frag<T>(dp, s2);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          adv[t] = M::mma(I::colfrag(ldsG, 32 * u, s2, 32 * t, lane), pf, adv[t]);
          adk[t] = M::mma(I::colfrag(ldsQ, 32 * u, s2, 32 * t, lane), sf, adk[t]);
        }
      }
    }
    if (more) {
      if (nbuf<T, DP>() == 1) __syncthreads();
      put(smem + (nbuf<T, DP>() == 2 ? ((qt + 1) & 1) : 0) * TB, qt + 1);
    }
    __syncthreads();
  }

  if constexpr (sizeof(T) == 2 && VEC) {
    if (active) {   // whole-row stores through a per-wave LDS scratch (buffers free)
      const int k0 = kb * kBKV + w * 32;
      char* scr = smem + w * 32 * DP * 2;
      T* DK = reinterpret_cast<T*>(a.dk) + b * a.dks[0] + hh * a.dks[2] + (long long)k0 * a.dks[1];
      T* DV = reinterpret_cast<T*>(a.dv) + b * a.dvs[0] + hh * a.dvs[2] + (long long)k0 * a.dvs[1];
      wave_store_rows<DP>(adk, a.scale, scr, reinterpret_cast<__bf16*>(DK), a.dks[1], a.Nk - k0, a.D, lane);
      wave_store_rows<DP>(adv, 1.f, scr, reinterpret_cast<__bf16*>(DV), a.dvs[1], a.Nk - k0, a.D, lane);
    }
  } else if (key < a.Nk) {
    T* DK = reinterpret_cast<T*>(a.dk) + b * a.dks[0] + hh * a.dks[2] + (long long)key * a.dks[1];
    T* DV = reinterpret_cast<T*>(a.dv) + b * a.dvs[0] + hh * a.dvs[2] + (long long)key * a.dvs[1];
    const float sc = a.scale;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d0 = 32 * t + 8 * g + 4 * h;
        store4<T, VEC>(DK, d0, a.D, adk[t][4 * g] * sc, adk[t][4 * g + 1] * sc, adk[t][4 * g + 2] * sc,
                       adk[t][4 * g + 3] * sc);
        store4<T, VEC>(DV, d0, a.D, adv[t][4 * g], adv[t][4 * g + 1], adv[t][4 * g + 2], adv[t][4 * g + 3]);
      }
  }
}

// ========================================================================= backward: dQ
template <typename T, int DP, bool VEC, bool REL>
__global__ __launch_bounds__(256, DP >= 128 ? 1 : 2) void attn_bwd_dq_kernel(AttnArgs a) {
  using M = MF<T>;
  using I = Img<T, DP>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TB = 2 * I::bytes(kBK);                              // [buf][K | V]
  float* ldsB = reinterpret_cast<float*>(smem + nbuf<T, DP>() * TB);  // REL: bias [4][32][RW]
  // REL: dbias accumulators [4][32][RW] follow the bias tables

  const int nqb = (a.Nq + kBQ - 1) / kBQ;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb;
  bid /= nqb;
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q = qb * kBQ + w * 32 + r32;
  const bool active = qb * kBQ + __builtin_amdgcn_readfirstlane(w) * 32 < a.Nq;

  const T* Q = reinterpret_cast<const T*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const T* K = reinterpret_cast<const T*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const T* V = reinterpret_cast<const T*>(a.v) + b * a.vs[0] + hh * a.vs[2];
  const T* G = reinterpret_cast<const T*>(a.dout) + b * a.dos[0] + hh * a.dos[2];
  const size_t rowoff = ((size_t)b * a.H + hh) * a.Nq;

  constexpr int NS = DP / M::KSTEP;
  constexpr int NP = 32 / M::KSTEP;
  constexpr int NT = DP / 32;

  typename M::frag qf[NS], gf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    qf[s] = gfrag<T, VEC>(Q, q, a.Nq, a.qs[1], a.D, s, h);
    gf[s] = gfrag<T, VEC>(G, q, a.Nq, a.dos[1], a.D, s, h);
  }
  const bool qok = q < a.Nq;
  // delta = rowsum(dO * O), from the dO fragments already in registers (this pass runs first
  // and publishes delta for the dK/dV pass)
  float dlt;
  {
    const T* O = reinterpret_cast<const T*>(a.o) + b * a.os[0] + hh * a.os[2];
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const typename M::frag of = gfrag<T, VEC>(O, q, a.Nq, a.os[1], a.D, s, h);
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) part += (float)of[j] * (float)gf[s][j];
      } else {
        part += of * gf[s];
      }
    }
    dlt = part + __shfl_xor(part, 32);
    if (qok && h == 0) a.delta[rowoff + q] = dlt;
  }
  const float lsc = qok ? -a.lse[rowoff + q] / a.scale : -kInf;   // S^T init: - lse / scale
  const int RW = a.rel_h + a.rel_w + 1;
  float* wb = ldsB + w * 32 * RW;
  float* wdb = ldsB + 4 * 32 * RW + w * 32 * RW;
  if constexpr (REL) {
    for (int i = lane; i < 32 * RW; i += 64) {
      const int rr = i / RW, cc = i % RW;
      const int qq = qb * kBQ + w * 32 + rr;
      float val = 0.f;
      if (qq < a.Nq && cc < RW - 1)
        val = cc < a.rel_h ? a.bias_h[(rowoff + qq) * a.rel_h + cc]
                           : a.bias_w[(rowoff + qq) * a.rel_w + (cc - a.rel_h)];
      wb[i] = val * kLog2e;
      wdb[i] = 0.f;
    }
  }

  f32x16 adq[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) adq[t] = zero16();
  const float sl2 = a.scale * kLog2e;
  const int nkt = (a.Nk + kBK - 1) / kBK;

  Stage<T, DP, kBK, VEC> kst, vst;
  const __amdgpu_buffer_rsrc_t rk = row_rsrc(K, a.Nk, a.ks[1]);
  const __amdgpu_buffer_rsrc_t rv = row_rsrc(V, a.Nk, a.vs[1]);
  if constexpr (VEC) {
    kst.load_buf(rk, 0, a.ks[1], a.D, tid);
    vst.load_buf(rv, 0, a.vs[1], a.D, tid);
  } else {
    kst.load(K, 0, a.Nk, a.ks[1], a.D, tid);
    vst.load(V, 0, a.Nk, a.vs[1], a.D, tid);
  }

  kst.write(smem, tid);
  vst.write(smem + I::bytes(kBK), tid);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const char* ldsK = smem + (nbuf<T, DP>() == 2 ? (kt & 1) : 0) * TB;
    const char* ldsV = ldsK + I::bytes(kBK);
    const bool more = kt + 1 < nkt;
    if (more) {
      if constexpr (VEC) {
        kst.load_buf(rk, (kt + 1) * kBK, a.ks[1], a.D, tid);
        vst.load_buf(rv, (kt + 1) * kBK, a.vs[1], a.D, tid);
      } else {
        kst.load(K, (kt + 1) * kBK, a.Nk, a.ks[1], a.D, tid);
        vst.load(V, (kt + 1) * kBK, a.Nk, a.vs[1], a.D, tid);
      }
    }
    const int nu = !active ? 0 : (kt * kBK + 32 < a.Nk ? 2 : 1);   // skip padding halves / idle waves
    const bool tail = (kt + 1) * kBK > a.Nk;           // only the last tile needs the key mask
#pragma unroll 1
    for (int u = 0; u < nu; ++u) {
      f32x16 sp, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sp[r] = lsc;
        dp[r] = -dlt;
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sp = M::mma(I::rowfrag(ldsK, 32 * u + r32, s, h), qf[s], sp);
        dp = M::mma(I::rowfrag(ldsV, 32 * u + r32, s, h), gf[s], dp);
      }
      // sp: S^T[key = kt*64 + 32u + row_of(r,h)][q = lane] - lse/scale; dp: dP^T - delta
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * kBK + 32 * u + row_of(r, h);
        float x = sp[r] * sl2;
        int kx = 0, ky = 0;
        if constexpr (REL) {
          const int kk = min(key, a.Nk - 1);
          kx = (kk * a.rel_magic) >> 20;
          ky = kk - kx * a.rel_w;
          x += wb[r32 * RW + kx] + wb[r32 * RW + a.rel_h + ky];
        }
        const float p = (!tail || key < a.Nk) ? ex2(x) : 0.f;
        const float ds = p * dp[r];
        dp[r] = ds;
        if constexpr (REL) {
          if (key < a.Nk) {
            atomicAdd(&wdb[r32 * RW + kx], ds);
            atomicAdd(&wdb[r32 * RW + a.rel_h + ky], ds);
          }
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < NP; ++s2) {
        const typename M::frag sf = acc_frag<T>(dp, s2);
#pragma unroll
        for (int t = 0; t < NT; ++t) adq[t] = M::mma(I::colfrag(ldsK, 32 * u, s2, 32 * t, lane), sf, adq[t]);
      }
    }
    if (more) {
      if (nbuf<T, DP>() == 1) __syncthreads();
      char* nk = smem + (nbuf<T, DP>() == 2 ? ((kt + 1) & 1) : 0) * TB;
      kst.write(nk, tid);
      vst.write(nk + I::bytes(kBK), tid);
    }
    __syncthreads();
  }

  if constexpr (sizeof(T) == 2 && VEC) {
    if (active) {
      const int q0 = qb * kBQ + w * 32;
      T* DQ = reinterpret_cast<T*>(a.dq) + b * a.dqs[0] + hh * a.dqs[2] + (long long)q0 * a.dqs[1];
      wave_store_rows<DP>(adq, a.scale, smem + w * 32 * DP * 2, reinterpret_cast<__bf16*>(DQ), a.dqs[1],
                          a.Nq - q0, a.D, lane);
    }
  } else if (qok) {
    T* DQ = reinterpret_cast<T*>(a.dq) + b * a.dqs[0] + hh * a.dqs[2] + (long long)q * a.dqs[1];
    const float sc = a.scale;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4<T, VEC>(DQ, 32 * t + 8 * g + 4 * h, a.D, adq[t][4 * g] * sc, adq[t][4 * g + 1] * sc,
                       adq[t][4 * g + 2] * sc, adq[t][4 * g + 3] * sc);
  }
  if constexpr (REL) {
    __syncthreads();   // LDS atomics of both lane halves complete (wave-local region, but be safe)
    for (int i = lane; i < 32 * (RW - 1); i += 64) {
      const int rr = i / (RW - 1), cc = i % (RW - 1);
      const int qq = qb * kBQ + w * 32 + rr;
      if (qq >= a.Nq) continue;
      const float val = wdb[rr * RW + cc];
      if (cc < a.rel_h) a.dbias_h[(rowoff + qq) * a.rel_h + cc] = val;
      else a.dbias_w[(rowoff + qq) * a.rel_w + (cc - a.rel_h)] = val;
    }
  }
}

}  // namespace sae
