// fwd3.h -- bf16 attention forward with TWO 32-row query blocks per wave (64 query rows).
//
// Same algorithm, layout and tile pipeline as fwd2.h (reference chain
// models/layers/attentions/attention.py:39-58).  What changes is the wave's share: every K row
// fragment and every transposed V fragment read from LDS feeds two MFMAs (one per query block),
// halving LDS read bytes per FLOP, and each 64-key tile carries two independent online-softmax
// chains, so the scheduler can issue one block's exp / max / convert VALU work between the other
// block's MFMAs instead of leaving the matrix pipe idle through a single dependent chain.
#pragma once
#include "fwd2.h"

namespace sae {

template <int DP, bool LSUM>
__device__ __forceinline__ void fwd3_tile(const char* ldsK, const char* ldsV, const bf16x8 (&qf)[2][F2<DP>::NS],
                                          f32x16 (&acco)[2][F2<DP>::NT], f32x16 (&lacc)[2], float (&m)[2],
                                          float (&l)[2], int nvalid, float sl2, const unsigned* ka,
                                          const unsigned* va, int h) {
  constexpr int NS = F2<DP>::NS, NT = F2<DP>::NT;
  const bool two = nvalid > 32;
  f32x16 s[2][2];
#pragma unroll
  for (int b = 0; b < 2; ++b) s[b][0] = s[b][1] = zero16();
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const bf16x8 k0 = *reinterpret_cast<const bf16x8*>(ldsK + ka[k]);
    s[0][0] = MF<__bf16>::mma(k0, qf[0][k], s[0][0]);
    s[1][0] = MF<__bf16>::mma(k0, qf[1][k], s[1][0]);
  }
  if (two) {
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const bf16x8 k1 = *reinterpret_cast<const bf16x8*>(ldsK + ka[k] + 32 * DP * 2);
      s[0][1] = MF<__bf16>::mma(k1, qf[0][k], s[0][1]);
      s[1][1] = MF<__bf16>::mma(k1, qf[1][k], s[1][1]);
    }
  }
  if (nvalid < 64) {   // tail tile: keys past the end score -inf (key = row_of(r, h) = c_r + 4h)
    const int nvh = nvalid - 4 * h;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = (r & 3) + 8 * (r >> 2);
        s[b][0][r] = c < nvh ? s[b][0][r] : -kInf;
        s[b][1][r] = c + 32 < nvh ? s[b][1][r] : -kInf;
      }
  }
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    float mx = s[b][0][0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[b][0][r]);
    if (two) {
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[b][1][r]);
    }
    mx = xhalf_max(mx) * sl2;
    if (!__all(mx - m[b] <= 8.f)) {
      const float mn = fmaxf(m[b], mx);
      const float alpha = ex2(m[b] - mn);
      m[b] = mn;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acco[b][t][r] *= alpha;
      if constexpr (LSUM) {
#pragma unroll
        for (int r = 0; r < 16; ++r) lacc[b][r] *= alpha;
      } else {
        l[b] *= alpha;
      }
    }
    const float mb = m[b];
#pragma unroll
    for (int r = 0; r < 16; ++r) s[b][0][r] = ex2(__builtin_fmaf(s[b][0][r], sl2, -mb));
    if (two) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[b][1][r] = ex2(__builtin_fmaf(s[b][1][r], sl2, -mb));
    }
    if constexpr (!LSUM) {
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) ls += s[b][0][r];
      if (two) {
#pragma unroll
        for (int r = 0; r < 16; ++r) ls += s[b][1][r];
      }
      l[b] += ls;
    }
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (u == 1 && !two) break;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 p0 = acc_frag<__bf16>(s[0][u], s2);
      const bf16x8 p1 = acc_frag<__bf16>(s[1][u], s2);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int ro = (32 * u + 16 * s2) * DP * 2;
        s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ldsV + va[2 * t] + ro));
        s16x4 x2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ldsV + va[2 * t + 1] + ro));
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        s16x8 vv = {x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
        const bf16x8 vf = __builtin_bit_cast(bf16x8, vv);
        acco[0][t] = MF<__bf16>::mma(vf, p0, acco[0][t]);
        acco[1][t] = MF<__bf16>::mma(vf, p1, acco[1][t]);
      }
      if constexpr (LSUM) {
        lacc[0] = MF<__bf16>::mma(ones, p0, lacc[0]);
        lacc[1] = MF<__bf16>::mma(ones, p1, lacc[1]);
      }
    }
  }
}

template <int DP, int NW, int MINW, bool LSUM>
__global__ __launch_bounds__(64 * NW, MINW) void attn_fwd3_kernel(AttnArgs a) {
  using FF = F2<DP>;
  constexpr int NS = FF::NS, NT = FF::NT, TILE = FF::TILE;
  constexpr int BQ = 64 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nqb = (a.Nq + BQ - 1) / BQ;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb;
  bid /= nqb;
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q0 = qb * BQ + w * 64;   // this wave's first query row (block 0: q0.., block 1: q0+32..)
  const bool active = qb * BQ + __builtin_amdgcn_readfirstlane(w) * 64 < a.Nq;

  const __bf16* Q = reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const __bf16* K = reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const __bf16* V = reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2];

  F2Stage<DP, NW> kst[2], vst[2];   // two register stages in flight, as in fwd2
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    kst[r].init(tid, a.ks[1], a.D);
    vst[r].init(tid, a.vs[1], a.D);
  }
  const __amdgpu_buffer_rsrc_t rk = row_rsrc(K, a.Nk, a.ks[1]);
  const __amdgpu_buffer_rsrc_t rv = row_rsrc(V, a.Nk, a.vs[1]);
  const unsigned kstep = (unsigned)(64 * a.ks[1] * 2), vstep = (unsigned)(64 * a.vs[1] * 2);
  const int nkt = (a.Nk + 63) / 64;
  kst[0].load(rk, 0);
  vst[0].load(rv, 0);
  if (nkt > 1) {
    kst[1].load(rk, kstep);
    vst[1].load(rv, vstep);
  }

  bf16x8 qf[2][NS];
  {
    const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
      const unsigned qo = (unsigned)((long long)(q0 + 32 * bb + r32) * a.qs[1] * 2);
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        const unsigned off = (16 * k + 8 * h < a.D) ? qo + (16 * k + 8 * h) * 2 : 0x80000000u;
        qf[bb][k] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, off, 0, 0));
      }
    }
  }
  unsigned ka[NS], va[2 * NT];
#pragma unroll
  for (int k = 0; k < NS; ++k) ka[k] = r32 * DP * 2 + 16 * ((2 * k + h) ^ swz<DP>(r32));
  {
    const int li = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int colb = 32 * t + 16 * (g & 1) + 4 * (li & 3);
      const int chunk = colb >> 3, half = (colb >> 2) & 1;
      const int r1 = 4 * h + (li >> 2), r2 = r1 + 8;
      va[2 * t] = r1 * DP * 2 + 16 * (chunk ^ swz<DP>(r1)) + 8 * half;
      va[2 * t + 1] = r2 * DP * 2 + 16 * (chunk ^ swz<DP>(r2)) + 8 * half;
    }
  }

  f32x16 acco[2][NT], lacc[2];
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
    lacc[bb] = zero16();
#pragma unroll
    for (int t = 0; t < NT; ++t) acco[bb][t] = zero16();
  }
  float m[2] = {-kInf, -kInf}, l[2] = {0.f, 0.f};
  const float sl2 = a.scale * kLog2e;

  kst[0].write(smem);
  vst[0].write(smem + TILE);
  vm_wait_all();
  __syncthreads();
  for (int kt = 0; kt < nkt; kt += 2) {
#pragma unroll
    for (int bsel = 0; bsel < 2; ++bsel) {
      const int t = kt + bsel;
      if (t >= nkt) break;
      char* cur = smem + bsel * 2 * TILE;
      char* nxt = smem + (bsel ^ 1) * 2 * TILE;
      if (t + 2 < nkt) {
        kst[bsel].load(rk, (unsigned)(t + 2) * kstep);
        vst[bsel].load(rv, (unsigned)(t + 2) * vstep);
      }
      if (active)
        fwd3_tile<DP, LSUM>(cur, cur + TILE, qf, acco, lacc, m, l, min(64, a.Nk - 64 * t), sl2, ka, va, h);
      if (t + 1 < nkt) {
        kst[bsel ^ 1].write(nxt);
        vst[bsel ^ 1].write(nxt + TILE);
      }
      __syncthreads();
    }
  }

  if (!active) return;
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
    const float lt = LSUM ? lacc[bb][0] : xhalf_sum(l[bb]);
    const float inv = 1.f / lt;
    const int qr = q0 + 32 * bb;
    __bf16* O = reinterpret_cast<__bf16*>(a.out) + b * a.os[0] + hh * a.os[2] + (long long)qr * a.os[1];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acco[bb][t][r] *= inv;
    wave_store_rows<DP>(acco[bb], 1.f, smem + (2 * w + bb) * 32 * DP * 2, O, a.os[1], a.Nq - qr, a.D, lane);
    const int q = qr + r32;
    if (q < a.Nq && h == 0 && a.lse) a.lse[((size_t)b * a.H + hh) * a.Nq + q] = (m[bb] + lg2(lt)) * kLn2;
  }
}

}  // namespace sae
