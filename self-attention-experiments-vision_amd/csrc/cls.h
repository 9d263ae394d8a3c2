// cls.h -- single-query attention (Nq = 1) as a memory-bound K/V stream on the VALU.
//
// CaiT's class attention (models/cait.py:10-15: the CLS row inputs[:, 0:1] attends over
// [cls, x], Nk = 197, H = 8, D = 48) and CeiT's last-token query (models/ceit.py:11-16) run the
// core of attention.py:39-58 with ONE query row.  On the 32 x 32 MFMA tiles of fwd2.h / bwd3.h that
// row is 1 of 32 (31/32 of the matrix work and of the softmax VALU is padding); per (batch, head)
// the op is a read of K and V (and a write of dK, dV in the backward), so it is an HBM stream:
//   * one 256-thread workgroup per (batch, head); 8 lanes per key row (16-byte chunks: D <= 64 in
//     one chunk per lane, D <= 128 in two), 32 key rows per pass -- each row segment is read by
//     8 consecutive lanes (coalesced) and exactly once;
//   * K and V rows of a batch of 256 keys loaded at once (all in flight), online softmax over
//     batches with block max / sum by shuffles + LDS;
//   * fp32 everywhere (P is not rounded to bf16 before P V), outputs rounded to bf16 once;
//   * fixed reduction orders: deterministic.
// Backward (same layout): per key s, p = exp(s - lse), dP = dO . V, dS = p (dP - delta),
// dV = p dO, dK = scale dS q written per key row, dQ = scale sum_k dS K summed over the 32
// key groups through LDS.  delta = dO . O is formed in the prologue (no workspace).
#pragma once
#include "common.h"

namespace sae {

constexpr int kClsLpk = 8;                     // lanes per key row
constexpr int kClsGroups = 256 / kClsLpk;      // key rows per pass

__device__ __forceinline__ float cls_sum8(float x) {   // sum over the 8 lanes of a key group
  x += __shfl_xor(x, 1);
  x += __shfl_xor(x, 2);
  x += __shfl_xor(x, 4);
  return x;
}

// chunk c (elements 8 (sub + 8c) .. + 7) of a bf16 row as fp32, zero past D
template <int NCH>
__device__ __forceinline__ void cls_load(const __bf16* row, int sub, int D, float (&v)[NCH][8]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int d0 = 8 * (sub + 8 * c);
    if (d0 < D) {
      const bf16x8 x = *reinterpret_cast<const bf16x8*>(row + d0);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = (float)x[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
}

template <int NCH>
__device__ __forceinline__ void cls_store(__bf16* row, int sub, int D, const float (&v)[NCH][8], float sc) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int d0 = 8 * (sub + 8 * c);
    if (d0 < D) {
      bf16x8 x;
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (__bf16)(v[c][j] * sc);
      *reinterpret_cast<bf16x8*>(row + d0) = x;
    }
  }
}

// block-wide max / sum of one value per thread (256 threads), result in every thread
__device__ __forceinline__ float cls_block_max(float x, float* red) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) x = fmaxf(x, __shfl_xor(x, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
__device__ __forceinline__ float cls_block_sum(float x, float* red) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// the [32 groups][D] fp32 partial rows of acc summed over the groups (fixed order) -> lane chunk
template <int NCH>
__device__ __forceinline__ void cls_group_sum(float (&acc)[NCH][8], float* part, int grp, int sub, int D) {
  const int DP = 64 * NCH;
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) part[grp * DP + 8 * (sub + 8 * c) + j] = acc[c][j];
  __syncthreads();
  if (grp == 0) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float s = 0.f;
        for (int g = 0; g < kClsGroups; ++g) s += part[g * DP + 8 * (sub + 8 * c) + j];
        acc[c][j] = s;
      }
  }
  (void)D;
}

// key rows per thread per batch: a batch (32 x kClsU = 256 keys) has all its K and V row loads in
// flight at once (the loop is latency-bound otherwise: one dependent HBM round trip per key pass)
constexpr int kClsU = 8;

// raw bf16 chunks of key row k (zero past Nk / D)
template <int NCH>
__device__ __forceinline__ void cls_raw(const __bf16* base, long long ld, int k, int Nk, int sub, int D,
                                        uint4 (&v)[NCH]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int d0 = 8 * (sub + 8 * c);
    v[c] = (k < Nk && d0 < D) ? *reinterpret_cast<const uint4*>(base + (long long)k * ld + d0) : uint4{0, 0, 0, 0};
  }
}
template <int NCH>
__device__ __forceinline__ float cls_dot(const float (&q)[NCH][8], const uint4 (&v)[NCH]) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const bf16x8 x = __builtin_bit_cast(bf16x8, v[c]);
#pragma unroll
    for (int j = 0; j < 8; ++j) s = __builtin_fmaf(q[c][j], (float)x[j], s);
  }
  return s;
}

// LDS: 4 reduction slots + [32][64 NCH] partial rows
template <int NCH> size_t cls_lds_bytes() { return (4 + (size_t)kClsGroups * 64 * NCH) * 4; }

// Online softmax over batches of 256 keys (one batch for CaiT's 197): per batch the block max,
// the rescale of the running (l, acc) by exp(m_old - m_new), then P and P V in fp32.
template <int NCH>
__global__ __launch_bounds__(256) void attn_cls_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float csm[];
  float* red = csm;                // [4]
  float* part = red + 4;           // [32][64 NCH]
  // XCD-aware order: the heads of one batch row share cache lines of the token-major K / V rows,
  // so consecutive (batch, head) pairs run on one XCD (one L2)
  const int bh = xcd_remap(blockIdx.x, gridDim.x), b = bh / a.H, hh = bh % a.H;
  const int tid = threadIdx.x, sub = tid & 7, grp = tid >> 3;
  const __bf16* Q = reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const __bf16* K = reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const __bf16* V = reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2];
  float qv[NCH][8];
  cls_load<NCH>(Q, sub, a.D, qv);
  float acc[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  float m = -kInf, l = 0.f;
  for (int kb = 0; kb < a.Nk; kb += kClsGroups * kClsU) {
    uint4 kr[kClsU][NCH], vr[kClsU][NCH];
#pragma unroll
    for (int u = 0; u < kClsU; ++u) {
      cls_raw<NCH>(K, a.ks[1], kb + grp + kClsGroups * u, a.Nk, sub, a.D, kr[u]);
      cls_raw<NCH>(V, a.vs[1], kb + grp + kClsGroups * u, a.Nk, sub, a.D, vr[u]);
    }
    float s[kClsU], mx = -kInf;
#pragma unroll
    for (int u = 0; u < kClsU; ++u) {
      s[u] = cls_sum8(cls_dot<NCH>(qv, kr[u])) * a.scale;
      if (kb + grp + kClsGroups * u >= a.Nk) s[u] = -kInf;
      mx = fmaxf(mx, s[u]);
    }
    const float mn = fmaxf(m, cls_block_max(mx, red));
    const float alpha = __expf(m - mn);   // 0 on the first batch (m = -inf)
    m = mn;
    float ls = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[c][j] *= alpha;
#pragma unroll
    for (int u = 0; u < kClsU; ++u) {
      const float p = __expf(s[u] - m);
      ls += p;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const bf16x8 x = __builtin_bit_cast(bf16x8, vr[u][c]);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[c][j] = __builtin_fmaf(p, (float)x[j], acc[c][j]);
      }
    }
    // every lane of a key group holds the same p: the sub == 0 lanes carry the row sum
    l = l * alpha + cls_block_sum(sub == 0 ? ls : 0.f, red);
  }
  cls_group_sum<NCH>(acc, part, grp, sub, a.D);
  if (grp == 0) {
    __bf16* O = reinterpret_cast<__bf16*>(a.out) + b * a.os[0] + hh * a.os[2];
    cls_store<NCH>(O, sub, a.D, acc, 1.f / l);
    if (sub == 0 && a.lse) a.lse[bh] = m + __logf(l);
  }
}

template <int NCH>
__global__ __launch_bounds__(256) void attn_cls_bwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float csm[];
  float* part = csm + 4;
  // XCD-aware order: the heads of one batch row share cache lines of the token-major K / V rows,
  // so consecutive (batch, head) pairs run on one XCD (one L2)
  const int bh = xcd_remap(blockIdx.x, gridDim.x), b = bh / a.H, hh = bh % a.H;
  const int tid = threadIdx.x, sub = tid & 7, grp = tid >> 3;
  const __bf16* Q = reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const __bf16* K = reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const __bf16* V = reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2];
  const __bf16* O = reinterpret_cast<const __bf16*>(a.o) + b * a.os[0] + hh * a.os[2];
  const __bf16* G = reinterpret_cast<const __bf16*>(a.dout) + b * a.dos[0] + hh * a.dos[2];
  __bf16* DK = reinterpret_cast<__bf16*>(a.dk) + b * a.dks[0] + hh * a.dks[2];
  __bf16* DV = reinterpret_cast<__bf16*>(a.dv) + b * a.dvs[0] + hh * a.dvs[2];
  float qv[NCH][8], gv[NCH][8];
  cls_load<NCH>(Q, sub, a.D, qv);
  cls_load<NCH>(G, sub, a.D, gv);
  float delta = 0.f;
  {
    float ov[NCH][8];
    cls_load<NCH>(O, sub, a.D, ov);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) delta = __builtin_fmaf(gv[c][j], ov[c][j], delta);
    delta = cls_sum8(delta);
  }
  const float lse = a.lse[bh];
  float acc[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  for (int kb = 0; kb < a.Nk; kb += kClsGroups * kClsU) {
    uint4 kr[kClsU][NCH], vr[kClsU][NCH];
#pragma unroll
    for (int u = 0; u < kClsU; ++u) {
      cls_raw<NCH>(K, a.ks[1], kb + grp + kClsGroups * u, a.Nk, sub, a.D, kr[u]);
      cls_raw<NCH>(V, a.vs[1], kb + grp + kClsGroups * u, a.Nk, sub, a.D, vr[u]);
    }
#pragma unroll
    for (int u = 0; u < kClsU; ++u) {
      const int k = kb + grp + kClsGroups * u;
      const float s = cls_sum8(cls_dot<NCH>(qv, kr[u]));
      const float dp = cls_sum8(cls_dot<NCH>(gv, vr[u]));
      if (k >= a.Nk) continue;   // uniform over the key group (after its shuffles)
      const float p = __expf(s * a.scale - lse);
      const float ds = p * (dp - delta);
      cls_store<NCH>(DV + (long long)k * a.dvs[1], sub, a.D, gv, p);
      cls_store<NCH>(DK + (long long)k * a.dks[1], sub, a.D, qv, ds * a.scale);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const bf16x8 x = __builtin_bit_cast(bf16x8, kr[u][c]);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[c][j] = __builtin_fmaf(ds, (float)x[j], acc[c][j]);
      }
    }
  }
  cls_group_sum<NCH>(acc, part, grp, sub, a.D);
  if (grp == 0) {
    __bf16* DQ = reinterpret_cast<__bf16*>(a.dq) + b * a.dqs[0] + hh * a.dqs[2];
    cls_store<NCH>(DQ, sub, a.D, acc, a.scale);
  }
}

}  // namespace sae
