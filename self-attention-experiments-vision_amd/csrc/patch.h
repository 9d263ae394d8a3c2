// patch.h -- the patch embedding (models/layers/stems/patch_embed.py:15-26) as ONE GEMM whose
// A operand is gathered straight from the images while it is staged: no patchified copy of the
// batch is ever written.
//
//   tokens[n][p][e] = sum_k A[m][k] W[k][e],  A[m][k] = image[n][py Ph + ky][px Pw + kx][c]
//   (einops 'b (h ph) (w pw) c -> b (h w) (ph pw c)': k = (ky Pw + kx) C + c, p = py gw + px)
//   dW[k][e] = sum_m A[m][k] dY[m][e]   (the images take no gradient)
//
// Two image layouts (PatchGeom in common.h):
//   * NHWC, the model's call signature: token row m = n L + p; eight consecutive k of one token
//     are contiguous (Pw C % 8 == 0), so a 16-byte chunk of the [128 tokens][64 k] operand image
//     is one 16-byte (bf16) or two (fp32) loads;
//   * HWCN, the train-step feed (train.py:80 rearranges 'H W C N -> N H W C' after the pipeline's
//     double-transpose, input_pipeline.py:187-191): the batch index is the contiguous one, so the
//     GEMM walks tokens as m = p Nb + n and a chunk is eight consecutive images at one k (one
//     16-byte load), scattered into eight operand rows; the epilogue stores row m at n L + p.
// fp32 images are rounded to bf16 while staged (train.py:81 casts the images to bf16).
// The rest is gemm_nt_kernel / gemm_dw_kernel with these loaders.
#pragma once
#include "gemm_dw.h"
#include "gemm_nt.h"

namespace sae {

// element offset of GEMM row m of the patch matrix (k = 0)
template <bool HWCN>
__device__ __forceinline__ unsigned patch_rowbase(const PatchGeom& g, int m) {
  int n, p;
  if constexpr (HWCN) {
    p = g.dNb.div(m);
    n = m - p * g.Nb;
  } else {
    n = g.dL.div(m);
    p = m - n * g.L;
  }
  const int py = g.dgw.div(p), px = p - py * g.gw;
  if constexpr (HWCN) return ((unsigned)(py * g.Ph) * g.Wimg + (unsigned)(px * g.Pw)) * g.C * g.Nb + n;
  return ((unsigned)(n * g.Himg + py * g.Ph) * g.Wimg + (unsigned)(px * g.Pw)) * g.C;
}
// element offset of column k (ky, then kx c within one contiguous patch row)
template <bool HWCN>
__device__ __forceinline__ unsigned patch_kofs(const PatchGeom& g, int k) {
  const int ky = g.dPwC.div(k), r2 = k - ky * g.PwC;
  const unsigned o = (unsigned)ky * g.WC + r2;
  return HWCN ? o * g.Nb : o;
}
// output row of GEMM row m
template <bool HWCN>
__device__ __forceinline__ long long patch_orow(const PatchGeom& g, int m) {
  if constexpr (!HWCN) return m;
  const int p = g.dNb.div(m), n = m - p * g.Nb;
  return (long long)n * g.L + p;
}
// eight consecutive image elements as bf16
template <bool F32>
__device__ __forceinline__ uint4 patch_load8(const void* x, unsigned e) {
  if constexpr (F32) {
    const f32x4* p = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(x) + e);
    const f32x4 u = p[0], v = p[1];
    const bf16x8 r = {(__bf16)u[0], (__bf16)u[1], (__bf16)u[2], (__bf16)u[3],
                      (__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    return __builtin_bit_cast(uint4, r);
  } else {
    return *reinterpret_cast<const uint4*>(reinterpret_cast<const __bf16*>(x) + e);
  }
}
__device__ __forceinline__ unsigned short u4_half(const uint4& v, int j) {
  const unsigned w = j < 2 ? v.x : j < 4 ? v.y : j < 6 ? v.z : v.w;
  return (unsigned short)((j & 1) ? (w >> 16) : (w & 0xffffu));
}

// ---- forward: gemm_nt A operand, [128 tokens][64 k] image (128-byte rows, swz<64>)
// Rows past M and columns past K load from clamped (valid) addresses: their values only reach
// output rows that are never stored, or stages that are never computed.
template <bool HWCN, bool F32>
struct NtPatchA {
  uint4 v[4];
  unsigned rb[HWCN ? 1 : 4];
  int tid;
  __device__ __forceinline__ void init(const NtArgs& a, int tid_, int m0) {
    tid = tid_;
    if constexpr (HWCN) {   // thread: rows 8 rg .. 8 rg + 7 (eight images of one patch), columns kk_i
      const int rg = tid & 15;
      rb[0] = patch_rowbase<true>(a.pg, min(m0 + 8 * rg, a.M - 8));
    } else {                // thread: rows (tid >> 3) + 32 i, columns 8 (tid & 7) .. + 7
#pragma unroll
      for (int i = 0; i < 4; ++i) rb[i] = patch_rowbase<false>(a.pg, min(m0 + (tid >> 3) + 32 * i, a.M - 1));
    }
  }
  __device__ __forceinline__ void load(const NtArgs& a, int st) {
    if constexpr (HWCN) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int k = st * kNtK + (tid >> 4) + 16 * i;
        k = k < a.K ? k : 0;
        v[i] = patch_load8<F32>(a.pg.x, rb[0] + patch_kofs<true>(a.pg, k));
      }
    } else {
      int k = st * kNtK + 8 * (tid & 7);
      k = k < a.K ? k : 0;
      const unsigned ko = patch_kofs<false>(a.pg, k);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = patch_load8<F32>(a.pg.x, rb[i] + ko);
    }
  }
  __device__ __forceinline__ void write(char* img) const {
    if constexpr (HWCN) {
      const int rg = tid & 15;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kk = (tid >> 4) + 16 * i;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = 8 * rg + j;
          *reinterpret_cast<unsigned short*>(img + r * 128 + 16 * ((kk >> 3) ^ swz<64>(r)) + 2 * (kk & 7)) =
              u4_half(v[i], j);
        }
      }
    } else {
      const int c = tid & 7;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = (tid >> 3) + 32 * i;
        *reinterpret_cast<uint4*>(img + r * 128 + 16 * (c ^ swz<64>(r))) = v[i];
      }
    }
  }
  static __device__ __forceinline__ long long orow(const NtArgs& a, int m) { return patch_orow<HWCN>(a.pg, m); }
};

// ---- weight gradient: gemm_dw X operand, [64 tokens][128 k] image (256-byte rows, swz<128>);
// rows past m1 (the split's end) and columns past I are zero
template <bool HWCN, bool F32>
struct DwPatchX {
  uint4 v[4];
  unsigned ko[HWCN ? 4 : 1];
  bool kok[HWCN ? 4 : 1];
  int tid, m0, m1;
  __device__ __forceinline__ void init(const DwArgs& a, int tid_, int m0_, int m1_, int col0) {
    tid = tid_;
    m0 = m0_;
    m1 = m1_;
    if constexpr (HWCN) {   // thread: token group tg = tid & 7 (8 images), columns (tid >> 3) + 32 i
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = col0 + (tid >> 3) + 32 * i;
        kok[i] = k < a.I;
        ko[i] = patch_kofs<true>(a.pg, kok[i] ? k : 0);
      }
    } else {                // thread: tokens (tid >> 4) + 16 i, columns 8 (tid & 15) .. + 7
      const int k = col0 + 8 * (tid & 15);
      kok[0] = k < a.I;
      ko[0] = patch_kofs<false>(a.pg, kok[0] ? k : 0);
    }
  }
  __device__ __forceinline__ void load(const DwArgs& a, int st) {
    if constexpr (HWCN) {
      const int m = m0 + st * kDwK + 8 * (tid & 7);
      const bool mok = m < m1;
      const unsigned rb = patch_rowbase<true>(a.pg, mok ? m : m0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        v[i] = (mok && kok[i]) ? patch_load8<F32>(a.pg.x, rb + ko[i]) : uint4{0, 0, 0, 0};
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + st * kDwK + (tid >> 4) + 16 * i;
        const bool ok = m < m1 && kok[0];
        v[i] = ok ? patch_load8<F32>(a.pg.x, patch_rowbase<false>(a.pg, m) + ko[0]) : uint4{0, 0, 0, 0};
      }
    }
  }
  __device__ __forceinline__ void write(char* img) const {
    if constexpr (HWCN) {
      const int tg = tid & 7;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kk = (tid >> 3) + 32 * i;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int r = 8 * tg + j;
          *reinterpret_cast<unsigned short*>(img + r * 256 + 16 * ((kk >> 3) ^ swz<128>(r)) + 2 * (kk & 7)) =
              u4_half(v[i], j);
        }
      }
    } else {
      const int c = tid & 15;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = (tid >> 4) + 16 * i;
        *reinterpret_cast<uint4*>(img + r * 256 + 16 * (c ^ swz<128>(r))) = v[i];
      }
    }
  }
};

// dY rows in the HWCN token order (row m of the GEMM is output row n L + p)
struct DwPermY {
  uint4 v[4];
  int tid, m0, m1, col;
  __device__ __forceinline__ void init(const DwArgs& a, int tid_, int m0_, int m1_, int col0) {
    tid = tid_;
    m0 = m0_;
    m1 = m1_;
    col = col0 + 8 * (tid & 15);
  }
  __device__ __forceinline__ void load(const DwArgs& a, int st) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + st * kDwK + (tid >> 4) + 16 * i;
      const bool ok = m < m1 && col < a.J;
      v[i] = ok ? *reinterpret_cast<const uint4*>(a.dy + patch_orow<true>(a.pg, m) * a.ldy + col) : uint4{0, 0, 0, 0};
    }
  }
  __device__ __forceinline__ void write(char* img) const {
    const int c = tid & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 4) + 16 * i;
      *reinterpret_cast<uint4*>(img + r * 256 + 16 * (c ^ swz<128>(r))) = v[i];
    }
  }
};


// The patch matrix itself (round 5, HWCN train-step feed): A[n L + p][k] bf16 written once, so the
// embedding GEMM and its weight gradient run on the LDS-DMA kernels (gemm8 / gemm_dw8) instead of
// gathering eight images per 16-byte chunk into eight operand rows (the fused HWCN loaders ran the
// 25,088 x 768 x 384 product at 1.3 TB/s of image reads, 59 + 56 us at DeiT-S).  Thread (n, kg)
// reads image elements k = 8 kg .. 8 kg + 7 of token row (n, p) -- for one k, consecutive n are
// consecutive addresses, so a wave's loads are whole 256-byte runs -- rounds them to bf16 (as the
// fused loaders do: the same operand bits) and stores one 16-byte chunk of the row.
template <bool F32>
__global__ __launch_bounds__(256) void patch_gather_hwcn_kernel(PatchGeom g, __bf16* out, int K) {
  const int kgs = K / 8;
  const int n = blockIdx.y * 64 + (threadIdx.x & 63);
  const int kg = blockIdx.z * 4 + (threadIdx.x >> 6);
  const int p = blockIdx.x;
  if (n >= g.Nb || kg >= kgs) return;
  const unsigned base = patch_rowbase<true>(g, p * g.Nb + n);
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const unsigned e = base + patch_kofs<true>(g, 8 * kg + j);
    v[j] = F32 ? (__bf16)reinterpret_cast<const float*>(g.x)[e] : reinterpret_cast<const __bf16*>(g.x)[e];
  }
  *reinterpret_cast<bf16x8*>(out + ((long long)n * g.L + p) * K + 8 * kg) = v;
}

}  // namespace sae
