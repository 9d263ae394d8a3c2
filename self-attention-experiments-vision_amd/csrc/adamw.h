// adamw.h -- the optimizer update of the data-parallel training step, one launch for every
// parameter of the model (the §8f "DP train-step harness" row).
//
// Reference: train.py:25-27,229-233 builds optax.adamw (b1 0.9, b2 0.999, eps 1e-8, decoupled
// weight decay 1e-4) and applies it once per batch (train.py:94-100; survey D9: descent, not the
// reference chain's ascent).  The update follows torch.optim.AdamW's order of operations, which
// the host-side harness used before this kernel (train.py) and the parity test compares against:
//   p *= 1 - lr wd;  m = lerp(m, g, 1 - b1);  v = b2 v + (1 - b2) g^2;
//   p -= (lr / (1 - b1^t)) m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// HBM-bound elementwise work (28 bytes per parameter: read p, g, m, v, write p, m, v): the
// parameters are cut into 2048-element chunks (one 256-thread workgroup, 8 consecutive elements
// per thread as two 16-byte accesses); a device-resident chunk table built once by the host
// names each chunk's four pointers, so ~150 tensors cost one launch instead of torch's five
// multi-tensor launches.  The step counter lives in device memory (incremented by a one-thread
// kernel in the same stream) so a captured HIP graph replays the correct bias corrections.
#pragma once
#include "common.h"

namespace sae {

constexpr int kAdamwChunk = 2048;   // elements per chunk (256 threads x 8)

struct AdamwChunk {
  float* p;
  const float* g;
  float* m;
  float* v;
  int32_t n;       // elements in this chunk (<= kAdamwChunk)
  int32_t vec;     // all four pointers 16-byte aligned and n == kAdamwChunk
};

__global__ void adamw_tick_kernel(int32_t* step) {
  if (threadIdx.x == 0) *step += 1;
}

__device__ __forceinline__ void adamw_one(float& p, float g, float& m, float& v, float decay, float b1c, float b2,
                                          float b2c, float step_size, float inv_bc2s, float eps) {
  p *= decay;
  m = __builtin_fmaf(b1c, g - m, m);                 // torch lerp (weight < 0.5): m + w (g - m)
  v = __builtin_fmaf(b2, v, b2c * g * g);            // v * b2 + (1 - b2) g^2 (addcmul)
  const float denom = __builtin_sqrtf(v) * inv_bc2s + eps;
  p = __builtin_fmaf(-step_size, m / denom, p);
}

struct AdamwConst {
  float decay, b1c, b2, b2c, step_size, inv_bc2s, eps;
  __device__ __forceinline__ AdamwConst(const int32_t* step, float lr, float b1, float b2_, float eps_, float wd) {
    const float t = (float)(*step);
    const float bc1 = 1.f - __builtin_powf(b1, t), bc2 = 1.f - __builtin_powf(b2_, t);
    step_size = lr / bc1;
    inv_bc2s = 1.f / __builtin_sqrtf(bc2);
    decay = 1.f - lr * wd;
    b1c = 1.f - b1;
    b2 = b2_;
    b2c = 1.f - b2_;
    eps = eps_;
  }
};

// one 2048-element chunk of the flat table
__device__ __forceinline__ void adamw_chunk(const AdamwChunk& c, const AdamwConst& k) {
  const float decay = k.decay, b1c = k.b1c, b2 = k.b2, b2c = k.b2c, step_size = k.step_size,
              inv_bc2s = k.inv_bc2s, eps = k.eps;
  const int i0 = threadIdx.x * 8;
  if (c.vec) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = i0 + 4 * h;
      float4 p = *reinterpret_cast<const float4*>(c.p + i);
      const float4 g = *reinterpret_cast<const float4*>(c.g + i);
      float4 m = *reinterpret_cast<const float4*>(c.m + i);
      float4 v = *reinterpret_cast<const float4*>(c.v + i);
      adamw_one(p.x, g.x, m.x, v.x, decay, b1c, b2, b2c, step_size, inv_bc2s, eps);
      adamw_one(p.y, g.y, m.y, v.y, decay, b1c, b2, b2c, step_size, inv_bc2s, eps);
      adamw_one(p.z, g.z, m.z, v.z, decay, b1c, b2, b2c, step_size, inv_bc2s, eps);
      adamw_one(p.w, g.w, m.w, v.w, decay, b1c, b2, b2c, step_size, inv_bc2s, eps);
      *reinterpret_cast<float4*>(c.p + i) = p;
      *reinterpret_cast<float4*>(c.m + i) = m;
      *reinterpret_cast<float4*>(c.v + i) = v;
    }
  } else {
    for (int i = i0; i < i0 + 8 && i < c.n; ++i) {
      float p = c.p[i], m = c.m[i], v = c.v[i];
      adamw_one(p, c.g[i], m, v, decay, b1c, b2, b2c, step_size, inv_bc2s, eps);
      c.p[i] = p;
      c.m[i] = m;
      c.v[i] = v;
    }
  }
}

__global__ __launch_bounds__(256) void adamw_kernel(const AdamwChunk* __restrict__ chunks,
                                                    const int32_t* __restrict__ step, float lr, float b1,
                                                    float b2, float eps, float wd) {
  adamw_chunk(chunks[blockIdx.x], AdamwConst(step, lr, b1, b2, eps, wd));
}

// A 64 x 64 tile of a Dense kernel [K][N]: the AdamW update (identical arithmetic to the chunk
// path) plus the bf16 compute copies the next forward reads, w16 [K][ld16] at column col0 and its
// transpose wt16 [.][ldT] at row col0 (the tile goes through LDS for the transposed 8-byte
// stores) -- what sae_weight_cast_multi does at the start of every forward, moved into the update
// that produces the values.
struct AdamwCastTile {
  float* p;
  const float* g;
  float* m;
  float* v;
  __bf16* w16;
  __bf16* wt16;
  int32_t K, N, ld16, ldT, col0, k0, n0, pad;
};

__device__ __forceinline__ void adamw_cast_tile(const AdamwCastTile& c, const AdamwConst& k, float (*tile)[65]) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = t + 256 * q, row = i >> 4, c4 = i & 15;
    const int kk = c.k0 + row, n = c.n0 + 4 * c4;
    float4 pv = {0.f, 0.f, 0.f, 0.f};
    if (kk < c.K && n < c.N) {
      const long long off = (long long)kk * c.N + n;
      pv = *reinterpret_cast<const float4*>(c.p + off);
      const float4 g = *reinterpret_cast<const float4*>(c.g + off);
      float4 m = *reinterpret_cast<const float4*>(c.m + off);
      float4 v = *reinterpret_cast<const float4*>(c.v + off);
      adamw_one(pv.x, g.x, m.x, v.x, k.decay, k.b1c, k.b2, k.b2c, k.step_size, k.inv_bc2s, k.eps);
      adamw_one(pv.y, g.y, m.y, v.y, k.decay, k.b1c, k.b2, k.b2c, k.step_size, k.inv_bc2s, k.eps);
      adamw_one(pv.z, g.z, m.z, v.z, k.decay, k.b1c, k.b2, k.b2c, k.step_size, k.inv_bc2s, k.eps);
      adamw_one(pv.w, g.w, m.w, v.w, k.decay, k.b1c, k.b2, k.b2c, k.step_size, k.inv_bc2s, k.eps);
      *reinterpret_cast<float4*>(c.p + off) = pv;
      *reinterpret_cast<float4*>(c.m + off) = m;
      *reinterpret_cast<float4*>(c.v + off) = v;
      if (c.w16)
        *reinterpret_cast<bf16x4*>(c.w16 + (long long)kk * c.ld16 + c.col0 + n) =
            bf16x4{(__bf16)pv.x, (__bf16)pv.y, (__bf16)pv.z, (__bf16)pv.w};
    }
    tile[row][4 * c4] = pv.x;
    tile[row][4 * c4 + 1] = pv.y;
    tile[row][4 * c4 + 2] = pv.z;
    tile[row][4 * c4 + 3] = pv.w;
  }
  if (!c.wt16) return;   // (uniform per tile)
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = t + 256 * q, nn = i >> 4, kq = i & 15;
    const int n = c.n0 + nn, kk = c.k0 + 4 * kq;
    if (n < c.N && kk < c.K)
      *reinterpret_cast<bf16x4*>(c.wt16 + (long long)(c.col0 + n) * c.ldT + kk) =
          bf16x4{(__bf16)tile[4 * kq][nn], (__bf16)tile[4 * kq + 1][nn], (__bf16)tile[4 * kq + 2][nn],
                 (__bf16)tile[4 * kq + 3][nn]};
  }
}

// workgroups [0, n_chunks): the flat chunks; [n_chunks, n_chunks + n_tiles): the Dense-kernel tiles
__global__ __launch_bounds__(256) void adamw_cast_kernel(const AdamwChunk* __restrict__ chunks, int n_chunks,
                                                         const AdamwCastTile* __restrict__ tiles,
                                                         const int32_t* __restrict__ step, float lr, float b1,
                                                         float b2, float eps, float wd) {
  __shared__ float tile[64][65];
  const AdamwConst k(step, lr, b1, b2, eps, wd);
  const int b = blockIdx.x;
  if (b < n_chunks) adamw_chunk(chunks[b], k);
  else adamw_cast_tile(tiles[b - n_chunks], k, tile);
}

}  // namespace sae
