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

__global__ __launch_bounds__(256) void adamw_kernel(const AdamwChunk* __restrict__ chunks,
                                                    const int32_t* __restrict__ step, float lr, float b1,
                                                    float b2, float eps, float wd) {
  const AdamwChunk c = chunks[blockIdx.x];
  const float t = (float)(*step);
  const float bc1 = 1.f - __builtin_powf(b1, t), bc2 = 1.f - __builtin_powf(b2, t);
  const float step_size = lr / bc1, inv_bc2s = 1.f / __builtin_sqrtf(bc2), decay = 1.f - lr * wd;
  const float b1c = 1.f - b1, b2c = 1.f - b2;
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

}  // namespace sae
