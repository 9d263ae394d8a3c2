// tokens.h -- the encoder input of ViT / DeiT: class token + patch tokens + absolute position
// embedding, forward and backward (the glue between the §8f patch-embedding row and the first
// encoder block).
//
// Reference: models/vit.py:82-85 (cls = tile(param, [b, 1, 1]); x = concatenate([cls, x], 1)) and
// vit.py:46 + layers/position_embed.py:48 (AddAbsPosEmbed: x + pos_embed), with the patch tokens
// promoted from the compute dtype to the fp32 residual stream:
//     x[b, 0, c] = cls[c] + pos[0, c];   x[b, 1 + p, c] = float(tok[b, p, c]) + pos[1 + p, c]
// Backward: dtok[b, p] = bf16(dx[b, 1 + p]), dpos[n] = sum_b dx[b, n], dcls = dpos[0].  One pass
// each way instead of the upcast, concatenate and add kernels (and their backward: slice, cast and
// two batch reductions).  HBM-bound: 2 B read + 4 B written per element forward, 4 B read + 2 B
// written backward.
#pragma once
#include "common.h"

namespace sae {

// one thread per 4 consecutive channels of one token
__global__ __launch_bounds__(256) void tokens_fwd_kernel(const __bf16* __restrict__ tok, const float* __restrict__ cls,
                                                         const float* __restrict__ pos, float* __restrict__ x, int B,
                                                         int L, int E) {
  const int E4 = E / 4, N = L + 1;
  const long long total = (long long)B * N * E4;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c4 = (int)(i % E4);
    const long long bn = i / E4;
    const int n = (int)(bn % N);
    const long long b = bn / N;
    const f32x4 p = reinterpret_cast<const f32x4*>(pos)[(long long)n * E4 + c4];
    f32x4 v;
    if (n == 0) {
      v = reinterpret_cast<const f32x4*>(cls)[c4];
    } else {
      const uint2 t = reinterpret_cast<const uint2*>(tok)[(b * L + n - 1) * E4 + c4];
      v = f32x4{__uint_as_float(t.x << 16), __uint_as_float(t.x & 0xffff0000u), __uint_as_float(t.y << 16),
                __uint_as_float(t.y & 0xffff0000u)};
    }
    reinterpret_cast<f32x4*>(x)[i] = v + p;
  }
}

// one workgroup per token position n: E / 4 channel groups x G batch groups (G = blockDim / (E/4));
// batch group g sums b = g, g + G, ... and the G partial sums are added in group order
// (deterministic).  LDS: G * E * 4 bytes.
__global__ __launch_bounds__(1024) void tokens_bwd_kernel(const float* __restrict__ dx, __bf16* __restrict__ dtok,
                                                          float* __restrict__ dcls, float* __restrict__ dpos, int B,
                                                          int L, int E) {
  extern __shared__ f32x4 part[];   // [G][E4]
  const int E4 = E / 4, N = L + 1, n = blockIdx.x;
  const int G = blockDim.x / E4;
  const int c4 = threadIdx.x % E4, g = threadIdx.x / E4;
  if (g < G) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int b = g; b < B; b += G) {
      const f32x4 v = reinterpret_cast<const f32x4*>(dx)[((long long)b * N + n) * E4 + c4];
      acc += v;
      if (n > 0) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        const bf16x4 t = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
        reinterpret_cast<bf16x4*>(dtok)[((long long)b * L + n - 1) * E4 + c4] = t;
      }
    }
    part[g * E4 + c4] = acc;
  }
  __syncthreads();
  if (g == 0) {
    f32x4 s = part[c4];
    for (int q = 1; q < G; ++q) s += part[q * E4 + c4];
    reinterpret_cast<f32x4*>(dpos)[(long long)n * E4 + c4] = s;
    if (n == 0 && dcls) reinterpret_cast<f32x4*>(dcls)[c4] = s;
  }
}

}  // namespace sae
