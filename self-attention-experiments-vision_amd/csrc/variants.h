// variants.h -- helper kernels for the attention variants (bandwidth-bound VALU work).
//
//   relpos_bias_fwd  : BoTNet RelativeLogits (models/botnet.py:70-141) in index-map form:
//                      bias_h[b,h,n,p] = <qhat[b,n,h,:], E_h[p - x_n + Hs - 1, :]>,
//                      bias_w[b,h,n,c] = <qhat[b,n,h,:], E_w[c - y_n + Ws - 1, :]>.
//                      The reference materialises [B,h,H,W,H,W] through pad/reshape/tile; the
//                      fused score tile only needs these (Hs + Ws) numbers per query row.
//   relpos_bias_bwd_*: dqhat += sum_p dbias_h E_h[..] + sum_c dbias_w E_w[..]; dE_h / dE_w
//                      reduced deterministically (per-batch partials, then a fixed-order sum).
//   rotary           : GPT-J interleaved rotary (position_embed.py:8-20) from fp32 tables.
#pragma once
#include "common.h"

namespace sae {

struct RelArgs {
  const void* qhat;
  long long qs[3];
  const float* eh;
  const float* ew;
  float* bias_h;
  float* bias_w;
  const float* dbias_h;
  const float* dbias_w;
  const void* dq_in;
  void* dq_out;
  long long dqs[3];
  float* demb_h;
  float* demb_w;
  float* part;      // workspace [B][(2Hs-1) + (2Ws-1)][D]
  int B, H, Hs, Ws, D;
};

template <typename T>
__device__ __forceinline__ float ldf(const T* p) { return (float)*p; }

// one thread per (b, h, n, j), j in [0, Hs + Ws)
template <typename T>
__global__ __launch_bounds__(256) void relpos_bias_fwd_kernel(RelArgs a) {
  const int N = a.Hs * a.Ws, J = a.Hs + a.Ws;
  const long long total = (long long)a.B * a.H * N * J;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int j = (int)(i % J);
  long long t = i / J;
  const int n = (int)(t % N);
  t /= N;
  const int hh = (int)(t % a.H);
  const int b = (int)(t / a.H);
  const int x = n / a.Ws, y = n % a.Ws;
  const T* qp = reinterpret_cast<const T*>(a.qhat) + b * a.qs[0] + (long long)n * a.qs[1] + hh * a.qs[2];
  const float* e;
  if (j < a.Hs) e = a.eh + (long long)(j - x + a.Hs - 1) * a.D;
  else e = a.ew + (long long)((j - a.Hs) - y + a.Ws - 1) * a.D;
  float acc = 0.f;
  for (int d = 0; d < a.D; ++d) acc += ldf(qp + d) * e[d];
  const long long row = ((long long)b * a.H + hh) * N + n;
  if (j < a.Hs) a.bias_h[row * a.Hs + j] = acc;
  else a.bias_w[row * a.Ws + (j - a.Hs)] = acc;
}

// dqhat: one thread per (b, n, h, d)
template <typename T>
__global__ __launch_bounds__(256) void relpos_bias_bwd_dq_kernel(RelArgs a) {
  const int N = a.Hs * a.Ws;
  const long long total = (long long)a.B * N * a.H * a.D;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int d = (int)(i % a.D);
  long long t = i / a.D;
  const int hh = (int)(t % a.H);
  t /= a.H;
  const int n = (int)(t % N);
  const int b = (int)(t / N);
  const int x = n / a.Ws, y = n % a.Ws;
  const long long row = ((long long)b * a.H + hh) * N + n;
  float acc = 0.f;
  for (int p = 0; p < a.Hs; ++p) acc += a.dbias_h[row * a.Hs + p] * a.eh[(long long)(p - x + a.Hs - 1) * a.D + d];
  for (int c = 0; c < a.Ws; ++c) acc += a.dbias_w[row * a.Ws + c] * a.ew[(long long)(c - y + a.Ws - 1) * a.D + d];
  const long long off_in = b * a.dqs[0] + (long long)n * a.dqs[1] + hh * a.dqs[2] + d;
  if (a.dq_in) acc += ldf(reinterpret_cast<const T*>(a.dq_in) + off_in);
  reinterpret_cast<T*>(a.dq_out)[off_in] = (T)acc;
}

// partial dE: one thread per (b, m, d) with m in [0, (2Hs-1) + (2Ws-1))
template <typename T>
__global__ __launch_bounds__(256) void relpos_bias_bwd_emb_partial_kernel(RelArgs a) {
  const int N = a.Hs * a.Ws;
  const int MH = 2 * a.Hs - 1, MW = 2 * a.Ws - 1, MT = MH + MW;
  const long long total = (long long)a.B * MT * a.D;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int d = (int)(i % a.D);
  long long t = i / a.D;
  const int mm = (int)(t % MT);
  const int b = (int)(t / MT);
  float acc = 0.f;
  for (int hh = 0; hh < a.H; ++hh) {
    const T* qb = reinterpret_cast<const T*>(a.qhat) + b * a.qs[0] + hh * a.qs[2] + d;
    const long long rowb = ((long long)b * a.H + hh) * N;
    for (int n = 0; n < N; ++n) {
      const int x = n / a.Ws, y = n % a.Ws;
      float g;
      if (mm < MH) {
        const int p = mm - a.Hs + 1 + x;
        if (p < 0 || p >= a.Hs) continue;
        g = a.dbias_h[(rowb + n) * a.Hs + p];
      } else {
        const int c = (mm - MH) - a.Ws + 1 + y;
        if (c < 0 || c >= a.Ws) continue;
        g = a.dbias_w[(rowb + n) * a.Ws + c];
      }
      acc += g * ldf(qb + (long long)n * a.qs[1]);
    }
  }
  a.part[i] = acc;
}

// fixed-order sum of the per-batch partials
__global__ __launch_bounds__(256) void relpos_bias_bwd_emb_reduce_kernel(RelArgs a) {
  const int MH = 2 * a.Hs - 1, MW = 2 * a.Ws - 1, MT = MH + MW;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= MT * a.D) return;
  float acc = 0.f;
  for (int b = 0; b < a.B; ++b) acc += a.part[(long long)b * MT * a.D + i];
  const int mm = i / a.D, d = i % a.D;
  if (mm < MH) a.demb_h[mm * a.D + d] = acc;
  else a.demb_w[(mm - MH) * a.D + d] = acc;
}

struct RotArgs {
  const void* x;
  void* y;
  long long xs[3], ys[3];
  const float* sin_t;
  const float* cos_t;
  int B, N, H, D;
  float sgn;
};

// one thread per rotation pair (b, n, h, i)
template <typename T>
__global__ __launch_bounds__(256) void rotary_kernel(RotArgs a) {
  const int P = a.D / 2;
  const long long total = (long long)a.B * a.N * a.H * P;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int i = (int)(idx % P);
  long long t = idx / P;
  const int hh = (int)(t % a.H);
  t /= a.H;
  const int n = (int)(t % a.N);
  const int b = (int)(t / a.N);
  const T* xp = reinterpret_cast<const T*>(a.x) + b * a.xs[0] + (long long)n * a.xs[1] + hh * a.xs[2] + 2 * i;
  T* yp = reinterpret_cast<T*>(a.y) + b * a.ys[0] + (long long)n * a.ys[1] + hh * a.ys[2] + 2 * i;
  const float s = a.sgn * a.sin_t[(long long)n * P + i];
  const float c = a.cos_t[(long long)n * P + i];
  const float x0 = (float)xp[0], x1 = (float)xp[1];
  // explicit FMAs, exactly as rope_pairs (common.h) in the fused kernels
  yp[0] = (T)__builtin_fmaf(x0, c, -(x1 * s));
  yp[1] = (T)__builtin_fmaf(x1, c, x0 * s);
}

}  // namespace sae
