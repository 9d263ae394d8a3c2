// loss.h -- the training step's label-smoothed softmax cross entropy, forward and backward (the
// §8f "DP train-step harness" row).
//
// Reference: train.py:77-90 -- y = optax.smooth_labels(one_hot(labels), alpha) = (1 - alpha) onehot
// + alpha / K, loss = mean_r optax.softmax_cross_entropy(logits_r, y_r) = mean_r -sum_c y_rc
// log_softmax(logits_r)_c, which per row is
//     lse_r - (1 - alpha) x[r, label_r] - (alpha / K) sum_c x[r, c]
// and whose gradient is  dlogits[r, c] = (g / R) (exp(x[r, c] - lse_r) - (1 - alpha) [c == label_r] - alpha / K).
// Replaces ~25 small framework launches (upcast, log-softmax, nll, smoothing sums, their
// backward) with three: the forward takes one workgroup per row (fp32 max / sum-exp / sum) and
// writes lse_r and the row's loss, one workgroup sums the row losses in a fixed order
// (deterministic), and the backward writes dlogits in the logits' dtype (bf16 or fp32), one
// workgroup per row.
#pragma once
#include "common.h"

namespace sae {

template <typename T> __device__ __forceinline__ float ce_ld(const T* p, long long i) { return (float)p[i]; }

__device__ __forceinline__ float ce_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float ce_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// forward, one 256-thread workgroup per row: lse_r and the row's smoothed loss
template <typename T>
__global__ __launch_bounds__(256) void smoothed_ce_fwd_kernel(const T* __restrict__ x, long long ld,
                                                              const int64_t* __restrict__ labels, int K, float alpha,
                                                              float* __restrict__ lse, float* __restrict__ row_loss) {
  __shared__ float red[2][4];
  const int r = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const T* xr = x + (long long)r * ld;
  float m = -INFINITY, sx = 0.f;
  for (int c = threadIdx.x; c < K; c += 256) {
    const float v = ce_ld(xr, c);
    m = fmaxf(m, v);
    sx += v;
  }
  m = ce_wave_max(m);
  sx = ce_wave_sum(sx);
  if (lane == 0) {
    red[0][w] = m;
    red[1][w] = sx;
  }
  __syncthreads();
  m = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
  sx = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
  __syncthreads();
  float se = 0.f;
  for (int c = threadIdx.x; c < K; c += 256) se += __expf(ce_ld(xr, c) - m);
  se = ce_wave_sum(se);
  if (lane == 0) red[0][w] = se;
  __syncthreads();
  if (threadIdx.x == 0) {
    se = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    const float l = m + __logf(se);
    const int64_t y = labels[r];
    const float xy = (y >= 0 && y < K) ? ce_ld(xr, (long long)y) : 0.f;
    lse[r] = l;
    row_loss[r] = l - (1.f - alpha) * xy - (alpha / (float)K) * sx;
  }
}

// the mean over rows, summed in row order by one workgroup (deterministic)
__global__ __launch_bounds__(256) void smoothed_ce_mean_kernel(const float* __restrict__ row_loss, int R,
                                                               float* __restrict__ loss) {
  __shared__ float part[256];
  // thread t sums the contiguous rows [t * per, (t + 1) * per), then thread 0 adds the 256 parts in order
  const int per = (R + 255) / 256;
  float s = 0.f;
  for (int r = threadIdx.x * per; r < min(R, (threadIdx.x + 1) * per); ++r) s += row_loss[r];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < 256; ++i) t += part[i];
    *loss = t / (float)R;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void smoothed_ce_bwd_kernel(const T* __restrict__ x, long long ld,
                                                              const int64_t* __restrict__ labels, int R, int K,
                                                              float alpha, const float* __restrict__ lse,
                                                              const float* __restrict__ gloss, T* __restrict__ dx,
                                                              long long ldd) {
  const int r = blockIdx.x;
  const float g = *gloss / (float)R, l = lse[r], off = alpha / (float)K;
  const int64_t y = labels[r];
  const T* xr = x + (long long)r * ld;
  T* dr = dx + (long long)r * ldd;
  for (int c = threadIdx.x; c < K; c += 256) {
    const float p = __expf(ce_ld(xr, c) - l);
    dr[c] = (T)(g * (p - (c == y ? 1.f - alpha : 0.f) - off));
  }
}

}  // namespace sae
