// ln.h -- the EncoderBlock glue around the attention hot path: residual add + LayerNorm.
//
// Reference: models/vit.py:19-31 (x = LN(inputs); x = attn(x) + inputs; y = LN(x); FF(y) + x)
// and vit.py:57 (final LayerNorm), Flax nn.LayerNorm(dtype): epsilon 1e-6, statistics in fp32,
// y = (x - mean) * rsqrt(var + eps) * scale + bias, output in the compute dtype.  Every residual
// add of the encoder is followed by a LayerNorm (the next block's LN0 or the final one), so one
// kernel does both:
//     x_out = x + delta            (fp32 residual stream; delta = attention / FF output, bf16)
//     y     = LN(x_out) in bf16    (+ per-row mean, rstd kept for the backward)
// and the backward
//     dx    = dx_in + LN_bwd(dy)   (fp32; the gradient of x and, cast to bf16, of delta)
//     dscale, dbias: per-workgroup partials, summed in a fixed order by a second kernel.
// One wave per row (C <= 1024 columns, float4 per lane), rows strided over the grid; HBM-bound.
#pragma once
#include "common.h"

namespace sae {

struct LnArgs {
  const float* x;        // [M][C] fp32 residual stream in
  const __bf16* delta;   // [M][C] bf16 addend (or null)
  float* xout;           // [M][C] fp32 x + delta (null if no delta)
  const float* gamma;    // [C] LayerNorm scale
  const float* beta;     // [C] LayerNorm bias
  __bf16* y;             // [M][C] bf16 output
  float* mean;           // [M]
  float* rstd;           // [M]
  // backward
  const __bf16* dy;      // [M][C] gradient of y
  const float* dxin;     // [M][C] gradient arriving at x_out from its other consumers (or null)
  float* dx;             // [M][C] fp32 gradient of x (and of delta)
  __bf16* ddelta;        // [M][C] bf16 copy of dx for delta (or null)
  float* part;           // [nblk][2][C] per-workgroup dscale / dbias partials
  float* dgamma;         // [C]
  float* dbeta;          // [C]
  // CaiT branch scale (layerscale.py:21-23 x stochastic_depth.py:19-28) folded into the add:
  // x_out = x + delta * bf16(lsc[c]) * rsc[row / rpb]   (lsc, rsc may be null = 1; the LayerScale
  // parameter is used at the compute dtype, layerscale.py:22, rounded here as it is loaded)
  const float* lsc;      // [C] LayerScale parameter (fp32)
  const float* rsc;      // [M / rpb] per-sample stochastic-depth factor (mask / keep)
  float* dlsc;           // [C] gradient of lsc (backward; needs delta)
  int rpb;               // rows per sample
  int M, C, nblk;
  float eps;
};

constexpr int kLnMaxV = 4;   // float4 chunks per lane: C <= 1024

__device__ __forceinline__ float ln_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ f32x4 ld_bf16x4(const __bf16* p) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}

__device__ __forceinline__ void st_bf16x4(__bf16* p, f32x4 v) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  *reinterpret_cast<bf16x4*>(p) = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
}

// fp32 -> the nearest bf16 value, as fp32 (the LayerScale parameter at the compute dtype;
// idempotent, so a caller passing already-rounded values gets the same result)
__device__ __forceinline__ f32x4 ln_bf16r(f32x4 v) {
  return f32x4{(float)(__bf16)v[0], (float)(__bf16)v[1], (float)(__bf16)v[2], (float)(__bf16)v[3]};
}

// Rows are software-pipelined: the next row's x / delta loads are issued before this row's
// reductions, so each wave keeps two rows of loads in flight (one row at a time left the HBM
// latency exposed between rows: 5.3 of 8 TB/s).
template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LnArgs a) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  const int C4 = a.C >> 2;
  f32x4 g[NV], bt[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = lane + 64 * k;
    g[k] = c < C4 ? reinterpret_cast<const f32x4*>(a.gamma)[c] : f32x4{};
    bt[k] = c < C4 ? reinterpret_cast<const f32x4*>(a.beta)[c] : f32x4{};
  }
  f32x4 ls[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = lane + 64 * k;
    ls[k] = (a.lsc && c < C4) ? ln_bf16r(reinterpret_cast<const f32x4*>(a.lsc)[c]) : f32x4{1.f, 1.f, 1.f, 1.f};
  }
  const float invC = 1.f / (float)a.C;
  const bool hasd = a.delta != nullptr;
  f32x4 nx[NV];    // the next row's x and delta, in flight during this row
  bf16x4 nd[NV];
  auto load = [&](int row) {
    const size_t ro = (size_t)row * a.C;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = lane + 64 * k;
      nx[k] = c < C4 ? reinterpret_cast<const f32x4*>(a.x + ro)[c] : f32x4{};
      nd[k] = (hasd && c < C4) ? *reinterpret_cast<const bf16x4*>(a.delta + ro + 4 * c) : bf16x4{};
    }
  };
  float nsf = 1.f;
  if (wave < a.M) {
    load(wave);
    if (a.rsc) nsf = a.rsc[wave / a.rpb];
  }
  for (int row = wave; row < a.M; row += nw) {
    const size_t ro = (size_t)row * a.C;
    const float rsf = nsf;
    f32x4 v[NV];
    bf16x4 dv[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      v[k] = nx[k];
      dv[k] = nd[k];
    }
    if (row + nw < a.M) {
      load(row + nw);
      if (a.rsc) nsf = a.rsc[(row + nw) / a.rpb];
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = lane + 64 * k;
      if (c < C4 && hasd) {
        v[k] += f32x4{(float)dv[k][0], (float)dv[k][1], (float)dv[k][2], (float)dv[k][3]} * (ls[k] * rsf);
        reinterpret_cast<f32x4*>(a.xout + ro)[c] = v[k];
      }
      s += v[k][0] + v[k][1] + v[k][2] + v[k][3];
    }
    const float mu = ln_wave_sum(s) * invC;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = lane + 64 * k;
      if (c < C4) {
        const f32x4 d = v[k] - mu;
        q += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
      }
    }
    const float rs = __builtin_amdgcn_rsqf(ln_wave_sum(q) * invC + a.eps);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = lane + 64 * k;
      if (c < C4) st_bf16x4(a.y + ro + 4 * c, (v[k] - mu) * rs * g[k] + bt[k]);
    }
    if (lane == 0) {
      a.mean[row] = mu;
      a.rstd[row] = rs;
    }
  }
}

// NP = 2: dgamma / dbeta partials; NP = 3: also the LayerScale gradient (a.lsc, a.delta set)
template <int NV, int NP = 2>
__global__ __launch_bounds__(256) void ln_bwd_kernel(LnArgs a) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  __shared__ f32x4 red[4][NP][64 * NV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wave = blockIdx.x * 4 + w;
  const int nw = gridDim.x * 4;
  const int C4 = a.C >> 2;
  f32x4 g[NV], pg[NV], pb[NV], pl[NV], ls[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = lane + 64 * k;
    g[k] = c < C4 ? reinterpret_cast<const f32x4*>(a.gamma)[c] : f32x4{};
    ls[k] = (NP == 3 && c < C4) ? ln_bf16r(reinterpret_cast<const f32x4*>(a.lsc)[c]) : f32x4{1.f, 1.f, 1.f, 1.f};
    pg[k] = pb[k] = pl[k] = f32x4{};
  }
  const float invC = 1.f / (float)a.C;
  const bool hasin = a.dxin != nullptr;
  // the next row's dy / x / dx_in (and mean / rstd; NP = 3: delta and the row scale), in flight
  // during this row (as ln_fwd_kernel)
  bf16x4 ndy[NV], nde[NP == 3 ? NV : 1];
  f32x4 nx[NV], ni[NV];
  float nmu = 0.f, nrs = 0.f, nsf = 1.f;
  auto load = [&](int row) {
    const size_t ro = (size_t)row * a.C;
    nmu = a.mean[row];
    nrs = a.rstd[row];
    if constexpr (NP == 3) nsf = a.rsc ? a.rsc[row / a.rpb] : 1.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = lane + 64 * k;
      ndy[k] = c < C4 ? *reinterpret_cast<const bf16x4*>(a.dy + ro + 4 * c) : bf16x4{};
      nx[k] = c < C4 ? reinterpret_cast<const f32x4*>(a.x + ro)[c] : f32x4{};
      ni[k] = (hasin && c < C4) ? reinterpret_cast<const f32x4*>(a.dxin + ro)[c] : f32x4{};
      if constexpr (NP == 3) nde[k] = c < C4 ? *reinterpret_cast<const bf16x4*>(a.delta + ro + 4 * c) : bf16x4{};
    }
  };
  if (wave < a.M) load(wave);
  for (int row = wave; row < a.M; row += nw) {
    const size_t ro = (size_t)row * a.C;
    const float mu = nmu, rs = nrs, rsf = nsf;
    f32x4 xh[NV], gy[NV], din[NV];
    bf16x4 dyr[NV], der[NP == 3 ? NV : 1];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      dyr[k] = ndy[k];
      xh[k] = nx[k];
      din[k] = ni[k];
      if constexpr (NP == 3) der[k] = nde[k];
    }
    if (row + nw < a.M) load(row + nw);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = lane + 64 * k;
      gy[k] = f32x4{};
      if (c < C4) {
        const f32x4 dyv = f32x4{(float)dyr[k][0], (float)dyr[k][1], (float)dyr[k][2], (float)dyr[k][3]};
        xh[k] = (xh[k] - mu) * rs;
        gy[k] = dyv * g[k];
        pg[k] += dyv * xh[k];
        pb[k] += dyv;
      } else {
        xh[k] = f32x4{};
      }
      s1 += gy[k][0] + gy[k][1] + gy[k][2] + gy[k][3];
      const f32x4 t = gy[k] * xh[k];
      s2 += t[0] + t[1] + t[2] + t[3];
    }
    const float m1 = ln_wave_sum(s1) * invC, m2 = ln_wave_sum(s2) * invC;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = lane + 64 * k;
      if (c < C4) {
        f32x4 d = (gy[k] - m1 - xh[k] * m2) * rs;
        if (hasin) d += din[k];
        reinterpret_cast<f32x4*>(a.dx + ro)[c] = d;
        if constexpr (NP == 3) {   // x_out = x + delta * ls * rsf
          pl[k] += d * f32x4{(float)der[k][0], (float)der[k][1], (float)der[k][2], (float)der[k][3]} * rsf;
          if (a.ddelta) st_bf16x4(a.ddelta + ro + 4 * c, d * ls[k] * rsf);
        } else {
          if (a.ddelta) st_bf16x4(a.ddelta + ro + 4 * c, d);
        }
      }
    }
  }
  // workgroup partial: the 4 waves' sums added in wave order
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    red[w][0][lane + 64 * k] = pg[k];
    red[w][1][lane + 64 * k] = pb[k];
    if constexpr (NP == 3) red[w][2][lane + 64 * k] = pl[k];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NP * C4; i += 256) {
    const int which = i / C4, c = i % C4;
    f32x4 s = red[0][which][c];
    s += red[1][which][c];
    s += red[2][which][c];
    s += red[3][which][c];
    reinterpret_cast<f32x4*>(a.part + ((size_t)blockIdx.x * NP + which) * a.C)[c] = s;
  }
}

// dgamma / dbeta (/ dlsc) = sum of the workgroup partials, deterministic, in ONE launch: thread
// (column chunk col, group g) sums partials g, g + 64, ... (float4 columns, L2-hot), then the 64
// group sums are added in group order.  A workgroup covers 4 float4 columns of the NP outputs
// (16 groups x 16 columns left each thread 64 dependent-latency partials on a dozen workgroups).
constexpr int kLnRedGroups = 64;
constexpr int kLnRedCols = 256 / kLnRedGroups;
template <int NP = 2>
__global__ __launch_bounds__(256) void ln_bwd_reduce_kernel(LnArgs a) {
  __shared__ f32x4 red[kLnRedGroups][kLnRedCols];
  const int C4 = a.C >> 2;
  const int cl = threadIdx.x % kLnRedCols, grp = threadIdx.x / kLnRedCols;
  const int col = blockIdx.x * kLnRedCols + cl;   // [0, NP * C4)
  const bool ok = col < NP * C4;
  const int which = ok ? col / C4 : 0, c4 = ok ? col % C4 : 0;
  f32x4 s0 = {}, s1 = {};
  if (ok) {
    const f32x4* src = reinterpret_cast<const f32x4*>(a.part) + (size_t)which * C4 + c4;
    const size_t step = (size_t)NP * C4;          // one workgroup partial
    int b = grp;
#pragma unroll 4
    for (; b + kLnRedGroups < a.nblk; b += 2 * kLnRedGroups) {
      s0 += src[(size_t)b * step];
      s1 += src[(size_t)(b + kLnRedGroups) * step];
    }
    if (b < a.nblk) s0 += src[(size_t)b * step];
  }
  red[grp][cl] = s0 + s1;
  __syncthreads();
  if (grp == 0 && ok) {
    f32x4 t = red[0][cl];
#pragma unroll
    for (int g = 1; g < kLnRedGroups; ++g) t += red[g][cl];
    float* dst = which == 0 ? a.dgamma : which == 1 ? a.dbeta : a.dlsc;
    reinterpret_cast<f32x4*>(dst)[c4] = t;
  }
}

}  // namespace sae
