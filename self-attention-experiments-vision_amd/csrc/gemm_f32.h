// gemm_f32.h -- fp32 projections on the f32-input MFMA (v_mfma_f32_32x32x2_f32).
//
// The Dense / DenseGeneral dot_generals of the path (attention.py:29-37,60-63, ff.py:8-34) at
// compute dtype float32 -- the reference's fp32 trunks (CaiT, cait.py:147-154) and every fp32
// parity run -- with their JAX-autodiff gradients:
//   forward  y  = x  W  (+ b)   A = x  [M][K] (k contiguous), B = W  [K][N] (n contiguous)
//   input    dx = dy W^T        A = dy [M][J] (k contiguous), B(k=j, n=i) = W[i][j] (k contiguous)
//   weight   dW = x^T dy        A(m=i, k=t) = x[t][i] (m contiguous), B = dy [T][J] (n contiguous)
//            db = colsum(dy)    the "ones row": A gets one extra row m = M of 1.0, whose output
//                               row is the column sum of B (one MFMA pass, no separate kernel)
// One kernel, templated on which index of A / B is contiguous.  The f32 MFMA is exact fp32 (a
// k-ordered fmaf chain per 2-deep step) at 1/16 of the bf16 rate, so a plainly staged 128 x 128
// tile is MFMA-bound: per 16-deep k tile a wave issues 32 MFMAs (2048 cycles per SIMD) against
// 16 KB of operand loads per workgroup -- no LDS-DMA, no ping-pong needed.
//
// Tile: 128 x 128 outputs, 4 waves as 2 x 2, each 64 x 64 = 2 x 2 MFMA blocks of 32 x 32
// (4 accumulators x 16 VGPRs).  LDS holds both operands k-major (As[k][m], Bs[k][n], rows padded
// to 132 floats), double-buffered: the next k tile's global loads are issued into registers before
// the current tile's MFMAs and written to the other buffer after them, one barrier per tile.
// Operand lanes: MFMA lane l reads As[k + (l >> 5)][m0 + (l & 31)] -- 32 consecutive floats per
// half-wave, conflict-free.  Transposing stores (the k-contiguous operands) write 4 scalars per
// float4 at rows kq*4 + j: with the 132-float row pitch the 64 lanes of one store (16 m x 4 kq)
// land in 64 distinct banks.
//
// Split-K (weight gradients: T = 25,216 tokens deep, 9 - 27 output tiles): grid.z splits write
// fp32 partials [S][M'][N] to the workspace and gemm_f32_reduce_kernel sums them in split order
// (deterministic, no atomics), adding the bias / accumulating into C and the column-sum row.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace sae {

constexpr int kF32T = 128;      // output tile (both dims)
constexpr int kF32K = 16;       // k tile
constexpr int kF32P = 132;      // LDS row pitch (floats)

struct F32Args {
  const float* a;
  const float* b;
  const float* bias;            // [N] or null (added once, by the kernel that writes C)
  float* c;
  float* colsum;                // [N] or null: the ones row's output (db)
  float* part;                  // split-K partials [S][M + (colsum != 0)][N]
  int64_t sam, sak, sbk, sbn, ldc;
  int M, N, K;
  int S, kchunk;                // splits, k depth per split (multiple of kF32K)
  int accumulate;
};

typedef float f32x16v __attribute__((ext_vector_type(16)));

template <bool AK, bool BK>
__global__ __launch_bounds__(256) void gemm_f32_kernel(F32Args g) {
  __shared__ float As[2][kF32K][kF32P];
  __shared__ float Bs[2][kF32K][kF32P];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * kF32T, n0 = blockIdx.y * kF32T;
  const int z = blockIdx.z;
  const int kbeg = z * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const bool ones = g.colsum != nullptr;
  const int Mx = g.M + (ones ? 1 : 0);   // rows incl. the ones row

  float4 ra[2], rb[2];
  // global -> registers for the k tile at k0 (zero outside the operand; the ones row is 1.0)
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int f = tid + 256 * i;
      if (AK) {                         // A[m][k], k contiguous: 4 lanes per 64-byte row piece
        const int m = m0 + (f >> 2), k = k0 + (f & 3) * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k < kend) {
          if (m < g.M) v = *reinterpret_cast<const float4*>(g.a + (size_t)m * g.sam + k);
          else if (m == g.M && ones) v = make_float4(1.f, 1.f, 1.f, 1.f);
        }
        ra[i] = v;
      } else {                          // A[k][m], m contiguous
        const int k = k0 + (f >> 5), m = m0 + (f & 31) * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k < kend) {
          if (m < g.M) v = *reinterpret_cast<const float4*>(g.a + (size_t)k * g.sak + m);
          else if (m == g.M && ones) v = make_float4(1.f, 0.f, 0.f, 0.f);
        }
        ra[i] = v;
      }
      if (BK) {                         // B[n][k], k contiguous
        const int n = n0 + (f >> 2), k = k0 + (f & 3) * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k < kend && n < g.N) v = *reinterpret_cast<const float4*>(g.b + (size_t)n * g.sbn + k);
        rb[i] = v;
      } else {                          // B[k][n], n contiguous
        const int k = k0 + (f >> 5), n = n0 + (f & 31) * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k < kend && n < g.N) v = *reinterpret_cast<const float4*>(g.b + (size_t)k * g.sbk + n);
        rb[i] = v;
      }
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int f = tid + 256 * i;
      if (AK) {
        const int m = f >> 2, kq = (f & 3) * 4;
        As[buf][kq + 0][m] = ra[i].x;
        As[buf][kq + 1][m] = ra[i].y;
        As[buf][kq + 2][m] = ra[i].z;
        As[buf][kq + 3][m] = ra[i].w;
      } else {
        *reinterpret_cast<float4*>(&As[buf][f >> 5][(f & 31) * 4]) = ra[i];
      }
      if (BK) {
        const int n = f >> 2, kq = (f & 3) * 4;
        Bs[buf][kq + 0][n] = rb[i].x;
        Bs[buf][kq + 1][n] = rb[i].y;
        Bs[buf][kq + 2][n] = rb[i].z;
        Bs[buf][kq + 3][n] = rb[i].w;
      } else {
        *reinterpret_cast<float4*>(&Bs[buf][f >> 5][(f & 31) * 4]) = rb[i];
      }
    }
  };

  f32x16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int lr = lane & 31, lk = lane >> 5;
  const int nk = (kend - kbeg + kF32K - 1) / kF32K;
  if (nk > 0) {
    load(kbeg);
    store(0);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    if (t + 1 < nk) load(kbeg + (t + 1) * kF32K);
#pragma unroll
    for (int kk = 0; kk < kF32K; kk += 2) {
      const float a0 = As[buf][kk + lk][wm + lr], a1 = As[buf][kk + lk][wm + 32 + lr];
      const float b0 = Bs[buf][kk + lk][wn + lr], b1 = Bs[buf][kk + lk][wn + 32 + lr];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (t + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  // C/D map of the 32 x 32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  const bool split = g.S > 1;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + j * 32 + lr;
      if (n >= g.N) continue;
      const float bn = (!split && g.bias) ? g.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (m >= Mx) continue;
        const float v = acc[i][j][r];
        if (split) {
          g.part[((size_t)z * Mx + m) * g.N + n] = v;
        } else if (m == g.M) {           // the ones row: db
          g.colsum[n] = g.accumulate ? g.colsum[n] + v : v;
        } else {
          float* cp = g.c + (size_t)m * g.ldc + n;
          *cp = g.accumulate ? *cp + v + bn : v + bn;
        }
      }
    }
}

// split-K reduction: C[m][n] (+)= sum_z part[z][m][n] (+ bias[n]) in split order; row M -> colsum
__global__ __launch_bounds__(256) void gemm_f32_reduce_kernel(F32Args g) {
  const int Mx = g.M + (g.colsum ? 1 : 0);
  const long long total = (long long)Mx * g.N;
  const size_t plane = (size_t)Mx * g.N;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int m = (int)(e / g.N), n = (int)(e % g.N);
    float s = 0.f;
    for (int z = 0; z < g.S; ++z) s += g.part[z * plane + e];
    if (m == g.M) {
      g.colsum[n] = g.accumulate ? g.colsum[n] + s : s;
    } else {
      if (g.bias) s += g.bias[n];
      float* cp = g.c + (size_t)m * g.ldc + n;
      *cp = g.accumulate ? *cp + s : s;
    }
  }
}

}  // namespace sae
