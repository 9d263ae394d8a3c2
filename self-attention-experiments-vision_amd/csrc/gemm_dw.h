// gemm_dw.h -- weight / bias gradients of the projections on the hot path, split over tokens.
//
// For every Dense / DenseGeneral of the path (QKV projection `queries|keys|values`,
// attention.py:29-37; output projection `DenseGeneral_0`, attention.py:60-63; the FF block's
// `Dense_0/1`, ff.py:8-34) the backward needs
//     dW[i][j] = sum_m X[m][i] dY[m][j]      (fp32, the parameter dtype)
//     db[j]    = sum_m dY[m][j]
// with m running over every token of the batch (M = B*N = 25,216 for DeiT-S) and a small
// output (384 x 1152 for the QKV projection).  Library GEMMs run this shape at 60-220 TF/s
// (tools/gemm_probe.py); here it is a split-K MFMA kernel:
//   * a workgroup owns a 128 x 128 output tile and one contiguous chunk of tokens; 4 waves,
//     each a 64 x 64 quarter (2 x 2 accumulators of v_mfma_f32_32x32x16_bf16);
//   * X and dY chunks of 64 tokens are staged global -> registers -> LDS as [token][column]
//     images (XOR-swizzled 256-byte rows), double-buffered in LDS with two register stages in
//     flight (loads issued two stages ahead of use), and both MFMA operands are read
//     with ds_read_b64_tr_b16 (K = tokens on the transposed axis, same permuted K order on both);
//   * db rides on the matrix pipe: an all-ones A operand times the dY fragment gives column sums;
//   * each split writes an fp32 partial tile; a second kernel sums the splits in a fixed order
//     (deterministic, no atomics) and writes / accumulates the fp32 gradient.
#pragma once
#include "common.h"

namespace sae {

struct DwArgs {
  const __bf16* x;    // [M][I] (row stride ldx elements)
  const __bf16* dy;   // [M][J] (row stride ldy)
  float* part;        // [S][I][J] fp32 partial sums
  float* bpart;       // [S][J] fp32 partial bias sums (or null)
  float* dw;          // [I][J] fp32 output (row stride ldw)
  float* db;          // [J] fp32 output (or null)
  int M, I, J, S, chunk;   // chunk = tokens per split (multiple of 64)
  long long ldx, ldy, ldw;
  int accumulate;     // dw / db += instead of =
  int jblock;         // > 0: dw is [J / jblock][I][jblock] (column blocks contiguous), ldw unused
  PatchGeom pg;       // patch-embedding X operand (patch.h), unused otherwise
};

constexpr int kDwT = 128;   // output tile edge
constexpr int kDwK = 64;    // tokens per staged stage

// tile images: [64 tokens][128 columns] bf16, 256-byte rows, swz<128>
template <int NCH>
struct DwStage {
  uint4 v[NCH];
  unsigned goff[NCH];
  unsigned loff[NCH];
  __device__ __forceinline__ void init(int tid, long long ld, int col0, int ncols) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int id = tid + 256 * i;
      const int r = id >> 4, c = id & 15;
      goff[i] = (col0 + 8 * c < ncols) ? (unsigned)(((long long)r * ld + col0 + 8 * c) * 2) : 0x80000000u;
      loff[i] = r * 256 + 16 * (c ^ swz<128>(r));
    }
  }
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, unsigned rowoff) {
#pragma unroll
    for (int i = 0; i < NCH; ++i)
      v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, goff[i] + rowoff, 0, 0));
  }
  __device__ __forceinline__ void write(char* img) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) *reinterpret_cast<uint4*>(img + loff[i]) = v[i];
  }
};

// Operand loaders of the plain kernel: token rows [m0, m1) of the row-major x [M][I] / dy [M][J]
// through buffer descriptors (rows past m1 read zero), columns col0 .. col0 + 127.  patch.h
// supplies the patch-gather loaders.
template <bool Y>
struct DwRow {
  DwStage<4> s;
  __amdgpu_buffer_rsrc_t rs;
  unsigned step;
  __device__ __forceinline__ void init(const DwArgs& a, int tid, int m0, int m1, int col0) {
    const __bf16* base = Y ? a.dy : a.x;
    const long long ld = Y ? a.ldy : a.ldx;
    rs = row_rsrc(base + (long long)m0 * ld, m1 - m0, ld);
    s.init(tid, ld, col0, Y ? a.J : a.I);
    step = (unsigned)(kDwK * ld * 2);
  }
  __device__ __forceinline__ void load(const DwArgs&, int st) { s.load(rs, (unsigned)st * step); }
  __device__ __forceinline__ void write(char* img) const { s.write(img); }
};

// transposed operand read: column col0 + (lane & 31) on the lane, K over rows 16s + permuted
__device__ __forceinline__ bf16x8 dw_colfrag(const char* img, const unsigned* ca, int s, int t) {
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  const int ro = 16 * s * 256;
  s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + ca[2 * t] + ro));
  s16x4 x2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + ca[2 * t + 1] + ro));
  s16x8 v = {x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// NG = 2: two groups of 4 waves per workgroup split the token chunk's stages (group g takes
// stages g, g + 2, ...; own LDS buffers) and add their accumulators through LDS at the end, group
// 0 first (fixed order): half the splits, so half the fp32 partial-tile traffic, at the same number
// of waves in flight (one 8-wave workgroup per CU instead of two 4-wave ones).
template <bool BIAS, class XL = DwRow<false>, class YL = DwRow<true>, int NG = 1>
__global__ __launch_bounds__(256 * NG, NG == 1 ? 2 : 1) void gemm_dw_kernel(DwArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem_all[];
  constexpr int IMG = kDwK * 256;     // 16 KiB per operand image
  const int ti = (a.I + kDwT - 1) / kDwT, tj = (a.J + kDwT - 1) / kDwT;
  // XCD-aware order: the logical blocks of one XCD are a contiguous range, tiles fastest, so
  // every tile of a token chunk runs on the same XCD at the same time and the chunk's X / dY
  // rows are fetched from HBM once per XCD (L2 hits for the other tiles), not once per tile
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid % (ti * tj), s = bid / (ti * tj);
  const int it = tile % ti, jt = tile / ti;
  const int i0 = it * kDwT, j0 = jt * kDwT;
  const int tid = threadIdx.x & 255, lane = tid & 63, h = lane >> 5;
  const int grp = NG == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8));
  char* const smem = smem_all + grp * 4 * IMG;   // this group's two stage buffers
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = w & 1, wj = w >> 1;  // this wave's 64 x 64 quarter
  const int m0 = s * a.chunk;
  const int m1 = min(a.M, m0 + a.chunk);
  const bool bias = BIAS && it == 0 && wi == 0;

  // two register stages in flight: the loads for stage st + 2 are issued while stage st computes
  // and stage st + 1 (issued one stage earlier) is written to LDS at its end
  XL xs[2];
  YL ys[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    xs[r].init(a, tid, m0, m1, i0);
    ys[r].init(a, tid, m0, m1, j0);
  }
  // this group's stage count (group g's stage q is the chunk's stage NG q + g; past the chunk's
  // end the rows read zero)
  const int nst = ((m1 - m0 + kDwK - 1) / kDwK + NG - 1) / NG;
  // straight-line staging (as gemm_nt.h): stage loads / LDS writes past the end are issued
  // unconditionally (they read zeros: rows past m1 are zero) so the waitcnt pass keeps two
  // register stages in flight instead of draining the queue before every reload
  xs[0].load(a, grp);
  ys[0].load(a, grp);
  xs[1].load(a, NG + grp);
  ys[1].load(a, NG + grp);

  unsigned ca[8];   // [operand x / dy][t = 0, 1][r1, r2] transposed-read addresses
  {
    const int li = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int op = 0; op < 2; ++op) {
        const int col0 = 64 * (op == 0 ? wi : wj) + 32 * t;
        const int colb = col0 + 16 * (g & 1) + 4 * (li & 3);
        const int chunk = colb >> 3, half = (colb >> 2) & 1;
        const int r1 = 4 * h + (li >> 2), r2 = r1 + 8;
        ca[4 * op + 2 * t] = r1 * 256 + 16 * (chunk ^ swz<128>(r1)) + 8 * half;
        ca[4 * op + 2 * t + 1] = r2 * 256 + 16 * (chunk ^ swz<128>(r2)) + 8 * half;
      }
    }
  }
  f32x16 acc[2][2], accb[2];
#pragma unroll
  for (int a2 = 0; a2 < 2; ++a2) {
    accb[a2] = zero16();
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2) acc[a2][b2] = zero16();
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;

  auto compute = [&](const char* imx, const char* imy) {
#pragma unroll
    for (int k = 0; k < kDwK / 16; ++k) {
      const bf16x8 a0 = dw_colfrag(imx, ca, k, 0), a1 = dw_colfrag(imx, ca, k, 1);
      const bf16x8 b0 = dw_colfrag(imy, ca + 4, k, 0), b1 = dw_colfrag(imy, ca + 4, k, 1);
      acc[0][0] = MF<__bf16>::mma(a0, b0, acc[0][0]);
      acc[0][1] = MF<__bf16>::mma(a0, b1, acc[0][1]);
      acc[1][0] = MF<__bf16>::mma(a1, b0, acc[1][0]);
      acc[1][1] = MF<__bf16>::mma(a1, b1, acc[1][1]);
      if (bias) {
        accb[0] = MF<__bf16>::mma(ones, b0, accb[0]);
        accb[1] = MF<__bf16>::mma(ones, b1, accb[1]);
      }
    }
  };
  xs[0].write(smem);
  ys[0].write(smem + IMG);
  __syncthreads();
  int st = 0;
  for (; st + 2 <= nst; st += 2) {
#pragma unroll
    for (int bsel = 0; bsel < 2; ++bsel) {
      const char* imx = smem + bsel * 2 * IMG;
      char* nxt = smem + (bsel ^ 1) * 2 * IMG;
      // register set bsel was written to LDS at the end of the previous stage: refill (stage + 2)
      xs[bsel].load(a, (st + bsel + 2) * NG + grp);
      ys[bsel].load(a, (st + bsel + 2) * NG + grp);
      compute(imx, imx + IMG);
      xs[bsel ^ 1].write(nxt);
      ys[bsel ^ 1].write(nxt + IMG);
      __syncthreads();
    }
  }
  if (st < nst) compute(smem, smem + IMG);   // odd stage count: the last stage sits in buffer 0
  if constexpr (NG == 2) {
    // group 1 hands its accumulators to group 0 through the (now free) stage buffers: per wave
    // 16 KiB of dW (+ 8 KiB of db), lane-contiguous
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem_all) + w * (4 * 16 * 64);
    float* redb = reinterpret_cast<float*>(smem_all + 4 * 16384) + w * (2 * 16 * 64);
    if (grp == 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(q * 16 + r) * 64 + lane] = acc[q >> 1][q & 1][r];
      if (bias) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int r = 0; r < 16; ++r) redb[(q * 16 + r) * 64 + lane] = accb[q][r];
      }
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[q >> 1][q & 1][r] += red[(q * 16 + r) * 64 + lane];
    if (bias) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) accb[q][r] += redb[(q * 16 + r) * 64 + lane];
    }
  }
  // fp32 partial tile: accumulator row = i (row_of), column = j (lane)
  float* P = a.part + (size_t)s * a.I * a.J;
  const int jc = j0 + 64 * wj + (lane & 31);
#pragma unroll
  for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2) {
      const int j = jc + 32 * b2;
      if (j >= a.J) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + 64 * wi + 32 * a2 + row_of(r, h);
        if (i < a.I) P[(size_t)i * a.J + j] = acc[a2][b2][r];
      }
    }
  if (bias && h == 0) {
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2) {
      const int j = jc + 32 * b2;
      if (j < a.J) a.bpart[(size_t)s * a.J + j] = accb[b2][0];
    }
  }
}

// dw[i][j] (+)= sum_s part[s][i][j]; db likewise (blockIdx.y == 1 for db).  A workgroup takes 64
// float4 columns x 4 split groups: group g sums its contiguous quarter of the splits in split order,
// then the four group sums are added in group order (fixed order: deterministic).  One thread per
// column summing all S partials (S = 14 .. 56 at the DeiT-S shapes) ran latency-bound on a few
// hundred workgroups.
constexpr int kDwRedCols = 64, kDwRedGroups = 4;
__global__ __launch_bounds__(256) void gemm_dw_reduce_kernel(DwArgs a) {
  if (blockIdx.y == 0) {
    __shared__ f32x4 red[kDwRedGroups][kDwRedCols];
    const long long n4 = (long long)a.I * a.J / 4;
    const long long stride = (long long)a.I * a.J;
    const int col = threadIdx.x % kDwRedCols, grp = threadIdx.x / kDwRedCols;
    const int per = (a.S + kDwRedGroups - 1) / kDwRedGroups;
    const int s0 = grp * per, s1 = min(a.S, s0 + per);
    for (long long base = blockIdx.x * (long long)kDwRedCols; base < n4; base += (long long)gridDim.x * kDwRedCols) {
      const long long e = base + col;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (e < n4 && s0 < s1) {
        acc = *reinterpret_cast<const f32x4*>(a.part + s0 * stride + 4 * e);
        for (int s = s0 + 1; s < s1; ++s) acc += *reinterpret_cast<const f32x4*>(a.part + s * stride + 4 * e);
      }
      red[grp][col] = acc;
      __syncthreads();
      if (grp == 0 && e < n4) {
#pragma unroll
        for (int g = 1; g < kDwRedGroups; ++g) acc += red[g][col];
      }
      __syncthreads();
      if (grp != 0 || e >= n4) continue;
      const long long i = (4 * e) / a.J, j = (4 * e) % a.J;
      f32x4* out = reinterpret_cast<f32x4*>(
          a.jblock ? a.dw + (j / a.jblock) * ((long long)a.I * a.jblock) + i * a.jblock + j % a.jblock
                   : a.dw + i * a.ldw + j);
      if (a.accumulate) acc += *out;
      *out = acc;
    }
  } else if (a.db) {
    for (int j = blockIdx.x * 256 + threadIdx.x; j < a.J; j += gridDim.x * 256) {
      float acc = a.bpart[j];
      for (int s = 1; s < a.S; ++s) acc += a.bpart[(size_t)s * a.J + j];
      a.db[j] = a.accumulate ? a.db[j] + acc : acc;
    }
  }
}

}  // namespace sae
