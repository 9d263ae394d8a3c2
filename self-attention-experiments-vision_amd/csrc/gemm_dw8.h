// gemm_dw8.h -- the projection weight / bias gradients (gemm_dw.h) with LDS-DMA operand staging.
//
// Same product, tiling and reduction as gemm_dw_kernel (128 x 128 output tile per 4-wave group,
// 64 x 64 per wave on v_mfma_f32_32x32x16_bf16, both operands read transposed with
// ds_read_b64_tr_b16 from [token][column] images, db on the matrix pipe, fp32 partial per split
// summed in split order by gemm_dw_reduce_kernel).  What changes is how a stage reaches LDS: the
// register path (buffer_load -> VGPR -> ds_write_b128) moved every operand byte through the LDS
// store port at ~79 B/clk/CU and, with the transposed reads, kept the LDS array busy for about as
// many cycles as the MFMAs run (MI355X_MICROARCH.md, LDS table).  Here the 32-token X and dY
// images are written by LDS-DMA (buffer_load_dwordx4 ... lds, one 1-KiB piece per
// wave-instruction, the LDS array written 64 dwords per clock), the 16-byte chunk swizzle of the
// images applied through the DMA SOURCE address (gemm8.h), and a 4-deep ring per wave group keeps
// three stages in flight with one barrier per stage:
//   stage g:  wait (counted vmcnt) for this wave's pieces of g, s_barrier (everyone's landed; every
//             wave is done with stage g - 1), issue stage g + 3 into g - 1's buffer, compute g.
// Columns past the operand width and rows past the split's chunk read zero through the
// descriptor's range check (no memory traffic).
#pragma once
#include "gemm8.h"
#include "gemm_dw.h"

namespace sae {

constexpr int kDw8K = 32;                  // tokens per stage
constexpr int kDw8NS = 4;                  // ring depth per wave group
constexpr int kDw8Img = kDw8K * 256;       // one [32][128] bf16 operand image (8 KiB)
constexpr int kDw8Stage = 2 * kDw8Img;     // X + dY
template <int NG, int NS = kDw8NS> constexpr int dw8_lds_bytes() {
  constexpr int ring = NG * NS * kDw8Stage;
  constexpr int red = NG == 2 ? 4 * 16384 + 4 * 8192 : 0;   // group 1 -> group 0 hand-off
  return ring > red ? ring : red;
}

// counted wait for the oldest stage with `ahead` younger stages (4 DMA instructions each) in flight
template <int N> __device__ __forceinline__ void dw8_wait(int ahead) {
  if constexpr (N > 0) {
    if (ahead >= N) {
      g8_wait_barrier<4 * N>();
      return;
    }
    dw8_wait<N - 1>(ahead);
  } else {
    g8_wait_barrier<0>();
  }
}

// STAG (NG = 2; dev A/B): the two wave groups (waves 0-3 / 4-7, SIMD partners) offset by one
// barrier -- 1: one barrier per stage (a whole stage apart); 2: a second barrier between the two
// k-steps of a stage (half a stage apart) -- so that partners do not read LDS and issue MFMAs in
// lockstep.  Each group reads only its own ring, so the offset moves no data hazard.
template <bool BIAS, int NG, int NS = kDw8NS, int STAG = 0>
__global__ __launch_bounds__(256 * NG, NG == 1 && NS <= 4 ? 2 : 1) void gemm_dw8_kernel(DwArgs a) {
  static_assert(STAG == 0 || NG == 2, "stagger: two wave groups");
  extern __shared__ __attribute__((aligned(16))) char smem_all[];
  const int ti = (a.I + kDwT - 1) / kDwT, tj = (a.J + kDwT - 1) / kDwT;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);   // as gemm_dw_kernel: a chunk's tiles on one XCD
  const int tile = bid % (ti * tj), s = bid / (ti * tj);
  const int it = tile % ti, jt = tile / ti;
  const int i0 = it * kDwT, j0 = jt * kDwT;
  const int tid = threadIdx.x & 255, lane = tid & 63, h = lane >> 5;
  const int grp = NG == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 8));
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = w & 1, wj = w >> 1;
  const int m0 = s * a.chunk;
  const int m1 = min(a.M, m0 + a.chunk);
  const bool bias = BIAS && it == 0 && wi == 0;
  const unsigned lring = __builtin_amdgcn_readfirstlane(
      (unsigned)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem_all)) +
      (unsigned)(grp * NS * kDw8Stage);
  const char* ring = smem_all + grp * NS * kDw8Stage;

  const g8_u32x4 rx = g8_rsrc(a.x + (long long)m0 * a.ldx, m1 - m0, a.ldx);
  const g8_u32x4 ry = g8_rsrc(a.dy + (long long)m0 * a.ldy, m1 - m0, a.ldy);
  // this wave's pieces: p = w and w + 4 of each 32-row image (rows 4p .. 4p + 3); lane L lands at
  // row 4p + L / 16, chunk L % 16 and fetches global chunk (L % 16) ^ swz<128>(row)
  unsigned vx[2], vy[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = w + 4 * q, r = 4 * p + (lane >> 4), c = (lane & 15) ^ swz<128>(r);
    const int cx = i0 + 8 * c, cy = j0 + 8 * c;
    vx[q] = cx < a.I ? (unsigned)(((long long)r * a.ldx + cx) * 2) : 0x80000000u;
    vy[q] = cy < a.J ? (unsigned)(((long long)r * a.ldy + cy) * 2) : 0x80000000u;
  }
  const unsigned stx = (unsigned)(kDw8K * a.ldx * 2), sty = (unsigned)(kDw8K * a.ldy * 2);
  // group g takes the chunk's stages g, g + NG, ...; both groups run the same count (past the
  // chunk's end the rows read zero) so their barriers pair up
  const int nst = ((m1 - m0 + kDw8K - 1) / kDw8K + NG - 1) / NG;
  auto issue = [&](int q) __attribute__((always_inline)) {
    const int st = q * NG + grp;
    const unsigned lb = lring + (unsigned)((q % NS) * kDw8Stage);
    g8_dma2(rx, vx[0] + (unsigned)st * stx, vx[1] + (unsigned)st * stx, lb + 1024u * w, lb + 1024u * (w + 4));
    g8_dma2(ry, vy[0] + (unsigned)st * sty, vy[1] + (unsigned)st * sty, lb + kDw8Img + 1024u * w,
            lb + kDw8Img + 1024u * (w + 4));
  };

  unsigned ca[8];   // [operand x / dy][t = 0, 1][r1, r2] transposed-read addresses (gemm_dw_kernel)
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

#pragma unroll
  for (int q = 0; q < NS - 1; ++q)
    if (q < nst) issue(q);
  if (STAG && grp == 1) asm volatile("s_barrier" ::: "memory");   // the offset
  for (int g = 0; g < nst; ++g) {
    dw8_wait<NS - 2>(min(NS - 2, nst - 1 - g));   // younger stages still in flight
    __builtin_amdgcn_sched_barrier(0);
    if (g + NS - 1 < nst) issue(g + NS - 1);
    const char* imx = ring + (g % NS) * kDw8Stage;
    const char* imy = imx + kDw8Img;
#pragma unroll
    for (int k = 0; k < kDw8K / 16; ++k) {
      if (STAG == 2 && k == 1) {
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
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
  }
  if (STAG && grp == 0) asm volatile("s_barrier" ::: "memory");   // balance the offset
  if constexpr (NG == 2) {
    // group 1 hands its accumulators to group 0 through the (now idle) ring, as gemm_dw_kernel
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

}  // namespace sae
