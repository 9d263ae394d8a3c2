// REJECTED EXPERIMENT (round 4) -- not built, not dispatched; kept as the record behind DESIGN.md §5
// "Rejected in round 4".  Measured as dev variants 10 / 11 of the bf16 forward: slower than fwd2.h
// on every ViT shape (VGPR spills at 3 waves/SIMD, 2 waves too few to hide the exp2 chain) and the
// fixed-max fallback drifted dv past tolerance (gpurun_out r04f logs, profiles/r04f_fwdp.txt).
// fwdp.h -- software-pipelined bf16 forward attention (D <= 64), no running max.
//
// Same layout and algorithm as attn_fwd2_kernel (fwd2.h; reference chain
// models/layers/attentions/attention.py:39-58: query on the MFMA lane, S^T = K Q^T, P V through
// V^T P^T, one wave per 32 query rows, 4 waves per workgroup, 64-key K / V tiles in LDS), with the
// per-tile VALU work cut and the tile's two dependency chains overlapped:
//   * no running max: q is pre-scaled once by scale * log2(e) (rounded to bf16, as the reference
//     rounds q / sqrt(d)), so the MFMA returns s' = log2(e) S and P = exp2(s') needs no subtract,
//     no max and no rescale.  O = sum P V / sum P is exact algebra without the max; the max only
//     guards fp32 range, so after the sweep any row whose sum left [2^-64, 2^64) (a score beyond
//     about +-60 log2 units) makes the workgroup redo its block with the tracking sweep of fwd2.h
//     (same inputs: bit-equal to fwd2's tracking path);
//   * K one tile ahead of V: iteration t runs the QK^T MFMAs of tile t + 1 beside the exp2 / row
//     sum / bf16 packing of tile t (independent, one basic block: the compiler interleaves the
//     matrix pipe with the VALU), then P V of tile t (T15, two named score states);
//   * the last tile's key mask is applied once, after the tile's QK^T, outside the hot block.
// K(t) sits in the K half of LDS buffer t & 1 and V(t) in the V half: iteration t reads K(t + 1)
// and V(t), writes K(t + 2) over K(t) and V(t + 1) over V(t - 1), one barrier per iteration.
#pragma once
#include <type_traits>

#include "fwd2.h"

namespace sae {

// exp2 of a score tile in place, the row-sum contribution returned (fp32, tree order)
__device__ __forceinline__ float fwdp_exp16(f32x16& s) {
#pragma unroll
  for (int r = 0; r < 16; ++r) s[r] = ex2(s[r]);
  float a0 = s[0] + s[1], a1 = s[2] + s[3], a2 = s[4] + s[5], a3 = s[6] + s[7];
  float a4 = s[8] + s[9], a5 = s[10] + s[11], a6 = s[12] + s[13], a7 = s[14] + s[15];
  return ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));
}

template <int DP, int MINW, int NSU = DP / 16, bool ROT = false>
__global__ __launch_bounds__(256, MINW) void attn_fwdp_kernel(AttnArgs a) {
  using FF = F2<DP>;
  constexpr int NW = 4, NS = NSU, NT = FF::NT, TILE = FF::TILE;
  constexpr int BQ = 32 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nqb = (a.Nq + BQ - 1) / BQ;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb;
  bid /= nqb;
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q = qb * BQ + w * 32 + r32;
  const bool active = qb * BQ + __builtin_amdgcn_readfirstlane(w) * 32 < a.Nq;

  const __bf16* Q = reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const __bf16* K = reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const __bf16* V = reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2];

  F2Stage<DP, NW> kst, vst;
  kst.init(tid, a.ks[1], a.D);
  vst.init(tid, a.vs[1], a.D);
  const __amdgpu_buffer_rsrc_t rk = row_rsrc(K, a.Nk, a.ks[1]);
  const __amdgpu_buffer_rsrc_t rv = row_rsrc(V, a.Nk, a.vs[1]);
  const unsigned kstep = (unsigned)(64 * a.ks[1] * 2), vstep = (unsigned)(64 * a.vs[1] * 2);
  const int nkt = (a.Nk + 63) / 64;

  // query fragments (row q, head-dim 16s + 8h .. +7), rotated (ROT), pre-scaled by scale log2(e)
  const float sl2 = a.scale * kLog2e;
  bf16x8 qf[NS];
  {
    const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
    const unsigned qo = (unsigned)((long long)q * a.qs[1] * 2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const unsigned off = (16 * s + 8 * h < a.D) ? qo + (16 * s + 8 * h) * 2 : 0x80000000u;
      qf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, off, 0, 0));
    }
    if constexpr (ROT) {
#pragma unroll
      for (int s = 0; s < NS; ++s) qf[s] = rope8<1>(qf[s], a.rope, q, 16 * s + 8 * h);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[s][j] = (__bf16)((float)qf[s][j] * sl2);
  }
  unsigned ka[NS], va[2 * NT];
#pragma unroll
  for (int s = 0; s < NS; ++s) ka[s] = r32 * DP * 2 + 16 * ((2 * s + h) ^ swz<DP>(r32));
  {
    const int li = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int colb = 32 * t + 16 * (g & 1) + 4 * (li & 3);
      const int chunk = colb >> 3, half = (colb >> 2) & 1;
      const int r1 = 4 * h + (li >> 2), r2 = r1 + 8;
      va[2 * t] = r1 * DP * 2 + 16 * (chunk ^ swz<DP>(r1)) + 8 * half;
      va[2 * t + 1] = r2 * DP * 2 + 16 * (chunk ^ swz<DP>(r2)) + 8 * half;
    }
  }

  // ---- prologue: K(0), V(0) into buffer 0, K(1) into buffer 1's K half
  kst.load(rk, 0);
  vst.load(rv, 0);
  if constexpr (ROT) kst.rope(a.rope, 0, tid);
  kst.write(smem);
  vst.write(smem + TILE);
  kst.load(rk, kstep);
  if constexpr (ROT) kst.rope(a.rope, 64, tid);
  kst.write(smem + 2 * TILE);
  vm_wait_all();
  __syncthreads();

  // score tile of the K image at ldsK (64 keys: two 32-key halves)
  auto qk = [&](const char* ldsK, f32x16& s0, f32x16& s1) __attribute__((always_inline)) {
    s0 = zero16();
    s1 = zero16();
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bf16x8 k0 = *reinterpret_cast<const bf16x8*>(ldsK + ka[s]);
      const bf16x8 k1 = *reinterpret_cast<const bf16x8*>(ldsK + ka[s] + 32 * DP * 2);
      s0 = MF<__bf16>::mma(k0, qf[s], s0);
      s1 = MF<__bf16>::mma(k1, qf[s], s1);
    }
  };
  // keys past Nk of the tile starting at key0 score -inf (key = row_of(r, h) (+32))
  auto mask = [&](f32x16& s0, f32x16& s1, int key0) __attribute__((always_inline)) {
    const int nvh = a.Nk - key0 - 4 * h;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = (r & 3) + 8 * (r >> 2);
      s0[r] = c < nvh ? s0[r] : -kInf;
      s1[r] = c + 32 < nvh ? s1[r] : -kInf;
    }
  };
  f32x16 acco[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acco[t] = zero16();
  float l = 0.f;
  // P V of one 64-key tile (P in s0 / s1, already exponentiated) with V^T from ldsV
  auto pv = [&](const char* ldsV, const f32x16& s0, const f32x16& s1) __attribute__((always_inline)) {
#pragma unroll
    for (int hk = 0; hk < 2; ++hk) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = acc_frag<__bf16>(hk ? s1 : s0, s2);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const char* p1 = ldsV + va[2 * t] + (32 * hk + 16 * s2) * DP * 2;
          const char* p2 = ldsV + va[2 * t + 1] + (32 * hk + 16 * s2) * DP * 2;
          acco[t] = MF<__bf16>::mma(tr2(p1, p2), pf, acco[t]);
        }
      }
    }
  };
  // iteration t: loads K(t + 2), V(t + 1); S(t + 1) beside exp2(S(t)); P V(t); stage; barrier
  auto iter = [&](int t, f32x16& c0, f32x16& c1, f32x16& n0, f32x16& n1, auto par_c, auto compute_c)
                  __attribute__((always_inline)) {
    constexpr int par = decltype(par_c)::value;       // t & 1
    constexpr bool compute = decltype(compute_c)::value;
    char* bufc = smem + par * 2 * TILE;                // K(t) / V(t) buffer
    char* bufn = smem + (par ^ 1) * 2 * TILE;          // K(t + 1) / V(t + 1) buffer
    kst.load(rk, (unsigned)(t + 2) * kstep);           // past Nk: zeros (range check), never read
    vst.load(rv, (unsigned)(t + 1) * vstep);
    if constexpr (compute) {
      qk(bufn, n0, n1);                                // S(t + 1)
      l += fwdp_exp16(c0) + fwdp_exp16(c1);            // P(t)
      pv(bufc + TILE, c0, c1);                         // O += P(t) V(t)
    }
    if constexpr (ROT) kst.rope(a.rope, 64 * (t + 2), tid);
    kst.write(bufc);                                   // K(t + 2) over K(t)
    vst.write(bufn + TILE);                            // V(t + 1) over V(t - 1)
    if constexpr (compute)
      if (t + 1 == nkt - 1 && (a.Nk & 63)) mask(n0, n1, 64 * (t + 1));
    __syncthreads();
  };
  auto sweep = [&](auto compute_c) __attribute__((always_inline)) {
    f32x16 sa0, sa1, sb0, sb1;
    if constexpr (decltype(compute_c)::value) {
      qk(smem, sa0, sa1);                              // S(0)
      if (nkt == 1 && (a.Nk & 63)) mask(sa0, sa1, 0);
    }
    __syncthreads();   // every wave has read K(0) before iteration 0 writes K(2) over it
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    for (int t = 0; t < nkt; t += 2) {
      iter(t, sa0, sa1, sb0, sb1, P0{}, compute_c);
      if (t + 1 < nkt) iter(t + 1, sb0, sb1, sa0, sa1, P1{}, compute_c);
    }
  };
  if (active) sweep(std::true_type{});
  else sweep(std::false_type{});

  // rows whose sum left [2^-64, 2^64): redo the block with fwd2's tracking sweep (running max)
  float m = 0.f;
  const float lt0 = xhalf_sum(l);
  if (__syncthreads_or(active && q < a.Nq && !(lt0 >= 0x1p-64f && lt0 < 0x1p64f))) {
    f32x16 lacc;
    m = -kInf;
    kst.load(rk, 0);
    vst.load(rv, 0);
    if constexpr (ROT) kst.rope(a.rope, 0, tid);
    kst.write(smem);
    vst.write(smem + TILE);
    vm_wait_all();
    __syncthreads();
    auto step = [&](int t, auto bsel_c, auto first_c, auto compute_c) __attribute__((always_inline)) {
      constexpr int bsel = decltype(bsel_c)::value;
      char* cur = smem + bsel * 2 * TILE;
      char* nxt = smem + (bsel ^ 1) * 2 * TILE;
      if (t + 1 < nkt) {
        kst.load(rk, (unsigned)(t + 1) * kstep);
        vst.load(rv, (unsigned)(t + 1) * vstep);
      }
      if constexpr (decltype(compute_c)::value)   // q already carries scale log2(e): sl2 = 1
        fwd2_tile<DP, NW, false, decltype(first_c)::value, NSU, false, false>(
            cur, cur + TILE, qf, acco, lacc, m, l, min(64, a.Nk - 64 * t), 1.f, ka, va, h);
      if (t + 1 < nkt) {
        if constexpr (ROT) kst.rope(a.rope, 64 * (t + 1), tid);
        kst.write(nxt);
        vst.write(nxt + TILE);
      }
      __syncthreads();
    };
    auto tsweep = [&](auto compute_c) __attribute__((always_inline)) {
      using B0 = std::integral_constant<int, 0>;
      using B1 = std::integral_constant<int, 1>;
      step(0, B0{}, std::true_type{}, compute_c);
      for (int t = 1; t < nkt; t += 2) {
        step(t, B1{}, std::false_type{}, compute_c);
        if (t + 1 < nkt) step(t + 1, B0{}, std::false_type{}, compute_c);
      }
    };
    if (active) tsweep(std::true_type{});
    else tsweep(std::false_type{});
  }

  if (!active) return;
  const float lt = xhalf_sum(l);
  const float inv = 1.f / lt;
  {  // O rows through a per-wave LDS scratch (the K/V images are free after the last barrier)
    const int q0 = qb * BQ + w * 32;
    __bf16* O = reinterpret_cast<__bf16*>(a.out) + b * a.os[0] + hh * a.os[2] + (long long)q0 * a.os[1];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acco[t][r] *= inv;
    wave_store_rows<DP>(acco, 1.f, smem + w * 32 * DP * 2, O, a.os[1], a.Nq - q0, a.D, lane);
  }
  if (q < a.Nq && h == 0 && a.lse) a.lse[((size_t)b * a.H + hh) * a.Nq + q] = (m + lg2(lt)) * kLn2;
}

}  // namespace sae
