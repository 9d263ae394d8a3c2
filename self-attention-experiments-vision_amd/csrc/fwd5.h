// fwd5.h -- round-5 bf16 attention forward for gfx950 at head_dim <= 64 (the ViT / DeiT / CaiT
// trunks; models/layers/attentions/attention.py:39-58).
//
// Same tiling as fwd2.h (one wave = 32 query rows with the query on the MFMA lane, S^T = K Q^T;
// NW waves share each 64-key K / V tile staged global -> registers -> LDS, one barrier per tile),
// rebuilt so that a full 64-key tile is ONE basic block whose VALU work is only what the softmax
// needs:
//   * the query fragments are pre-scaled by scale * log2(e) (rounded to bf16 once, at load), so the
//     score accumulator already holds the exponent's argument in log2 units;
//   * the running max is fixed by the first tile (fwd2.h FIX: the block is redone with the tracking
//     sweep if any row's sum leaves [1, 2^64)), and its negation is the score MFMAs' initial
//     accumulator: p = 2^(acc) is ONE v_exp_f32 per score, no multiply, no subtract, no max;
//   * full tiles and the ragged last tile are separate code (the tail's masking and the "second
//     32-key half exists" test were branches inside fwd2's tile, which split it into basic blocks
//     the scheduler could not interleave across);
//   * the row sum is a pairwise tree per tile (fwd2's serial chain of 32 dependent adds sat on the
//     critical path) or, LSUM, an MFMA with an all-ones operand;
//   * the next tile's global loads and LDS writes are unconditional (past the last key the
//     descriptor's range check reads zeros into a buffer nobody reads).
#pragma once
#include <type_traits>

#include "fwd2.h"

namespace sae {

// x * s for 8 bf16 values, rounded back to bf16 (round-to-nearest-even)
__device__ __forceinline__ bf16x8 bf16x8_scale(bf16x8 x, float s) {
  bf16x8 y;
#pragma unroll
  for (int j = 0; j < 8; ++j) y[j] = (__bf16)((float)x[j] * s);
  return y;
}

// pairwise sum of the 16 accumulator values of a 32 x 32 tile (depth 4, not a 16-long chain)
__device__ __forceinline__ float tree16(const f32x16& x) {
  const float a0 = (x[0] + x[1]) + (x[2] + x[3]), a1 = (x[4] + x[5]) + (x[6] + x[7]);
  const float a2 = (x[8] + x[9]) + (x[10] + x[11]), a3 = (x[12] + x[13]) + (x[14] + x[15]);
  return (a0 + a1) + (a2 + a3);
}
__device__ __forceinline__ float tmax16(const f32x16& x) {
  const float a0 = fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])), a1 = fmaxf(fmaxf(x[4], x[5]), fmaxf(x[6], x[7]));
  const float a2 = fmaxf(fmaxf(x[8], x[9]), fmaxf(x[10], x[11])), a3 = fmaxf(fmaxf(x[12], x[13]), fmaxf(x[14], x[15]));
  return fmaxf(fmaxf(a0, a1), fmaxf(a2, a3));
}

// Tile kinds: FIRST (sets the running max), TAIL (keys past nvalid masked; nvalid <= 32 skips the
// second half), TRACK (the fallback sweep: a tile whose max exceeds the running max by more than
// 2^8 moves it and rescales what was accumulated).
template <int NS, int NT, bool LSUM, bool FIRST, bool TAIL, bool TRACK>
__device__ __forceinline__ void fwd5_tile(const char* ldsK, const char* ldsV, const bf16x8* qf, f32x16* acco,
                                          f32x16& lacc, float& lsum, float& m, f32x16& negm, int nvalid,
                                          const unsigned* ka, const unsigned* va, int h) {
  constexpr int DP = 64;
  const bool two = !TAIL || nvalid > 32;
  bf16x8 kk0[NS], kk1[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) kk0[s] = *reinterpret_cast<const bf16x8*>(ldsK + ka[s]);
  if (two) {
#pragma unroll
    for (int s = 0; s < NS; ++s) kk1[s] = *reinterpret_cast<const bf16x8*>(ldsK + ka[s] + 32 * DP * 2);
  }
  f32x16 s0 = FIRST ? zero16() : negm, s1 = FIRST ? zero16() : negm;
#pragma unroll
  for (int s = 0; s < NS; ++s) s0 = MF<__bf16>::mma(kk0[s], qf[s], s0);
  if (two) {
#pragma unroll
    for (int s = 0; s < NS; ++s) s1 = MF<__bf16>::mma(kk1[s], qf[s], s1);
  }
  if constexpr (TAIL) {   // keys past the end score -inf (key = 32 u + row_of(r, h))
    const int nvh = nvalid - 4 * h;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = (r & 3) + 8 * (r >> 2);
      s0[r] = c < nvh ? s0[r] : -kInf;
      s1[r] = (two && c + 32 < nvh) ? s1[r] : -kInf;
    }
  }
  if constexpr (FIRST) {   // the running max starts at this tile's max
    float mx = two ? fmaxf(tmax16(s0), tmax16(s1)) : tmax16(s0);
    m = xhalf_max(mx);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      negm[r] = -m;
      s0[r] -= m;
      s1[r] -= m;
    }
  } else if constexpr (TRACK) {   // accumulators are relative to m; move it if a score left 2^8
    float mx = two ? fmaxf(tmax16(s0), tmax16(s1)) : tmax16(s0);
    mx = xhalf_max(mx);
    if (!__all(mx <= 8.f)) {
      const float mv = fmaxf(mx, 0.f);
      const float alpha = ex2(-mv);
      m += mv;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        negm[r] = -m;
        s0[r] -= mv;
        s1[r] -= mv;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acco[t][r] *= alpha;
      if constexpr (LSUM) {
#pragma unroll
        for (int r = 0; r < 16; ++r) lacc[r] *= alpha;
      } else {
        lsum *= alpha;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) s0[r] = ex2(s0[r]);
  if (two) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s1[r] = ex2(s1[r]);
  }
  if constexpr (!LSUM) {
    const float ts = two ? tree16(s0) + tree16(s1) : tree16(s0);
    lsum = FIRST ? ts : lsum + ts;
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (u == 1 && !two) break;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pf = acc_frag<__bf16>(u == 0 ? s0 : s1, s2);
      const bool z = FIRST && u == 0 && s2 == 0;   // first tile, first 16 keys: zero C operand
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int ro = (32 * u + 16 * s2) * DP * 2;
        const bf16x8 vv = tr2(ldsV + va[2 * t] + ro, ldsV + va[2 * t + 1] + ro);
        acco[t] = MF<__bf16>::mma(vv, pf, z ? zero16() : acco[t]);
      }
      if constexpr (LSUM) lacc = MF<__bf16>::mma(ones, pf, z ? zero16() : lacc);
    }
  }
}

// NW waves x 32 query rows per workgroup, MINW workgroups' worth of waves per SIMD.
template <int NW, int MINW, bool LSUM, int NSU>
__global__ __launch_bounds__(64 * NW, MINW) void attn_fwd5_kernel(AttnArgs a) {
  constexpr int DP = 64;
  using FF = F2<DP>;
  constexpr int NS = NSU, NT = FF::NT, TILE = FF::TILE;
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
  const int nfull = a.Nk / 64;
  kst.load(rk, 0);
  vst.load(rv, 0);

  const float sl2 = a.scale * kLog2e;
  bf16x8 qf[NS];
  {
    const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
    const unsigned qo = (unsigned)((long long)q * a.qs[1] * 2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const unsigned off = (16 * s + 8 * h < a.D) ? qo + (16 * s + 8 * h) * 2 : 0x80000000u;
      qf[s] = bf16x8_scale(__builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, off, 0, 0)), sl2);
    }
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

  f32x16 acco[NT], lacc, negm;
  float m = 0.f, lsum = 0.f;

  kst.write(smem);
  vst.write(smem + TILE);
  vm_wait_all();
  __syncthreads();
  // one K/V tile: load t + 1 (unconditionally: past the end it reads zeros into a buffer nobody
  // reads), compute t from buffer BSEL, stage t + 1 into the other buffer, barrier
  auto step = [&](int t, auto bsel_c, auto first_c, auto tail_c, auto track_c, auto compute_c) {
    constexpr int bsel = decltype(bsel_c)::value;
    const char* cur = smem + bsel * 2 * TILE;
    char* nxt = smem + (bsel ^ 1) * 2 * TILE;
    kst.load(rk, (unsigned)(t + 1) * kstep);
    vst.load(rv, (unsigned)(t + 1) * vstep);
    if constexpr (decltype(compute_c)::value)
      fwd5_tile<NS, NT, LSUM, decltype(first_c)::value, decltype(tail_c)::value, decltype(track_c)::value>(
          cur, cur + TILE, qf, acco, lacc, lsum, m, negm, decltype(tail_c)::value ? a.Nk - 64 * t : 64, ka, va, h);
    kst.write(nxt);
    vst.write(nxt + TILE);
    __syncthreads();
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  using T_ = std::true_type;
  using F_ = std::false_type;
  auto sweep = [&](auto compute_c, auto track_c) {
    if (nfull == 0) {   // a single, partial tile
      step(0, B0{}, T_{}, T_{}, track_c, compute_c);
      return;
    }
    step(0, B0{}, T_{}, F_{}, track_c, compute_c);
    int t = 1;
    for (; t + 1 < nfull; t += 2) {
      step(t, B1{}, F_{}, F_{}, track_c, compute_c);
      step(t + 1, B0{}, F_{}, F_{}, track_c, compute_c);
    }
    if (t < nfull) {   // t odd: one more full tile in buffer 1
      step(t, B1{}, F_{}, F_{}, track_c, compute_c);
      ++t;
    }
    if (t < nkt) {     // the ragged last tile, buffer t & 1
      if (t & 1) step(t, B1{}, F_{}, T_{}, track_c, compute_c);
      else step(t, B0{}, F_{}, T_{}, track_c, compute_c);
    }
  };
  if (active) sweep(T_{}, F_{});
  else sweep(F_{}, F_{});
  // a row whose sum left [1, 2^64) (a later score far above the first tile's max): redo the block
  // with the tracking sweep (fwd2.h FIX)
  const float lt0 = LSUM ? lacc[0] : xhalf_sum(lsum);
  if (__syncthreads_or(active && q < a.Nq && !(lt0 < 0x1p64f))) {
    kst.load(rk, 0);
    vst.load(rv, 0);
    kst.write(smem);
    vst.write(smem + TILE);
    vm_wait_all();
    __syncthreads();
    if (active) sweep(T_{}, T_{});
    else sweep(F_{}, T_{});
  }
  if (!active) return;
  const float lt = LSUM ? lacc[0] : xhalf_sum(lsum);
  const float inv = 1.f / lt;
  {  // O rows through a per-wave LDS scratch (the K/V images are free after the last barrier)
    const int q0 = qb * BQ + w * 32;
    __bf16* O = reinterpret_cast<__bf16*>(a.out) + b * a.os[0] + hh * a.os[2] + (long long)q0 * a.os[1];
    wave_store_rows<DP>(acco, inv, smem + w * 32 * DP * 2, O, a.os[1], a.Nq - q0, a.D, lane);
  }
  if (q < a.Nq && h == 0 && a.lse) a.lse[((size_t)b * a.H + hh) * a.Nq + q] = (m + lg2(lt)) * kLn2;
}

}  // namespace sae

namespace sae {

// ------------------------------------------------------------------ forward, ping-pong form
// 8 waves = 2 groups x 4; waves w and w + 4 hold the same 32 query rows (query group w & 3, query
// on the MFMA lane) and split each 64-key K / V tile: group u takes key half u, with its own running
// max m, row sum l and O accumulator.  Each group alternates
//   M(t): O^T += V^T P^T of tile t - 1 (its 32 keys, 4 MFMAs) and S^T = K Q^T of tile t (4 MFMAs)
//   V(t): P = 2^(S sl2 - m) (the first tile sets m: fwd2.h FIX), row sums, bf16 packing
// group 1 one phase behind group 0, one barrier per phase for all 8 waves, K / V tiles in a 3-deep
// LDS ring (as attn_bwd6_dkdv_kernel).  At the end the two groups' (m, l, O) merge through LDS:
// m = max(m0, m1), O = O0 2^(m0 - m) + O1 2^(m1 - m), l likewise.  A row whose sum left [1, 2^64)
// in either group (a later score far above its first tile's max) makes the workgroup redo the sweep
// with per-tile max tracking (TRACK).
// PRIO: waves 4-7 (the second-dispatched group, which loses VALU arbitration) at s_setprio 1
template <int PRIO = 0>
__global__ __launch_bounds__(512, 1) void attn_fwd6_kernel(AttnArgs a) {
  constexpr int DP = 64, NW = 8;
  using FF = F2<DP>;
  constexpr int NS = FF::NS, NT = FF::NT, TILE = FF::TILE;
  constexpr int BQ = 128;
  constexpr int TB = 2 * TILE;
  constexpr int NBUF = 3;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nqb = (a.Nq + BQ - 1) / BQ;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb;
  bid /= nqb;
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qg = w & 3, u = w >> 2;
  const int q = qb * BQ + qg * 32 + r32;
  const bool active = qb * BQ + qg * 32 < a.Nq;

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
  auto fetch = [&](int t) {
    kst.load(rk, (unsigned)t * kstep);
    vst.load(rv, (unsigned)t * vstep);
  };
  auto put = [&](int t) {
    char* buf = smem + (t % NBUF) * TB;
    kst.write(buf);
    vst.write(buf + TILE);
  };

  bf16x8 qf[NS];
  {
    const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
    const unsigned qo = (unsigned)((long long)q * a.qs[1] * 2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const unsigned off = (16 * s + 8 * h < a.D) ? qo + (16 * s + 8 * h) * 2 : 0x80000000u;
      qf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, off, 0, 0));
    }
  }
  const float sl2 = a.scale * kLog2e;
  unsigned ka[NS], va[2 * NT];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int rr = 32 * u + r32;
    ka[s] = rr * DP * 2 + 16 * ((2 * s + h) ^ swz<DP>(rr));
  }
  {
    const int li = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int colb = 32 * t + 16 * (g & 1) + 4 * (li & 3);
      const int chunk = colb >> 3, half = (colb >> 2) & 1;
      const int r1 = 32 * u + 4 * h + (li >> 2), r2 = r1 + 8;
      va[2 * t] = r1 * DP * 2 + 16 * (chunk ^ swz<DP>(r1)) + 8 * half;
      va[2 * t + 1] = r2 * DP * 2 + 16 * (chunk ^ swz<DP>(r2)) + 8 * half;
    }
  }

  f32x16 acco[NT], sp;
  bf16x8 pf[2];
  float m = 0.f, lsum = 0.f;
  bool started = false;   // this group has seen a tile with keys (its max is set)

  auto sweep = [&](auto track_c) {
    constexpr bool TRACK = decltype(track_c)::value;
#pragma unroll
    for (int t = 0; t < NT; ++t) acco[t] = zero16();
#pragma unroll
    for (int i = 0; i < 2; ++i) pf[i] = bf16x8{};
    m = 0.f;
    lsum = 0.f;
    started = false;
    fetch(0);
    vm_wait_all();
    put(0);
    fetch(1);
    vm_wait_all();
    put(1);
    fetch(2);
    __syncthreads();
    auto mphase = [&](int t) {
      if (t > 0) {   // O^T += V^T P^T of tile t - 1
        const char* ldsV = smem + ((t - 1) % NBUF) * TB + TILE;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int tt = 0; tt < NT; ++tt) {
            const int ro = 16 * s2 * DP * 2;
            const bf16x8 vv = tr2(ldsV + va[2 * tt] + ro, ldsV + va[2 * tt + 1] + ro);
            acco[tt] = MF<__bf16>::mma(vv, pf[s2], acco[tt]);
          }
      }
      if (t < nkt) {   // S^T = K Q^T of tile t
        const char* ldsK = smem + (t % NBUF) * TB;
        sp = zero16();
#pragma unroll
        for (int s = 0; s < NS; ++s) sp = MF<__bf16>::mma(*reinterpret_cast<const bf16x8*>(ldsK + ka[s]), qf[s], sp);
      }
    };
    auto vphase = [&](int t) {
      const int nvh = a.Nk - 64 * t - 32 * u - 4 * h;   // keys of this half that exist, per lane half
      const bool full = a.Nk - 64 * t - 32 * u >= 32;    // wave-uniform
      if (!full) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sp[r] = ((r & 3) + 8 * (r >> 2)) < nvh ? sp[r] * sl2 : -kInf;
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) sp[r] *= sl2;
      }
      if (!started || TRACK) {
        const float mx = xhalf_max(tmax16(sp));
        if (!started) {
          if (__all(mx == -kInf)) {   // no key of this group in the tile (nothing to add)
#pragma unroll
            for (int i = 0; i < 2; ++i) pf[i] = bf16x8{};
            return;
          }
          m = mx;
          started = true;
        } else if (!__all(mx - m <= 8.f)) {
          const float mn = fmaxf(m, mx);
          const float alpha = ex2(m - mn);
          m = mn;
#pragma unroll
          for (int tt = 0; tt < NT; ++tt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acco[tt][r] *= alpha;
          lsum *= alpha;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) sp[r] = ex2(sp[r] - m);
      lsum += tree16(sp);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) pf[s2] = acc_frag<__bf16>(sp, s2);
    };
    const int nph = 2 * nkt + 2;
    if (PRIO && u == 1) __builtin_amdgcn_s_setprio(1);
    for (int p = 0; p < nph; ++p) {
      if ((p & 1) == 0 && p >= 2) {
        const int t = p / 2 - 1;
        if (t + 2 <= nkt) {
          vm_wait_all();
          put(t + 2);
          fetch(t + 3);
        }
      }
      const int qq = p - u;
      if (active && qq >= 0 && qq <= 2 * nkt) {
        if ((qq & 1) == 0) mphase(qq / 2);
        else vphase(qq / 2);
      }
      __syncthreads();
    }
  };
  sweep(std::false_type{});
  {
    const float lt = xhalf_sum(lsum);
    if (__syncthreads_or(active && q < a.Nq && !(lt < 0x1p64f))) sweep(std::true_type{});
  }
  // merge group 1 into group 0 through LDS: [query group][m | l] and O^T partials
  float* red = reinterpret_cast<float*>(smem);
  float* redml = red + 4 * NT * 16 * 64;
  const float lt = xhalf_sum(lsum);
  if (u == 1 && active) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((qg * NT + t) * 16 + r) * 64 + lane] = acco[t][r];
    if (h == 0) {
      redml[qg * 64 + r32] = started ? m : -kInf;
      redml[qg * 64 + 32 + r32] = lt;
    }
  }
  __syncthreads();
  if (u == 0 && active) {
    const float m1 = redml[qg * 64 + r32], l1 = redml[qg * 64 + 32 + r32];
    const float m0 = started ? m : -kInf;
    const float mm = fmaxf(m0, m1);
    const float a0 = m0 == -kInf ? 0.f : ex2(m0 - mm), a1 = m1 == -kInf ? 0.f : ex2(m1 - mm);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acco[t][r] = acco[t][r] * a0 + red[((qg * NT + t) * 16 + r) * 64 + lane] * a1;
    const float ltot = lt * a0 + l1 * a1;
    m = mm;
    lsum = ltot;
  }
  __syncthreads();
  if (u == 0 && active) {
    const float inv = 1.f / lsum;
    const int q0 = qb * BQ + qg * 32;
    __bf16* O = reinterpret_cast<__bf16*>(a.out) + b * a.os[0] + hh * a.os[2] + (long long)q0 * a.os[1];
    wave_store_rows<DP>(acco, inv, smem + qg * 32 * DP * 2, O, a.os[1], a.Nq - q0, a.D, lane);
    if (q < a.Nq && h == 0 && a.lse) a.lse[((size_t)b * a.H + hh) * a.Nq + q] = (m + lg2(lsum)) * kLn2;
  }
}

}  // namespace sae
