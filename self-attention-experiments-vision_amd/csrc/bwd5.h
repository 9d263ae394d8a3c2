// bwd5.h -- round-5 bf16 attention backward for gfx950 at head_dim <= 64, key ranges > 256 (the
// ViT-B/16@384 headline, N = 577): the two passes of bwd2.h (dQ, then dK / dV; the JAX autodiff of
// models/layers/attentions/attention.py:39-58) rebuilt so that one wave keeps the matrix pipe busy
// on its own.  What bounded bwd2 (ISA of the N = 577 instances, profiles/r05*): each 32-row half
// of a tile ran as MFMA burst -> ~55 dependent VALU -> MFMA burst, with a branch between the halves
// (the last tile's empty half), so one wave's softmax never overlapped its own MFMAs and the two
// waves of a SIMD (separate workgroups, same program) mostly stalled in the same phase.
// Here a tile's two halves are one basic block, software-pipelined by hand:
//   phase A  S1 = Q1 K^T, dP1 = dO1 V^T           (8 MFMAs)   beside   softmax of half 0
//   phase B  dV^T += dO0^T P0, dK^T += Q0^T dS0    (8 MFMAs)   beside   softmax of half 1
//   phase C  dV^T += dO1^T P1, dK^T += Q1^T dS1    (8 MFMAs)   then the next tile's S0 / dP0 (8)
// with __builtin_amdgcn_sched_group_barrier fixing the interleave (MFMA : VALU : LDS-read groups),
// so the compiler cannot hoist a whole half and blow the register budget.  Padded query rows
// (past Nq) carry lse = +inf and delta = 0: their P and dS are exactly zero, so the last tile runs
// the same branch-free body.  -delta enters as the dP MFMAs' initial accumulator (read from LDS),
// replacing bwd2's extra MFMA per half.
#pragma once
#include <type_traits>

#include "fwd2.h"

namespace sae {

// sched_group_barrier masks (LLVM SchedGroupMask)
constexpr int kSgMfma = 0x8, kSgValu = 0x402, kSgDsRead = 0x100, kSgDsWrite = 0x200, kSgVmemRead = 0x20;
#define SAE_SGB(mask, n, id) __builtin_amdgcn_sched_group_barrier((mask), (n), (id))

// --------------------------------------------------------------------------- dK / dV pass
// One wave = 32 keys (key on the MFMA lane), K / V fragments in registers; NW waves share each
// 64-query Q / dO tile and its row constants (lse * log2 e, -delta), double-buffered in LDS.
template <int NW, int MINW, int SCHED>
__global__ __launch_bounds__(64 * NW, MINW) void attn_bwd5_dkdv_kernel(AttnArgs a) {
  constexpr int DP = 64;
  using FF = F2<DP>;
  constexpr int NS = FF::NS, NT = FF::NT, TILE = FF::TILE;
  constexpr int BK = 32 * NW;
  constexpr int TB = 2 * TILE + 2 * 64 * 4;   // [Q img | dO img | lse2[64] | -delta[64]]
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nkb = (a.Nk + BK - 1) / BK;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = bid % nkb;
  bid /= nkb;
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int key = kb * BK + w * 32 + r32;
  const bool active = kb * BK + __builtin_amdgcn_readfirstlane(w) * 32 < a.Nk;
  const size_t rowoff = ((size_t)b * a.H + hh) * a.Nq;

  const __bf16* Q = reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const __bf16* K = reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const __bf16* V = reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2];
  const __bf16* G = reinterpret_cast<const __bf16*>(a.dout) + b * a.dos[0] + hh * a.dos[2];

  // Q / dO tiles staged through registers: NSTG = 1 -- tile t + 1 loaded while tile t computes;
  // NSTG = 2 (SCHED 2) -- tile t + 2 (two register sets in flight, as bwd2.h)
  constexpr int NSTG = SCHED == 2 ? 2 : 1;
  F2Stage<DP, NW> qst[NSTG], gst[NSTG];
#pragma unroll
  for (int r = 0; r < NSTG; ++r) {
    qst[r].init(tid, a.qs[1], a.D);
    gst[r].init(tid, a.dos[1], a.D);
  }
  const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
  const __amdgpu_buffer_rsrc_t rg = row_rsrc(G, a.Nq, a.dos[1]);
  const unsigned qstep = (unsigned)(64 * a.qs[1] * 2), gstep = (unsigned)(64 * a.dos[1] * 2);
  const int nqt = (a.Nq + 63) / 64;
  float rc_l[NSTG], rc_d[NSTG];   // raw row constants of a staged tile (threads 0 .. 63)
#pragma unroll
  for (int r = 0; r < NSTG; ++r) rc_l[r] = rc_d[r] = 0.f;
  auto fetch_r = [&](int r, int qt) {
    qst[r].load(rq, (unsigned)qt * qstep);
    gst[r].load(rg, (unsigned)qt * gstep);
    if (tid < 64) {
      const int qq = min(qt * 64 + tid, a.Nq - 1);
      rc_l[r] = a.lse[rowoff + qq];
      rc_d[r] = a.delta[rowoff + qq];
    }
  };
  auto put_r = [&](int r, char* buf, int qt) {
    qst[r].write(buf);
    gst[r].write(buf + TILE);
    if (tid < 64) {
      const bool ok = qt * 64 + tid < a.Nq;
      reinterpret_cast<float*>(buf + 2 * TILE)[tid] = ok ? rc_l[r] * kLog2e : kInf;
      reinterpret_cast<float*>(buf + 2 * TILE + 256)[tid] = ok ? -rc_d[r] : 0.f;
    }
  };
  auto fetch = [&](int qt) { fetch_r(0, qt); };
  auto put = [&](char* buf, int qt) { put_r(0, buf, qt); };
  fetch(0);
  if constexpr (NSTG == 2) fetch_r(1, 1);

  bf16x8 kf[NS], vf[NS];
  {
    const __amdgpu_buffer_rsrc_t rk = row_rsrc(K, a.Nk, a.ks[1]);
    const __amdgpu_buffer_rsrc_t rv = row_rsrc(V, a.Nk, a.vs[1]);
    const unsigned ko = (unsigned)((long long)key * a.ks[1] * 2);
    const unsigned vo = (unsigned)((long long)key * a.vs[1] * 2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int d0 = 16 * s + 8 * h;
      const bool ok = d0 < a.D;
      kf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rk, ok ? ko + d0 * 2 : 0x80000000u, 0, 0));
      vf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rv, ok ? vo + d0 * 2 : 0x80000000u, 0, 0));
    }
  }
  const float sl2 = a.scale * kLog2e;
  unsigned ra[NS], ca[2 * NT];
#pragma unroll
  for (int s = 0; s < NS; ++s) ra[s] = r32 * DP * 2 + 16 * ((2 * s + h) ^ swz<DP>(r32));
  {
    const int li = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int colb = 32 * t + 16 * (g & 1) + 4 * (li & 3);
      const int chunk = colb >> 3, half = (colb >> 2) & 1;
      const int r1 = 4 * h + (li >> 2), r2 = r1 + 8;
      ca[2 * t] = r1 * DP * 2 + 16 * (chunk ^ swz<DP>(r1)) + 8 * half;
      ca[2 * t + 1] = r2 * DP * 2 + 16 * (chunk ^ swz<DP>(r2)) + 8 * half;
    }
  }
  f32x16 adk[NT], adv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    adk[t] = zero16();
    adv[t] = zero16();
  }

  put(smem, 0);
  vm_wait_all();
  __syncthreads();

  // S / dP of query half u of the tile in `buf` (rows 32u + row_of(r, h)): returns the two
  // accumulators, -delta as dP's initial value; l4 = the half's lse2 constants
  auto sdp = [&](const char* buf, int u, f32x16& sp, f32x16& dp, f32x4* l4) {
    const char* ldsQ = buf;
    const char* ldsG = buf + TILE;
    const float* ldsL = reinterpret_cast<const float*>(buf + 2 * TILE);
    const float* ldsD = ldsL + 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(ldsD + 32 * u + 8 * g + 4 * h);
      l4[g] = *reinterpret_cast<const f32x4*>(ldsL + 32 * u + 8 * g + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) dp[4 * g + j] = d4[j];
    }
    sp = zero16();
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bf16x8 qr = *reinterpret_cast<const bf16x8*>(ldsQ + ra[s] + 32 * u * DP * 2);
      const bf16x8 gr = *reinterpret_cast<const bf16x8*>(ldsG + ra[s] + 32 * u * DP * 2);
      sp = MF<__bf16>::mma(qr, kf[s], sp);
      dp = MF<__bf16>::mma(gr, vf[s], dp);
    }
  };
  // P = 2^(S sl2 - lse2), dS = P o dP' (in place)
  auto softmax = [&](f32x16& sp, f32x16& dp, const f32x4* l4) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = ex2(__builtin_fmaf(sp[4 * g + j], sl2, -l4[g][j]));
        sp[4 * g + j] = p;
        dp[4 * g + j] *= p;
      }
  };
  // dV^T += dO_u^T P, dK^T += Q_u^T dS
  auto dkdv = [&](const char* buf, int u, const f32x16& sp, const f32x16& dp) {
    const char* ldsQ = buf;
    const char* ldsG = buf + TILE;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pf = acc_frag<__bf16>(sp, s2);
      const bf16x8 sf = acc_frag<__bf16>(dp, s2);
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        const int ro = (32 * u + 16 * s2) * DP * 2;
        const bf16x8 gv = tr2(ldsG + ca[2 * tt] + ro, ldsG + ca[2 * tt + 1] + ro);
        adv[tt] = MF<__bf16>::mma(gv, pf, adv[tt]);
        const bf16x8 qv = tr2(ldsQ + ca[2 * tt] + ro, ldsQ + ca[2 * tt + 1] + ro);
        adk[tt] = MF<__bf16>::mma(qv, sf, adk[tt]);
      }
    }
  };

  // one tile: fetch t + 1 (registers), the pipelined body on buffer BSEL, stage t + 1 into the
  // other buffer, barrier.  Loads / writes past the last tile read zeros into a dead buffer.
  auto step_sgb = [&](int qt, auto bsel_c) {
    constexpr int bsel = decltype(bsel_c)::value;
    const char* buf = smem + bsel * TB;
    char* nxt = smem + (bsel ^ 1) * TB;
    fetch(qt + 1);
    f32x16 sp0, dp0, sp1, dp1;
    f32x4 l40[4], l41[4];
    sdp(buf, 0, sp0, dp0, l40);
    sdp(buf, 1, sp1, dp1, l41);
    softmax(sp0, dp0, l40);
    dkdv(buf, 0, sp0, dp0);
    softmax(sp1, dp1, l41);
    dkdv(buf, 1, sp1, dp1);
    // the interleave (sched_group_barrier: groups filled in program order, dependencies permitting)
    SAE_SGB(kSgDsRead, 16, 0);   // half 0: Q / dO row fragments, lse2 / -delta
    SAE_SGB(kSgMfma, 8, 0);      // S0, dP0
    SAE_SGB(kSgDsRead, 16, 0);   // half 1 rows
#pragma unroll
    for (int i = 0; i < 8; ++i) {   // S1 / dP1 beside half 0's softmax
      SAE_SGB(kSgMfma, 1, 0);
      SAE_SGB(kSgValu, 8, 0);
    }
    SAE_SGB(kSgDsRead, 16, 0);   // half 0 transposed reads
#pragma unroll
    for (int i = 0; i < 8; ++i) {   // half 0's dV / dK beside half 1's softmax
      SAE_SGB(kSgMfma, 1, 0);
      SAE_SGB(kSgValu, 8, 0);
    }
    SAE_SGB(kSgDsRead, 16, 0);   // half 1 transposed reads
    SAE_SGB(kSgMfma, 8, 0);      // half 1's dV / dK
    put(nxt, qt + 1);
    __syncthreads();
  };

  // Hand-ordered body: slots fenced by sched_barrier(0), so the emitted order is this one.  Each
  // slot is one MFMA plus the LDS reads and VALU placed in its shadow.
#define SAE_FENCE() __builtin_amdgcn_sched_barrier(0)
  auto step_hand = [&](int qt, auto bsel_c) {
    // PROBE (dev timing probes, wrong results): 1 = half 1 reuses half 0's row fragments,
    // 2 = no lse / -delta reads, 3 = half 1 reuses half 0's transposed fragments, 4 = no global
    // Q / dO loads (tiles never restaged), 5 = no barrier, 6 = no softmax VALU, 7 = no LDS reads
    constexpr int PROBE = SCHED >= 10 ? SCHED - 10 : 0;
    constexpr int bsel = decltype(bsel_c)::value;
    const char* ldsQ = smem + bsel * TB;
    const char* ldsG = ldsQ + TILE;
    const float* ldsL = reinterpret_cast<const float*>(ldsQ + 2 * TILE);
    const float* ldsD = ldsL + 64;
    char* nxt = smem + (bsel ^ 1) * TB;
    if constexpr (PROBE != 4) {
      if constexpr (NSTG == 2) fetch_r(bsel, qt + 2);   // set bsel went to LDS at the end of tile qt - 1
      else fetch(qt + 1);
    }
    SAE_FENCE();
    bf16x8 q0[NS], g0[NS], q1[NS], g1[NS];
    f32x4 l0[4], l1[4];
    f32x16 sp0 = zero16(), dp0, sp1 = zero16(), dp1;
    auto rowrd = [&](int u, int s, bf16x8& qr, bf16x8& gr) {
      if constexpr (PROBE == 7) {
        qr = kf[(s + u) & 3];
        gr = vf[(s + 2 * u) & 3];
      } else {
        qr = *reinterpret_cast<const bf16x8*>(ldsQ + ra[s] + 32 * u * DP * 2);
        gr = *reinterpret_cast<const bf16x8*>(ldsG + ra[s] + 32 * u * DP * 2);
      }
    };
    auto drd = [&](int u, int g, f32x16& dp) {
      const f32x4 d4 = (PROBE == 2 || PROBE == 7) ? f32x4{-0.1f, 0.f, 0.1f, 0.f}
                                                  : *reinterpret_cast<const f32x4*>(ldsD + 32 * u + 8 * g + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) dp[4 * g + j] = d4[j];
    };
    auto lrd = [&](int u, int g, f32x4* l4) {
      l4[g] = (PROBE == 2 || PROBE == 7) ? f32x4{9.f, 9.f, 9.f, 9.f}
                                         : *reinterpret_cast<const f32x4*>(ldsL + 32 * u + 8 * g + 4 * h);
    };
    auto sm2 = [&](f32x16& sp, f32x16& dp, const f32x4* l4, int r) {   // two softmax elements r, r + 1
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        if constexpr (PROBE == 6) continue;
        const float p = ex2(__builtin_fmaf(sp[r + e], sl2, -l4[(r + e) >> 2][(r + e) & 3]));
        sp[r + e] = p;
        dp[r + e] *= p;
      }
    };
    // ---- reads of half 0 (rows, -delta, lse) ahead of segment 0
#pragma unroll
    for (int g = 0; g < 4; ++g) drd(0, g, dp0);
    rowrd(0, 0, q0[0], g0[0]);
    rowrd(0, 1, q0[1], g0[1]);
    SAE_FENCE();
    // ---- segment 0: S0 / dP0 (8 MFMAs); half-0 rows 2 ahead, then lse0, -delta1, half-1 rows
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      sp0 = MF<__bf16>::mma(q0[s], kf[s], sp0);
      if (s + 2 < NS) rowrd(0, s + 2, q0[s + 2], g0[s + 2]);
      else { lrd(0, 2 * (s - 2), l0); lrd(0, 2 * (s - 2) + 1, l0); }
      SAE_FENCE();
      dp0 = MF<__bf16>::mma(g0[s], vf[s], dp0);
      if (s < 2) { drd(1, 2 * s, dp1); drd(1, 2 * s + 1, dp1); }
      else if constexpr (PROBE == 1) { q1[s - 2] = q0[s - 2]; g1[s - 2] = g0[s - 2]; }
      else rowrd(1, s - 2, q1[s - 2], g1[s - 2]);
      SAE_FENCE();
    }
    // ---- segment 1: S1 / dP1 (8 MFMAs) beside half 0's softmax (2 elements per slot)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      sp1 = MF<__bf16>::mma(q1[s], kf[s], sp1);
      if (s + 2 < NS) {
        if constexpr (PROBE == 1) { q1[s + 2] = q0[s + 2]; g1[s + 2] = g0[s + 2]; }
        else rowrd(1, s + 2, q1[s + 2], g1[s + 2]);
      }
      sm2(sp0, dp0, l0, 4 * s);
      SAE_FENCE();
      dp1 = MF<__bf16>::mma(g1[s], vf[s], dp1);
      if (s >= 2) { lrd(1, 2 * (s - 2), l1); lrd(1, 2 * (s - 2) + 1, l1); }
      sm2(sp0, dp0, l0, 4 * s + 2);
      SAE_FENCE();
    }
    // ---- segment 2: half 0's dV / dK (8 MFMAs) beside half 1's softmax; half-0 bf16 packing
    //      and transposed reads just ahead of their MFMAs
    bf16x8 tv[2][NT], tq[2][NT];
    auto trd = [&](int u, int s2, int tt, bf16x8& gv, bf16x8& qv) {
      if constexpr (PROBE == 7) {
        gv = kf[(s2 + tt + u) & 3];
        qv = vf[(s2 + 2 * tt + u) & 3];
        return;
      }
      const int ro = (32 * u + 16 * s2) * DP * 2;
      gv = tr2(ldsG + ca[2 * tt] + ro, ldsG + ca[2 * tt + 1] + ro);
      qv = tr2(ldsQ + ca[2 * tt] + ro, ldsQ + ca[2 * tt + 1] + ro);
    };
    trd(0, 0, 0, tv[0][0], tq[0][0]);
    trd(0, 0, 1, tv[0][1], tq[0][1]);
    bf16x8 pf = acc_frag<__bf16>(sp0, 0), sf = acc_frag<__bf16>(dp0, 0);
    SAE_FENCE();
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        adv[tt] = MF<__bf16>::mma(tv[s2][tt], pf, adv[tt]);
        if (s2 == 0) trd(0, 1, tt, tv[1][tt], tq[1][tt]);
        sm2(sp1, dp1, l1, 8 * s2 + 4 * tt);
        SAE_FENCE();
        adk[tt] = MF<__bf16>::mma(tq[s2][tt], sf, adk[tt]);
        sm2(sp1, dp1, l1, 8 * s2 + 4 * tt + 2);
        SAE_FENCE();
      }
      if (s2 == 0) {
        pf = acc_frag<__bf16>(sp0, 1);
        sf = acc_frag<__bf16>(dp0, 1);
        SAE_FENCE();
      }
    }
    // ---- segment 3: half 1's dV / dK (8 MFMAs); the next tile's staging in their shadow
    if constexpr (PROBE != 3) {
      trd(1, 0, 0, tv[0][0], tq[0][0]);
      trd(1, 0, 1, tv[0][1], tq[0][1]);
    }
    pf = acc_frag<__bf16>(sp1, 0);
    sf = acc_frag<__bf16>(dp1, 0);
    SAE_FENCE();
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        adv[tt] = MF<__bf16>::mma(tv[s2][tt], pf, adv[tt]);
        if (s2 == 0 && PROBE != 3) trd(1, 1, tt, tv[1][tt], tq[1][tt]);
        SAE_FENCE();
        adk[tt] = MF<__bf16>::mma(tq[s2][tt], sf, adk[tt]);
        SAE_FENCE();
      }
      if (s2 == 0) {
        pf = acc_frag<__bf16>(sp1, 1);
        sf = acc_frag<__bf16>(dp1, 1);
        SAE_FENCE();
      }
    }
    if constexpr (PROBE != 4) {
      if constexpr (NSTG == 2) put_r(bsel ^ 1, nxt, qt + 1);
      else put(nxt, qt + 1);
    }
    if constexpr (PROBE != 5) __syncthreads();
  };
  auto step = [&](int qt, auto bsel_c) {
    if constexpr (SCHED == 1 || SCHED == 2 || SCHED >= 10) step_hand(qt, bsel_c);
    else step_sgb(qt, bsel_c);
  };
  if (active) {
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    int qt = 0;
    for (; qt + 1 < nqt; qt += 2) {
      step(qt, B0{});
      step(qt + 1, B1{});
    }
    if (qt < nqt) step(qt, B0{});
  } else {   // waves past the last key only stage tiles and meet the barriers
    for (int qt = 0; qt < nqt; ++qt) {
      if constexpr (NSTG == 2) {
        fetch_r(qt & 1, qt + 2);
        put_r((qt + 1) & 1, smem + ((qt + 1) & 1) * TB, qt + 1);
      } else {
        fetch(qt + 1);
        put(smem + ((qt + 1) & 1) * TB, qt + 1);
      }
      __syncthreads();
    }
  }
  if (active) {
    const int k0 = kb * BK + w * 32;
    char* scr = smem + w * 32 * DP * 2;
    __bf16* DK = reinterpret_cast<__bf16*>(a.dk) + b * a.dks[0] + hh * a.dks[2] + (long long)k0 * a.dks[1];
    __bf16* DV = reinterpret_cast<__bf16*>(a.dv) + b * a.dvs[0] + hh * a.dvs[2] + (long long)k0 * a.dvs[1];
    wave_store_rows<DP>(adk, a.scale, scr, DK, a.dks[1], a.Nk - k0, a.D, lane);
    wave_store_rows<DP>(adv, 1.f, scr, DV, a.dvs[1], a.Nk - k0, a.D, lane);
  }
  (void)key;
}

}  // namespace sae

namespace sae {

// ------------------------------------------------------------ dK / dV pass, ping-pong form
// 8 waves = 2 groups x 4; waves w and w + 4 hold the same 32 keys (key group w & 3) and split each
// 64-query tile: group u = w >> 2 takes query half u.  Each group alternates an MFMA phase
//   M(t): dV^T += dO^T P, dK^T += Q^T dS of tile t - 1 (its half) and S, dP of tile t   (16 MFMAs)
// with a VALU phase
//   V(t): P = 2^(S sl2 - lse2), dS = P o dP', both packed to bf16
// and group 1 runs one phase behind group 0, with one s_barrier per phase for all 8 waves: on every
// SIMD one wave is in its MFMA phase while its partner is in its VALU phase (MI355X_MICROARCH.md,
// two waves per SIMD; the role split by wave number >= 4, item 9).  Tiles sit in a 3-deep LDS ring:
// tile t is read by group 0 in phases 2t, 2t + 2 and by group 1 in 2t + 1, 2t + 3; tile t + 2 is
// written (from registers loaded two phases earlier) at the start of phase 2t + 2, after the last
// read of tile t - 1, its buffer.  The two groups' dK / dV partials are summed through LDS at the end
// (fixed order: deterministic).
// PRIO: waves 4-7 (the second-dispatched group, which loses VALU arbitration) at s_setprio 1
template <int PRIO = 0>
__global__ __launch_bounds__(512, 1) void attn_bwd6_dkdv_kernel(AttnArgs a) {
  constexpr int DP = 64, NW = 8;
  using FF = F2<DP>;
  constexpr int NS = FF::NS, NT = FF::NT, TILE = FF::TILE;
  constexpr int BK = 128;                      // keys per workgroup (4 key groups of 32)
  constexpr int TB = 2 * TILE + 2 * 64 * 4;    // [Q img | dO img | lse2[64] | -delta[64]]
  constexpr int NBUF = 3;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nkb = (a.Nk + BK - 1) / BK;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = bid % nkb;
  bid /= nkb;
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = w & 3, u = w >> 2;            // key group, query half
  const int key = kb * BK + kg * 32 + r32;
  const bool active = kb * BK + kg * 32 < a.Nk;   // wave-uniform
  const size_t rowoff = ((size_t)b * a.H + hh) * a.Nq;

  const __bf16* Q = reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const __bf16* K = reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const __bf16* V = reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2];
  const __bf16* G = reinterpret_cast<const __bf16*>(a.dout) + b * a.dos[0] + hh * a.dos[2];

  F2Stage<DP, NW> qst, gst;   // one 16-byte chunk of Q and of dO per thread and tile
  qst.init(tid, a.qs[1], a.D);
  gst.init(tid, a.dos[1], a.D);
  const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
  const __amdgpu_buffer_rsrc_t rg = row_rsrc(G, a.Nq, a.dos[1]);
  const unsigned qstep = (unsigned)(64 * a.qs[1] * 2), gstep = (unsigned)(64 * a.dos[1] * 2);
  const int nqt = (a.Nq + 63) / 64;
  float rc_l = 0.f, rc_d = 0.f;
  auto fetch = [&](int qt) {   // tiles past the end read zeros (range check), constants clamp
    qst.load(rq, (unsigned)qt * qstep);
    gst.load(rg, (unsigned)qt * gstep);
    if (tid < 64) {
      const int qq = min(qt * 64 + tid, a.Nq - 1);
      rc_l = a.lse[rowoff + qq];
      rc_d = a.delta[rowoff + qq];
    }
  };
  auto put = [&](int qt) {
    char* buf = smem + (qt % NBUF) * TB;
    qst.write(buf);
    gst.write(buf + TILE);
    if (tid < 64) {
      const bool ok = qt * 64 + tid < a.Nq;
      reinterpret_cast<float*>(buf + 2 * TILE)[tid] = ok ? rc_l * kLog2e : kInf;
      reinterpret_cast<float*>(buf + 2 * TILE + 256)[tid] = ok ? -rc_d : 0.f;
    }
  };

  bf16x8 kf[NS], vf[NS];
  {
    const __amdgpu_buffer_rsrc_t rk = row_rsrc(K, a.Nk, a.ks[1]);
    const __amdgpu_buffer_rsrc_t rv = row_rsrc(V, a.Nk, a.vs[1]);
    const unsigned ko = (unsigned)((long long)key * a.ks[1] * 2);
    const unsigned vo = (unsigned)((long long)key * a.vs[1] * 2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int d0 = 16 * s + 8 * h;
      const bool ok = d0 < a.D;
      kf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rk, ok ? ko + d0 * 2 : 0x80000000u, 0, 0));
      vf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rv, ok ? vo + d0 * 2 : 0x80000000u, 0, 0));
    }
  }
  const float sl2 = a.scale * kLog2e;
  // this wave's query half: row reads at rows 32u + r32, transposed reads at rows 32u + ...
  unsigned ra[NS], ca[2 * NT];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int rr = 32 * u + r32;
    ra[s] = rr * DP * 2 + 16 * ((2 * s + h) ^ swz<DP>(rr));
  }
  {
    const int li = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int colb = 32 * t + 16 * (g & 1) + 4 * (li & 3);
      const int chunk = colb >> 3, half = (colb >> 2) & 1;
      const int r1 = 32 * u + 4 * h + (li >> 2), r2 = r1 + 8;   // swz<64> depends on r & 15 only
      ca[2 * t] = r1 * DP * 2 + 16 * (chunk ^ swz<DP>(r1)) + 8 * half;
      ca[2 * t + 1] = r2 * DP * 2 + 16 * (chunk ^ swz<DP>(r2)) + 8 * half;
    }
  }
  f32x16 adk[NT], adv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    adk[t] = zero16();
    adv[t] = zero16();
  }

  // prologue: tiles 0 and 1 in the ring, tile 2 in registers
  fetch(0);
  vm_wait_all();
  put(0);
  fetch(1);
  vm_wait_all();
  put(1);
  fetch(2);
  __syncthreads();

  f32x16 sp, dp;            // S / dP of the current tile (MFMA phase -> VALU phase)
  bf16x8 pf[2], sf[2];      // bf16 P / dS of the previous tile (VALU phase -> next MFMA phase)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    pf[i] = bf16x8{};
    sf[i] = bf16x8{};
  }
  // MFMA phase of tile t (t == nqt: only the dV / dK of tile nqt - 1)
  auto mphase = [&](int t) {
    if (t > 0) {   // dV^T += dO^T P, dK^T += Q^T dS of tile t - 1
      const char* ldsQ = smem + ((t - 1) % NBUF) * TB;
      const char* ldsG = ldsQ + TILE;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
          const int ro = 16 * s2 * DP * 2;
          const bf16x8 gv = tr2(ldsG + ca[2 * tt] + ro, ldsG + ca[2 * tt + 1] + ro);
          adv[tt] = MF<__bf16>::mma(gv, pf[s2], adv[tt]);
          const bf16x8 qv = tr2(ldsQ + ca[2 * tt] + ro, ldsQ + ca[2 * tt + 1] + ro);
          adk[tt] = MF<__bf16>::mma(qv, sf[s2], adk[tt]);
        }
    }
    if (t < nqt) {   // S, dP of tile t (-delta as dP's initial accumulator)
      const char* ldsQ = smem + (t % NBUF) * TB;
      const char* ldsG = ldsQ + TILE;
      const float* ldsD = reinterpret_cast<const float*>(ldsQ + 2 * TILE) + 64;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(ldsD + 32 * u + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) dp[4 * g + j] = d4[j];
      }
      sp = zero16();
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8 qr = *reinterpret_cast<const bf16x8*>(ldsQ + ra[s]);
        const bf16x8 gr = *reinterpret_cast<const bf16x8*>(ldsG + ra[s]);
        sp = MF<__bf16>::mma(qr, kf[s], sp);
        dp = MF<__bf16>::mma(gr, vf[s], dp);
      }
    }
  };
  // VALU phase of tile t
  auto vphase = [&](int t) {
    const float* ldsL = reinterpret_cast<const float*>(smem + (t % NBUF) * TB + 2 * TILE);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 l4 = *reinterpret_cast<const f32x4*>(ldsL + 32 * u + 8 * g + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = ex2(__builtin_fmaf(sp[4 * g + j], sl2, -l4[j]));
        sp[4 * g + j] = p;
        dp[4 * g + j] *= p;
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      pf[s2] = acc_frag<__bf16>(sp, s2);
      sf[s2] = acc_frag<__bf16>(dp, s2);
    }
  };
  // phase p (0 .. 2 nqt): group 0 runs M(p / 2) on even p and V((p - 1) / 2) on odd p; group 1
  // the same sequence one phase later.  Staging: at the start of every even phase p = 2t + 2 the
  // registers holding tile t + 2 go to the ring and tile t + 3 is fetched.
  const int nph = 2 * nqt + 2;
  if (PRIO && u == 1) __builtin_amdgcn_s_setprio(1);
  for (int p = 0; p < nph; ++p) {
    if ((p & 1) == 0 && p >= 2) {
      const int t = p / 2 - 1;   // p = 2t + 2
      if (t + 2 <= nqt) {
        vm_wait_all();
        put(t + 2);
        fetch(t + 3);
      }
    }
    const int q = p - u;   // this group's own phase index
    if (active && q >= 0 && q <= 2 * nqt) {
      if ((q & 1) == 0) mphase(q / 2);
      else vphase(q / 2);
    }
    __syncthreads();
  }
  // dK / dV: group 1's partials through LDS (fp32 [key group][tile][16 regs][64 lanes]), group 0 adds
  float* red = reinterpret_cast<float*>(smem);
  if (u == 1 && active) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        red[((kg * 2 * NT + t) * 16 + r) * 64 + lane] = adk[t][r];
        red[((kg * 2 * NT + NT + t) * 16 + r) * 64 + lane] = adv[t][r];
      }
  }
  __syncthreads();
  if (u == 0 && active) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        adk[t][r] += red[((kg * 2 * NT + t) * 16 + r) * 64 + lane];
        adv[t][r] += red[((kg * 2 * NT + NT + t) * 16 + r) * 64 + lane];
      }
  }
  __syncthreads();   // partials read: the LDS becomes the store scratch
  if (u == 0 && active) {
    const int k0 = kb * BK + kg * 32;
    char* scr = smem + kg * 32 * DP * 2;
    __bf16* DK = reinterpret_cast<__bf16*>(a.dk) + b * a.dks[0] + hh * a.dks[2] + (long long)k0 * a.dks[1];
    __bf16* DV = reinterpret_cast<__bf16*>(a.dv) + b * a.dvs[0] + hh * a.dvs[2] + (long long)k0 * a.dvs[1];
    wave_store_rows<DP>(adk, a.scale, scr, DK, a.dks[1], a.Nk - k0, a.D, lane);
    wave_store_rows<DP>(adv, 1.f, scr, DV, a.dvs[1], a.Nk - k0, a.D, lane);
  }
}

}  // namespace sae

namespace sae {

// --------------------------------------------------------------------- dQ pass, ping-pong form
// 8 waves = 2 groups x 4; waves w and w + 4 hold the same 32 query rows (query group w & 3, query
// on the MFMA lane) and split each 64-key K / V tile: group u takes key half u.  Phases as in
// attn_bwd6_dkdv_kernel:
//   M(t): dQ^T += K^T dS^T of tile t - 1 (its 32 keys) and S^T = K Q^T, dP^T = V dO^T of tile t
//   V(t): P = 2^(S sl2 - lse2), dS = P o dP', packed to bf16
// group 1 one phase behind group 0, one barrier per phase, K / V tiles in a 3-deep LDS ring.
// delta = rowsum(dO o O) is formed from the fragments in registers and published for the dK / dV
// pass; -delta and -lse2 are per-lane constants (the query is on the lane): -delta is the dP^T
// MFMAs' initial accumulator.  The groups' dQ partials are summed through LDS at the end.
// PRIO: waves 4-7 (the second-dispatched group, which loses VALU arbitration) at s_setprio 1
template <int PRIO = 0>
__global__ __launch_bounds__(512, 1) void attn_bwd6_dq_kernel(AttnArgs a) {
  constexpr int DP = 64, NW = 8;
  using FF = F2<DP>;
  constexpr int NS = FF::NS, NT = FF::NT, TILE = FF::TILE;
  constexpr int BQ = 128;
  constexpr int TB = 2 * TILE;   // [K img | V img]
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
  const size_t rowoff = ((size_t)b * a.H + hh) * a.Nq;

  const __bf16* Q = reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const __bf16* K = reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const __bf16* V = reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2];
  const __bf16* O = reinterpret_cast<const __bf16*>(a.o) + b * a.os[0] + hh * a.os[2];
  const __bf16* G = reinterpret_cast<const __bf16*>(a.dout) + b * a.dos[0] + hh * a.dos[2];

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

  bf16x8 qf[NS], gf[NS];
  float dlt;
  {
    const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
    const __amdgpu_buffer_rsrc_t rg = row_rsrc(G, a.Nq, a.dos[1]);
    const __amdgpu_buffer_rsrc_t ro = row_rsrc(O, a.Nq, a.os[1]);
    const unsigned qo = (unsigned)((long long)q * a.qs[1] * 2);
    const unsigned go = (unsigned)((long long)q * a.dos[1] * 2);
    const unsigned oo = (unsigned)((long long)q * a.os[1] * 2);
    float part = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int d0 = 16 * s + 8 * h;
      const bool ok = d0 < a.D;
      qf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rq, ok ? qo + d0 * 2 : 0x80000000u, 0, 0));
      gf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rg, ok ? go + d0 * 2 : 0x80000000u, 0, 0));
      const bf16x8 of = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ro, ok ? oo + d0 * 2 : 0x80000000u, 0, 0));
#pragma unroll
      for (int j = 0; j < 8; ++j) part += (float)of[j] * (float)gf[s][j];
    }
    dlt = xhalf_sum(part);
  }
  const bool qok = q < a.Nq;
  if (qok && h == 0 && u == 0) a.delta[rowoff + q] = dlt;
  const float lsc2 = qok ? -a.lse[rowoff + q] * kLog2e : -kInf;
  const float sl2 = a.scale * kLog2e;
  f32x16 ndl;   // -delta of this lane's query: the dP^T MFMAs' initial accumulator
#pragma unroll
  for (int r = 0; r < 16; ++r) ndl[r] = -dlt;

  // K / V row reads at rows 32u + r32 of the tile; transposed K reads at rows 32u + ...
  unsigned ka[NS], ca[2 * NT];
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
      ca[2 * t] = r1 * DP * 2 + 16 * (chunk ^ swz<DP>(r1)) + 8 * half;
      ca[2 * t + 1] = r2 * DP * 2 + 16 * (chunk ^ swz<DP>(r2)) + 8 * half;
    }
  }
  f32x16 adq[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) adq[t] = zero16();

  fetch(0);
  vm_wait_all();
  put(0);
  fetch(1);
  vm_wait_all();
  put(1);
  fetch(2);
  __syncthreads();

  f32x16 sp, dp;
  bf16x8 sf[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) sf[i] = bf16x8{};
  auto mphase = [&](int t) {
    if (t > 0) {   // dQ^T += K^T dS^T of tile t - 1 (this group's 32 keys)
      const char* ldsK = smem + ((t - 1) % NBUF) * TB;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
          const int ro = 16 * s2 * DP * 2;
          const bf16x8 kv = tr2(ldsK + ca[2 * tt] + ro, ldsK + ca[2 * tt + 1] + ro);
          adq[tt] = MF<__bf16>::mma(kv, sf[s2], adq[tt]);
        }
    }
    if (t < nkt) {   // S^T = K Q^T, dP^T = V dO^T (-delta initial) of tile t
      const char* ldsK = smem + (t % NBUF) * TB;
      const char* ldsV = ldsK + TILE;
      sp = zero16();
      dp = ndl;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const bf16x8 kr = *reinterpret_cast<const bf16x8*>(ldsK + ka[s]);
        const bf16x8 vr = *reinterpret_cast<const bf16x8*>(ldsV + ka[s]);
        sp = MF<__bf16>::mma(kr, qf[s], sp);
        dp = MF<__bf16>::mma(vr, gf[s], dp);
      }
    }
  };
  auto vphase = [&](int t) {
    // keys past Nk (zero K / V rows, score 0) must not contribute: P forced to 0
    const int nvh = a.Nk - 64 * t - 32 * u - 4 * h;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = ((r & 3) + 8 * (r >> 2)) < nvh ? ex2(__builtin_fmaf(sp[r], sl2, lsc2)) : 0.f;
      dp[r] *= p;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) sf[s2] = acc_frag<__bf16>(dp, s2);
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
  float* red = reinterpret_cast<float*>(smem);
  if (u == 1 && active) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((qg * NT + t) * 16 + r) * 64 + lane] = adq[t][r];
  }
  __syncthreads();
  if (u == 0 && active) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) adq[t][r] += red[((qg * NT + t) * 16 + r) * 64 + lane];
  }
  __syncthreads();
  if (u == 0 && active) {
    const int q0 = qb * BQ + qg * 32;
    __bf16* DQ = reinterpret_cast<__bf16*>(a.dq) + b * a.dqs[0] + hh * a.dqs[2] + (long long)q0 * a.dqs[1];
    wave_store_rows<DP>(adq, a.scale, smem + qg * 32 * DP * 2, DQ, a.dqs[1], a.Nq - q0, a.D, lane);
  }
}

}  // namespace sae

namespace sae {

// one 1-KiB LDS-DMA piece (16 bytes per lane at LDS byte address lds + 16 lane; M0 saved and
// restored inside the statement, as gemm8.h g8_dma1) and the 256-byte dword form
__device__ __forceinline__ void b7_dma16(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds) : "memory");
}
__device__ __forceinline__ void b7_dma4(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
               "buffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(rs), "s"(lds) : "memory");
}
template <int N> __device__ __forceinline__ void b7_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// --------------------------------------------- dK / dV pass, LDS-DMA staged, hand-ordered body
// As attn_bwd5_dkdv_kernel (SCHED 1: both query halves of a 64-query tile in one hand-ordered
// block), with the Q / dO tiles and their row constants staged by LDS-DMA into a 3-deep ring:
// tile t + 2 is issued at the top of tile t (its buffer held tile t - 1, whose readers all passed
// the barrier that ended tile t - 1), and the counted vmcnt + barrier at the end of tile t makes
// tile t + 1 visible -- two tiles of load latency hidden, no staging registers, no ds_write.  The
// row constants come ready from the dQ pass (attn_bwd2_dq_kernel PUB2: -delta, lse log2 e); query
// rows past Nq read as zeros (range check), which leaves their dS and their dV / dK terms zero.
// The DMA writes lane-linearly: the XOR swizzle of the tile images goes into the source address.
template <int MINW>
__global__ __launch_bounds__(256, MINW) void attn_bwd7_dkdv_kernel(AttnArgs a) {
  constexpr int DP = 64, NW = 4;
  using FF = F2<DP>;
  constexpr int NS = FF::NS, NT = FF::NT, TILE = FF::TILE;
  constexpr int BK = 32 * NW;
  constexpr int TB = 2 * TILE + 2 * 64 * 4;   // [Q img | dO img | lse2[64] | -delta[64]]
  constexpr int NBUF = 3;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nkb = (a.Nk + BK - 1) / BK;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int kb = bid % nkb;
  bid /= nkb;
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int key = kb * BK + w * 32 + r32;
  const bool active = kb * BK + w * 32 < a.Nk;
  const size_t rowoff = ((size_t)b * a.H + hh) * a.Nq;

  const __bf16* Q = reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const __bf16* K = reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const __bf16* V = reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2];
  const __bf16* G = reinterpret_cast<const __bf16*>(a.dout) + b * a.dos[0] + hh * a.dos[2];
  const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
  const __amdgpu_buffer_rsrc_t rg = row_rsrc(G, a.Nq, a.dos[1]);
  const __amdgpu_buffer_rsrc_t rdl = row_rsrc(a.delta + rowoff, a.Nq, 1);   // -delta
  const __amdgpu_buffer_rsrc_t rl2 = row_rsrc(a.delta + (size_t)a.B * a.H * a.Nq + rowoff, a.Nq, 1);   // lse log2 e
  const int nqt = (a.Nq + 63) / 64;
  const unsigned lbase = __builtin_amdgcn_readfirstlane(
      (unsigned)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem));
  // this wave's pieces: Q / dO rows 8p .. 8p + 7 for p = w, w + 4; lane L: row 8p + L / 8, image
  // chunk L % 8 = global chunk (L % 8) ^ swz(row) (chunks past the head dim read zero)
  unsigned goq[2], gog[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 8 * (w + 4 * i) + (lane >> 3);
    const int c = (lane & 7) ^ swz<DP>(row);
    const bool ok = c * 8 < a.D;
    goq[i] = ok ? (unsigned)(((long long)row * a.qs[1] + 8 * c) * 2) : 0x80000000u;
    gog[i] = ok ? (unsigned)(((long long)row * a.dos[1] + 8 * c) * 2) : 0x80000000u;
  }
  const unsigned qstep = (unsigned)(64 * a.qs[1] * 2), gstep = (unsigned)(64 * a.dos[1] * 2);
  // pieces per tile: 4 per wave, + the lse2 piece (wave 0) / the -delta piece (wave 1)
  auto issue = [&](int t) {
    const unsigned lb = lbase + (unsigned)((t % NBUF) * TB);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const unsigned p = (unsigned)(w + 4 * i) * 1024u;
      b7_dma16(rq, goq[i] + (unsigned)t * qstep, lb + p);
      b7_dma16(rg, gog[i] + (unsigned)t * gstep, lb + TILE + p);
    }
    if (w == 0) b7_dma4(rl2, (unsigned)(t * 64 + lane) * 4u, lb + 2 * TILE);
    if (w == 1) b7_dma4(rdl, (unsigned)(t * 64 + lane) * 4u, lb + 2 * TILE + 256);
  };
  // wait for tile t (all older pieces; the pieces of tile t + 1 may stay in flight) + barrier
  auto wait_tile = [&](bool next_in_flight) {
    if (next_in_flight) {
      if (w < 2) b7_wait_barrier<5>(); else b7_wait_barrier<4>();
    } else {
      b7_wait_barrier<0>();
    }
  };

  bf16x8 kf[NS], vf[NS];
  {
    const __amdgpu_buffer_rsrc_t rk = row_rsrc(K, a.Nk, a.ks[1]);
    const __amdgpu_buffer_rsrc_t rv = row_rsrc(V, a.Nk, a.vs[1]);
    const unsigned ko = (unsigned)((long long)key * a.ks[1] * 2);
    const unsigned vo = (unsigned)((long long)key * a.vs[1] * 2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int d0 = 16 * s + 8 * h;
      const bool ok = d0 < a.D;
      kf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rk, ok ? ko + d0 * 2 : 0x80000000u, 0, 0));
      vf[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rv, ok ? vo + d0 * 2 : 0x80000000u, 0, 0));
    }
  }
  vm_wait_all();   // K / V fragments resident (the waitcnt pass cannot see the asm DMA)
  issue(0);
  if (nqt > 1) issue(1);
  wait_tile(nqt > 1);

  const float sl2 = a.scale * kLog2e;
  unsigned ra[NS], ca[2 * NT];
#pragma unroll
  for (int s = 0; s < NS; ++s) ra[s] = r32 * DP * 2 + 16 * ((2 * s + h) ^ swz<DP>(r32));
  {
    const int li = lane & 15, g = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int colb = 32 * t + 16 * (g & 1) + 4 * (li & 3);
      const int chunk = colb >> 3, half = (colb >> 2) & 1;
      const int r1 = 4 * h + (li >> 2), r2 = r1 + 8;
      ca[2 * t] = r1 * DP * 2 + 16 * (chunk ^ swz<DP>(r1)) + 8 * half;
      ca[2 * t + 1] = r2 * DP * 2 + 16 * (chunk ^ swz<DP>(r2)) + 8 * half;
    }
  }
  f32x16 adk[NT], adv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    adk[t] = zero16();
    adv[t] = zero16();
  }

#define SAE_FENCE7() __builtin_amdgcn_sched_barrier(0)
  for (int qt = 0; qt < nqt; ++qt) {
    if (qt + 2 < nqt) issue(qt + 2);
    SAE_FENCE7();
    if (active) {
      const char* ldsQ = smem + (qt % NBUF) * TB;
      const char* ldsG = ldsQ + TILE;
      const float* ldsL = reinterpret_cast<const float*>(ldsQ + 2 * TILE);
      const float* ldsD = ldsL + 64;
      bf16x8 q0[NS], g0[NS], q1[NS], g1[NS];
      f32x4 l0[4], l1[4];
      f32x16 sp0 = zero16(), dp0, sp1 = zero16(), dp1;
      auto rowrd = [&](int u, int s, bf16x8& qr, bf16x8& gr) {
        qr = *reinterpret_cast<const bf16x8*>(ldsQ + ra[s] + 32 * u * DP * 2);
        gr = *reinterpret_cast<const bf16x8*>(ldsG + ra[s] + 32 * u * DP * 2);
      };
      auto drd = [&](int u, int g, f32x16& dp) {
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(ldsD + 32 * u + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) dp[4 * g + j] = d4[j];
      };
      auto lrd = [&](int u, int g, f32x4* l4) { l4[g] = *reinterpret_cast<const f32x4*>(ldsL + 32 * u + 8 * g + 4 * h); };
      auto sm2 = [&](f32x16& sp, f32x16& dp, const f32x4* l4, int r) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float p = ex2(__builtin_fmaf(sp[r + e], sl2, -l4[(r + e) >> 2][(r + e) & 3]));
          sp[r + e] = p;
          dp[r + e] *= p;
        }
      };
#pragma unroll
      for (int g = 0; g < 4; ++g) drd(0, g, dp0);
      rowrd(0, 0, q0[0], g0[0]);
      rowrd(0, 1, q0[1], g0[1]);
      SAE_FENCE7();
#pragma unroll
      for (int s = 0; s < NS; ++s) {   // segment 0: S0 / dP0
        sp0 = MF<__bf16>::mma(q0[s], kf[s], sp0);
        if (s + 2 < NS) rowrd(0, s + 2, q0[s + 2], g0[s + 2]);
        else { lrd(0, 2 * (s - 2), l0); lrd(0, 2 * (s - 2) + 1, l0); }
        SAE_FENCE7();
        dp0 = MF<__bf16>::mma(g0[s], vf[s], dp0);
        if (s < 2) { drd(1, 2 * s, dp1); drd(1, 2 * s + 1, dp1); }
        else rowrd(1, s - 2, q1[s - 2], g1[s - 2]);
        SAE_FENCE7();
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {   // segment 1: S1 / dP1 beside half 0's softmax
        sp1 = MF<__bf16>::mma(q1[s], kf[s], sp1);
        if (s + 2 < NS) rowrd(1, s + 2, q1[s + 2], g1[s + 2]);
        sm2(sp0, dp0, l0, 4 * s);
        SAE_FENCE7();
        dp1 = MF<__bf16>::mma(g1[s], vf[s], dp1);
        if (s >= 2) { lrd(1, 2 * (s - 2), l1); lrd(1, 2 * (s - 2) + 1, l1); }
        sm2(sp0, dp0, l0, 4 * s + 2);
        SAE_FENCE7();
      }
      bf16x8 tv[2][NT], tq[2][NT];
      auto trd = [&](int u, int s2, int tt, bf16x8& gv, bf16x8& qv) {
        const int ro = (32 * u + 16 * s2) * DP * 2;
        gv = tr2(ldsG + ca[2 * tt] + ro, ldsG + ca[2 * tt + 1] + ro);
        qv = tr2(ldsQ + ca[2 * tt] + ro, ldsQ + ca[2 * tt + 1] + ro);
      };
      trd(0, 0, 0, tv[0][0], tq[0][0]);
      trd(0, 0, 1, tv[0][1], tq[0][1]);
      bf16x8 pf = acc_frag<__bf16>(sp0, 0), sf = acc_frag<__bf16>(dp0, 0);
      SAE_FENCE7();
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {   // segment 2: half 0's dV / dK beside half 1's softmax
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
          adv[tt] = MF<__bf16>::mma(tv[s2][tt], pf, adv[tt]);
          if (s2 == 0) trd(0, 1, tt, tv[1][tt], tq[1][tt]);
          sm2(sp1, dp1, l1, 8 * s2 + 4 * tt);
          SAE_FENCE7();
          adk[tt] = MF<__bf16>::mma(tq[s2][tt], sf, adk[tt]);
          sm2(sp1, dp1, l1, 8 * s2 + 4 * tt + 2);
          SAE_FENCE7();
        }
        if (s2 == 0) {
          pf = acc_frag<__bf16>(sp0, 1);
          sf = acc_frag<__bf16>(dp0, 1);
          SAE_FENCE7();
        }
      }
      trd(1, 0, 0, tv[0][0], tq[0][0]);
      trd(1, 0, 1, tv[0][1], tq[0][1]);
      pf = acc_frag<__bf16>(sp1, 0);
      sf = acc_frag<__bf16>(dp1, 0);
      SAE_FENCE7();
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {   // segment 3: half 1's dV / dK
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
          adv[tt] = MF<__bf16>::mma(tv[s2][tt], pf, adv[tt]);
          if (s2 == 0) trd(1, 1, tt, tv[1][tt], tq[1][tt]);
          SAE_FENCE7();
          adk[tt] = MF<__bf16>::mma(tq[s2][tt], sf, adk[tt]);
          SAE_FENCE7();
        }
        if (s2 == 0) {
          pf = acc_frag<__bf16>(sp1, 1);
          sf = acc_frag<__bf16>(dp1, 1);
          SAE_FENCE7();
        }
      }
    }
    // tile qt + 1 landed (the pieces of qt + 2 may stay in flight) and every wave done with qt
    if (qt + 1 < nqt) wait_tile(qt + 2 < nqt);
    else b7_wait_barrier<0>();
  }
  if (active) {
    const int k0 = kb * BK + w * 32;
    char* scr = smem + w * 32 * DP * 2;
    __bf16* DK = reinterpret_cast<__bf16*>(a.dk) + b * a.dks[0] + hh * a.dks[2] + (long long)k0 * a.dks[1];
    __bf16* DV = reinterpret_cast<__bf16*>(a.dv) + b * a.dvs[0] + hh * a.dvs[2] + (long long)k0 * a.dvs[1];
    wave_store_rows<DP>(adk, a.scale, scr, DK, a.dks[1], a.Nk - k0, a.D, lane);
    wave_store_rows<DP>(adv, 1.f, scr, DV, a.dvs[1], a.Nk - k0, a.D, lane);
  }
}

}  // namespace sae
