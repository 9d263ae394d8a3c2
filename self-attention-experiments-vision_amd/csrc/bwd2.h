// bwd2.h -- lean bf16 attention backward for gfx950 (dQ pass, then dK/dV pass).
//
// Same two deterministic passes as attn_bwd_dq_kernel / attn_bwd_dkdv_kernel (attn_kernels.h;
// the JAX autodiff of models/layers/attentions/attention.py:39-58), rebuilt the way fwd2.h is:
//   * every per-tile address precomputed once (buffer-descriptor offsets, VGPR + immediate LDS
//     addresses, tile loop unrolled over the two LDS buffers);
//   * score accumulators start at zero (a free immediate C operand) and the row constants enter
//     through the exponent's FMA: p = 2^(s * scale * log2e - lse * log2e), dS = p (dP - delta);
//   * the dK/dV pass prefetches the per-query row constants with the Q / dO tile (issue early,
//     write late): no dependent global load inside the loop;
//   * results leave through a per-wave LDS scratch as whole 16-byte row chunks (wave_store_rows).
#pragma once
#include "fwd2.h"

namespace sae {

// ------------------------------------------------------------------------------- dQ pass
// One wave = 32 query rows (query on the MFMA lane), NW waves share each 64-key K/V tile.
// delta = rowsum(dO o O) is computed from the fragments in registers and published for the
// dK/dV pass.  Per 32-key half: S^T = K Q^T, dP^T = V dO^T (row reads of the K / V images),
// dS^T = P^T o (dP^T - delta), dQ^T += K^T dS^T (transposed reads of the K image).
// ROT (both passes): q / k rotated as they are staged, dq / dk rotated back as they are stored.
// REL (both passes): the BoTNet relative logits enter the recomputed scores as two extra k-steps
// (fwd2.h rel_onehot8 / rel_qrow8); the dQ pass also forms dbias^T = onehot^T dS^T on the matrix
// pipe -- one more 32 x 32 accumulator, complete per query row because the pass sweeps every key
// -- and stores dbias_h / dbias_w (deterministic, no atomics).
template <int DP, int NW, int MINW, bool ROT = false, bool REL = false>
__global__ __launch_bounds__(64 * NW, MINW) void attn_bwd2_dq_kernel(AttnArgs a) {
  using FF = F2<DP>;
  constexpr int NS = FF::NS, NT = FF::NT, TILE = FF::TILE;
  constexpr int BQ = 32 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nqb = (a.Nq + BQ - 1) / BQ;
  SAE_STAMPO(4096, 0);
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = bid % nqb;
  bid /= nqb;
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r32 = lane & 31;
  const int q = qb * BQ + w * 32 + r32;
  const bool active = qb * BQ + __builtin_amdgcn_readfirstlane(w) * 32 < a.Nq;
  const size_t rowoff = ((size_t)b * a.H + hh) * a.Nq;

  const __bf16* Q = reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const __bf16* K = reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const __bf16* V = reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2];
  const __bf16* O = reinterpret_cast<const __bf16*>(a.o) + b * a.os[0] + hh * a.os[2];
  const __bf16* G = reinterpret_cast<const __bf16*>(a.dout) + b * a.dos[0] + hh * a.dos[2];

  F2Stage<DP, NW> kst, vst;   // K/V tile t + 1 loaded while tile t computes
  kst.init(tid, a.ks[1], a.D);
  vst.init(tid, a.vs[1], a.D);
  const __amdgpu_buffer_rsrc_t rk = row_rsrc(K, a.Nk, a.ks[1]);
  const __amdgpu_buffer_rsrc_t rv = row_rsrc(V, a.Nk, a.vs[1]);
  const unsigned kstep = (unsigned)(64 * a.ks[1] * 2), vstep = (unsigned)(64 * a.vs[1] * 2);
  const int nkt = (a.Nk + 63) / 64;
  kst.load(rk, 0);
  vst.load(rv, 0);

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
    if constexpr (ROT) {
#pragma unroll
      for (int s = 0; s < NS; ++s) qf[s] = rope8<1>(qf[s], a.rope, q, 16 * s + 8 * h);
    }
  }
  const bool qok = q < a.Nq;
  if (qok && h == 0) a.delta[rowoff + q] = dlt;
  const float lsc2 = qok ? -a.lse[rowoff + q] * kLog2e : -kInf;
  const float sl2 = a.scale * kLog2e;

  unsigned ka[NS], ca[2 * NT];
#pragma unroll
  for (int s = 0; s < NS; ++s) ka[s] = r32 * DP * 2 + 16 * ((2 * s + h) ^ swz<DP>(r32));
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

  // -delta as the initial dP^T accumulator, made by one MFMA: ones (k = 0, 1) times the
  // bf16 hi / lo split of -delta (k = 0, 1 of this lane's query column); dS = P o dP' then
  // needs one multiply per element instead of a subtract and a multiply
  bf16x8 dl_b, dl_a;
  {
    const __bf16 hi = (__bf16)(-dlt);
    const __bf16 lo = (__bf16)(-dlt - (float)hi);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dl_b[j] = (__bf16)0.f;
      dl_a[j] = (__bf16)0.f;
    }
    if (h == 0) {
      dl_b[0] = hi;
      dl_b[1] = lo;
      dl_a[0] = dl_a[1] = (__bf16)1.f;
    }
  }
  f32x16 adq[NT];   // written first by the peeled first tile (zero C operand)
  // REL: query-bias fragments, one-hot row reads (scores) and transposed reads (dbias^T)
  char* const rimg = smem + 4 * TILE;
  bf16x8 qa[2];
  unsigned rra[2], rca[2];
  f32x16 adb = zero16();
  if constexpr (REL) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      qa[s] = __builtin_bit_cast(bf16x8, rel_qrow8(a, rowoff + q, qok, 2 * s + h, 1.f / a.scale));
      rra[s] = r32 * 64 + 16 * ((2 * s + h) ^ swz<32>(r32));
    }
    const int li = lane & 15, g = lane >> 4;
    const int colb = 16 * (g & 1) + 4 * (li & 3);
    const int chunk = colb >> 3, half = (colb >> 2) & 1;
    const int r1 = 4 * h + (li >> 2), r2 = r1 + 8;
    rca[0] = r1 * 64 + 16 * (chunk ^ swz<32>(r1)) + 8 * half;
    rca[1] = r2 * 64 + 16 * (chunk ^ swz<32>(r2)) + 8 * half;
  }

  if constexpr (ROT) kst.rope(a.rope, 0, tid);
  kst.write(smem);
  vst.write(smem + TILE);
  if constexpr (REL) rel_put_onehot<NW>(a, rimg, 0, tid);
  vm_wait_all();   // Q / dO fragments resident before the loop (see vm_wait_all)
  __syncthreads();
  SAE_STAMPO(4096, 1);
  // one K/V tile: load t + 1, compute t from LDS buffer BSEL, stage t + 1, barrier (as fwd2.h)
  auto step = [&](int t, auto bsel_c, auto first_c, auto compute_c) {
    constexpr int bsel = decltype(bsel_c)::value;
    constexpr bool FIRST = decltype(first_c)::value;
    const char* ldsK = smem + bsel * 2 * TILE;
    const char* ldsV = ldsK + TILE;
    const char* ldsR = rimg + bsel * kRelImg;
    char* nxt = smem + (bsel ^ 1) * 2 * TILE;
    if (t + 1 < nkt) {
      kst.load(rk, (unsigned)(t + 1) * kstep);
      vst.load(rv, (unsigned)(t + 1) * vstep);
    }
    const int nvalid = min(64, a.Nk - 64 * t);
    if constexpr (decltype(compute_c)::value) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && nvalid <= 32) break;
        f32x16 sp = zero16();
        f32x16 dp = MF<__bf16>::mma(dl_a, dl_b, zero16());
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bf16x8 kr = *reinterpret_cast<const bf16x8*>(ldsK + ka[s] + 32 * u * DP * 2);
          const bf16x8 vr = *reinterpret_cast<const bf16x8*>(ldsV + ka[s] + 32 * u * DP * 2);
          sp = MF<__bf16>::mma(kr, qf[s], sp);
          dp = MF<__bf16>::mma(vr, gf[s], dp);
        }
        if constexpr (REL) {
#pragma unroll
          for (int s = 0; s < 2; ++s)
            sp = MF<__bf16>::mma(*reinterpret_cast<const bf16x8*>(ldsR + rra[s] + 32 * u * 64), qa[s], sp);
        }
        if (nvalid < 64) {   // tail: keys past the end contribute nothing
          const int nvh = nvalid - 32 * u - 4 * h;
#pragma unroll
          for (int r = 0; r < 16; ++r) sp[r] = ((r & 3) + 8 * (r >> 2)) < nvh ? sp[r] : -kInf;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) dp[r] *= ex2(__builtin_fmaf(sp[r], sl2, lsc2));
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 sf = acc_frag<__bf16>(dp, s2);
#pragma unroll
          for (int tt = 0; tt < NT; ++tt) {
            const int ro = (32 * u + 16 * s2) * DP * 2;
            s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ldsK + ca[2 * tt] + ro));
            s16x4 x2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ldsK + ca[2 * tt + 1] + ro));
            typedef __attribute__((ext_vector_type(8))) short s16x8;
            s16x8 vv = {x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
            adq[tt] = MF<__bf16>::mma(__builtin_bit_cast(bf16x8, vv), sf,
                                      (FIRST && u == 0 && s2 == 0) ? zero16() : adq[tt]);
          }
          if constexpr (REL) {   // dbias^T += onehot^T dS^T (the one-hot image read transposed)
            const int ro = (32 * u + 16 * s2) * 64;
            s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ldsR + rca[0] + ro));
            s16x4 x2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ldsR + rca[1] + ro));
            typedef __attribute__((ext_vector_type(8))) short s16x8;
            s16x8 ov = {x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
            adb = MF<__bf16>::mma(__builtin_bit_cast(bf16x8, ov), sf, adb);
          }
        }
      }
    }
    if (t + 1 < nkt) {
      if constexpr (ROT) kst.rope(a.rope, 64 * (t + 1), tid);
      kst.write(nxt);
      vst.write(nxt + TILE);
      if constexpr (REL) rel_put_onehot<NW>(a, rimg + (bsel ^ 1) * kRelImg, 64 * (t + 1), tid);
    }
    __syncthreads();
    SAE_STAMPO(4096, 2 + (t < 27 ? t : 27));
  };
  auto sweep = [&](auto compute_c) {
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    step(0, B0{}, std::true_type{}, compute_c);
    for (int t = 1; t < nkt; t += 2) {
      step(t, B1{}, std::false_type{}, compute_c);
      if (t + 1 < nkt) step(t + 1, B0{}, std::false_type{}, compute_c);
    }
  };
  if (active) sweep(std::true_type{});   // waves past the last query row only stage and sync
  else sweep(std::false_type{});
  if constexpr (REL) {   // dbias^T: accumulator row = table column row_of(r, h), lane = query
    if (active && qok) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int col = row_of(r, h);
        if (col < a.rel_h) a.dbias_h[(rowoff + q) * a.rel_h + col] = adb[r];
        else if (col < a.rel_h + a.rel_w) a.dbias_w[(rowoff + q) * a.rel_w + col - a.rel_h] = adb[r];
      }
    }
  }
  SAE_STAMPO(4096, 30);
  if (active) {
    const int q0 = qb * BQ + w * 32;
    __bf16* DQ = reinterpret_cast<__bf16*>(a.dq) + b * a.dqs[0] + hh * a.dqs[2] + (long long)q0 * a.dqs[1];
    wave_store_rows<DP, ROT ? -1 : 0>(adq, a.scale, smem + w * 32 * DP * 2, DQ, a.dqs[1], a.Nq - q0, a.D, lane,
                                      &a.rope, q0);
  }
  SAE_STAMPO(4096, 31);
}

// --------------------------------------------------------------------------- dK / dV pass
// One wave = 32 keys (key on the MFMA lane) with K, V fragments in registers; NW waves share
// each 64-query Q / dO tile and its row constants (lse * log2 e, delta).  Per 32-query half:
// S = Q K^T, dP = dO V^T (row reads), P = 2^(S sl2 - lse2), dS = P o (dP - delta),
// dV^T += dO^T P and dK^T += Q^T dS (transposed reads of the dO / Q images).
// REL: the staged tile also carries the query-bias rows of its 64 queries ([64][32] bf16 image),
// the wave's keys hold their one-hot rows in registers.
// PIPE: full 64-query tiles issue both halves' S / dP chains back to back so that the scheduler
// can run one half's exponentials under the other half's MFMAs (needs the registers of a
// one-wave-per-SIMD build: MINW = 1, accumulators in AGPRs -- the bwd_agpr.hip instances).
template <int DP, int NW, int MINW, bool ROT = false, bool REL = false, bool PIPE = false>
__global__ __launch_bounds__(64 * NW, MINW) void attn_bwd2_dkdv_kernel(AttnArgs a) {
  using FF = F2<DP>;
  constexpr int NS = FF::NS, NT = FF::NT, TILE = FF::TILE;
  constexpr int BK = 32 * NW;
  // [Q img | dO img | lse2[64] | delta[64] (| query-bias img)]
  constexpr int TB = 2 * TILE + 2 * 64 * 4 + (REL ? kRelImg : 0);
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nkb = (a.Nk + BK - 1) / BK;
  SAE_STAMP(0);
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

  // Q / dO tiles and their row constants: two register stages in flight (as in fwd2.h)
  F2Stage<DP, NW> qst[2], gst[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    qst[r].init(tid, a.qs[1], a.D);
    gst[r].init(tid, a.dos[1], a.D);
  }
  const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
  const __amdgpu_buffer_rsrc_t rg = row_rsrc(G, a.Nq, a.dos[1]);
  const unsigned qstep = (unsigned)(64 * a.qs[1] * 2), gstep = (unsigned)(64 * a.dos[1] * 2);
  const int nqt = (a.Nq + 63) / 64;
  float rc_l[2] = {0.f, 0.f}, rc_d[2] = {0.f, 0.f};   // row constants of a staged tile (threads 0..63)
  uint4 rq8[2];   // REL: this thread's query-bias chunk of a staged tile (threads 0..255)
  auto fetch = [&](int r, int qt) {
    qst[r].load(rq, (unsigned)qt * qstep);
    gst[r].load(rg, (unsigned)qt * gstep);
    // raw values only: scaling or selecting them here would make the compiler wait for these
    // loads (and, vmcnt counting in order, for the Q / dO loads above) right after issue, which
    // drained the two-tile register prefetch every step; put() scales and masks them
    if (tid < 64) {
      const int qq = min(qt * 64 + tid, a.Nq - 1);
      rc_l[r] = a.lse[rowoff + qq];
      rc_d[r] = a.delta[rowoff + qq];
    }
    if constexpr (REL) {
      static_assert(NW == 4, "REL staging: one query-bias chunk per thread");
      const int qq = qt * 64 + (tid >> 2);
      rq8[r] = rel_qrow8(a, rowoff + qq, qq < a.Nq, tid & 3, 1.f / a.scale);
    }
  };
  fetch(0, 0);
  if (nqt > 1) fetch(1, 1);

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
    if constexpr (ROT) {
#pragma unroll
      for (int s = 0; s < NS; ++s) kf[s] = rope8<1>(kf[s], a.rope, key, 16 * s + 8 * h);
    }
  }
  // REL: the one-hot row of this lane's key (B operand) and the query-bias image row reads
  bf16x8 kfa[2];
  unsigned rra[2];
  if constexpr (REL) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      kfa[s] = __builtin_bit_cast(bf16x8, rel_onehot8(a, key, 2 * s + h));
      rra[s] = r32 * 64 + 16 * ((2 * s + h) ^ swz<32>(r32));
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

  f32x16 adk[NT], adv[NT];   // written first by the peeled first tile (zero C operand)
  // -delta as the initial dP accumulator (one MFMA, as in the dQ pass): A = bf16 hi / lo split
  // of -delta of this lane's query row at k = 0, 1, B = ones at k = 0, 1
  bf16x8 one01;
#pragma unroll
  for (int j = 0; j < 8; ++j) one01[j] = (__bf16)((h == 0 && j < 2) ? 1.f : 0.f);
  auto put = [&](int r, char* buf, int qt) {
    if constexpr (ROT) qst[r].rope(a.rope, 64 * qt, tid);
    qst[r].write(buf);
    gst[r].write(buf + TILE);
    if (tid < 64) {
      const bool ok = qt * 64 + tid < a.Nq;
      reinterpret_cast<float*>(buf + 2 * TILE)[tid] = ok ? rc_l[r] * kLog2e : kInf;
      reinterpret_cast<float*>(buf + 2 * TILE + 256)[tid] = ok ? rc_d[r] : 0.f;
    }
    if constexpr (REL) {
      const int rr = tid >> 2, c = tid & 3;
      *reinterpret_cast<uint4*>(buf + 2 * TILE + 512 + rr * 64 + 16 * (c ^ swz<32>(rr))) = rq8[r];
    }
  };
  put(0, smem, 0);
  vm_wait_all();   // K / V fragments resident before the loop (see vm_wait_all)
  __syncthreads();
  SAE_STAMP(1);
  auto step = [&](int qt, auto bsel_c, auto first_c, auto compute_c) {
    constexpr int bsel = decltype(bsel_c)::value;
    constexpr bool FIRST = decltype(first_c)::value;
    const char* ldsQ = smem + bsel * TB;
    const char* ldsG = ldsQ + TILE;
    const float* ldsL = reinterpret_cast<const float*>(ldsQ + 2 * TILE);
    const float* ldsD = ldsL + 64;
    char* nxt = smem + (bsel ^ 1) * TB;
    if (qt + 2 < nqt) fetch(bsel, qt + 2);   // register set bsel went to LDS at the end of tile qt - 1
    bool piped = false;
    if constexpr (PIPE && !REL && decltype(compute_c)::value) {
      if (qt * 64 + 32 < a.Nq) {   // both halves hold query rows
        piped = true;
        f32x16 sp[2], dp[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          bf16x8 dla;
          const float nd = -ldsD[32 * u + r32];
          const __bf16 hi = (__bf16)nd;
          const __bf16 lo = (__bf16)(nd - (float)hi);
#pragma unroll
          for (int j = 0; j < 8; ++j) dla[j] = (__bf16)0.f;
          if (h == 0) {
            dla[0] = hi;
            dla[1] = lo;
          }
          sp[u] = zero16();
          dp[u] = MF<__bf16>::mma(dla, one01, zero16());
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            const bf16x8 qr = *reinterpret_cast<const bf16x8*>(ldsQ + ra[s] + 32 * u * DP * 2);
            const bf16x8 gr = *reinterpret_cast<const bf16x8*>(ldsG + ra[s] + 32 * u * DP * 2);
            sp[u] = MF<__bf16>::mma(qr, kf[s], sp[u]);
            dp[u] = MF<__bf16>::mma(gr, vf[s], dp[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 l4 = *reinterpret_cast<const f32x4*>(ldsL + 32 * u + 8 * g + 4 * h);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float p = ex2(__builtin_fmaf(sp[u][4 * g + j], sl2, -l4[j]));
              sp[u][4 * g + j] = p;
              dp[u][4 * g + j] *= p;
            }
          }
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            const bf16x8 pf = acc_frag<__bf16>(sp[u], s2);
            const bf16x8 sf = acc_frag<__bf16>(dp[u], s2);
            const bool z = FIRST && u == 0 && s2 == 0;
#pragma unroll
            for (int tt = 0; tt < NT; ++tt) {
              const int ro = (32 * u + 16 * s2) * DP * 2;
              const bf16x8 gv = tr2(ldsG + ca[2 * tt] + ro, ldsG + ca[2 * tt + 1] + ro);
              adv[tt] = MF<__bf16>::mma(gv, pf, z ? zero16() : adv[tt]);
              const bf16x8 qv = tr2(ldsQ + ca[2 * tt] + ro, ldsQ + ca[2 * tt + 1] + ro);
              adk[tt] = MF<__bf16>::mma(qv, sf, z ? zero16() : adk[tt]);
            }
          }
        }
      }
    }
    if (!piped && decltype(compute_c)::value) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && qt * 64 + 32 >= a.Nq) break;
        bf16x8 dla;
        {
          const float nd = -ldsD[32 * u + r32];
          const __bf16 hi = (__bf16)nd;
          const __bf16 lo = (__bf16)(nd - (float)hi);
#pragma unroll
          for (int j = 0; j < 8; ++j) dla[j] = (__bf16)0.f;
          if (h == 0) {
            dla[0] = hi;
            dla[1] = lo;
          }
        }
        f32x16 sp = zero16();
        f32x16 dp = MF<__bf16>::mma(dla, one01, zero16());
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bf16x8 qr = *reinterpret_cast<const bf16x8*>(ldsQ + ra[s] + 32 * u * DP * 2);
          const bf16x8 gr = *reinterpret_cast<const bf16x8*>(ldsG + ra[s] + 32 * u * DP * 2);
          sp = MF<__bf16>::mma(qr, kf[s], sp);
          dp = MF<__bf16>::mma(gr, vf[s], dp);
        }
        if constexpr (REL) {
          const char* ldsR = ldsQ + 2 * TILE + 512;
#pragma unroll
          for (int s = 0; s < 2; ++s)
            sp = MF<__bf16>::mma(*reinterpret_cast<const bf16x8*>(ldsR + rra[s] + 32 * u * 64), kfa[s], sp);
        }
        // rows q = 32u + row_of(r, h): constants for r = 4g + j at 32u + 8g + 4h + j
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
          const bf16x8 pf = acc_frag<__bf16>(sp, s2);
          const bf16x8 sf = acc_frag<__bf16>(dp, s2);
          const bool z = FIRST && u == 0 && s2 == 0;
#pragma unroll
          for (int tt = 0; tt < NT; ++tt) {
            const int ro = (32 * u + 16 * s2) * DP * 2;
            typedef __attribute__((ext_vector_type(8))) short s16x8;
            s16x4 g1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ldsG + ca[2 * tt] + ro));
            s16x4 g2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ldsG + ca[2 * tt + 1] + ro));
            s16x8 gv = {g1[0], g1[1], g1[2], g1[3], g2[0], g2[1], g2[2], g2[3]};
            adv[tt] = MF<__bf16>::mma(__builtin_bit_cast(bf16x8, gv), pf, z ? zero16() : adv[tt]);
            s16x4 q1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ldsQ + ca[2 * tt] + ro));
            s16x4 q2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(ldsQ + ca[2 * tt + 1] + ro));
            s16x8 qv = {q1[0], q1[1], q1[2], q1[3], q2[0], q2[1], q2[2], q2[3]};
            adk[tt] = MF<__bf16>::mma(__builtin_bit_cast(bf16x8, qv), sf, z ? zero16() : adk[tt]);
          }
        }
      }
    }
    if (qt + 1 < nqt) put(bsel ^ 1, nxt, qt + 1);
    __syncthreads();
    SAE_STAMP(2 + (qt < 27 ? qt : 27));
  };
  auto sweep = [&](auto compute_c) {
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    step(0, B0{}, std::true_type{}, compute_c);
    for (int qt = 1; qt < nqt; qt += 2) {
      step(qt, B1{}, std::false_type{}, compute_c);
      if (qt + 1 < nqt) step(qt + 1, B0{}, std::false_type{}, compute_c);
    }
  };
  if (active) sweep(std::true_type{});   // waves past the last key only stage and sync
  else sweep(std::false_type{});
  SAE_STAMP(30);
  if (active) {
    const int k0 = kb * BK + w * 32;
    char* scr = smem + w * 32 * DP * 2;
    __bf16* DK = reinterpret_cast<__bf16*>(a.dk) + b * a.dks[0] + hh * a.dks[2] + (long long)k0 * a.dks[1];
    __bf16* DV = reinterpret_cast<__bf16*>(a.dv) + b * a.dvs[0] + hh * a.dvs[2] + (long long)k0 * a.dvs[1];
    wave_store_rows<DP, ROT ? -1 : 0>(adk, a.scale, scr, DK, a.dks[1], a.Nk - k0, a.D, lane, &a.rope, k0);
    wave_store_rows<DP>(adv, 1.f, scr, DV, a.dvs[1], a.Nk - k0, a.D, lane);
  }
  (void)key;
  SAE_STAMP(31);
}

}  // namespace sae
