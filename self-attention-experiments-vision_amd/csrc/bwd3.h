// bwd3.h -- single-pass bf16 attention backward for gfx950 (dQ, dK, dV from ONE sweep).
//
// The JAX autodiff of models/layers/attentions/attention.py:39-58 (A18 of SURVEY §8a):
//   dV = P^T dO,  dP = dO V^T,  dS = P o (dP - delta),  dK = scale dS^T Q,  dQ = scale dS K,
// with P recomputed from Q, K and the forward's log-sum-exp.  bwd2.h runs it as two passes
// (dQ, then dK/dV), each recomputing S, exp(S) and dP: 7 MFMA products and two exp passes per
// (query, key) tile.  Here one workgroup owns a block of 32 * NW keys of one (batch, head):
//   * wave w keeps K, V fragments of its 32 keys and the dK^T / dV^T accumulators in registers
//     (key on the MFMA lane) and sweeps every 32-row query tile once: S = Q K^T, dP = dO V^T
//     (-delta as the initial accumulator), P = 2^(S scale log2 e - lse log2 e), dS = P o dP',
//     dV^T += dO^T P, dK^T += Q^T dS -- exp is computed once per score;
//   * dS crosses LDS once, as a [keys][32 q] bf16 image, and dQ^T = K^T dS^T for the tile is
//     split over the waves as 16 x 16 output tiles (v_mfma_f32_16x16x32_bf16), each summing over
//     all keys of the block, the K^T operand fragments held in registers for the whole sweep;
//   * delta = rowsum(dO o O) is formed while the dO / O tile is staged (no separate pass).
// Five products per tile instead of seven, and dQ needs no sum across workgroups: the kernel takes
// key ranges of up to 32 * NW * KPW = 256 keys (every N <= 256 config: DeiT / ViT at 224 px, CaiT,
// BoTNet, CeiT, TNT), one workgroup per (batch, head).  Longer key ranges stay on bwd2.h: split
// over several workgroups, the fp32 dQ partials plus their ordered sum cost more than the two-pass
// recompute (ViT-B/16@384: 441 vs 335 us, profiles/r02_bwd3_ab.txt).  Software pipeline: tile t's
// dQ runs in iteration t + 1 from the other dS image, so each query tile costs ONE barrier.
// Deterministic: no atomics.
#pragma once
#include "fwd2.h"

namespace sae {

template <int DP, int NW, int KPW> struct B3 {
  static constexpr int CPR = DP / 8;            // 16-byte chunks per row
  static constexpr int NS = DP / 16;            // bf16 k-steps over the head dim
  static constexpr int NT = DP / 32;            // 32-row tiles of dK^T / dV^T
  static constexpr int BK = 32 * NW * KPW;      // keys per workgroup
  static constexpr int KS = BK / 32;            // 32-key steps of the dQ^T product
  static constexpr int QIMG = 32 * DP * 2;      // one 32-row Q (or dO) image
  static constexpr int TB = 2 * QIMG + 2 * 32 * 4;   // [Q | dO | lse2[32] | -delta[32]]
  static constexpr int DSIMG = BK * 64;         // dS^T image: [BK keys][32 q] bf16, 64-B rows
  static constexpr int KIMG = BK * DP * 2;      // K image (prologue only; aliases the dS images)
  static constexpr int NDB = DP / 16;           // 16-wide head-dim blocks of dQ^T
  static constexpr int NDQ = NDB * 2;           // 16 x 16 dQ^T tiles per query tile
  static constexpr int TPW = NDQ > NW ? NDQ / NW : 1;   // dQ^T tiles per wave (same head-dim block)
  static constexpr int LDS = 2 * TB + (2 * DSIMG > KIMG ? 2 * DSIMG : KIMG);
  static_assert(32 * CPR <= 64 * NW, "one staged chunk per thread");
  static_assert(NDQ % NW == 0 || NW % NDQ == 0, "dQ tiles split evenly");
  static_assert(NDQ <= NW || NW % NDB == 0, "a wave's dQ tiles share one head-dim block");
  static_assert(KIMG <= 2 * DSIMG, "K image fits the dS images");
};

// dS^T image addressing: 8-byte slot s (4 query columns) of key row r, XOR-swizzled so that the
// ds_write_b64 of 16 consecutive key rows and the ds_read_b64_tr_b16 of 4-row blocks are both
// bank-conflict free.
__device__ __forceinline__ int ds_off(int r, int s) { return r * 64 + 8 * (s ^ ((r >> 1) & 7)); }


template <int CTRL> __device__ __forceinline__ float dpp_mov(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}

// One 32-row query tile of Q, dO and O staged global -> registers -> LDS, plus its row
// constants: lse * log2 e and -delta, delta = rowsum(dO o O) formed from the staged chunks.
template <int DP, int NW> struct B3Stage {
  using C = B3<DP, NW, 1>;
  unsigned oq, og, oo;   // byte offsets of this thread's chunk in query tile 0
  unsigned loff;         // LDS byte offset in an image
  int row, col;
  bool has;
  uint4 q, g, o;
  float lse2;            // raw lse of row qt_ * 32 + tid (tid < 32), scaled by log2 e in write()
  int qt_;               // query tile held in the registers (rotary position base)
  int nq_;

  __device__ __forceinline__ void init(int tid, const AttnArgs& a) {
    row = tid / C::CPR;
    col = tid % C::CPR;
    has = tid < 32 * C::CPR;
    const bool ok = has && col * 8 < a.D;
    oq = ok ? (unsigned)(((long long)row * a.qs[1] + col * 8) * 2) : 0x80000000u;
    og = ok ? (unsigned)(((long long)row * a.dos[1] + col * 8) * 2) : 0x80000000u;
    oo = ok ? (unsigned)(((long long)row * a.os[1] + col * 8) * 2) : 0x80000000u;
    loff = (unsigned)(row * DP * 2 + 16 * (col ^ swz<DP>(row)));
  }
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rq, __amdgpu_buffer_rsrc_t rg,
                                       __amdgpu_buffer_rsrc_t ro, const AttnArgs& a, int qt, size_t rowoff,
                                       int tid) {
    qt_ = qt;
    nq_ = a.Nq;
    q = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                      rq, oq + (unsigned)(qt * 32 * a.qs[1] * 2), 0, 0));
    g = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                      rg, og + (unsigned)(qt * 32 * a.dos[1] * 2), 0, 0));
    o = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                      ro, oo + (unsigned)(qt * 32 * a.os[1] * 2), 0, 0));
    // the raw lse only: scaling or selecting it here would make the compiler wait for this load --
    // and with it for the q / dO / O loads above (vmcnt counts in order) -- right after issue,
    // turning the register prefetch into a synchronous load at the top of every tile
    if (tid < 32) lse2 = a.lse[rowoff + min(qt * 32 + tid, a.Nq - 1)];
  }
  template <bool ROT = false>
  __device__ __forceinline__ void write(char* buf, int tid, const RopeTab* rope = nullptr) const {
    const bf16x8 gv = __builtin_bit_cast(bf16x8, g), ov = __builtin_bit_cast(bf16x8, o);
    float part = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) part += (float)gv[j] * (float)ov[j];
    // the CPR chunks of one row sit on consecutive lanes: DPP sums (quad xor 1, xor 2, half-row mirror)
    part += dpp_mov<0xB1>(part);
    part += dpp_mov<0x4E>(part);
    if constexpr (C::CPR == 8) part += dpp_mov<0x141>(part);
    if (has) {
      if constexpr (ROT)
        *reinterpret_cast<uint4*>(buf + loff) = rope8<1>(q, *rope, qt_ * 32 + row, 8 * col);
      else
        *reinterpret_cast<uint4*>(buf + loff) = q;
      *reinterpret_cast<uint4*>(buf + C::QIMG + loff) = g;
      if (col == 0) reinterpret_cast<float*>(buf + 2 * C::QIMG + 128)[row] = -part;
    }
    if (tid < 32) reinterpret_cast<float*>(buf + 2 * C::QIMG)[tid] = qt_ * 32 + tid < nq_ ? lse2 * kLog2e : kInf;
  }
};

// NW waves x KPW sub-blocks of 32 keys per workgroup.  KPW = 2 (four waves, one per SIMD, the
// whole register file each): the two sub-blocks of a wave share every Q / dO operand read and give
// the scheduler two independent MFMA / exp chains; KPW = 1 (eight waves, two per SIMD).
// ROT: q / k rotated as they are staged (the K fragments also feed the K image, so dQ uses the
// rotated K as it must), dq / dk rotated back as they are stored.
// NSU: the 16-wide k-steps of S / dP that carry head-dim columns (3 for D = 48 at DP = 64)
// STAG (8 waves, two per SIMD): waves 4-7 -- each the SIMD partner of one of waves 0-3 -- run the
// previous tile's dQ product at the START of a step instead of at its end, so the two waves of a
// SIMD are in different phases of the step (one's exponentials beside the other's MFMAs) instead of
// in lockstep (MI355X_MICROARCH.md, two waves per SIMD, item 9); PRIO: waves 4-7 at s_setprio 1
template <int DP, int NW, int KPW, bool ROT = false, int NSU = DP / 16, bool STAG = false, bool PRIO = false>
__global__ __launch_bounds__(64 * NW, (NW * KPW == 8 && KPW == 1) ? 2 : 1) void attn_bwd3_kernel(AttnArgs a) {
  using C = B3<DP, NW, KPW>;
  constexpr int NS = NSU, NT = C::NT, TB = C::TB, KS = C::KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const dsb = smem + 2 * TB;   // two dS^T images (the K image during the prologue)

  SAE_STAMP(0);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int hh = bid % a.H;
  const int b = bid / a.H;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int key0 = 0;                     // the whole key range is this workgroup's (Nk <= BK)
  const int wrow = w * 32 * KPW;              // first key (image row) of this wave
  const bool active = key0 + wrow < a.Nk;     // wave-uniform: this wave holds at least one key
  const size_t rowoff = ((size_t)b * a.H + hh) * a.Nq;

  const __bf16* Q = reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2];
  const __bf16* K = reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2];
  const __bf16* V = reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2];
  const __bf16* O = reinterpret_cast<const __bf16*>(a.o) + b * a.os[0] + hh * a.os[2];
  const __bf16* G = reinterpret_cast<const __bf16*>(a.dout) + b * a.dos[0] + hh * a.dos[2];
  const __amdgpu_buffer_rsrc_t rq = row_rsrc(Q, a.Nq, a.qs[1]);
  const __amdgpu_buffer_rsrc_t rg = row_rsrc(G, a.Nq, a.dos[1]);
  const __amdgpu_buffer_rsrc_t ro = row_rsrc(O, a.Nq, a.os[1]);
  const int nqt = (a.Nq + 31) / 32;

  B3Stage<DP, NW> st;
  st.init(tid, a);
  st.load(rq, rg, ro, a, 0, rowoff, tid);

  // K / V fragments of the wave's sub-blocks: key on the lane, head dim 16s + 8h .. + 7 (zero past
  // Nk / D); the K image [BK keys][DP] (the dQ^T = K^T dS^T operand) is written from them
  bf16x8 kf[KPW][NS], vf[KPW][NS];
  {
    const __amdgpu_buffer_rsrc_t rk = row_rsrc(K, a.Nk, a.ks[1]);
    const __amdgpu_buffer_rsrc_t rv = row_rsrc(V, a.Nk, a.vs[1]);
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
      const int key = key0 + wrow + 32 * j + r32;
      const unsigned ko = (unsigned)((long long)key * a.ks[1] * 2);
      const unsigned vo = (unsigned)((long long)key * a.vs[1] * 2);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int d0 = 16 * s + 8 * h;
        const bool ok = d0 < a.D;
        kf[j][s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rk, ok ? ko + d0 * 2 : 0x80000000u, 0, 0));
        vf[j][s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rv, ok ? vo + d0 * 2 : 0x80000000u, 0, 0));
      }
      if constexpr (ROT) {
#pragma unroll
        for (int s = 0; s < NS; ++s) kf[j][s] = rope8<1>(kf[j][s], a.rope, key, 16 * s + 8 * h);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < KPW; ++j)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int rr = wrow + 32 * j + r32;
      *reinterpret_cast<bf16x8*>(dsb + rr * DP * 2 + 16 * ((2 * s + h) ^ swz<DP>(rr))) = kf[j][s];
    }
  st.template write<ROT>(smem, tid, &a.rope);
  vm_wait_all();
  __syncthreads();
  SAE_STAMP(1);

  // dQ^T tiles of this wave: head-dim block db (16 wide) x query halves qh (16 rows) of each tile
  const int db = w % C::NDB;
  const bool dqw = w < C::NDQ;
  const int li = lane & 15, gq = lane >> 4;
  bf16x8 aq[KS];   // K^T fragments: rows d = 16 db + li, k = 32 ks + 8 gq + j
  if (dqw) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int r1 = 32 * ks + 8 * gq + (li >> 2), r2 = r1 + 4;
      const int col = 16 * db + 4 * (li & 3);
      const int ch = col >> 3, hf = (col >> 2) & 1;
      aq[ks] = tr2(dsb + r1 * DP * 2 + 16 * (ch ^ swz<DP>(r1)) + 8 * hf,
                   dsb + r2 * DP * 2 + 16 * (ch ^ swz<DP>(r2)) + 8 * hf);
    }
  }
  // per-lane read addresses of the dS^T image (B operand of the dQ^T product), per dQ tile
  unsigned da[C::TPW][2];
  int qhs[C::TPW];
#pragma unroll
  for (int t = 0; t < C::TPW; ++t) {
    const int tile = w + t * NW;
    qhs[t] = tile / C::NDB;
    const int r1 = 8 * gq + (li >> 2);
    da[t][0] = (unsigned)ds_off(r1, 4 * qhs[t] + (li & 3));
    da[t][1] = (unsigned)ds_off(r1 + 4, 4 * qhs[t] + (li & 3));
  }
  // Q / dO image row reads (S, dP) and transposed reads (dK, dV)
  unsigned ra[NS], ca[2 * NT];
#pragma unroll
  for (int s = 0; s < NS; ++s) ra[s] = r32 * DP * 2 + 16 * ((2 * s + h) ^ swz<DP>(r32));
  {
    const int g = lane >> 4;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int colb = 32 * t + 16 * (g & 1) + 4 * (li & 3);
      const int chunk = colb >> 3, half = (colb >> 2) & 1;
      const int r1 = 4 * h + (li >> 2), r2 = r1 + 8;
      ca[2 * t] = r1 * DP * 2 + 16 * (chunk ^ swz<DP>(r1)) + 8 * half;
      ca[2 * t + 1] = r2 * DP * 2 + 16 * (chunk ^ swz<DP>(r2)) + 8 * half;
    }
  }
  // dS^T write addresses: key row wrow + 32 j + r32, slots 2g + h (query rows 8g + 4h .. + 3)
  unsigned wa[KPW][4];
#pragma unroll
  for (int j = 0; j < KPW; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) wa[j][g] = (unsigned)ds_off(wrow + 32 * j + r32, 2 * g + h);

  f32x16 adk[KPW][NT], adv[KPW][NT];
#pragma unroll
  for (int j = 0; j < KPW; ++j)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      adk[j][t] = zero16();
      adv[j][t] = zero16();
    }
  bf16x8 one01;
#pragma unroll
  for (int j = 0; j < 8; ++j) one01[j] = (__bf16)((h == 0 && j < 2) ? 1.f : 0.f);
  const float sl2 = a.scale * kLog2e;
  __syncthreads();   // every wave holds its K^T fragments: the K image becomes the dS images
  SAE_STAMP(2);
  if (!active) {     // a wave past the last key writes zero dS once (its K rows are zero)
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    const bf16x4 z = {};
#pragma unroll
    for (int j = 0; j < KPW; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        *reinterpret_cast<bf16x4*>(dsb + wa[j][g]) = z;
        *reinterpret_cast<bf16x4*>(dsb + C::DSIMG + wa[j][g]) = z;
      }
  }

  // dQ^T for the query tile whose dS^T sits in image `img`
  auto dq_tile = [&](const char* img, int qt) {
    if (!dqw) return;
#pragma unroll
    for (int t = 0; t < C::TPW; ++t) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 bq = tr2(img + da[t][0] + ks * 32 * 64, img + da[t][1] + ks * 32 * 64);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[ks], bq, acc, 0, 0, 0);
      }
      // acc[j] = dQ^T[d = 16 db + 4 gq + j][q = qt * 32 + 16 qh + li]
      const int qq = qt * 32 + 16 * qhs[t] + li;
      const int d0 = 16 * db + 4 * gq;
      if (qq < a.Nq && d0 < a.D) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 v = {(__bf16)(acc[0] * a.scale), (__bf16)(acc[1] * a.scale), (__bf16)(acc[2] * a.scale),
                    (__bf16)(acc[3] * a.scale)};
        if constexpr (ROT) {   // back by -theta from the bf16 values (as the standalone pass would)
          float x[4] = {(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
          rope_pairs<2, -1>(x, a.rope, qq, d0 / 2);
          v = bf16x4{(__bf16)x[0], (__bf16)x[1], (__bf16)x[2], (__bf16)x[3]};
        }
        __bf16* DQ = reinterpret_cast<__bf16*>(a.dq) + b * a.dqs[0] + hh * a.dqs[2] + (long long)qq * a.dqs[1];
        *reinterpret_cast<bf16x4*>(DQ + d0) = v;
      }
    }
  };

  // one query tile: stage qt + 1, compute qt from buffer BSEL (dS^T into image BSEL), dQ of
  // qt - 1 from the other image, write the staged tile, barrier
  auto step = [&](int qt, auto bsel_c) {
    constexpr int bsel = decltype(bsel_c)::value;
    const char* ldsQ = smem + bsel * TB;
    const char* ldsG = ldsQ + C::QIMG;
    const float* ldsL = reinterpret_cast<const float*>(ldsQ + 2 * C::QIMG);
    const float* ldsD = ldsL + 32;
    char* img = dsb + bsel * C::DSIMG;
    if (qt + 1 < nqt) st.load(rq, rg, ro, a, qt + 1, rowoff, tid);
    const bool late = STAG && w >= NW / 2;   // this wave runs the previous tile's dQ first
    if (late && qt > 0) dq_tile(dsb + (bsel ^ 1) * C::DSIMG, qt - 1);
    if (active) {
      bf16x8 qr[NS], gr[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        qr[s] = *reinterpret_cast<const bf16x8*>(ldsQ + ra[s]);
        gr[s] = *reinterpret_cast<const bf16x8*>(ldsG + ra[s]);
      }
      f32x4 l4[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) l4[g] = *reinterpret_cast<const f32x4*>(ldsL + 8 * g + 4 * h);
      bf16x8 dla;
      {
        const float nd = ldsD[r32];
        const __bf16 hi = (__bf16)nd;
        const __bf16 lo = (__bf16)(nd - (float)hi);
#pragma unroll
        for (int j = 0; j < 8; ++j) dla[j] = (__bf16)0.f;
        if (h == 0) {
          dla[0] = hi;
          dla[1] = lo;
        }
      }
      f32x16 sp[KPW], dp[KPW];
#pragma unroll
      for (int j = 0; j < KPW; ++j) {
        sp[j] = zero16();
        dp[j] = MF<__bf16>::mma(dla, one01, zero16());
      }
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < KPW; ++j) {
          sp[j] = MF<__bf16>::mma(qr[s], kf[j][s], sp[j]);
          dp[j] = MF<__bf16>::mma(gr[s], vf[j][s], dp[j]);
        }
      // rows q = row_of(r, h): constants for r = 4g + i at 8g + 4h + i.  P <= 1 always (lse bounds
      // every score of the row); the clamp keeps keys past Nk (zero K rows) finite.
#pragma unroll
      for (int j = 0; j < KPW; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __builtin_amdgcn_fmed3f(ex2(__builtin_fmaf(sp[j][4 * g + i], sl2, -l4[g][i])), 0.f, 1.f);
            sp[j][4 * g + i] = p;
            dp[j][4 * g + i] *= p;
          }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int ro_ = 16 * s2 * DP * 2;
        bf16x8 gt[NT], qt_[NT];
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
          gt[tt] = tr2(ldsG + ca[2 * tt] + ro_, ldsG + ca[2 * tt + 1] + ro_);
          qt_[tt] = tr2(ldsQ + ca[2 * tt] + ro_, ldsQ + ca[2 * tt + 1] + ro_);
        }
#pragma unroll
        for (int j = 0; j < KPW; ++j) {
          const bf16x8 pf = acc_frag<__bf16>(sp[j], s2);
          const bf16x8 sf = acc_frag<__bf16>(dp[j], s2);
          // dS^T (bf16) for the dQ product: registers 8 s2 .. + 7 = query rows 16 s2 + 4h + {0..3, 8..11}
          // (whole dwords of the packed fragment: element-wise bf16 extraction made the compiler
          // convert every dS value a second time and re-pack the pairs with v_perm)
          const uint4 su = __builtin_bit_cast(uint4, sf);
          *reinterpret_cast<uint2*>(img + wa[j][2 * s2]) = make_uint2(su.x, su.y);
          *reinterpret_cast<uint2*>(img + wa[j][2 * s2 + 1]) = make_uint2(su.z, su.w);
#pragma unroll
          for (int tt = 0; tt < NT; ++tt) {
            adv[j][tt] = MF<__bf16>::mma(gt[tt], pf, adv[j][tt]);
            adk[j][tt] = MF<__bf16>::mma(qt_[tt], sf, adk[j][tt]);
          }
        }
      }
    }
    if (!late && qt > 0) dq_tile(dsb + (bsel ^ 1) * C::DSIMG, qt - 1);
    if (qt + 1 < nqt) st.template write<ROT>(smem + (bsel ^ 1) * TB, tid, &a.rope);
    __syncthreads();
    SAE_STAMP(3 + (qt < 26 ? qt : 26));
  };
  if (PRIO && w >= NW / 2) __builtin_amdgcn_s_setprio(1);
  {
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    for (int qt = 0; qt < nqt; qt += 2) {
      step(qt, B0{});
      if (qt + 1 < nqt) step(qt + 1, B1{});
    }
  }
  if (PRIO && w >= NW / 2) __builtin_amdgcn_s_setprio(0);
  dq_tile(dsb + ((nqt - 1) & 1) * C::DSIMG, nqt - 1);
  __syncthreads();   // every image read: the LDS becomes the per-wave store scratch
  SAE_STAMP(30);
  if (active) {
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
      const int k0 = key0 + wrow + 32 * j;
      if (k0 >= a.Nk) break;
      char* scr = smem + w * 32 * DP * 2;
      __bf16* DK = reinterpret_cast<__bf16*>(a.dk) + b * a.dks[0] + hh * a.dks[2] + (long long)k0 * a.dks[1];
      __bf16* DV = reinterpret_cast<__bf16*>(a.dv) + b * a.dvs[0] + hh * a.dvs[2] + (long long)k0 * a.dvs[1];
      wave_store_rows<DP, ROT ? -1 : 0>(adk[j], a.scale, scr, DK, a.dks[1], a.Nk - k0, a.D, lane, &a.rope, k0);
      wave_store_rows<DP>(adv[j], 1.f, scr, DV, a.dvs[1], a.Nk - k0, a.D, lane);
    }
  }
  SAE_STAMP(31);
}

}  // namespace sae
