// gemm8.h -- the projection / FF GEMMs on 256-row tiles of one 8-wave workgroup per CU.
//
//   c[m][n] = epi( sum_k a[m][k] * bt[n][k] (+ bias[n]) )          (NtArgs, gemm_nt.h epilogues)
//
// Why a second GEMM structure: sae_gemm_nt's 128 x 128 tiles read 64 FLOP per
// L2 byte, so at two workgroups per CU the operand stream from L2 takes as long as the MFMAs
// (profiles/r02_pmc_gemm_nt.txt: MFMA busy 0.23).  Here a workgroup owns a 256 x BN tile (BN = 128,
// 192 or 256: 85 / 110 / 128 FLOP per L2 byte) and its 8 waves (2 per SIMD) share one LDS ring:
//   * operands staged by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction, no VGPR
//     round trip), NS stage buffers of BK-deep A [256][BK] and B [BN][BK] images, NS - 1 stages in
//     flight; each wave waits with a counted vmcnt for its own pieces of the stage it is about to
//     read, one s_barrier per stage publishes them and frees the buffer the next issue overwrites;
//   * 16-byte chunks of the images XOR-swizzled per row through the DMA SOURCE address (the DMA
//     writes lane-linearly), so the v_mfma_f32_16x16x32_bf16 fragment reads (ds_read_b128, 16 rows
//     x 4 chunks per wave-instruction) are bank-conflict free;
//   * waves as 2 (M) x 4 (N): wave tile 128 x BN / 4, accumulators D = C^T (the output feature on
//     the accumulator row, the token on the lane), so the epilogue writes each token's features
//     as bf16x4 into a per-wave LDS image and stores whole row segments (16 B per lane);
//   * waves 4-7 (the second half to be dispatched, which loses VALU arbitration to its SIMD
//     partner) run at s_setprio 1 for the main loop (MI355X_MICROARCH.md, two waves per SIMD,
//     item 4).
#pragma once
#include "gemm_nt.h"

namespace sae {

typedef __attribute__((ext_vector_type(4))) unsigned g8_u32x4;

// descriptor words over rows [0, nrows) of a [rows][ld] bf16 operand (range check = zero fill)
__device__ __forceinline__ g8_u32x4 g8_rsrc(const __bf16* base, int nrows, long long ld) {
  const unsigned long long p = reinterpret_cast<unsigned long long>(base);
  g8_u32x4 w;
  w[0] = __builtin_amdgcn_readfirstlane((unsigned)p);
  w[1] = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32)) & 0xffffu;
  w[2] = __builtin_amdgcn_readfirstlane((unsigned)((long long)nrows * ld * 2));
  w[3] = 0x00020000u;
  return w;
}

// one 1-KiB LDS-DMA piece: lane L's 16 bytes (global byte offset voff in the descriptor's range)
// land at LDS byte address lds + 16 L.  M0 is saved / restored inside the statement.
__device__ __forceinline__ void g8_dma1(g8_u32x4 rs, unsigned voff, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(lds)
      : "memory");
}
__device__ __forceinline__ void g8_dma2(g8_u32x4 rs, unsigned voff0, unsigned voff1, unsigned lds0, unsigned lds1) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff0), "v"(voff1), "s"(rs), "s"(lds0), "s"(lds1)
      : "memory");
}

template <int N>
__device__ __forceinline__ void g8_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// chunk swizzle of a BK-deep bf16 image row (BK = 32: 64-byte rows, BK = 64: 128-byte rows),
// chosen for the 16x16x32 fragment read: lane l reads row base + (l & 15), chunk 4 kk + (l >> 4);
// within each 16-lane group of a ds_read_b128 the 16 chunks then hit distinct 16-byte bank slots
template <int BK> __device__ __forceinline__ int g8_swz(int r) {
  if constexpr (BK == 32) return (0x1320 >> (4 * ((r >> 2) & 3))) & 3;   // [0, 2, 3, 1][(r >> 2) & 3]
  else return (r >> 1) & 7;
}

// BM: tile rows (256, or 224 where 256-row tiles leave CUs idle: M = 25,216 into 384 features is
// 198 tiles of 256 x 192 on 256 CUs but 226 of 224 x 192; the A image keeps 256 rows, the rows past
// BM read as zero through the descriptor's range check -- no memory traffic)
// WGM: waves along M (2: 2 x 4 waves; 4: 4 x 2 -- 64 x 64 wave tiles at 256 x 128, so each wave's
// epilogue row segment is a whole 128-byte line)
template <int BN, int BM = 256, int WGM = 2> struct G8Cfg {
  static_assert(BM % 32 == 0 && BM <= 256, "tile rows");
  static constexpr int WM = BM / WGM, WN = BN / (8 / WGM);  // wave tile
  static constexpr int MT = WM / 16, NT = WN / 16; // 16 x 16 accumulator tiles per wave
};

// LDS: the stage ring, then one 32-row epilogue scratch per wave (rows padded by 16 bytes)
template <int BN, int BK, int NS> constexpr int g8_ring_bytes() { return NS * (256 + BN) * BK * 2; }
template <int BN, int WGM = 2> constexpr int g8_scratch_bytes() { return 32 * (BN / (8 / WGM) * 2 + 16); }
template <int BN, int BK, int NS, int WGM = 2> constexpr int g8_lds_bytes() {
  return g8_ring_bytes<BN, BK, NS>() + 8 * g8_scratch_bytes<BN, WGM>();
}
constexpr int kG8TickBytes = 16;   // the DYN ticket word after the scratch images

// Persistent: workgroup b walks tiles xcd_remap(b) + i G (G = gridDim.x <= #tiles; consecutive
// logical tiles -- the N tiles of one 256-row block -- run on one XCD at the same time, so the A
// rows come from HBM once per XCD).  The stage stream runs on across tiles: the next tile's first
// NS - 1 stages are in flight while a tile's epilogue drains its accumulators (through the
// per-wave scratch, 32 rows at a time: 16-byte row-segment stores), so neither the prologue's load
// latency nor the epilogue's stores stall the ring.
// DYN (launches with more tiles than workgroups): work stealing.  The tiles are dealt to the 8
// placement groups of the static walk (group x = hardware blocks b with b % 8 = x, which the
// dispatcher puts on one XCD; xcd_remap gives group x the logical range R_x, and with it the tiles
// R_x + i G), and each group's tiles are handed out in that order by a ticket counter of the group,
// t(k) = R_x.start + k % |R_x| + (k / |R_x|) G -- the first tile of a workgroup too: a workgroup that
// starts late (its CU held by an RCCL all-reduce kernel on the communication stream) finds its
// group's tiles taken and leaves at once, where the static walk would hold the kernel's end back by
// its whole tile list.  Wave 0 draws the ticket (one returning atomic) of the tile after the one the
// issue cursor enters, a whole tile ahead, keeps it in an LDS word, and every wave reads it when the
// cursor crosses the next tile boundary; the atomic is issued after a stage's DMA pieces and is
// covered by the next stage's vmcnt(0) wait (NS = 2).  Each workgroup that draws a ticket past its
// group's tiles adds to the slot's done counter; the last of the G resets the slot for the next
// launch (capi.hip g8_slot: one slot per stream).  Every tile is computed the same way whoever takes
// it: results are bit-identical to the static walk (tools/g8_dyn_check.py).  Placement only decides
// speed: every group has workgroups (G >= 8), and each drains its own counter.
// MODE (probe builds only): 0 = the kernel; 1 = no global stores; 2 = no MFMAs (staging only)
// XW (plain epilogue, 2 x 4 waves): the four waves of a wave row stage their 32-row pieces into one
// shared [32][BN] image and store whole rows (BN = 192: three full 128-byte lines per row instead of
// four 96-byte pieces), two workgroup barriers per 32-row group
template <int EPI, int BN, int BK, int NS, int MODE = 0, int BM = 256, bool DYN = false, int WGM = 2, bool XW = false>
__global__ __launch_bounds__(512, 1) void gemm8_nt_kernel(NtArgs a) {
  static_assert(!XW || (EPI == kEpiNone && WGM == 2 && 64 * (BN * 2 + 16) <= 8 * g8_scratch_bytes<BN, WGM>()),
                "XW: plain epilogue, 2 x 4 waves, the two row images fit the scratch");
  static_assert(!DYN || NS == 2, "dynamic walk: the ticket atomic rides on the vmcnt(0) stage waits of NS = 2");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using C = G8Cfg<BN, BM, WGM>;
  constexpr int RB = BK * 2;                  // image row bytes
  constexpr int CPR = BK / 8;                 // 16-byte chunks per row
  constexpr int RPP = 64 / CPR;               // rows per 1-KiB piece
  constexpr int IMGA = 256 * RB, STAGE = (256 + BN) * RB;
  constexpr int PA = 256 / RPP / 8;           // A pieces per wave per stage
  constexpr int PBT = BN / RPP;               // B pieces per stage (all waves)
  static_assert(PA * RPP * 8 == 256, "A pieces");
  constexpr int PB0 = (PBT + 7) / 8;          // B pieces of waves 0 .. PBT % 8 - 1
  constexpr int PB1 = PBT / 8;                // B pieces of the other waves
  constexpr int PBX = PBT % 8;                // waves with PB0 pieces (0: every wave has PB1)

  const int tn = (a.N + BN - 1) / BN;
  const int ntiles = ((a.M + BM - 1) / BM) * tn;
  const int G = gridDim.x;
  const int b0 = xcd_remap(blockIdx.x, G);
  // static: tiles b0, b0 + G, ...; DYN: one ticket of the placement group per tile
  const int myt = DYN ? 0x3fffffff : (ntiles - b0 + G - 1) / G;
  const int nst = a.K / BK;
  int total = DYN ? 0x7fffffff : myt * nst;   // stages of this workgroup's stream (DYN: found at the end)
  volatile unsigned* tick = reinterpret_cast<volatile unsigned*>(smem + g8_lds_bytes<BN, BK, NS, WGM>());
  unsigned tkv = 0;                           // wave 0: the returning ticket atomic in flight
  int tile_e = b0, tile_o = b0;               // DYN: tile ids of the even / odd local tiles
  auto tile_of = [&](int it) { return __builtin_amdgcn_readfirstlane((it & 1) ? tile_o : tile_e); };
  // DYN: this workgroup's placement group and the group's logical range R_x (xcd_remap's blocks)
  const int grp_x = blockIdx.x & 7, gq = G >> 3, gr = G & 7;
  const int r_cnt = gq + (grp_x < gr), r_start = grp_x < gr ? grp_x * (gq + 1) : gr * (gq + 1) + (grp_x - gr) * gq;
  unsigned* gctr = DYN ? a.ctr + 32 * grp_x : nullptr;   // the group's counter (its own 128-byte line)
  auto ticket_tile = [&](unsigned k) { return r_start + (int)(k % (unsigned)r_cnt) + (int)(k / (unsigned)r_cnt) * G; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w / (8 / WGM), wc = w % (8 / WGM);
  const unsigned lbase = __builtin_amdgcn_readfirstlane(
      (unsigned)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem));

  // this wave's pieces: A pieces w + 8 i (rows RPP (w + 8 i) ...), B pieces w + 8 i
  const int prow = lane / CPR, pc = lane % CPR;
  unsigned goa[PA], gob[PB0 > 0 ? PB0 : 1];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    const int row = RPP * (w + 8 * i) + prow;
    goa[i] = (unsigned)(((long long)row * a.lda + 8 * (pc ^ g8_swz<BK>(row))) * 2);
  }
#pragma unroll
  for (int i = 0; i < (PB0 > 0 ? PB0 : 1); ++i) {
    const int row = RPP * (w + 8 * i) + prow;
    gob[i] = (unsigned)(((long long)row * a.ldb + 8 * (pc ^ g8_swz<BK>(row))) * 2);
  }
  const bool bx = PBX == 0 || w < PBX;   // this wave issues PB0 B pieces (else PB1)

  // issue cursor: stage ist of local tile iti, with that tile's descriptors
  int iti = 0, ist = 0, ibuf = 0;
  g8_u32x4 ra, rb;
  auto set_issue_tile = [&](int it) {
    const int t = DYN ? tile_of(it) : b0 + it * G;
    const int m0 = (t / tn) * BM, n0 = (t % tn) * BN;
    ra = g8_rsrc(a.a + (long long)m0 * a.lda, min(BM, a.M - m0), a.lda);
    rb = g8_rsrc(a.bt + (long long)n0 * a.ldb, min(BN, a.N - n0), a.ldb);
  };
  // DYN: wave 0 draws the ticket of the tile after the one the issue cursor is entering
  auto draw_ticket = [&]() {
    if (w == 0) {
      if (lane == 0) tkv = __hip_atomic_fetch_add(gctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  };
  auto issue_next = [&]() {
    const unsigned ko = (unsigned)ist * RB;
    const unsigned lb = lbase + (unsigned)(ibuf * STAGE);
#pragma unroll
    for (int i = 0; i < PA; i += 2) {
      if (i + 1 < PA)
        g8_dma2(ra, goa[i] + ko, goa[i + 1] + ko, lb + 1024u * (w + 8 * i), lb + 1024u * (w + 8 * (i + 1)));
      else
        g8_dma1(ra, goa[i] + ko, lb + 1024u * (w + 8 * i));
    }
#pragma unroll
    for (int i = 0; i < PB0; ++i) {
      if (i < PB1 || bx) g8_dma1(rb, gob[i] + ko, lb + IMGA + 1024u * (w + 8 * i));
    }
    ibuf = ibuf + 1 == NS ? 0 : ibuf + 1;
    if (++ist == nst) {
      ist = 0;
      if constexpr (DYN) {
        const int t = __builtin_amdgcn_readfirstlane(ticket_tile(tick[0]));   // published at least one barrier ago
        if (t < ntiles) {
          if ((iti + 1) & 1) tile_o = t;
          else tile_e = t;
          ++iti;
          set_issue_tile(iti);
          draw_ticket();
        } else {
          total = (iti + 1) * nst;       // every stage of this workgroup's stream is issued
        }
      } else {
        if (++iti < myt) set_issue_tile(iti);
      }
    }
  };
  // DYN: wave 0 publishes a returned ticket (after the stage wait that covered its atomic)
  bool tpend = false;
  auto publish_ticket = [&]() {
    if (w == 0 && tpend) {
      const unsigned v = __builtin_amdgcn_readfirstlane(tkv);
      if (lane == 0) tick[0] = v;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      tpend = false;
    }
  };

  f32x4 acc[C::MT][C::NT];
#pragma unroll
  for (int i = 0; i < C::MT; ++i)
#pragma unroll
    for (int j = 0; j < C::NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets: row base + (lane & 15), chunk 4 kk + (lane >> 4)
  const int fr = lane & 15, fg = lane >> 4;
  const int sw = g8_swz<BK>(fr);   // rows are 16-aligned + fr: the swizzle depends on fr only
  const char* pa0 = smem + (C::WM * wr + fr) * RB;   // WM a multiple of 16: the swizzle stays g8_swz(fr)
  const char* pb0 = smem + IMGA + (C::WN * wc + fr) * RB;
  constexpr int SRB = C::WN * 2 + 16;             // scratch row bytes (wave tile row + pad)
  constexpr int SCH = C::WN / 8;                  // 16-byte chunks per tile row
  uint4 hv[EPI == kEpiDGelu ? (C::MT + 1) / 2 : 1][EPI == kEpiDGelu ? 32 * SCH / 64 : 1];   // GELU' aux tile
  char* scratch = smem + g8_ring_bytes<BN, BK, NS>() + w * g8_scratch_bytes<BN, WGM>();

  if constexpr (DYN) {
    // the first tile: drawn, published through LDS, then the second tile's ticket goes out
    draw_ticket();
    if (w == 0) {
      const unsigned v = __builtin_amdgcn_readfirstlane(tkv);
      if (lane == 0) tick[0] = v;
    }
    __syncthreads();
    const int t0 = __builtin_amdgcn_readfirstlane(ticket_tile(tick[0]));
    __syncthreads();            // every wave read the word before wave 0 publishes the next ticket
    if (t0 >= ntiles) {
      total = 0;                // this group's tiles are all taken: nothing to do
    } else {
      tile_e = t0;
      draw_ticket();            // the ticket of this workgroup's second tile
      tpend = true;
    }
  }
  if (total > 0) set_issue_tile(0);
#pragma unroll
  for (int q = 0; q < NS - 1; ++q)
    if (q < total) issue_next();
  if (w >= 4) __builtin_amdgcn_s_setprio(1);
  int cur = 0, cst = 0, cti = 0;   // compute cursor: buffer, stage, local tile
  for (int g = 0; g < total; ++g) {
    // stage g landed (this wave's pieces; the barrier: everyone's), buffer of g - 1 free
    const int ahead = min(NS - 2, total - 1 - g);   // younger stages still in flight
    if (ahead >= 2) {
      if (bx) g8_wait_barrier<2 * (PA + PB0)>(); else g8_wait_barrier<2 * (PA + PB1)>();
    } else if (ahead == 1) {
      if (bx) g8_wait_barrier<PA + PB0>(); else g8_wait_barrier<PA + PB1>();
    } else {
      g8_wait_barrier<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (DYN) {
      publish_ticket();                    // covered by the vmcnt(0) above
      const int it0 = iti;
      if (g + NS - 1 < total) issue_next();
      if (iti != it0) tpend = true;        // a new ticket atomic went out with this issue
    } else {
      if (g + NS - 1 < total) issue_next();
    }
    if constexpr (EPI == kEpiDGelu) {
      // GELU' epilogue: the tile's aux (h) chunks are loaded in one batch at the start of its last
      // stage, so the epilogue's stores do not each wait out a dependent HBM round trip
      if (cst == nst - 1) {
        const int t = DYN ? tile_of(cti) : b0 + cti * G;
        const int m0 = (t / tn) * BM + C::WM * wr, nw = (t % tn) * BN + C::WN * wc;
#pragma unroll
        for (int ip = 0; ip < (C::MT + 1) / 2; ++ip)
#pragma unroll
          for (int it = 0; it < 32 * SCH / 64; ++it) {
            const int id = it * 64 + lane;
            const int rr = id / SCH, c = id % SCH;
            const int m = m0 + 32 * ip + rr, n = nw + 8 * c;
            const bool in = 32 * ip + rr < C::WM && m < a.M && n < a.N;
            if (a.nts & 2) {   // aux streamed (non-temporal load): read once, not kept in L2
              typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
              const u32x4 v = in ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.aux + (long long)m * a.ldaux + n))
                                 : u32x4{0u, 0u, 0u, 0u};
              hv[ip][it] = uint4{v[0], v[1], v[2], v[3]};
            } else {
              hv[ip][it] = in ? *reinterpret_cast<const uint4*>(a.aux + (long long)m * a.ldaux + n) : uint4{0u, 0u, 0u, 0u};
            }
          }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const char* ia = pa0 + cur * STAGE;
    const char* ib = pb0 + cur * STAGE;
#pragma unroll
    for (int kk = 0; kk < (MODE == 2 ? 0 : BK / 32); ++kk) {
      const int co = 16 * ((4 * kk + fg) ^ sw);
      bf16x8 bf[C::NT], af[C::MT];
#pragma unroll
      for (int j = 0; j < C::NT; ++j) bf[j] = *reinterpret_cast<const bf16x8*>(ib + 16 * j * RB + co);
#pragma unroll
      for (int i = 0; i < C::MT; ++i) af[i] = *reinterpret_cast<const bf16x8*>(ia + 16 * i * RB + co);
#pragma unroll
      for (int i = 0; i < C::MT; ++i)
#pragma unroll
        for (int j = 0; j < C::NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    }
    cur = cur + 1 == NS ? 0 : cur + 1;
    if (++cst < nst) continue;
    cst = 0;

    // ---- epilogue of local tile cti.  acc[i][j] = D[n][m]: n = WN wc + 16 j + 4 fg + e,
    // m = 128 wr + 16 i + fr (tile-relative); through the wave's scratch 32 rows at a time
    const int t = DYN ? tile_of(cti) : b0 + cti * G;
    ++cti;
    const int m0 = (t / tn) * BM + C::WM * wr, nw = (t % tn) * BN + C::WN * wc;
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    f32x4 bv[C::NT];
#pragma unroll
    for (int j = 0; j < C::NT; ++j) {
      const int n = nw + 16 * j + 4 * fg;
      bv[j] = (EPI != kEpiDGelu && a.bias && n < a.N) ? *reinterpret_cast<const f32x4*>(a.bias + n)
                                                        : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (XW) {
      constexpr int XRB = BN * 2 + 16, XCH = BN / 8;   // row image bytes, 16-byte chunks per row
      char* const xs = smem + g8_ring_bytes<BN, BK, NS>() + wr * 32 * XRB;
      const int mrow = (t / tn) * BM + C::WM * wr, ncol = (t % tn) * BN;
#pragma unroll
      for (int ip = 0; ip < (C::MT + 1) / 2; ++ip) {
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int i = 2 * ip + h2;
          if (i >= C::MT) break;
#pragma unroll
          for (int j = 0; j < C::NT; ++j) {
            const bf16x4 v = {(__bf16)(acc[i][j][0] + bv[j][0]), (__bf16)(acc[i][j][1] + bv[j][1]),
                              (__bf16)(acc[i][j][2] + bv[j][2]), (__bf16)(acc[i][j][3] + bv[j][3])};
            *reinterpret_cast<bf16x4*>(xs + (16 * h2 + fr) * XRB + 2 * (C::WN * wc + 16 * j + 4 * fg)) = v;
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < 32 * XCH / 256; ++it) {
          const int id = (4 * it + wc) * 64 + lane;
          const int rr = id / XCH, c = id % XCH;
          const uint4 raw = *reinterpret_cast<const uint4*>(xs + rr * XRB + 16 * c);
          const int m = mrow + 32 * ip + rr, n = ncol + 8 * c;
          if (32 * ip + rr < C::WM && m < a.M && n < a.N) {
            __bf16* const cp = a.c + (long long)m * a.ldc + n;
            if (a.nts & 1) st16<true>(cp, raw);
            else st16(cp, raw);
          }
        }
        __syncthreads();
      }
      continue;
    }
#pragma unroll
    for (int ip = 0; ip < (C::MT + 1) / 2; ++ip) {
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int i = 2 * ip + h2;
        if (i >= C::MT) break;   // odd MT: the last group holds 16 rows
#pragma unroll
        for (int j = 0; j < C::NT; ++j) {
          const bf16x4 v = {(__bf16)(acc[i][j][0] + bv[j][0]), (__bf16)(acc[i][j][1] + bv[j][1]),
                            (__bf16)(acc[i][j][2] + bv[j][2]), (__bf16)(acc[i][j][3] + bv[j][3])};
          *reinterpret_cast<bf16x4*>(scratch + (16 * h2 + fr) * SRB + 2 * (16 * j + 4 * fg)) = v;
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int it = 0; it < 32 * SCH / 64; ++it) {
        const int id = it * 64 + lane;
        const int rr = id / SCH, c = id % SCH;
        const uint4 raw = *reinterpret_cast<const uint4*>(scratch + rr * SRB + 16 * c);
        const int m = m0 + 32 * ip + rr, n = nw + 8 * c;
        if (32 * ip + rr >= C::WM) continue;
        if (MODE == 1) {
          if (raw.x == 0x7fc07fc0u && raw.y == 0x12345678u) a.c[0] = (__bf16)1.f;   // keep the reads
        } else if (m < a.M && n < a.N) {
          __bf16* const cp = a.c + (long long)m * a.ldc + n;
          if (a.nts & 1) {   // (wave-uniform)
            if constexpr (EPI == kEpiNone) st16<true>(cp, raw);
            else if constexpr (EPI == kEpiGelu) gelu_store8<true>(raw, a.gp, cp, a.c2 + (long long)m * a.ldc + n);
            else st16<true>(cp, dgelu8(raw, hv[ip][it], a.gp));
          } else {
            if constexpr (EPI == kEpiNone) st16(cp, raw);
            else if constexpr (EPI == kEpiGelu) gelu_store8(raw, a.gp, cp, a.c2 + (long long)m * a.ldc + n);
            else st16(cp, dgelu8(raw, hv[ip][it], a.gp));
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (w >= 4) __builtin_amdgcn_s_setprio(0);
  if constexpr (DYN) {
    // this workgroup drew its ticket past its group's tiles (its stream ended on it): count it in
    // the slot's done word; the last of the G workgroups resets the slot -- every draw of this
    // launch has returned by then
    if (threadIdx.x == 0) {
      const unsigned d = __hip_atomic_fetch_add(a.ctr + 256, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == (unsigned)G - 1u) {
        for (int x = 0; x < 8; ++x) __hip_atomic_store(a.ctr + 32 * x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.ctr + 256, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

}  // namespace sae

namespace sae {

// ---------------------------------------------------------------------------------------------
// Ping-pong variant (long reductions): one 256 x BN tile per workgroup (not persistent), K-tiles of
// 32 through a 4-deep LDS ring (K-tile t + 2 issued while t computes), and the two wave groups
// -- waves 0-3 (tile rows 0-127) and 4-7 (rows 128-255) -- one barrier apart: each K-tile is two
// phases per group, a load segment (LDS-DMA issue, fragment reads, the stage wait) and an MFMA
// segment (16 MFMAs at s_setprio 1), so on every SIMD one wave's load segment runs beside its
// partner's MFMAs (cdna_hip_programming.md section 5, the 8-phase template; MI355X_MICROARCH.md,
// two waves per SIMD).  RAW: a stage is waited for (counted vmcnt) in the load segment of the
// phase before the one that first reads it, and every group passes a barrier in between; WAR:
// K-tile t + 2 overwrites the buffer of t - 2, read four phases (eight barriers) earlier.
// BAL: the A pieces of K-tile t + 2 go out in phase 0, its B pieces in phase 1 after that phase's
// wait (both load segments carry DMA; the wait counts only the two A pieces, for every wave)
template <int EPI, int BN, bool BAL = false, int BM = 256>
__global__ __launch_bounds__(512, 1) void gemm8x_nt_kernel(NtArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using C = G8Cfg<BN, BM>;
  static_assert(C::MT > 4 && C::MT <= 8, "phase 0 computes rows 0-63 of a wave tile, phase 1 the rest");
  static_assert(C::WM * (C::WN / 8) % 64 == 0, "epilogue: whole 64-lane store rounds");
  constexpr int RB = 64;                       // image row bytes (BK = 32)
  constexpr int IMGA = 256 * RB, STAGE = (256 + BN) * RB;
  constexpr int PBT = BN / 16;                 // B pieces per stage (16 rows per piece)
  constexpr int PB0 = (PBT + 7) / 8, PB1 = PBT / 8, PBX = PBT % 8;

  const int tn = (a.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / tn) * BM, n0 = (bid % tn) * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2, wc = w & 3;
  const g8_u32x4 ra = g8_rsrc(a.a + (long long)m0 * a.lda, min(BM, a.M - m0), a.lda);
  const g8_u32x4 rb = g8_rsrc(a.bt + (long long)n0 * a.ldb, min(BN, a.N - n0), a.ldb);
  const unsigned lbase = __builtin_amdgcn_readfirstlane(
      (unsigned)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem));
  const int prow = lane >> 2, pc = lane & 3;
  unsigned goa[2], gob[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * (w + 8 * i) + prow;
    goa[i] = (unsigned)(((long long)row * a.lda + 8 * (pc ^ g8_swz<32>(row))) * 2);
    gob[i] = (unsigned)(((long long)row * a.ldb + 8 * (pc ^ g8_swz<32>(row))) * 2);
  }
  const bool bx = PBX == 0 || w < PBX;
  auto issue_a = [&](int kt) __attribute__((always_inline)) {
    const unsigned ko = (unsigned)kt * RB;
    const unsigned lb = lbase + (unsigned)((kt & 3) * STAGE);
    g8_dma2(ra, goa[0] + ko, goa[1] + ko, lb + 1024u * w, lb + 1024u * (w + 8));
  };
  auto issue_b = [&](int kt) __attribute__((always_inline)) {
    const unsigned ko = (unsigned)kt * RB;
    const unsigned lb = lbase + (unsigned)((kt & 3) * STAGE);
    if (PB0 == 2 && bx)
      g8_dma2(rb, gob[0] + ko, gob[1] + ko, lb + IMGA + 1024u * w, lb + IMGA + 1024u * (w + 8));
    else if (PB0 >= 1 && (PB1 >= 1 || bx))
      g8_dma1(rb, gob[0] + ko, lb + IMGA + 1024u * w);
  };
  auto issue = [&](int kt) __attribute__((always_inline)) {
    issue_a(kt);
    issue_b(kt);
  };
  const int fr = lane & 15, fg = lane >> 4;
  const int co = 16 * (fg ^ g8_swz<32>(fr));
  const char* pa0 = smem + (C::WM * grp + fr) * RB + co;
  const char* pb0 = smem + IMGA + (C::WN * wc + fr) * RB + co;
  f32x4 acc[C::MT][C::NT];
#pragma unroll
  for (int i = 0; i < C::MT; ++i)
#pragma unroll
    for (int j = 0; j < C::NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkt = a.K / 32;
  issue(0);
  if (nkt > 1) issue(1);
  if (nkt > 1) {
    if (bx) g8_wait_barrier<2 + PB0>(); else g8_wait_barrier<2 + PB1>();
  } else {
    g8_wait_barrier<0>();
  }
  if (grp == 1) asm volatile("s_barrier" ::: "memory");   // the stagger
  __builtin_amdgcn_sched_barrier(0);
  for (int kt = 0; kt < nkt; ++kt) {
    const char* ia = pa0 + (kt & 3) * STAGE;
    const char* ib = pb0 + (kt & 3) * STAGE;
    // ---- phase 0: read B and the first half of A, issue K-tile kt + 2 (BAL: its A pieces)
    bf16x8 bf[C::NT], af[4];
#pragma unroll
    for (int j = 0; j < C::NT; ++j) bf[j] = *reinterpret_cast<const bf16x8*>(ib + 16 * j * RB);
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(ia + 16 * i * RB);
    if (kt + 2 < nkt) {
      if constexpr (BAL) issue_a(kt + 2);
      else issue(kt + 2);
    }
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < C::NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase 1: read the second half of A; K-tile kt + 1 must have landed before the next
    // phase's reads (BAL: then the B pieces of kt + 2)
#pragma unroll
    for (int i = 0; i < C::MT - 4; ++i) af[i] = *reinterpret_cast<const bf16x8*>(ia + 16 * (4 + i) * RB);
    if (kt + 1 < nkt) {
      if (kt + 2 < nkt) {
        if constexpr (BAL) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else if (bx) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 + PB0) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 + PB1) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    if constexpr (BAL)
      if (kt + 2 < nkt) issue_b(kt + 2);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < C::MT - 4; ++i)
#pragma unroll
      for (int j = 0; j < C::NT; ++j)
        acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  if (grp == 0) asm volatile("s_barrier" ::: "memory");   // balance the stagger
  asm volatile("s_barrier" ::: "memory");                  // every wave done with the ring

  // ---- epilogue through a per-wave scratch (the ring is free): acc[i][j] = D[n][m]
  constexpr int SRB = C::WN * 2 + 16, SCH = C::WN / 8;
  char* scratch = smem + w * (C::WM * SRB);
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  const int nw = n0 + C::WN * wc;
  f32x4 bv[C::NT];
#pragma unroll
  for (int j = 0; j < C::NT; ++j) {
    const int n = nw + 16 * j + 4 * fg;
    bv[j] = (a.bias && n < a.N) ? *reinterpret_cast<const f32x4*>(a.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < C::MT; ++i)
#pragma unroll
    for (int j = 0; j < C::NT; ++j) {
      const bf16x4 v = {(__bf16)(acc[i][j][0] + bv[j][0]), (__bf16)(acc[i][j][1] + bv[j][1]),
                        (__bf16)(acc[i][j][2] + bv[j][2]), (__bf16)(acc[i][j][3] + bv[j][3])};
      *reinterpret_cast<bf16x4*>(scratch + (16 * i + fr) * SRB + 2 * (16 * j + 4 * fg)) = v;
    }
  __builtin_amdgcn_wave_barrier();
  const int mw = m0 + C::WM * grp;
#pragma unroll 4
  for (int it = 0; it < C::WM * SCH / 64; ++it) {
    const int id = it * 64 + lane;
    const int rr = id / SCH, c = id % SCH;
    const uint4 raw = *reinterpret_cast<const uint4*>(scratch + rr * SRB + 16 * c);
    const int m = mw + rr, n = nw + 8 * c;
    if (m < a.M && n < a.N) {
      if constexpr (EPI == kEpiNone) {
        *reinterpret_cast<uint4*>(a.c + (long long)m * a.ldc + n) = raw;
      } else {
        gelu_store8(raw, a.gp, a.c + (long long)m * a.ldc + n, a.c2 + (long long)m * a.ldc + n);
      }
    }
  }
}

template <int BN, int BM = 256> constexpr int g8x_lds_bytes() {
  constexpr int ring = 4 * (256 + BN) * 64, scratch = 8 * (BM / 2) * (BN / 4 * 2 + 16);
  return ring > scratch ? ring : scratch;
}

}  // namespace sae
