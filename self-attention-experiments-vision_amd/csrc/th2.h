// th2.h -- talking-heads attention (CaiT trunk) for gfx950 with the head mixes on the matrix pipe.
//
// Reference: models/layers/attentions/attention.py:41-58 with talking_heads=True and
// models/layers/attentions/talking_heads.py:9-14 (T is [h_in, h_out]):
//   S_h = scale Q_h K_h^T ; S1_i = sum_h T1[h,i] S_h ; P_i = softmax_k(S1_i) ;
//   P2_i = sum_h T2[h,i] P_h ; O_i = P2_i V_i
// A workgroup owns one 32-row query block (th2_fwd, th2_bwd_q) or one 32-key block (th2_bwd_kv)
// for ALL H <= 16 heads; wave w computes head w's 32 x 32 score tiles on the MFMA (key on the
// accumulator rows, query on the lane, as fwd2.h).  The head mix is a tiny [H x H] x [H x 1024]
// product per tile, done on the MFMA instead of the VALU (th_kernels.h spends 2 x H^2 FMAs per
// score there):
//   * every wave writes its tile as bf16 into an exchange image [head][key * 32 + query] (the
//     reference's scores are bf16 values: attention.py:41-42 returns dtype);
//   * position block `key` (32 queries) of the tile belongs to wave key mod H, which reads the H
//     head values of its positions with ds_read_b64_tr_b16 (B operand: 16 heads x 32 positions)
//     and runs v_mfma_f32_32x32x16_bf16 with A = the [H x H] transform, split into a bf16 high and
//     low part (two MFMAs: ~16-bit transform precision; the reference promotes the mix to fp32,
//     talking_heads.py:11-13).  The result has the query on the lane and the mixed head in the
//     accumulator rows, so the softmax statistics of every (head, query) row live in registers
//     and the second mix takes the accumulator as its B operand with no lane movement;
//   * what the next product needs per head goes back through the images.
// The softmax needs the row statistics of the MIXED logits before P can be mixed again, so the
// forward sweeps the keys twice (statistics, then output), as the reference's materialised
// softmax implies.  dT1 / dT2 are 16 x 16 MFMA sums over the score positions of each tile
// (v_mfma_f32_16x16x32_bf16), reduced over waves and workgroups in a fixed order.
// bf16 only (the fp32 path keeps th_kernels.h: exact fp32 mixing).
#pragma once
#include "common.h"
#include "th_kernels.h"

namespace sae {

constexpr int kTh2MaxH = 16;
// An image row (one head) holds 1024 positions = 32 blocks of 32 bf16; each block is padded to
// 80 bytes (a multiple of 16 for the 16-byte reads), so that the lanes of a transposed tile write
// (lane = block, four consecutive positions each) spread over the banks instead of sharing 8;
// head rows are 64 bytes (16 banks) past a multiple of 256, so that the mixes' transposed reads
// (4 head rows x 64 contiguous bytes) and the dT reads (one 16-byte piece per head row) do not
// pile onto the same banks (with rows a multiple of 256 bytes apart they conflicted 4- to 16-way)
constexpr int kTh2Blk = 80;                      // bytes per 32-position block
constexpr int kTh2Row = 32 * kTh2Blk + 64;       // bytes per head row (2624 = 10 x 256 + 64)
// KST ("K-stacked", H <= 8): a mix is ONE MFMA whose K = 16 holds the 8 heads twice, the high
// bf16 part of T against the first copy and the low part against the second, and the images
// need only 8 rows; otherwise (H <= 16) two MFMAs (high, low) over 16 image rows.
// Row r starts at th2_ro(r): rows 4-7 and 12-15 sit 32 bytes (8 banks) further, so that the dT
// reads (ds_read_b128, one 16-byte piece of each of 8 / 16 rows in a 16-lane group) find rows r
// and r + 4 on different banks (2-way conflicts with a uniform stride); the mixes' transposed
// reads take rows 0-3 and 4-7 in separate instructions, so the shift costs them nothing.
template <bool KST> constexpr int th2_rows() { return KST ? 8 : kTh2MaxH; }
__host__ __device__ constexpr int th2_ro(int r) { return r * kTh2Row + 32 * ((r >> 2) & 1); }
template <bool KST> constexpr int th2_img() { return th2_rows<KST>() * kTh2Row + 32; }   // one exchange image
constexpr int kTh2MixTbl = 4 * 64 * 32;          // th2_bwd_kv: four mix operands (hi, lo) per lane

typedef __attribute__((ext_vector_type(8))) short th_s16x8;

__device__ __forceinline__ bf16x8 th2_tr2(const char* p1, const char* p2) {
  const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
  const s16x4 x2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p2));
  const th_s16x8 v = {x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// A operand of a head mix, high and low bf16 parts: A[row][k] = TR ? T[row][k] : T[k][row]
// (T fp32 [H][H], [h_in][h_out]).  K order: standard (k = 8 (lane >> 5) + j: the B operand comes
// from an image) or PERM (the B operand is a 32 x 32 accumulator: element j of lane half g is
// row 8 (j >> 2) + 4 g + (j & 3)).  Rows / k >= H are zero.  KST: one operand in `hi` whose k < 8
// carry the high parts of heads k and k >= 8 the low parts of heads k - 8.
struct Th2Mix {
  bf16x8 hi, lo;
};
// n mix operands per lane in LDS: the high parts of all n, then the low parts -- a 16-byte lane
// stride (conflict-free ds_read_b128; {hi, lo} pairs at a 32-byte stride conflicted 2-way)
__device__ __forceinline__ void th2_mx_put(char* t, int n, int k, int lane, const Th2Mix& m) {
  reinterpret_cast<bf16x8*>(t)[k * 64 + lane] = m.hi;
  reinterpret_cast<bf16x8*>(t)[(n + k) * 64 + lane] = m.lo;
}
__device__ __forceinline__ Th2Mix th2_mx_get(const char* t, int n, int k, int lane) {
  return Th2Mix{reinterpret_cast<const bf16x8*>(t)[k * 64 + lane], reinterpret_cast<const bf16x8*>(t)[(n + k) * 64 + lane]};
}
// `mul` scales T before the split (th2_fwd: log2 e, so the mixed logits come out in the log2 domain)
template <bool TR, bool PERM, bool KST>
__device__ __forceinline__ Th2Mix th2_mix(const float* T, int H, int lane, float mul = 1.f) {
  Th2Mix m;
  const int row = lane & 31, g = lane >> 5;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = PERM ? 8 * (j >> 2) + 4 * g + (j & 3) : 8 * g + j;
    const int hd = KST ? (k & 7) : k;
    const float t = (row < H && hd < H) ? (TR ? T[row * H + hd] : T[hd * H + row]) * mul : 0.f;
    const __bf16 hi = (__bf16)t;
    const __bf16 lo = (__bf16)(t - (float)hi);
    if constexpr (KST) {
      m.hi[j] = k < 8 ? hi : lo;
      m.lo[j] = (__bf16)0.f;
    } else {
      m.hi[j] = hi;
      m.lo[j] = lo;
    }
  }
  return m;
}

// mixed tile of position block `blk` (32 positions) from an image: C[row][pos], pos on the lane
template <bool KST>
__device__ __forceinline__ f32x16 th2_mix_img(const char* img, int blk, const Th2Mix& m, int lane) {
  const int li = lane & 15;
  const int r1 = (KST ? 0 : 8 * (lane >> 5)) + (li >> 2);   // KST: both lane halves read rows 0..7
  const int col = blk * kTh2Blk + (16 * ((lane >> 4) & 1) + 4 * (li & 3)) * 2;
  const bf16x8 b = th2_tr2(img + th2_ro(r1) + col, img + th2_ro(r1 + 4) + col);
  const f32x16 c = MF<__bf16>::mma(m.hi, b, zero16());
  if constexpr (KST) return c;
  return MF<__bf16>::mma(m.lo, b, c);
}

// two fp32 values -> one dword of two bf16 (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ unsigned th2_pk(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f2v;
  typedef __attribute__((ext_vector_type(2))) __bf16 b2v;
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f2v{a, b}, b2v));
}

// mixed tile from an accumulator (rows = heads < 16, lanes = positions); KST: registers 4..7
// (rows 8..15) take a copy of 0..3 (rows 0..7), the second K half of the stacked operand.  The
// operand is packed pairwise (element-wise conversion left single-value conversions plus v_perm
// re-packing in the hot loops)
template <bool KST>
__device__ __forceinline__ f32x16 th2_mix_acc(const f32x16& x, const Th2Mix& m) {
  if constexpr (KST) {
    const unsigned p0 = th2_pk(x[0], x[1]), p1 = th2_pk(x[2], x[3]);
    return MF<__bf16>::mma(m.hi, __builtin_bit_cast(bf16x8, uint4{p0, p1, p0, p1}), zero16());
  } else {
    const bf16x8 b = __builtin_bit_cast(
        bf16x8, uint4{th2_pk(x[0], x[1]), th2_pk(x[2], x[3]), th2_pk(x[4], x[5]), th2_pk(x[6], x[7])});
    f32x16 c = MF<__bf16>::mma(m.hi, b, zero16());
    return MF<__bf16>::mma(m.lo, b, c);
  }
}

// bf16 score tile in the transposed accumulator layout (query row_of(r, h) on register r, key on
// the lane) into image row `head` at position key * 32 + query: registers 4g .. 4g + 3 are four
// consecutive positions, one 8-byte write
__device__ __forceinline__ void th2_put(char* img, int head, const f32x16& v, float sc, int lane) {
  char* p = img + th2_ro(head) + (lane & 31) * kTh2Blk + 8 * (lane >> 5);
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *reinterpret_cast<bf16x4*>(p + 16 * g) = bf16x4{(__bf16)(v[4 * g] * sc), (__bf16)(v[4 * g + 1] * sc),
                                                   (__bf16)(v[4 * g + 2] * sc), (__bf16)(v[4 * g + 3] * sc)};
}

// rows i < H of a mixed block (accumulator rows = heads; registers r < NR) into the images at
// block `blk`
template <int NR>
__device__ __forceinline__ void th2_put_block(char* img, int blk, const f32x16& v, int H, int lane) {
  char* p = img + blk * kTh2Blk + (lane & 31) * 2;
  const int h = lane >> 5;
  if (H >= 2 * NR) {   // every row of the registers is a head (wave-uniform): no per-lane branches
#pragma unroll
    for (int r = 0; r < NR; ++r) *reinterpret_cast<__bf16*>(p + th2_ro(row_of(r, h))) = (__bf16)v[r];
    return;
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int i = row_of(r, h);
    if (i < H) *reinterpret_cast<__bf16*>(p + th2_ro(i)) = (__bf16)v[r];
  }
}

// zero image rows [H, rows) once (read as the padded k of the mixes; must be finite)
template <bool KST>
__device__ __forceinline__ void th2_zero_pad(char* img, int H, int tid, int nthreads) {
  uint4* p = reinterpret_cast<uint4*>(img + th2_ro(H));
  const int n = (th2_img<KST>() - th2_ro(H)) / 16;
  for (int i = tid; i < n; i += nthreads) p[i] = uint4{0, 0, 0, 0};
}

// 16 x 16 dT partial for position block blk: acc[h = 4 (lane >> 4) + j][i = lane & 15] +=
// sum over the block's 32 positions of A-image[h] * B-image[i]
template <bool KST>
__device__ __forceinline__ f32x4 th2_dt(const char* ia, const char* ib, int blk, f32x4 acc, int lane) {
  // KST: 8-row images; lanes 8..15 re-read rows 0..7 (their dT rows / columns are discarded)
  const int row = lane & (KST ? 7 : 15), o = blk * kTh2Blk + 16 * (lane >> 4);
  const bf16x8 a = *reinterpret_cast<const bf16x8*>(ia + th2_ro(row) + o);
  const bf16x8 b = *reinterpret_cast<const bf16x8*>(ib + th2_ro(row) + o);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
}

// B operand of the per-head products, paired with Img::colfrag (K = tile rows in the accumulator
// order: element j of k-step s, lane half g <-> row 16 s + 8 (j >> 2) + 4 g + (j & 3)).
// th2_colB: image row `head` read as a [row][column = lane] matrix (position = row * 32 + column),
// transposed reads.
__device__ __forceinline__ bf16x8 th2_colB(const char* img, int head, int s, int lane) {
  const int li = lane & 15;
  const int r1 = 16 * s + 4 * (lane >> 5) + (li >> 2);
  const int col = (16 * ((lane >> 4) & 1) + 4 * (li & 3)) * 2;
  const char* base = img + th2_ro(head) + col;
  return th2_tr2(base + r1 * kTh2Blk, base + (r1 + 8) * kTh2Blk);
}

// operand fragment of row `row` (head-dim columns 16 s + 8 h .. + 7) through a buffer descriptor
// over the valid rows (row_rsrc): rows past the end and columns >= D read as zero.  (gfrag's
// branch-per-load form made hipcc wait vmcnt(0) after every fragment load: no prefetch survived.)
__device__ __forceinline__ bf16x8 th2_frag(__amdgpu_buffer_rsrc_t rsrc, int row, long long rs, int D, int s, int h) {
  const int d0 = 16 * s + 8 * h;
  const unsigned off = d0 < D ? (unsigned)(((long long)row * rs + d0) * 2) : 0x80000000u;
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
}

// th2_rowB: image row `head` read as a [column = lane][row] matrix (position = column * 32 + row:
// the key-block kernel, B[k = query][column = key]): two 8-byte reads of query runs
__device__ __forceinline__ bf16x8 th2_rowB(const char* img, int head, int s, int lane) {
  const char* base = img + th2_ro(head) + (lane & 31) * kTh2Blk + (16 * s + 4 * (lane >> 5)) * 2;
  const s16x4 x1 = *reinterpret_cast<const s16x4*>(base);
  const s16x4 x2 = *reinterpret_cast<const s16x4*>(base + 16);
  const th_s16x8 v = {x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Head-dim tail on v_mfma_f32_16x16x32_bf16 (TAIL: D <= 48 at DP 64, rows d 32..47 of the query
// pass's dQ^T product as two 16 x 16 blocks instead of half of a second 32 x 32 tile).  Operand k order:
// standard, k = 8 (lane >> 4) + j.
// A: image column col0 + (lane & 15) of a [row][DP] Img tile, k = image rows 8 (lane >> 4) + j
template <int DP> __device__ __forceinline__ bf16x8 th2_colA16(const char* lds, int col0, int lane) {
  const int li = lane & 15, g = lane >> 4;
  const int colb = col0 + 4 * (li & 3), chunk = colb >> 3, half = (colb >> 2) & 1;
  const int r1 = 8 * g + (li >> 2), r2 = r1 + 4;
  return th2_tr2(lds + r1 * (DP * 2) + 16 * (chunk ^ swz<DP>(r1)) + 8 * half,
                 lds + r2 * (DP * 2) + 16 * (chunk ^ swz<DP>(r2)) + 8 * half);
}
// B of the query pass: image row `head` at position k * 32 + n, k = key, n = 16 bb + (lane & 15) (query)
__device__ __forceinline__ bf16x8 th2_colB16(const char* img, int head, int bb, int lane) {
  const int li = lane & 15, k1 = 8 * (lane >> 4) + (li >> 2);
  const char* base = img + th2_ro(head) + (16 * bb + 4 * (li & 3)) * 2;
  return th2_tr2(base + k1 * kTh2Blk, base + (k1 + 4) * kTh2Blk);
}
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// sum of per-wave 16 x 16 partials (one per wave of the NW, in LDS scratch) -> this workgroup's dT
// slot (the first 256 threads: NW >= 4 when H > 4)
__device__ __forceinline__ void th2_dt_store(float* scratch, f32x4 acc, float* out, int H, int NW, int w, int lane,
                                             int tid, bool transpose_out) {
  // acc[j] = dT[h = 4 (lane >> 4) + j][i = lane & 15]
  f32x4* s4 = reinterpret_cast<f32x4*>(scratch);
  s4[w * 64 + lane] = acc;
  __syncthreads();
  if (tid < 256) {
    const int ln = tid & 63, j = tid >> 6;   // element j of lane ln: h = 4 (ln >> 4) + j, i = ln & 15
    float s = 0.f;
    for (int ww = 0; ww < NW; ++ww) s += scratch[(ww * 64 + ln) * 4 + j];
    const int h = 4 * (ln >> 4) + j, i = ln & 15;
    if (h < H && i < H) out[transpose_out ? i * H + h : h * H + i] = s;
  }
  __syncthreads();
}

// ================================================================================= forward
// (Measured and dropped: double-buffered images with the next tile's scores issued before this
// tile's mixes and one barrier per tile -- 238 vs 221 us at cait_s24: in-order issue stalls on
// the score tile's MFMA results before the mixes can start, so nothing overlapped.)
// HPW heads per wave (1, or 2 for 9..16 heads: eight waves of up to 256 registers instead of
// sixteen of 128, which spilled); wave w owns heads w + NW e, e < HPW, NW = ceil(H / HPW) waves.
// LEAN: <= 128 VGPRs (four waves per SIMD: two workgroups per CU at <= 8 heads) -- no K prefetch,
// mix groups of two
// NSU: 16-wide head-dim k-steps held and multiplied (D <= 16 NSU; CaiT's D = 48 at DP 64: 3, which
// frees the registers of an all-zero fourth Q / K fragment)
template <int DP, int NWMAX, bool ROT = false, int HPW = 1, bool LEAN = false, int NSU = DP / 16>
__global__ __launch_bounds__(64 * NWMAX, LEAN ? 4 : 1) void th2_fwd_kernel(ThArgs a) {
  using I = Img<__bf16, DP>;
  constexpr int NS = NSU, NT = DP / 32;
  constexpr bool KST = NWMAX * HPW <= 8;     // H <= 8: stacked mixes, heads in registers 0..3
  constexpr int NR = KST ? 4 : 8;            // registers r < NR hold the mixed heads row_of(r, h)
  constexpr int IMG = th2_img<KST>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H, NW = (H + HPW - 1) / HPW;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* const XS = smem;                    // scores S_h (bf16), then statistics scratch
  char* const XP = smem + IMG;              // mixed probabilities P2_j (bf16)

  const int nqb = (a.Nq + 31) / 32;
  // XCD-aware order: the query blocks of one image run on one XCD and share its K / V in L2
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = lb % nqb, b = lb / nqb;
  const int q = qb * 32 + r32;
  int hd[HPW];                              // this wave's heads (hd[e] >= H: none, e > 0 only)
  bool hv[HPW];
  char* ldsV[HPW];
  __amdgpu_buffer_rsrc_t rQ[HPW], rK[HPW], rV[HPW];
#pragma unroll
  for (int e = 0; e < HPW; ++e) {
    hd[e] = w + NW * e;
    hv[e] = hd[e] < H;
    const int he = hv[e] ? hd[e] : w;
    ldsV[e] = smem + 2 * IMG + he * I::bytes(32);
    rQ[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + he * a.qs[2], a.Nq, a.qs[1]);
    rK[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + he * a.ks[2], a.Nk, a.ks[1]);
    rV[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + he * a.vs[2], a.Nk, a.vs[1]);
  }

  th2_zero_pad<KST>(XS, H, tid, 64 * NW);
  th2_zero_pad<KST>(XP, H, tid, 64 * NW);
  constexpr bool rot = ROT;   // rotary: q / k rotated as they are loaded
  // the last 16-wide k-step holds head-dim columns (NSU < DP / 16: dispatched for 16 (NSU - 1) < D)
  const bool full = NSU < DP / 16 || a.D > 16 * (NS - 1);
  bf16x8 qf[HPW][NS];
#pragma unroll
  for (int e = 0; e < HPW; ++e)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qf[e][s] = th2_frag(rQ[e], q, a.qs[1], a.D, s, h);
      if (rot) qf[e][s] = rope8<1>(qf[e][s], a.rope, q, 16 * s + 8 * h);
    }
  // S1 = T1^T S with T1 scaled by log2 e: the mixed logits come out in the log2 domain, so the
  // statistics and probabilities need no per-element scaling
  // LEAN (128 registers): the two operands live in an LDS table written by wave 0 before the first
  // barrier and are re-read per use (held in registers they were spilled to scratch and reloaded in
  // the output sweep)
  Th2Mix m1r, m2r;
  char* const mxt = smem + 2 * IMG + H * I::bytes(32);
  if constexpr (LEAN) {
    if (w == 0) {
      th2_mx_put(mxt, 2, 0, lane, th2_mix<false, false, KST>(a.th1, H, lane, kLog2e));
      th2_mx_put(mxt, 2, 1, lane, th2_mix<false, true, KST>(a.th2, H, lane));
    }
  } else {
    m1r = th2_mix<false, false, KST>(a.th1, H, lane, kLog2e);
    m2r = th2_mix<false, true, KST>(a.th2, H, lane);    // P2 = T2^T P (accumulator operand)
  }
  auto m1 = [&]() -> Th2Mix { if constexpr (LEAN) return th2_mx_get(mxt, 2, 0, lane); else return m1r; };
  auto m2 = [&]() -> Th2Mix { if constexpr (LEAN) return th2_mx_get(mxt, 2, 1, lane); else return m2r; };
  const int nkt = (a.Nk + 31) / 32;

  // ---- pass 0: row statistics (log2 domain) of the mixed logits, per (head i, query) in this
  //      wave's key blocks: register r <-> head row_of(r, h), lane <-> query
  float m[NR], l[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    m[r] = -kInf;
    l[r] = 0.f;
  }
  // K fragments of the next key tile are loaded while this one computes (the global latency
  // would otherwise sit in front of every tile's first MFMA)
  // one head per wave: the next key tile's K fragments are in flight while this one computes; two
  // heads: the registers hold the second head's Q instead and each head's K loads directly
  constexpr bool PF = HPW == 1 && !LEAN;
  bf16x8 kn[NS];
  auto load_k = [&](int e, int kt) {
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) kn[s_] = th2_frag(rK[e], kt * 32 + r32, a.ks[1], a.D, s_, h);
  };
  auto scores = [&](int kt, int ktn) {   // ktn: the tile whose K fragments PF prefetches
#pragma unroll
    for (int e = 0; e < HPW; ++e) {
      if constexpr (!PF) load_k(e, kt);
      bf16x8 kc[NS];
#pragma unroll
      for (int s_ = 0; s_ < NS; ++s_) kc[s_] = rot ? rope8<1>(kn[s_], a.rope, kt * 32 + r32, 16 * s_ + 8 * h) : kn[s_];
      if constexpr (PF) load_k(0, ktn);
      f32x16 s = zero16();
#pragma unroll
      for (int s_ = 0; s_ < NS; ++s_)
        if (s_ < NS - 1 || full) s = MF<__bf16>::mma(qf[e][s_], kc[s_], s);   // S^T: query rows, key lanes
      if (hv[e]) th2_put(XS, hd[e], s, a.scale, lane);
    }
  };
  auto stats = [&](int kt) {   // this wave's blocks of tile kt, groups of SG: one max update each
    constexpr int SG = 4;   // (LEAN too since its mix operands moved to LDS: no extra spills)
    const char* xs = XS;
    for (int b0 = w; b0 < 32; b0 += SG * NW) {
      f32x16 c[SG];
      bool ok[SG];
#pragma unroll
      for (int u = 0; u < SG; ++u) {   // independent chains: issued together, blocks past the end clamped
        const int blk = b0 + u * NW;
        ok[u] = blk < 32 && kt * 32 + blk < a.Nk;
        c[u] = th2_mix_img<KST>(xs, blk & 31, m1(), lane);
      }
      if (!ok[0]) break;   // (the later blocks of the group lie further out)
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        float mx = -kInf;
#pragma unroll
        for (int u = 0; u < SG; ++u)
          if (ok[u]) mx = fmaxf(mx, c[u][r]);
        const float mn = fmaxf(m[r], mx);
        float sum = l[r] * ex2(m[r] - mn);
#pragma unroll
        for (int u = 0; u < SG; ++u)
          if (ok[u]) sum += ex2(c[u][r] - mn);
        l[r] = sum;
        m[r] = mn;
      }
    }
  };
  if constexpr (PF) load_k(0, 0);
  for (int kt = 0; kt < nkt; ++kt) {
    scores(kt, kt + 1 < nkt ? kt + 1 : nkt - 1);   // (the last prefetch: pass 1's first tile)
    __syncthreads();
    stats(kt);
    __syncthreads();
  }
  // combine the per-wave statistics: scratch [w][r][lane] (m, l) in the images
  {
    float2* st = reinterpret_cast<float2*>(smem);
#pragma unroll
    for (int r = 0; r < NR; ++r) st[(w * NR + r) * 64 + lane] = make_float2(m[r], l[r]);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      float mm = -kInf, ll = 0.f;
      for (int ww = 0; ww < NW; ++ww) {
        const float2 v = st[(ww * NR + r) * 64 + lane];
        const float mn = fmaxf(mm, v.x);
        ll = (mm == -kInf ? 0.f : ll * ex2(mm - mn)) + (v.x == -kInf ? 0.f : v.y * ex2(v.x - mn));
        mm = mn;
      }
      m[r] = mm + lg2(ll);   // from here on: log2 of the row's normaliser, P = 2^(S1 - m)
      const int i = row_of(r, h);
      if (w == 0 && i < H && q < a.Nq) a.lse[((size_t)b * H + i) * a.Nq + q] = m[r] * kLn2;
    }
    __syncthreads();
    th2_zero_pad<KST>(XS, H, tid, 64 * NW);   // the scratch overwrote the pad rows
    th2_zero_pad<KST>(XP, H, tid, 64 * NW);
  }

  // ---- pass 1: P_i = 2^(S1 - m) / l, P2 = T2^T P into XP, O_w += P2_w V_w
  f32x16 acco[HPW][NT];
#pragma unroll
  for (int e = 0; e < HPW; ++e)
#pragma unroll
    for (int t = 0; t < NT; ++t) acco[e][t] = zero16();
  auto probs = [&](int kt) {   // this wave's blocks of tile kt: P2 = T2^T P into XP
    const char* xs = XS;
    char* xp = XP;
    constexpr int G = KST && !LEAN ? 4 : (LEAN && NSU < DP / 16 ? 1 : 2);   // blocks per group: independent chains issued together
    const bool whole = kt * 32 + 32 <= a.Nk;   // every key of the tile exists (wave-uniform)
    for (int b0 = w; b0 < 32; b0 += G * NW) {
      f32x16 c[G];
#pragma unroll
      for (int u = 0; u < G; ++u) c[u] = th2_mix_img<KST>(xs, (b0 + u * NW) & 31, m1(), lane);
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int blk = b0 + u * NW;
        if (whole || kt * 32 + blk < a.Nk) {
#pragma unroll
          for (int r = 0; r < NR; ++r) c[u][r] = ex2(c[u][r] - m[r]);
        } else {   // keys past the end: P = 0
#pragma unroll
          for (int r = 0; r < NR; ++r) c[u][r] = 0.f;
        }
        if constexpr (!KST) {
#pragma unroll
          for (int r = 8; r < 16; ++r) c[u][r] = 0.f;
        }
        c[u] = th2_mix_acc<KST>(c[u], m2());
      }
#pragma unroll
      for (int u = 0; u < G; ++u)
        if (b0 + u * NW < 32) th2_put_block<NR>(xp, b0 + u * NW, c[u], H, lane);
    }
  };
  auto pv = [&]() {
#pragma unroll
    for (int e = 0; e < HPW; ++e)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = th2_colB(XP, hv[e] ? hd[e] : w, s2, lane);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acco[e][t] = MF<__bf16>::mma(I::colfrag(ldsV[e], 0, s2, 32 * t, lane), pf, acco[e][t]);
      }
  };
  // pass 1 sweeps the key tiles in reverse: the tiles pass 0 read last are the most recently used
  // in L2 (the forward's excess reads, 1.37x, turned out to be its spilled registers' scratch
  // traffic, gone with NSU 3: profiles/r06p_th_traffic.txt)
  WStage<__bf16, DP, true> vst[HPW];   // V tile kt - 1 in flight while tile kt computes (wave-private images)
#pragma unroll
  for (int e = 0; e < HPW; ++e) {
    vst[e].load_buf(rV[e], (nkt - 1) * 32, a.vs[1], a.D, lane);
    vst[e].write(ldsV[e], lane);
  }
  for (int kt = nkt - 1; kt >= 0; --kt) {
    if (kt > 0)
#pragma unroll
      for (int e = 0; e < HPW; ++e) vst[e].load_buf(rV[e], (kt - 1) * 32, a.vs[1], a.D, lane);
    scores(kt, kt > 0 ? kt - 1 : 0);
    __syncthreads();
    probs(kt);
    __syncthreads();
    pv();
    if (kt > 0)   // wave-private: after this wave's own reads
#pragma unroll
      for (int e = 0; e < HPW; ++e) vst[e].write(ldsV[e], lane);
    __syncthreads();
  }
  // O through LDS: the workgroup holds every head of its 32 queries, i.e. whole token rows of the
  // [B, N, H, D] output; staged as [query][head][d] and stored in 16-byte chunks, consecutive lanes on
  // consecutive chunks (instead of 8-byte pieces of 96-byte head rows per lane)
  {
    const int rowb = H * a.D * 2 + 16;   // bytes per staged query row (+16: spreads the rows' banks)
#pragma unroll
    for (int e = 0; e < HPW; ++e) {
      if (!hv[e]) continue;
      char* rp = smem + r32 * rowb + hd[e] * a.D * 2;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d0 = 32 * t + 8 * g + 4 * h;
          if (d0 < a.D) {
            typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
            const bf16x4 v = {(__bf16)acco[e][t][4 * g], (__bf16)acco[e][t][4 * g + 1], (__bf16)acco[e][t][4 * g + 2],
                              (__bf16)acco[e][t][4 * g + 3]};
            *reinterpret_cast<bf16x4*>(rp + d0 * 2) = v;
          }
        }
    }
    __syncthreads();
    const int cpd = a.D / 8, cpr = H * cpd;   // 16-byte chunks per head row / per query row
    const int nq = min(32, a.Nq - qb * 32);
    __bf16* const O = reinterpret_cast<__bf16*>(a.o) + b * a.os[0] + (long long)(qb * 32) * a.os[1];
    for (int c = tid; c < nq * cpr; c += 64 * NW) {
      const int r = c / cpr, rem = c - r * cpr, hh = rem / cpd, dc = rem - hh * cpd;
      const uint4 v = *reinterpret_cast<const uint4*>(smem + r * rowb + (hh * a.D + 8 * dc) * 2);
      *reinterpret_cast<uint4*>(O + (long long)r * a.os[1] + hh * a.os[2] + 8 * dc) = v;
    }
  }
}

// ============================================================================ bwd: query
// pass A: delta_i = rowsum(P_i o dP_i), dP = T2 dP2, dP2_j = dO_j V_j^T; dT2 = sum P (x) dP2.
// pass B: dS1 = P o (dP - delta), dT1 = sum S (x) dS1, dS = T1 dS1, dQ_w += scale dS_w K_w.
// LEAN (H <= 8): <= 128 VGPRs, two workgroups per CU -- mix operands in the LDS table, no K / V
// prefetch, one mix chain per group (the forward's LEAN recipe)
template <int DP, int NWMAX, bool ROT = false, int HPW = 1, bool LEAN = false, int NSU = DP / 16>
__global__ __launch_bounds__(64 * NWMAX, LEAN ? 4 : 1) void th2_bwd_q_kernel(ThArgs a) {
  static_assert(!LEAN || HPW == 1, "LEAN: one head per wave");
  using I = Img<__bf16, DP>;
  constexpr bool TAIL = DP == 64 && NSU == 3;   // dQ^T rows d 32..47 on 16 x 16 MFMAs (th2_colA16)
  constexpr int NS = NSU, NT = TAIL ? 1 : DP / 32;   // (NSU as in th2_fwd_kernel)
  constexpr bool KST = NWMAX * HPW <= 8;
  constexpr int NR = KST ? 4 : 8;
  constexpr int IMG = th2_img<KST>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H, NW = (H + HPW - 1) / HPW;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* XS = smem;
  char* XG = smem + IMG;

  const int nqb = (a.Nq + 31) / 32;
  // XCD-aware order: the query blocks of one image run on one XCD and share its K / V in L2
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = lb % nqb, b = lb / nqb;
  const int q = qb * 32 + r32;
  int hd[HPW];                              // this wave's heads (as th2_fwd_kernel)
  bool hv[HPW];
  char* ldsK[HPW];
  __amdgpu_buffer_rsrc_t rQ[HPW], rK[HPW], rV[HPW], rG[HPW];
#pragma unroll
  for (int e = 0; e < HPW; ++e) {
    hd[e] = w + NW * e;
    hv[e] = hd[e] < H;
    const int he = hv[e] ? hd[e] : w;
    ldsK[e] = smem + 2 * IMG + he * I::bytes(32);
    rQ[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + he * a.qs[2], a.Nq, a.qs[1]);
    rK[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + he * a.ks[2], a.Nk, a.ks[1]);
    rV[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + he * a.vs[2], a.Nk, a.vs[1]);
    rG[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.dout) + b * a.dos[0] + he * a.dos[2], a.Nq, a.dos[1]);
  }

  th2_zero_pad<KST>(XS, H, tid, 64 * NW);
  th2_zero_pad<KST>(XG, H, tid, 64 * NW);
  constexpr bool rot = ROT;   // rotary: q / k rotated as loaded, dq rotated back
  // (a compile-time `full` for NSU < DP / 16, as in th2_fwd_kernel, spilled 12 registers here vs 4;
  // re-reading the dO fragments per tile instead of holding them: no spills but 508 vs 474 us)
  const bool full = a.D > 16 * (NS - 1);
  bf16x8 qf[HPW][NS], gf[HPW][NS];
#pragma unroll
  for (int e = 0; e < HPW; ++e)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qf[e][s] = th2_frag(rQ[e], q, a.qs[1], a.D, s, h);
      if (rot) qf[e][s] = rope8<1>(qf[e][s], a.rope, q, 16 * s + 8 * h);
      gf[e][s] = th2_frag(rG[e], q, a.dos[1], a.D, s, h);
    }
  // the mix operands: registers (one head per wave) or, with two heads per wave, an LDS table that
  // wave 0 writes before the first barrier (the registers go to the second head's operands)
  Th2Mix m1r, m2tr, m1tr;
  char* const mxt = smem + 2 * IMG + H * I::bytes(32);
  constexpr bool MXR = HPW == 1 && !LEAN;   // mix operands held in registers
  if constexpr (MXR) {
    m1r = th2_mix<false, false, KST>(a.th1, H, lane, kLog2e);   // S1 = T1^T S, log2 domain (image)
    m2tr = th2_mix<true, false, KST>(a.th2, H, lane);    // dP = T2 dP2        (image)
    m1tr = th2_mix<true, true, KST>(a.th1, H, lane);     // dS = T1 dS1        (accumulator)
  } else if (w == 0) {
    th2_mx_put(mxt, 3, 0, lane, th2_mix<false, false, KST>(a.th1, H, lane, kLog2e));
    th2_mx_put(mxt, 3, 1, lane, th2_mix<true, false, KST>(a.th2, H, lane));
    th2_mx_put(mxt, 3, 2, lane, th2_mix<true, true, KST>(a.th1, H, lane));
  }
  auto m1 = [&]() -> Th2Mix { if constexpr (MXR) return m1r; else return th2_mx_get(mxt, 3, 0, lane); };
  auto m2t = [&]() -> Th2Mix { if constexpr (MXR) return m2tr; else return th2_mx_get(mxt, 3, 1, lane); };
  auto m1t = [&]() -> Th2Mix { if constexpr (MXR) return m1tr; else return th2_mx_get(mxt, 3, 2, lane); };
  // lse (log2 domain) of the mixed rows of this lane's query, register r <-> head row_of(r, h)
  float lse2[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int i = row_of(r, h);
    lse2[r] = (i < H && q < a.Nq) ? a.lse[((size_t)b * H + i) * a.Nq + q] * kLog2e : kInf;
  }
  const int nkt = (a.Nk + 31) / 32;
  // next key tile's K / V fragments, in flight while this one computes (one head per wave: with
  // two, the registers go to the second head's operands instead and the loads are direct)
  constexpr bool PF = HPW == 1 && !LEAN;
  bf16x8 kn[NS], vn[NS];
  auto load_kv = [&](int e, int kt) {
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
      kn[s_] = th2_frag(rK[e], kt * 32 + r32, a.ks[1], a.D, s_, h);
      vn[s_] = th2_frag(rV[e], kt * 32 + r32, a.vs[1], a.D, s_, h);
    }
  };
  // S_h -> XS, dP2_h -> XG for this wave's heads; stage_k: the (rotated) K fragments also form the
  // head's K image, the dQ product's operand (key rows, the WStage layout)
  auto tiles = [&](int kt, bool stage_k) {
    if constexpr (LEAN) {   // one operand set and one accumulator live at a time: K -> S, then V -> dP2
      f32x16 s = zero16();
      {
        bf16x8 kc[NS];
#pragma unroll
        for (int s_ = 0; s_ < NS; ++s_) {
          kc[s_] = th2_frag(rK[0], kt * 32 + r32, a.ks[1], a.D, s_, h);
          if (rot) kc[s_] = rope8<1>(kc[s_], a.rope, kt * 32 + r32, 16 * s_ + 8 * h);
        }
        if (stage_k)
#pragma unroll
          for (int s_ = 0; s_ < DP / 16; ++s_)   // (columns past NSU k-steps: zero)
            *reinterpret_cast<bf16x8*>(ldsK[0] + r32 * (DP * 2) + 16 * ((2 * s_ + h) ^ swz<DP>(r32))) =
                s_ < NS ? kc[s_ < NS ? s_ : 0] : bf16x8{};
#pragma unroll
        for (int s_ = 0; s_ < NS; ++s_)
          if (s_ < NS - 1 || full) s = MF<__bf16>::mma(qf[0][s_], kc[s_], s);
      }
      if (hv[0]) th2_put(XS, hd[0], s, a.scale, lane);
      f32x16 g = zero16();
      {
        bf16x8 vc[NS];
#pragma unroll
        for (int s_ = 0; s_ < NS; ++s_) vc[s_] = th2_frag(rV[0], kt * 32 + r32, a.vs[1], a.D, s_, h);
#pragma unroll
        for (int s_ = 0; s_ < NS; ++s_)
          if (s_ < NS - 1 || full) g = MF<__bf16>::mma(gf[0][s_], vc[s_], g);
      }
      if (hv[0]) th2_put(XG, hd[0], g, 1.f, lane);
      return;
    }
#pragma unroll
    for (int e = 0; e < HPW; ++e) {
      if constexpr (!PF) load_kv(e, kt);
      bf16x8 kc[NS], vc[NS];
#pragma unroll
      for (int s_ = 0; s_ < NS; ++s_) {
        kc[s_] = rot ? rope8<1>(kn[s_], a.rope, kt * 32 + r32, 16 * s_ + 8 * h) : kn[s_];
        vc[s_] = vn[s_];
      }
      if constexpr (PF) load_kv(0, kt + 1 < nkt ? kt + 1 : 0);
      if (stage_k)
#pragma unroll
        for (int s_ = 0; s_ < DP / 16; ++s_)   // (columns past NSU k-steps: zero)
          *reinterpret_cast<bf16x8*>(ldsK[e] + r32 * (DP * 2) + 16 * ((2 * s_ + h) ^ swz<DP>(r32))) =
              s_ < NS ? kc[s_ < NS ? s_ : 0] : bf16x8{};
      f32x16 s = zero16(), g = zero16();
#pragma unroll
      for (int s_ = 0; s_ < NS; ++s_) {
        if (s_ < NS - 1 || full) {   // S^T, dP2^T: query rows, key lanes
          s = MF<__bf16>::mma(qf[e][s_], kc[s_], s);
          g = MF<__bf16>::mma(gf[e][s_], vc[s_], g);
        }
      }
      if (hv[e]) {
        th2_put(XS, hd[e], s, a.scale, lane);
        th2_put(XG, hd[e], g, 1.f, lane);
      }
    }
  };
  if constexpr (PF) load_kv(0, 0);

  // ---- pass A
  float dl[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) dl[r] = 0.f;
  f32x4 dt2 = {0.f, 0.f, 0.f, 0.f};
  for (int kt = 0; kt < nkt; ++kt) {
    tiles(kt, false);
    __syncthreads();
    constexpr int G = LEAN ? 1 : 2;   // blocks per group: independent chains issued together
    for (int b0 = w; b0 < 32 && kt * 32 + b0 < a.Nk; b0 += G * NW) {
      f32x16 p[G], dp[G];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        p[u] = th2_mix_img<KST>(XS, (b0 + u * NW) & 31, m1(), lane);
        dp[u] = th2_mix_img<KST>(XG, (b0 + u * NW) & 31, m2t(), lane);
      }
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int blk = b0 + u * NW;
        const bool ok = blk < 32 && kt * 32 + blk < a.Nk;   // (wave-uniform)
        if (ok) {
#pragma unroll
          for (int r = 0; r < NR; ++r) {
            p[u][r] = ex2(p[u][r] - lse2[r]);   // (S1 in the log2 domain: T1 carries log2 e)
            dl[r] += p[u][r] * dp[u][r];
          }
          th2_put_block<NR>(XS, blk, p[u], H, lane);   // P over S at this block (only this wave touches it)
          dt2 = th2_dt<KST>(XS, XG, blk, dt2, lane);   // dT2[h][i] += sum P_h dP2_i
        }
      }
    }
    __syncthreads();
  }
  // delta: sum of the per-wave partials (scratch [w][r][lane]) -> registers + workspace
  {
    float* st = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int r = 0; r < NR; ++r) st[(w * NR + r) * 64 + lane] = dl[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      float s = 0.f;
      for (int ww = 0; ww < NW; ++ww) s += st[(ww * NR + r) * 64 + lane];
      dl[r] = s;
      const int i = row_of(r, h);
      if (w == 0 && i < H && q < a.Nq) a.delta[((size_t)b * H + i) * a.Nq + q] = s;
    }
    __syncthreads();
  }
  float* pb = a.part + (size_t)blockIdx.x * 2 * H * H;
  th2_dt_store(reinterpret_cast<float*>(smem), dt2, pb + H * H, H, NW, w, lane, tid, false);
  th2_zero_pad<KST>(XS, H, tid, 64 * NW);
  th2_zero_pad<KST>(XG, H, tid, 64 * NW);   // (the last tile of pass A prefetched key tile 0)

  // ---- pass B
  f32x16 adq[HPW][NT];
  f32x4 adqt[HPW][2];   // TAIL: d 32..47, queries 16 bb + (lane & 15)
#pragma unroll
  for (int e = 0; e < HPW; ++e) {
#pragma unroll
    for (int t = 0; t < NT; ++t) adq[e][t] = zero16();
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) adqt[e][bb] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x4 dt1 = {0.f, 0.f, 0.f, 0.f};
  for (int kt = 0; kt < nkt; ++kt) {
    tiles(kt, true);   // (wave-private K images: after this wave's previous dQ reads)
    __syncthreads();
    constexpr int G = HPW == 1 && !LEAN ? 2 : 1;   // (two heads per wave / LEAN: one chain, the registers are short)
    for (int b0 = w; b0 < 32; b0 += G * NW) {
      f32x16 ds1[G], dp[G];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        ds1[u] = th2_mix_img<KST>(XS, (b0 + u * NW) & 31, m1(), lane);
        dp[u] = th2_mix_img<KST>(XG, (b0 + u * NW) & 31, m2t(), lane);
      }
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int blk = b0 + u * NW;
        const bool ok = kt * 32 + blk < a.Nk;   // keys past the end: dS = 0 (wave-uniform)
        if (ok) {
#pragma unroll
          for (int r = 0; r < NR; ++r) ds1[u][r] = ex2(ds1[u][r] - lse2[r]) * (dp[u][r] - dl[r]);
        } else {
#pragma unroll
          for (int r = 0; r < NR; ++r) ds1[u][r] = 0.f;
        }
        if constexpr (!KST) {
#pragma unroll
          for (int r = 8; r < 16; ++r) ds1[u][r] = 0.f;
        }
        if (blk < 32) {
          th2_put_block<NR>(XG, blk, ds1[u], H, lane);   // dS1 over dP2 at this block
          if (ok) dt1 = th2_dt<KST>(XS, XG, blk, dt1, lane);   // dT1[h][i] += sum S_h dS1_i
          th2_put_block<NR>(XS, blk, th2_mix_acc<KST>(ds1[u], m1t()), H, lane);   // dS_h over S_h
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < HPW; ++e)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 sf = th2_colB(XS, hv[e] ? hd[e] : w, s2, lane);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          adq[e][t] = MF<__bf16>::mma(I::colfrag(ldsK[e], 0, s2, 32 * t, lane), sf, adq[e][t]);
      }
    if constexpr (TAIL) {
#pragma unroll
      for (int e = 0; e < HPW; ++e) {
        const bf16x8 at = th2_colA16<DP>(ldsK[e], 32, lane);
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
          adqt[e][bb] = mfma16(at, th2_colB16(XS, hv[e] ? hd[e] : w, bb, lane), adqt[e][bb]);
      }
    }
    __syncthreads();
  }
  // dT1 partial: XS held the SCALED scores (S = scale q k, the reference's logits)
  th2_dt_store(reinterpret_cast<float*>(smem), dt1, pb, H, NW, w, lane, tid, false);
  if (q < a.Nq) {
    const float sc = a.scale;
#pragma unroll
    for (int e = 0; e < HPW; ++e) {
      if (!hv[e]) continue;
      __bf16* DQ = reinterpret_cast<__bf16*>(a.dq) + b * a.dqs[0] + hd[e] * a.dqs[2] + (long long)q * a.dqs[1];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 32 * t + 8 * g4 + 4 * h;
          float x[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) x[c] = (float)(__bf16)(adq[e][t][4 * g4 + c] * sc);
          if (rot && d0 < a.D) rope_pairs<2, -1>(x, a.rope, q, d0 / 2);
          store4<__bf16, true>(DQ, d0, a.D, x[0], x[1], x[2], x[3]);
        }
    }
  }
  if constexpr (TAIL) {   // query 16 bb + (lane & 15), d 32 + 4 (lane >> 4) .. + 3
#pragma unroll
    for (int e = 0; e < HPW; ++e) {
      if (!hv[e]) continue;
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) {
        const int qq = qb * 32 + 16 * bb + (lane & 15), d0 = 32 + 4 * (lane >> 4);
        if (qq >= a.Nq) continue;
        __bf16* DQ = reinterpret_cast<__bf16*>(a.dq) + b * a.dqs[0] + hd[e] * a.dqs[2] + (long long)qq * a.dqs[1];
        float x[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) x[c] = (float)(__bf16)(adqt[e][bb][c] * a.scale);
        if (rot && d0 < a.D) rope_pairs<2, -1>(x, a.rope, qq, d0 / 2);
        store4<__bf16, true>(DQ, d0, a.D, x[0], x[1], x[2], x[3]);
      }
    }
  }
}

// =============================================================================== bwd: kv
// One 32-key block for all heads, sweeping the query tiles: P2 = T2^T P and dS = T1 dS1 per tile
// (same mixes), dV_w^T += dO_w^T P2_w, dK_w^T += scale Q_w^T dS_w.  The score tiles keep the key
// on the accumulator rows and the query on the lane, so image position = key * 32 + query and the
// per-head operands read query runs of a key: plain 16-byte row reads.
// HPW = 2 (9..16 heads, eight waves of <= 256 registers): each wave keeps the dK / dV accumulators
// of its two heads; the key block's K / V fragments are re-read per query tile (L2-resident, 4 KiB
// per head) instead of held, and the dO / Q tiles go through one staging buffer per head.
// (NSU 3 with the 16 x 16 head-dim tail, as in the query pass, measured level here: 230.4 vs
// 229.9 us, 206 vs 226 VGPRs at the same occupancy -- profiles/r06u_th_tail_ab.txt)
template <int DP, int NWMAX, bool ROT = false, int HPW = 1>
__global__ __launch_bounds__(64 * NWMAX) void th2_bwd_kv_kernel(ThArgs a) {
  using I = Img<__bf16, DP>;
  constexpr int NS = DP / 16, NT = DP / 32;
  constexpr bool KST = NWMAX * HPW <= 8;
  constexpr int NR = KST ? 4 : 8;
  constexpr int IMG = th2_img<KST>();
  constexpr bool KVR = HPW == 1;   // K / V fragments held in registers for the whole sweep
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H, NW = (H + HPW - 1) / HPW;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* XS = smem;
  char* XG = smem + IMG;
  char* MX = smem + 2 * IMG;   // the four mix operands, per lane (registers are short here)

  const int nkb = (a.Nk + 31) / 32;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);   // the key blocks of one image on one XCD
  const int kb = lb % nkb, b = lb / nkb;
  const int key = kb * 32 + r32;
  // per-wave dO / Q tiles: with <= 8 heads both images stay resident (the S / dP2 operands are read
  // from them and the next tile is in flight during this one); otherwise one 4 KiB buffer per head
  // (dO for dV, then Q for dK) and the S / dP2 operands come from global memory
  constexpr bool TWO = NWMAX * HPW <= 8 && HPW == 1;
  int hd[HPW];
  bool hv[HPW];
  char *buf[HPW], *bufQ[HPW];
  __amdgpu_buffer_rsrc_t rQ[HPW], rK[HPW], rV[HPW], rG[HPW];
#pragma unroll
  for (int e = 0; e < HPW; ++e) {
    hd[e] = w + NW * e;
    hv[e] = hd[e] < H;
    const int he = hv[e] ? hd[e] : w;
    buf[e] = MX + kTh2MixTbl + he * I::bytes(32);
    bufQ[e] = TWO ? buf[e] + NWMAX * I::bytes(32) : buf[e];
    rQ[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + he * a.qs[2], a.Nq, a.qs[1]);
    rK[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + he * a.ks[2], a.Nk, a.ks[1]);
    rV[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + he * a.vs[2], a.Nk, a.vs[1]);
    rG[e] = row_rsrc(reinterpret_cast<const __bf16*>(a.dout) + b * a.dos[0] + he * a.dos[2], a.Nq, a.dos[1]);
  }

  th2_zero_pad<KST>(XS, H, tid, 64 * NW);
  th2_zero_pad<KST>(XG, H, tid, 64 * NW);
  constexpr bool rot = ROT;   // rotary: q / k rotated as loaded, dk rotated back
  const bool full = a.D > 16 * (NS - 1);
  bf16x8 kf[NS], vf[NS];   // A operands: key rows of this block (KVR: loaded once)
  auto load_kv = [&](int e) {
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
      kf[s_] = th2_frag(rK[e], key, a.ks[1], a.D, s_, h);
      if (rot) kf[s_] = rope8<1>(kf[s_], a.rope, key, 16 * s_ + 8 * h);
      vf[s_] = th2_frag(rV[e], key, a.vs[1], a.D, s_, h);
    }
  };
  if constexpr (KVR) load_kv(0);
  if (w == 0) {
    th2_mx_put(MX, 4, 0, lane, th2_mix<false, false, KST>(a.th1, H, lane, kLog2e));   // log2 e T1^T, image operand
    th2_mx_put(MX, 4, 1, lane, th2_mix<false, true, KST>(a.th2, H, lane));    // T2^T, accumulator operand
    th2_mx_put(MX, 4, 2, lane, th2_mix<true, false, KST>(a.th2, H, lane));    // T2, image operand
    th2_mx_put(MX, 4, 3, lane, th2_mix<true, true, KST>(a.th1, H, lane));     // T1, accumulator operand
  }
  auto mx = [&](int k) { return th2_mx_get(MX, 4, k, lane); };
  f32x16 adk[HPW][NT], adv[HPW][NT];
#pragma unroll
  for (int e = 0; e < HPW; ++e)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      adk[e][t] = zero16();
      adv[e][t] = zero16();
    }
  const int nqt = (a.Nq + 31) / 32;
  WStage<__bf16, DP, true> gst, qst;
  if constexpr (TWO) {
    gst.load_buf(rG[0], 0, a.dos[1], a.D, lane);
    qst.load_buf(rQ[0], 0, a.qs[1], a.D, lane);
    if (rot) qst.rope(a.rope, 0, lane);
    gst.write(buf[0], lane);
    qst.write(bufQ[0], lane);
  }
  for (int qt = 0; qt < nqt; ++qt) {
    const int q = qt * 32 + r32;
    // this tile's row constants, raw (scaled / masked where used, after the barrier), issued
    // BEFORE the next tile's Q / dO prefetch: waiting for them then leaves the prefetch in flight
    // (vmcnt counts in order; loaded after it, the wait drained the prefetch every tile)
    float lse2[NR], dl[NR];
    auto load_rows = [&]() {
      if constexpr (HPW == 1) {   // rows past H clamped (masked after the barrier)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const size_t o = ((size_t)b * H + min(row_of(r, h), H - 1)) * a.Nq + min(q, a.Nq - 1);
          lse2[r] = a.lse[o];
          dl[r] = a.delta[o];
        }
      } else {
        // one per-lane base (head 4h, query q) plus wave-uniform row offsets: the 64-bit offsets
        // per register above, hoisted out of the loop, were what spilled at two heads per wave
        const size_t base = ((size_t)b * H + 4 * h) * a.Nq + min(q, a.Nq - 1);
        const float* lrow = a.lse + base;
        const float* drow = a.delta + base;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int off = ((r & 3) + 8 * (r >> 2)) * a.Nq;   // (row_of(r, h) - 4h) Nq
          const bool in = row_of(r, h) < H;
          lse2[r] = in ? lrow[off] : 0.f;
          dl[r] = in ? drow[off] : 0.f;
        }
      }
    };
    if constexpr (TWO) load_rows();   // (no prefetch without TWO: loaded after the score tiles)
    if constexpr (TWO) {
      if (qt + 1 < nqt) {
        gst.load_buf(rG[0], (qt + 1) * 32, a.dos[1], a.D, lane);
        qst.load_buf(rQ[0], (qt + 1) * 32, a.qs[1], a.D, lane);
      }
    }
#pragma unroll
    for (int e = 0; e < HPW; ++e) {
      if constexpr (!TWO) gst.load_buf(rG[e], qt * 32, a.dos[1], a.D, lane);
      if constexpr (!KVR) load_kv(e);
      f32x16 s = zero16(), g = zero16();
#pragma unroll
      for (int s_ = 0; s_ < NS; ++s_) {
        bf16x8 qa, ga;
        if constexpr (TWO) {
          qa = I::rowfrag(bufQ[0], r32, s_, h);
          ga = I::rowfrag(buf[0], r32, s_, h);
        } else {
          qa = th2_frag(rQ[e], q, a.qs[1], a.D, s_, h);
          if (rot) qa = rope8<1>(qa, a.rope, q, 16 * s_ + 8 * h);
          ga = th2_frag(rG[e], q, a.dos[1], a.D, s_, h);
        }
        if (s_ < NS - 1 || full) {   // query rows, key lanes (th2_put)
          s = MF<__bf16>::mma(qa, kf[s_], s);
          g = MF<__bf16>::mma(ga, vf[s_], g);
        }
      }
      if (hv[e]) {
        th2_put(XS, hd[e], s, a.scale, lane);
        th2_put(XG, hd[e], g, 1.f, lane);
      }
      if constexpr (!TWO) gst.write(buf[e], lane);
    }
    if constexpr (!TWO) load_rows();
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const bool ok = row_of(r, h) < H && q < a.Nq;
      lse2[r] = ok ? lse2[r] * kLog2e : kInf;
      dl[r] = ok ? dl[r] : 0.f;
    }
    constexpr int G = HPW == 1 ? 2 : 1;   // blocks (keys) per group: independent chains issued together
    for (int b0 = w; b0 < 32; b0 += G * NW) {
      f32x16 p[G], dp[G];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        p[u] = th2_mix_img<KST>(XS, (b0 + u * NW) & 31, mx(0), lane);
        dp[u] = th2_mix_img<KST>(XG, (b0 + u * NW) & 31, mx(2), lane);
      }
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int blk = b0 + u * NW;   // blk = key of this block
        const bool ok = kb * 32 + blk < a.Nk;   // keys past the end: P2 = dS = 0 (wave-uniform)
        if (ok) {
#pragma unroll
          for (int r = 0; r < NR; ++r) {   // dp[u] becomes dS1 in place
            p[u][r] = ex2(p[u][r] - lse2[r]);
            dp[u][r] = p[u][r] * (dp[u][r] - dl[r]);
          }
        } else {
#pragma unroll
          for (int r = 0; r < NR; ++r) p[u][r] = dp[u][r] = 0.f;
        }
        if constexpr (!KST) {
#pragma unroll
          for (int r = 8; r < 16; ++r) {
            p[u][r] = 0.f;
            dp[u][r] = 0.f;
          }
        }
        if (blk < 32) {
          th2_put_block<NR>(XS, blk, th2_mix_acc<KST>(p[u], mx(1)), H, lane);       // P2_h over S_h at this key
          th2_put_block<NR>(XG, blk, th2_mix_acc<KST>(dp[u], mx(3)), H, lane);  // dS_h over dP2_h
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < HPW; ++e) {
      const int he = hv[e] ? hd[e] : w;
      if constexpr (!TWO) qst.load_buf(rQ[e], qt * 32, a.qs[1], a.D, lane);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pf = th2_rowB(XS, he, s2, lane);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          adv[e][t] = MF<__bf16>::mma(I::colfrag(buf[e], 0, s2, 32 * t, lane), pf, adv[e][t]);
      }

      if constexpr (!TWO) {   // one buffer: Q after this wave's own dO reads
        if (rot) qst.rope(a.rope, qt * 32, lane);
        qst.write(bufQ[e], lane);
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 sf = th2_rowB(XG, he, s2, lane);
#pragma unroll
        for (int t = 0; t < NT; ++t)
          adk[e][t] = MF<__bf16>::mma(I::colfrag(bufQ[e], 0, s2, 32 * t, lane), sf, adk[e][t]);
      }

    }
    if constexpr (TWO) {
      if (qt + 1 < nqt) {   // wave-private images: after this wave's own reads
        if (rot) qst.rope(a.rope, (qt + 1) * 32, lane);
        gst.write(buf[0], lane);
        qst.write(bufQ[0], lane);
      }
    }
    __syncthreads();
  }
  if (key < a.Nk) {
    const float sc = a.scale;
#pragma unroll
    for (int e = 0; e < HPW; ++e) {
      if (!hv[e]) continue;
      __bf16* DK = reinterpret_cast<__bf16*>(a.dk) + b * a.dks[0] + hd[e] * a.dks[2] + (long long)key * a.dks[1];
      __bf16* DV = reinterpret_cast<__bf16*>(a.dv) + b * a.dvs[0] + hd[e] * a.dvs[2] + (long long)key * a.dvs[1];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 32 * t + 8 * g4 + 4 * h;
          float x[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) x[c] = (float)(__bf16)(adk[e][t][4 * g4 + c] * sc);
          if (rot && d0 < a.D) rope_pairs<2, -1>(x, a.rope, key, d0 / 2);
          store4<__bf16, true>(DK, d0, a.D, x[0], x[1], x[2], x[3]);
          store4<__bf16, true>(DV, d0, a.D, adv[e][t][4 * g4], adv[e][t][4 * g4 + 1], adv[e][t][4 * g4 + 2],
                               adv[e][t][4 * g4 + 3]);
        }
    }
  }
}

// LDS: two exchange images + per-head 32-row staging (two per head in th2_bwd_kv at <= 8 waves);
// th2_bwd_q with two heads per wave adds its mix-operand table (3 x 64 lanes x 32 bytes)
// (th2_fwd LEAN: its two mix operands, 2 x 64 lanes x 32 bytes)
template <int DP, bool KST> constexpr size_t th2_lds_bytes(int H, int hpw = 1, bool lean = false) {
  return 2 * (size_t)th2_img<KST>() + (size_t)H * Img<__bf16, DP>::bytes(32) + (hpw > 1 ? 3 * 64 * 32 : 0) +
         (lean ? 2 * 64 * 32 : 0);
}

template <int DP, bool KST> constexpr size_t th2_kv_lds_bytes(int H, bool two_buffers) {
  return 2 * (size_t)th2_img<KST>() + kTh2MixTbl + (size_t)(two_buffers ? 16 : H) * Img<__bf16, DP>::bytes(32);
}

}  // namespace sae
