// fwd2.h -- lean bf16 forward attention for gfx950 (the hot path of every ViT/DeiT/CaiT layer).
//
// Same algorithm and layout as attn_fwd_kernel (attn_kernels.h; reference chain
// models/layers/attentions/attention.py:39-58), re-built around the VALU budget of one
// 32x32 score tile, which is what bounds a D <= 64 attention forward on CDNA4:
//   * every per-tile address is precomputed once per thread: global offsets are 32-bit buffer
//     offsets (hardware range check = zero fill for tail rows / padded head-dim columns), LDS
//     read/write addresses are VGPR + immediate, the K/V tile loop is unrolled over the two
//     LDS buffers so buffer selection is an immediate as well;
//   * the softmax row sum l runs on the matrix pipe: an all-ones A operand turns the P^T fed
//     to O^T = V^T P^T into one more MFMA per 16 keys whose accumulator rows are sum_k P
//     (the 32 f32 adds per tile it replaces are the single largest VALU item after exp);
//   * the running max uses v_max3 and one v_permlane32_swap for the lane-half exchange;
//   * lazy rescale (T13, threshold 2^8) decided wave-uniformly before any P of the tile is
//     exponentiated, as in the v1 kernel.
// One wave owns 32 query rows (query on the MFMA lane, "swapped" S^T = K Q^T), NW waves share
// each 64-key K/V tile staged global -> registers -> LDS (issue early, write late; one barrier
// per tile).
#pragma once
#include <type_traits>

#include "common.h"

namespace sae {

template <int DP> struct F2 {
  static constexpr int NS = DP / 16;        // bf16 k-steps over the head dim
  static constexpr int NT = DP / 32;        // 32-row tiles of O^T
  static constexpr int CPR = DP / 8;        // 16-byte chunks per row
  static constexpr int TILE = 64 * DP * 2;  // bytes of one 64-key image
};

__device__ __forceinline__ float xhalf_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// pairwise sum of the 16 accumulator values of a 32 x 32 tile
__device__ __forceinline__ float f2_tree16(const f32x16& x) {
  const float a0 = (x[0] + x[1]) + (x[2] + x[3]), a1 = (x[4] + x[5]) + (x[6] + x[7]);
  const float a2 = (x[8] + x[9]) + (x[10] + x[11]), a3 = (x[12] + x[13]) + (x[14] + x[15]);
  return (a0 + a1) + (a2 + a3);
}

__device__ __forceinline__ float xhalf_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// BoTNet relative logits on the matrix pipe (REL, botnet.py:191-192 in the index-map form of
// sae_attn.h): bias_h[q][k / Ws] + bias_w[q][k % Ws] is the dot product of a per-query row
// [bias_h[q][0 .. Hs) | bias_w[q][0 .. Ws) | 0] / scale (bf16) with a per-key one-hot row (1 at
// k / Ws and at Hs + k % Ws), i.e. two more 16-deep k-steps of the score MFMA (Hs + Ws <= 32) in
// place of two gathers and two adds per score on the VALU.  The one-hot rows of a 64-key tile
// are a [64][32] bf16 image (64-byte rows, swz<32>) generated while the tile is staged; the
// dQ pass also reads it transposed, as the A operand of dbias^T = onehot^T dS^T.
constexpr int kRelCols = 32;
constexpr int kRelImg = 64 * kRelCols * 2;

// one-hot row of `key`, columns 8c .. 8c + 7 (zero past Nk)
__device__ __forceinline__ uint4 rel_onehot8(const AttnArgs& a, int key, int c) {
  unsigned m = 0;
  if (key < a.Nk) {
    const int kx = (key * a.rel_magic) >> 20;
    m = (1u << kx) | (1u << (a.rel_h + key - kx * a.rel_w));
  }
  const unsigned b = m >> (8 * c);
  uint4 r;
  r.x = ((b & 1u) ? 0x3F80u : 0u) | ((b & 2u) ? 0x3F800000u : 0u);
  r.y = ((b & 4u) ? 0x3F80u : 0u) | ((b & 8u) ? 0x3F800000u : 0u);
  r.z = ((b & 16u) ? 0x3F80u : 0u) | ((b & 32u) ? 0x3F800000u : 0u);
  r.w = ((b & 64u) ? 0x3F80u : 0u) | ((b & 128u) ? 0x3F800000u : 0u);
  return r;
}

// query-bias row of score row `row` = (b H + h) Nq + q, columns 8c .. 8c + 7, times inv (1 / scale)
__device__ __forceinline__ uint4 rel_qrow8(const AttnArgs& a, size_t row, bool ok, int c, float inv) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = 8 * c + j;
    float v = 0.f;
    if (ok && col < a.rel_h) v = a.bias_h[row * a.rel_h + col];
    else if (ok && col < a.rel_h + a.rel_w) v = a.bias_w[row * a.rel_w + col - a.rel_h];
    r[j] = (__bf16)(v * inv);
  }
  return __builtin_bit_cast(uint4, r);
}

// the one-hot image of keys key0 .. key0 + 63 (threads 0 .. 255 one 16-byte chunk each)
template <int NW>
__device__ __forceinline__ void rel_put_onehot(const AttnArgs& a, char* img, int key0, int tid) {
#pragma unroll
  for (int i = 0; i < (256 + 64 * NW - 1) / (64 * NW); ++i) {
    const int id = tid + 64 * NW * i;
    if (256 % (64 * NW) == 0 || id < 256) {
      const int r = id >> 2, c = id & 3;
      *reinterpret_cast<uint4*>(img + r * 64 + 16 * (c ^ swz<32>(r))) = rel_onehot8(a, key0 + r, c);
    }
  }
}

template <int DP, int NW>
struct F2Stage {
  static constexpr int NCH = (64 * F2<DP>::CPR + 64 * NW - 1) / (64 * NW);
  unsigned goff[NCH];   // byte offset inside a tile (0x80000000 = padded column: reads zero)
  unsigned loff[NCH];   // LDS byte offset inside an image (0xffffffff = no chunk)
  uint4 v[NCH];

  __device__ __forceinline__ void init(int tid, long long rs, int D) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int id = tid + 64 * NW * i;
      const int r = id / F2<DP>::CPR, c = id % F2<DP>::CPR;
      const bool ok = id < 64 * F2<DP>::CPR;
      goff[i] = (ok && c * 8 < D) ? (unsigned)(((long long)r * rs + c * 8) * 2) : 0x80000000u;
      loff[i] = ok ? (unsigned)(r * DP * 2 + 16 * (c ^ swz<DP>(r))) : 0xffffffffu;
    }
  }
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, unsigned tileoff) {
#pragma unroll
    for (int i = 0; i < NCH; ++i)
      v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, goff[i] + tileoff, 0, 0));
  }
  __device__ __forceinline__ void write(char* img) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i)
      if (64 * F2<DP>::CPR % (64 * NW) == 0 || loff[i] != 0xffffffffu)
        *reinterpret_cast<uint4*>(img + loff[i]) = v[i];
  }
  // rotary on the staged chunks (rows = positions pos0 .. pos0 + 63), before write()
  __device__ __forceinline__ void rope(const RopeTab& t, int pos0, int tid) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int id = tid + 64 * NW * i;
      if (id < 64 * F2<DP>::CPR) v[i] = rope8<1>(v[i], t, pos0 + id / F2<DP>::CPR, 8 * (id % F2<DP>::CPR));
    }
  }
};

// NSU: the 16-wide k-steps of QK^T that carry head-dim columns (3 for D = 48 at DP = 64: the
// fourth would multiply zero padding)
// REL: ldsR = the tile's one-hot image, ra = this lane's row reads of it, qa = query-bias rows
// FIX: the running max stays where the first tile put it (no per-tile row max, no rescale); the
// kernel checks the row sums after the sweep and redoes the block with the tracking sweep if any
// row's sum left [1, 2^64) (a later tile's score more than 64 log2 units above the first tile's
// max).  P is fed to the MFMA in bf16, whose relative precision does not depend on magnitude,
// so the result is that of the tracking sweep up to fp32 summation order.
// PSC: the query fragments arrive pre-scaled by scale * log2 e (bf16), so the scores come out of
// the MFMA in the log2 domain; with FIX the score chains of every tile after the first start from
// C = -m (the fixed running max, `cneg`), so the exponent is the accumulator itself: no per-score
// FMA on the VALU (the tile's largest VALU item after exp).
template <int DP, int NW, bool LSUM, bool FIRST, int NSU = F2<DP>::NS, bool REL = false, bool FIX = false,
          bool PSC = false>
__device__ __forceinline__ void fwd2_tile(const char* ldsK, const char* ldsV, const bf16x8* qf, f32x16* acco,
                                          f32x16& lacc, float& m, float& l, int nvalid, float sl2,
                                          const unsigned* ka, const unsigned* va, int h,
                                          const char* ldsR = nullptr, const unsigned* ra = nullptr,
                                          const bf16x8* qa = nullptr, const f32x16* cneg = nullptr) {
  constexpr int NS = NSU, NT = F2<DP>::NT;
  constexpr bool CIN = PSC && FIX && !FIRST;   // chains start from -m: s0 / s1 are exponents
  // nvalid: keys of this tile that exist (64 for every tile but the tail)
  const bool two = nvalid > 32;
  f32x16 s0, s1;
  if constexpr (CIN) {
    s0 = *cneg;
    s1 = *cneg;
  } else {
    s0 = zero16();
    s1 = zero16();
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const bf16x8 k0 = *reinterpret_cast<const bf16x8*>(ldsK + ka[s]);
    s0 = MF<__bf16>::mma(k0, qf[s], s0);
  }
  if constexpr (REL) {
#pragma unroll
    for (int s = 0; s < 2; ++s) s0 = MF<__bf16>::mma(*reinterpret_cast<const bf16x8*>(ldsR + ra[s]), qa[s], s0);
  }
  if (two) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bf16x8 k1 = *reinterpret_cast<const bf16x8*>(ldsK + ka[s] + 32 * DP * 2);
      s1 = MF<__bf16>::mma(k1, qf[s], s1);
    }
    if constexpr (REL) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
        s1 = MF<__bf16>::mma(*reinterpret_cast<const bf16x8*>(ldsR + ra[s] + 32 * 64), qa[s], s1);
    }
  }
  if (nvalid < 64) {   // tail tile: keys past the end score -inf (key = row_of(r, h) = c_r + 4h)
    const int nvh = nvalid - 4 * h;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = (r & 3) + 8 * (r >> 2);
      s0[r] = c < nvh ? s0[r] : -kInf;
      s1[r] = c + 32 < nvh ? s1[r] : -kInf;
    }
  }
  if constexpr (FIRST || !FIX) {
  float mx = s0[0];
#pragma unroll
  for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s0[r]);
  if (two) {
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s1[r]);
  }
  mx = PSC ? xhalf_max(mx) : xhalf_max(mx) * sl2;
  if constexpr (FIRST) {   // first tile: nothing accumulated yet, the running max starts here
    m = mx;
  } else if (!__all(mx - m <= 8.f)) {
    const float mn = fmaxf(m, mx);
    const float alpha = ex2(m - mn);
    m = mn;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acco[t][r] *= alpha;
    if constexpr (LSUM) {
#pragma unroll
      for (int r = 0; r < 16; ++r) lacc[r] *= alpha;
    } else {
      l *= alpha;
    }
  }
  }
  if constexpr (CIN) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s0[r] = ex2(s0[r]);
    if (two) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s1[r] = ex2(s1[r]);
    }
  } else if constexpr (PSC) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s0[r] = ex2(s0[r] - m);
    if (two) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s1[r] = ex2(s1[r] - m);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) s0[r] = ex2(__builtin_fmaf(s0[r], sl2, -m));
    if (two) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s1[r] = ex2(__builtin_fmaf(s1[r], sl2, -m));
    }
  }
  if constexpr (!LSUM) {
    // pairwise (depth 4 per half): a serial chain of 32 dependent adds sat on the tile's critical
    // path (round-5 ISA of the N = 577 instance)
    float ls = f2_tree16(s0);
    if (two) ls += f2_tree16(s1);
    l = FIRST ? ls : l + ls;
  }
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const bf16x8 pf = acc_frag<__bf16>(s0, s2);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const char* p1 = ldsV + va[2 * t] + 16 * s2 * DP * 2;
      const char* p2 = ldsV + va[2 * t + 1] + 16 * s2 * DP * 2;
      s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
      s16x4 x2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p2));
      typedef __attribute__((ext_vector_type(8))) short s16x8;
      s16x8 vv = {x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
      // first tile, first 16 keys: the accumulators start from the MFMA's zero C operand
      acco[t] = MF<__bf16>::mma(__builtin_bit_cast(bf16x8, vv), pf, (FIRST && s2 == 0) ? zero16() : acco[t]);
    }
    if constexpr (LSUM) lacc = MF<__bf16>::mma(ones, pf, (FIRST && s2 == 0) ? zero16() : lacc);
  }
  if (two) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 pf = acc_frag<__bf16>(s1, s2);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const char* p1 = ldsV + va[2 * t] + (32 + 16 * s2) * DP * 2;
        const char* p2 = ldsV + va[2 * t + 1] + (32 + 16 * s2) * DP * 2;
        s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
        s16x4 x2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p2));
        typedef __attribute__((ext_vector_type(8))) short s16x8;
        s16x8 vv = {x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
        acco[t] = MF<__bf16>::mma(__builtin_bit_cast(bf16x8, vv), pf, acco[t]);
      }
      if constexpr (LSUM) lacc = MF<__bf16>::mma(ones, pf, lacc);
    }
  }
}

// ROT: q and k are rotated (rotary, common.h rope8) as they are staged -- q fragments once, each
// K tile as it goes to LDS -- so the rotated tensors never exist in HBM.
// REL: BoTNet relative logits as two extra score k-steps (rel_onehot8 / rel_qrow8 above); the
// one-hot images follow the K / V buffers in LDS.
template <int DP, int NW, int MINW, bool LSUM, bool ROT = false, int NSU = DP / 16, bool REL = false,
          bool FIX = false, bool PSC = false>
__global__ __launch_bounds__(64 * NW, MINW) void attn_fwd2_kernel(AttnArgs a) {
  using FF = F2<DP>;
  constexpr int NS = NSU, NT = FF::NT, TILE = FF::TILE;
  constexpr int BQ = 32 * NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  SAE_STAMP(0);
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

  // K/V tiles staged global -> registers -> LDS: tile t + 1 is loaded while tile t computes
  // (a second register stage in flight measured no faster and costs the third wave per SIMD)
  F2Stage<DP, NW> kst, vst;
  kst.init(tid, a.ks[1], a.D);
  vst.init(tid, a.vs[1], a.D);
  const __amdgpu_buffer_rsrc_t rk = row_rsrc(K, a.Nk, a.ks[1]);
  const __amdgpu_buffer_rsrc_t rv = row_rsrc(V, a.Nk, a.vs[1]);
  const unsigned kstep = (unsigned)(64 * a.ks[1] * 2), vstep = (unsigned)(64 * a.vs[1] * 2);
  const int nkt = (a.Nk + 63) / 64;
  kst.load(rk, 0);
  vst.load(rv, 0);

  // query fragments (row q, head-dim 16s + 8h .. +7), zero past Nq / D
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
    if constexpr (PSC) {   // q * scale * log2 e, rounded to bf16 (the scores come out in log2 units)
      const float c = a.scale * kLog2e;
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[s][j] = (__bf16)((float)qf[s][j] * c);
    }
  }
  // REL: query-bias fragments (columns 16s + 8h .. + 7) and the one-hot row reads
  bf16x8 qa[2];
  unsigned ra[2];
  if constexpr (REL) {
    const size_t row = ((size_t)b * a.H + hh) * a.Nq + q;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      qa[s] = __builtin_bit_cast(bf16x8, rel_qrow8(a, row, q < a.Nq, 2 * s + h, 1.f / a.scale));
      ra[s] = r32 * 64 + 16 * ((2 * s + h) ^ swz<32>(r32));
    }
  }
  char* const rimg = smem + 4 * TILE;   // REL: two one-hot images
  // per-lane LDS read addresses: K rows r32 (+32 as an immediate), V^T transposed reads
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

  f32x16 acco[NT], lacc;   // written first by the peeled first tile (zero C operand)
  f32x16 cneg;             // PSC + FIX: -m, the C operand of every later tile's score chains
  float m = -kInf, l = 0.f;
  const float sl2 = a.scale * kLog2e;

  if constexpr (ROT) kst.rope(a.rope, 0, tid);
  kst.write(smem);
  vst.write(smem + TILE);
  if constexpr (REL) rel_put_onehot<NW>(a, rimg, 0, tid);
  vm_wait_all();   // Q fragments resident before the loop (see vm_wait_all)
  __syncthreads();
  SAE_STAMP(1);
  // one K/V tile: load t + 1, compute t from LDS buffer BSEL, stage t + 1 into the other
  // buffer, barrier.  Buffer selection and the peeled first tile are compile-time, so the
  // first tile's zero accumulators become the MFMA's C operand and its rescale disappears.
  auto step = [&](int t, auto bsel_c, auto first_c, auto compute_c, auto fix_c) {
    constexpr int bsel = decltype(bsel_c)::value;
    char* cur = smem + bsel * 2 * TILE;
    char* nxt = smem + (bsel ^ 1) * 2 * TILE;
    if (t + 1 < nkt) {
      kst.load(rk, (unsigned)(t + 1) * kstep);
      vst.load(rv, (unsigned)(t + 1) * vstep);
    }
    if constexpr (decltype(compute_c)::value) {
      fwd2_tile<DP, NW, LSUM, decltype(first_c)::value, NSU, REL, decltype(fix_c)::value, PSC>(
          cur, cur + TILE, qf, acco, lacc, m, l, min(64, a.Nk - 64 * t), sl2, ka, va, h, rimg + bsel * kRelImg, ra,
          qa, &cneg);
      if constexpr (PSC && decltype(first_c)::value) {
#pragma unroll
        for (int r = 0; r < 16; ++r) cneg[r] = -m;
      }
    }
    if (t + 1 < nkt) {
      if constexpr (ROT) kst.rope(a.rope, 64 * (t + 1), tid);
      kst.write(nxt);
      vst.write(nxt + TILE);
      if constexpr (REL) rel_put_onehot<NW>(a, rimg + (bsel ^ 1) * kRelImg, 64 * (t + 1), tid);
    }
    __syncthreads();
    SAE_STAMP(2 + (t < 27 ? t : 27));
  };
  auto sweep = [&](auto compute_c, auto fix_c) {
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    step(0, B0{}, std::true_type{}, compute_c, fix_c);
    for (int t = 1; t < nkt; t += 2) {
      step(t, B1{}, std::false_type{}, compute_c, fix_c);
      if (t + 1 < nkt) step(t + 1, B0{}, std::false_type{}, compute_c, fix_c);
    }
  };
  // waves past the last query row only stage tiles and meet the barriers
  if (active) sweep(std::true_type{}, std::bool_constant<FIX>{});
  else sweep(std::false_type{}, std::bool_constant<FIX>{});
  if constexpr (FIX) {   // a row whose sum left [1, 2^64): redo the block with the tracking sweep
    const float lt0 = LSUM ? lacc[0] : xhalf_sum(l);
    if (__syncthreads_or(active && q < a.Nq && !(lt0 < 0x1p64f))) {
      kst.load(rk, 0);
      vst.load(rv, 0);
      if constexpr (ROT) kst.rope(a.rope, 0, tid);
      kst.write(smem);
      vst.write(smem + TILE);
      if constexpr (REL) rel_put_onehot<NW>(a, rimg, 0, tid);
      vm_wait_all();
      __syncthreads();
      if (active) sweep(std::true_type{}, std::false_type{});
      else sweep(std::false_type{}, std::false_type{});
    }
  }

  SAE_STAMP(30);
  if (!active) return;
  float lt;
  if constexpr (LSUM) lt = lacc[0];
  else lt = xhalf_sum(l);
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
  SAE_STAMP(31);
}

}  // namespace sae
