// gemm_nt.h -- forward / input-gradient GEMMs of the projections and the FF block, with the
// FF block's tanh-GELU and its derivative fused into the epilogue.
//
//   c[m][n] = epi( sum_k a[m][k] * bt[n][k] (+ bias[n]) )
//
// a [M][K] bf16 (tokens, row stride lda), bt [N][K] bf16 (output features, row stride ldb): both
// operands are K-contiguous ("NT").  The forward of a Flax Dense (kernel [in, out]) passes the
// transposed bf16 kernel copy; its input gradient dX = dY W^T passes the kernel as it is.
// Epilogues (ff.py:8-34: Dense -> nn.gelu (tanh form) -> Dense):
//   kEpiNone : c = bf16(acc + bias)
//   kEpiGelu : c2 = h = bf16(acc + bias) (saved for the backward), c = bf16(gelu(h))
//   kEpiDGelu: c = bf16(bf16(acc) * gelu'(aux))   (aux = the saved h; the FF block's dH)
// with NtArgs::gp set (the C ABI's SAE_EPI_GELU_GRAD / SAE_EPI_MUL_AUX, the FF block's pair) the
// forward saves g = bf16(gelu'(h)) instead of h (same sigmoid, a few more packed FMAs) and the
// backward epilogue is one multiply, c = bf16(bf16(acc) * g): the sigmoid / rcp work of GELU'
// leaves the input-gradient GEMM, whose epilogue bounded it.
// which removes the two elementwise HBM passes (GELU forward, GELU backward) per FF block.
//
// Structure (gfx950): a 128 x 128 output tile per 256-thread workgroup, 4 waves of 64 x 64 (2 x 2
// v_mfma_f32_32x32x16_bf16 accumulators); BK-deep K stages staged global -> registers -> LDS
// ([128 rows][BK k] images, rows XOR-swizzled per row: conflict-free ds_read_b128), two LDS
// buffers, loads issued two stages ahead.  BK = 64 (64 KiB of LDS, 2 workgroups per CU) by
// default; BK = 32 (32 KiB, 3-4 workgroups per CU) for the GELU / GELU' epilogues at K <= 384,
// where more resident tiles let one tile's epilogue VALU run under other tiles' MFMAs.  The MFMA runs with the output feature as the
// accumulator row and the token on the lane, so the epilogue writes each token's features as
// packed bf16x4 into a per-wave LDS image and stores whole 128-byte row segments.
// XCD-aware order: the N tiles of one token block are consecutive on one XCD (the token rows are
// fetched from HBM once per XCD; the small weight stays L2-resident).
#pragma once
#include "common.h"

namespace sae {

enum { kEpiNone = 0, kEpiGelu = 1, kEpiDGelu = 2 };

struct NtArgs {
  const __bf16* a;     // [M][K], row stride lda
  const __bf16* bt;    // [N][K], row stride ldb
  const float* bias;   // [N] or null
  const __bf16* aux;   // [M][N] row stride ldaux (kEpiDGelu)
  __bf16* c;           // [M][N] row stride ldc
  __bf16* c2;          // [M][N] row stride ldc (kEpiGelu: pre-activation)
  int M, N, K;
  long long lda, ldb, ldc, ldaux;
  PatchGeom pg;        // patch-embedding A operand (patch.h), unused otherwise
  int gp;              // kEpiGelu: c2 = gelu'(h) instead of h; kEpiDGelu: aux holds gelu'(h)
  unsigned* ctr;       // gemm8 dynamic tile walk: {ticket, done} counters of this launch's slot
  int nts;             // gemm8: 1 = epilogue stores non-temporal (streamed past L2's normal
                       // allocation), 2 = the gelu' aux tile loaded non-temporal
};

constexpr int kNtT = 128;   // output tile edge
constexpr int kNtK = 64;    // K per stage

// tanh-GELU (Flax nn.gelu default; torch approximate="tanh"): 0.5 x (1 + tanh(y)),
// y = sqrt(2/pi) (x + 0.044715 x^3) = x * sigmoid(2y)
constexpr float kGeluB = 0.7978845608028654f;
constexpr float kGeluK = 0.044715f;

__device__ __forceinline__ float gelu_sig(float x) {   // sigmoid(2y)
  const float y2 = x * (kGeluB + (kGeluB * kGeluK) * x * x);
  return __builtin_amdgcn_rcpf(1.f + ex2(-2.f * kLog2e * y2));
}
__device__ __forceinline__ float gelu_f(float x) { return x * gelu_sig(x); }
__device__ __forceinline__ float dgelu_f(float x) {
  const float s = gelu_sig(x);
  return s + 2.f * x * s * (1.f - s) * (kGeluB + (3.f * kGeluB * kGeluK) * x * x);
}

// The epilogues on pairs of elements: the polynomial / sigmoid algebra in packed f32
// (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32: two elements per VALU issue), the two
// transcendentals per element scalar.  A bf16 pair is one 32-bit word: lo = w << 16, hi = w & ~0xffff.
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ __forceinline__ f32x2 bf2_to_f2(unsigned w) {
  return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
__device__ __forceinline__ unsigned f2_to_bf2(f32x2 v) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
  const bf16x2 b = {(__bf16)v.x, (__bf16)v.y};
  return __builtin_bit_cast(unsigned, b);
}
__device__ __forceinline__ f32x2 gelu_sig2(f32x2 x) {   // sigmoid(2y) of both elements
  constexpr float c1 = -2.f * kLog2e * kGeluB, c2 = -2.f * kLog2e * kGeluB * kGeluK;
  const f32x2 t = x * (c1 + c2 * (x * x));
  const f32x2 d = f32x2{ex2(t.x), ex2(t.y)} + 1.f;
  return f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
__device__ __forceinline__ unsigned gelu_bf2(unsigned hw) {
  const f32x2 x = bf2_to_f2(hw);
  return f2_to_bf2(x * gelu_sig2(x));
}
__device__ __forceinline__ unsigned dgelu_bf2(unsigned dw, unsigned hw) {   // d * gelu'(h)
  const f32x2 x = bf2_to_f2(hw);
  const f32x2 s = gelu_sig2(x);
  const f32x2 q = s - s * s;                                    // s (1 - s)
  const f32x2 poly = (2.f * kGeluB) + (6.f * kGeluB * kGeluK) * (x * x);
  return f2_to_bf2(bf2_to_f2(dw) * ((x * q) * poly + s));
}
// gelu(h) and gelu'(h) of a bf16 pair from one sigmoid (the gp forward epilogue)
__device__ __forceinline__ unsigned gelu_grad_bf2(unsigned hw, unsigned& gw) {
  const f32x2 x = bf2_to_f2(hw);
  const f32x2 s = gelu_sig2(x);
  const f32x2 q = s - s * s;
  const f32x2 poly = (2.f * kGeluB) + (6.f * kGeluB * kGeluK) * (x * x);
  gw = f2_to_bf2((x * q) * poly + s);
  return f2_to_bf2(x * s);
}
__device__ __forceinline__ unsigned mul_bf2(unsigned dw, unsigned gw) {   // d * g (the gp backward epilogue)
  return f2_to_bf2(bf2_to_f2(dw) * bf2_to_f2(gw));
}
// a 16-byte output store; NT: non-temporal (the output stream does not displace the operands in L2)
template <bool NT = false> __device__ __forceinline__ void st16(__bf16* p, const uint4& v) {
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
  if constexpr (NT) __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<uint4*>(p) = v;
}
// the GELU / GELU' epilogue stores of one 16-byte row segment (8 outputs)
template <bool NT = false>
__device__ __forceinline__ void gelu_store8(const uint4& raw, bool gp, __bf16* c, __bf16* c2) {
  if (gp) {
    uint4 g, y;
    y.x = gelu_grad_bf2(raw.x, g.x);
    y.y = gelu_grad_bf2(raw.y, g.y);
    y.z = gelu_grad_bf2(raw.z, g.z);
    y.w = gelu_grad_bf2(raw.w, g.w);
    st16<NT>(c2, g);
    st16<NT>(c, y);
  } else {
    st16<NT>(c2, raw);
    st16<NT>(c, uint4{gelu_bf2(raw.x), gelu_bf2(raw.y), gelu_bf2(raw.z), gelu_bf2(raw.w)});
  }
}
__device__ __forceinline__ uint4 dgelu8(const uint4& raw, const uint4& hv, bool gp) {
  if (gp) return uint4{mul_bf2(raw.x, hv.x), mul_bf2(raw.y, hv.y), mul_bf2(raw.z, hv.z), mul_bf2(raw.w, hv.w)};
  return uint4{dgelu_bf2(raw.x, hv.x), dgelu_bf2(raw.y, hv.y), dgelu_bf2(raw.z, hv.z), dgelu_bf2(raw.w, hv.w)};
}

// one operand's ROWS x BK stage: ROWS * BK / 8 16-byte chunks, ROWS * BK / 2048 per thread.
// KT (K a multiple of 8 but not of BK: the CaiT-XXS / XS 288-wide, CvT 368-wide and TNT inner
// 24 / 40-wide projections): chunks at or past column K of the last stage read zero through the
// descriptor's range check (offset 0x80000000), so the MFMAs add zeros there.
template <int BK, int ROWS = 128, bool KT = false> struct NtStageT {
  static constexpr int CPR = BK / 8;         // 16-byte chunks per row
  static constexpr int PER = ROWS * CPR / 256;
  uint4 v[PER];
  unsigned goff[PER];
  unsigned loff[PER];
  int kc[KT ? PER : 1];                      // KT: the chunk's first column inside the stage
  __device__ __forceinline__ void init(int tid, long long ld) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = tid + 256 * i;
      const int r = id / CPR, c = id % CPR;
      goff[i] = (unsigned)(((long long)r * ld + 8 * c) * 2);
      loff[i] = r * (BK * 2) + 16 * (c ^ swz<BK>(r));
      if constexpr (KT) kc[i] = 8 * c;
    }
  }
  // kleft: columns of this stage that exist (K - st BK; only read with KT)
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, unsigned koff, int kleft = BK) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      unsigned off = goff[i] + koff;
      if constexpr (KT) off = kc[i] < kleft ? off : 0x80000000u;
      v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  }
  __device__ __forceinline__ void write(char* img) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) *reinterpret_cast<uint4*>(img + loff[i]) = v[i];
  }
};
using NtStage = NtStageT<kNtK>;

// A-operand loader of the plain GEMM: rows m0 .. m0 + ROWS - 1 of the row-major a [M][K] through
// a buffer descriptor (rows past M read zero).  patch.h supplies the patch-gather loaders (64-deep
// stages, 128 rows); a loader also maps GEMM row m to its output row (orow).
template <int BK, int ROWS = 128, bool KT = false> struct NtRowAT {
  static constexpr int kBK = BK;
  static constexpr bool kKT = KT;
  NtStageT<BK, ROWS, KT> s;
  __amdgpu_buffer_rsrc_t rs;
  __device__ __forceinline__ void init(const NtArgs& a, int tid, int m0) {
    rs = row_rsrc(a.a + (long long)m0 * a.lda, min(ROWS, a.M - m0), a.lda);
    s.init(tid, a.lda);
  }
  __device__ __forceinline__ void load(const NtArgs& a, int st) { s.load(rs, (unsigned)st * (BK * 2), a.K - st * BK); }
  __device__ __forceinline__ void write(char* img) const { s.write(img); }
  static __device__ __forceinline__ long long orow(const NtArgs&, int m) { return m; }
};
using NtRowA = NtRowAT<kNtK>;

// marker loader: A and B staged by LDS-DMA through NB stage buffers (32-deep stages, 128 rows)
template <int NB> struct NtDmaA {
  static constexpr int kBK = 32;
  static constexpr int kNB = NB;
  static __device__ __forceinline__ long long orow(const NtArgs&, int m) { return m; }
};

template <class AL> struct NtDepth { static constexpr int value = kNtK; };
template <int BK, int ROWS, bool KT> struct NtDepth<NtRowAT<BK, ROWS, KT>> { static constexpr int value = BK; };
template <int NB> struct NtDepth<NtDmaA<NB>> { static constexpr int value = 32; };
template <class AL> struct NtIsDma { static constexpr bool value = false; };
template <int NB> struct NtIsDma<NtDmaA<NB>> { static constexpr bool value = true; };
template <class AL> struct NtRows { static constexpr int value = kNtT; };
template <int BK, int ROWS, bool KT> struct NtRows<NtRowAT<BK, ROWS, KT>> { static constexpr int value = ROWS; };
template <class AL> struct NtKT { static constexpr bool value = false; };
template <int BK, int ROWS> struct NtKT<NtRowAT<BK, ROWS, true>> { static constexpr bool value = true; };

// Main loop, operands staged global -> registers -> LDS: two LDS buffers, two register sets in
// flight.  Straight-line staging (no data-dependent branches around the loads and LDS writes):
// the loads of stages st + 2 and the LDS writes of stage st + 1 are issued unconditionally -- past
// the end they read zeros (descriptor range check) or unused bytes into a buffer nobody reads
// again -- so the waitcnt pass can prove each register set's loads retired and keeps two stages
// in flight (with conditional loads it waited vmcnt(0) before every reload).
template <class AL, int BK, int TM, class Pre, class Compute>
__device__ __forceinline__ void nt_loop_regs(const NtArgs& a, int m0, int n0, int tid, char* smem, Pre&& preload,
                                             Compute&& compute) {
  constexpr int IMGA = TM * BK * 2, IMG = kNtT * BK * 2, BUF = IMGA + IMG;
  // rows past N read zero through the descriptor's range check
  const __amdgpu_buffer_rsrc_t rb = row_rsrc(a.bt + (long long)n0 * a.ldb, min(kNtT, a.N - n0), a.ldb);
  constexpr bool KT = NtKT<AL>::value;
  AL as[2];
  NtStageT<BK, 128, KT> bs[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    as[q].init(a, tid, m0);
    bs[q].init(tid, a.ldb);
  }
  const int nst = (a.K + BK - 1) / BK;   // KT: the last stage is partial
  as[0].load(a, 0);
  bs[0].load(rb, 0, a.K);
  as[1].load(a, 1);
  bs[1].load(rb, BK * 2, a.K - BK);
  preload();
  as[0].write(smem);
  bs[0].write(smem + IMGA);
  __syncthreads();
  int st = 0;
  for (; st + 2 <= nst; st += 2) {
#pragma unroll
    for (int bsel = 0; bsel < 2; ++bsel) {
      const char* ima = smem + bsel * BUF;
      char* nxt = smem + (bsel ^ 1) * BUF;
      // register set bsel went to LDS at the end of the previous stage: refill it (stage + 2)
      as[bsel].load(a, st + bsel + 2);
      bs[bsel].load(rb, (unsigned)(st + bsel + 2) * (BK * 2), a.K - (st + bsel + 2) * BK);
      compute(ima, ima + IMGA);
      as[bsel ^ 1].write(nxt);
      bs[bsel ^ 1].write(nxt + IMGA);
      __syncthreads();
    }
  }
  if (st < nst) {   // odd stage count: the last stage sits in buffer 0
    compute(smem, smem + IMGA);
    __syncthreads();   // every wave done with buffer 0 before the epilogue reuses it as scratch
  }
}

// One 16-byte-per-lane LDS-DMA piece (1 KiB at the wave-uniform LDS byte address `lds`: lane L's
// 16 bytes land at lds + 16 L).  Inline asm on purpose: through the builtin, hipcc cannot tell the
// DMA's LDS bytes from the ones a later ds_read reads and puts an s_waitcnt vmcnt(0) in front of
// it, which drains every stage in flight.  The waits are counted by hand instead (nt_loop_dma).
// M0 is compiler-reserved: saved and restored inside the statement (s_nop 4 for a descriptor
// just written by SALU, s_nop 0 after the M0 write).
typedef __attribute__((ext_vector_type(4))) unsigned nt_u32x4;
__device__ __forceinline__ void nt_dma16(nt_u32x4 rs, unsigned voff, unsigned lds) {
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

// the four words of row_rsrc's descriptor (common.h), for the inline-asm DMA
template <typename T>
__device__ __forceinline__ nt_u32x4 nt_rsrc_words(const T* base, int nrows, long long rs) {
  const unsigned long long p = reinterpret_cast<unsigned long long>(base);
  nt_u32x4 w;
  w[0] = __builtin_amdgcn_readfirstlane((unsigned)p);
  w[1] = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32)) & 0xffffu;   // stride 0
  w[2] = __builtin_amdgcn_readfirstlane((unsigned)((long long)nrows * rs * sizeof(T)));
  w[3] = 0x00020000u;
  return w;
}

// s_waitcnt vmcnt(N) + s_barrier as one statement: the "memory" clobber keeps the compiler from
// moving LDS accesses across it (the builtin barrier is not a memory operation to the compiler)
template <int N>
__device__ __forceinline__ void nt_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Main loop, operands staged by LDS-DMA (no VGPR round trip, no ds_write): 128 x 32 A and B
// images per stage (8 KiB each = 8 one-KiB pieces, XOR-swizzled like Img<bf16, 32>: lane L of a
// piece fetches the global chunk (L & 3) ^ swz(row) so the image holds chunk c at c ^ swz(row)),
// NB stage buffers, NB - 1 stages in flight.  Each wave issues 4 pieces per stage; at the top of
// stage st it waits until only the (NB - 2) newer stages' pieces are outstanding, and the barrier
// makes every wave's pieces of stage st visible and frees the buffer the next issue overwrites
// (computed at st - 1).  Stages past K are issued anyway (rows read zero or bytes nobody reads)
// so that the count stays uniform.
template <int NB, class Pre, class Compute>
__device__ __forceinline__ void nt_loop_dma(const NtArgs& a, int m0, int n0, int w, int lane, char* smem,
                                            Pre&& preload, Compute&& compute) {
  constexpr int BK = 32, IMG = kNtT * BK * 2, BUF = 2 * IMG;
  const nt_u32x4 ra = nt_rsrc_words(a.a + (long long)m0 * a.lda, min(kNtT, a.M - m0), a.lda);
  const nt_u32x4 rb = nt_rsrc_words(a.bt + (long long)n0 * a.ldb, min(kNtT, a.N - n0), a.ldb);
  const unsigned lbase = __builtin_amdgcn_readfirstlane(
      (unsigned)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)smem));
  // this wave's pieces: A pieces w and w + 4, B pieces w and w + 4 (16 rows of 64 bytes each)
  unsigned goa[2], gob[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * (w + 4 * i) + (lane >> 2);
    const int c = (lane & 3) ^ swz<BK>(row);
    goa[i] = (unsigned)(((long long)row * a.lda + 8 * c) * 2);
    gob[i] = (unsigned)(((long long)row * a.ldb + 8 * c) * 2);
  }
  auto issue = [&](int st, int buf) {
    const unsigned ko = (unsigned)st * (BK * 2);
    const unsigned lb = lbase + (unsigned)(buf * BUF) + (unsigned)(w * 1024);
    // the stage's four pieces in one statement: one M0 save / restore, one descriptor settle
    unsigned keep;
    asm volatile(
        "s_nop 4\n\t"
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %7\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %5, 0 offen lds\n\t"
        "s_add_u32 m0, %7, 4096\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %5, 0 offen lds\n\t"
        "s_add_u32 m0, %7, 8192\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %3, %6, 0 offen lds\n\t"
        "s_add_u32 m0, %7, 12288\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %4, %6, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(goa[0] + ko), "v"(goa[1] + ko), "v"(gob[0] + ko), "v"(gob[1] + ko), "s"(ra), "s"(rb), "s"(lb)
        : "memory", "scc");
  };
  static_assert(IMG == 8192, "piece layout: A pieces w, w + 4 at +0 / +4 KiB, B at +8 / +12 KiB");
  const int nst = a.K / BK;
#pragma unroll
  for (int q = 0; q < NB - 1; ++q) issue(q, q);
  preload();
  int cur = 0, nxt = NB - 1;
  for (int st = 0; st < nst; ++st) {
    nt_wait_barrier<4 * (NB - 2)>();
    issue(st + NB - 1, nxt);
    compute(smem + cur * BUF, smem + cur * BUF + IMG);
    cur = cur + 1 == NB ? 0 : cur + 1;
    nxt = nxt + 1 == NB ? 0 : nxt + 1;
  }
  nt_wait_barrier<0>();   // every piece landed and every wave done before the epilogue's scratch
}

// Tiles: TM (128 or 256) tokens x 128 features per workgroup, each wave TM / 2 tokens x 64
// features (UM = TM / 64 token sub-tiles of 32).  The 256-token tile reads 6 fragments from LDS
// per 8 MFMAs instead of 4 per 4 (43 vs 32 flop per LDS byte: the 128-token tile saturates LDS
// bandwidth before the MFMA pipe) and fetches the weight once per 256 tokens; it runs 32-deep
// stages so that the two staged register sets still fit beside the 128 accumulator registers.
template <int EPI, class AL>
constexpr int nt_min_blocks() {
  if constexpr (NtIsDma<AL>::value) return AL::kNB <= 3 ? 3 : 2;
  return NtRows<AL>::value == 256 ? 2 : NtDepth<AL>::value == 32 ? (EPI == kEpiDGelu ? 3 : 4) : 2;
}

template <int EPI, class AL = NtRowA>
__global__ __launch_bounds__(256, (nt_min_blocks<EPI, AL>())) void gemm_nt_kernel(NtArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BK = NtDepth<AL>::value;   // K per stage
  constexpr int TM = NtRows<AL>::value;    // tokens per tile
  constexpr int UM = TM / 64;              // 32-token sub-tiles per wave
  const int tn = (a.N + kNtT - 1) / kNtT;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / tn, nt = bid % tn;
  const int m0 = mt * TM, n0 = nt * kNtT;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w & 1, wn = w >> 1;   // this wave's TM / 2 (tokens) x 64 (features) quarter
  constexpr int WT = TM / 2;

  // kEpiDGelu: this lane's eight aux chunks (the epilogue's row groups) are loaded before the
  // main loop, so their HBM traffic overlaps the MFMAs instead of following them
  const int c8 = lane & 7;                 // 16-byte chunk of an epilogue row segment
  const int n = n0 + 64 * wn + 8 * c8;     // its first feature
  // (the 256-token tile has no registers left for all of them: it loads each sub-tile's chunks
  // at the start of that sub-tile's epilogue)
  constexpr int UA = UM == 2 ? 2 : 1;
  uint4 auxv[UA][4];
  auto load_aux = [&](int ua, int u) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int m = m0 + WT * wm + 32 * u + 8 * it + (lane >> 3);
      auxv[ua][it] = (m < a.M && n < a.N) ? *reinterpret_cast<const uint4*>(a.aux + AL::orow(a, m) * a.ldaux + n)
                                          : uint4{0, 0, 0, 0};
    }
  };
  auto preload = [&]() {
    if constexpr (EPI == kEpiDGelu && UM == 2) {
      load_aux(0, 0);
      load_aux(1, 1);
    }
  };
  f32x16 acc[2][UM];   // [feature sub-tile t][token sub-tile u]
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < UM; ++u) acc[t][u] = zero16();

  auto compute = [&](const char* ima, const char* imb) {
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const bf16x8 b0 = Img<__bf16, BK>::rowfrag(imb, 64 * wn + r, s, h);
      const bf16x8 b1 = Img<__bf16, BK>::rowfrag(imb, 64 * wn + 32 + r, s, h);
      bf16x8 av[UM];
#pragma unroll
      for (int u = 0; u < UM; ++u) av[u] = Img<__bf16, BK>::rowfrag(ima, WT * wm + 32 * u + r, s, h);
#pragma unroll
      for (int u = 0; u < UM; ++u) {
        acc[0][u] = MF<__bf16>::mma(b0, av[u], acc[0][u]);
        acc[1][u] = MF<__bf16>::mma(b1, av[u], acc[1][u]);
      }
    }
  };
  if constexpr (NtIsDma<AL>::value)
    nt_loop_dma<AL::kNB>(a, m0, n0, w, lane, smem, preload, compute);
  else
    nt_loop_regs<AL, BK, TM>(a, m0, n0, tid, smem, preload, compute);

  // ---- epilogue: accumulator row = feature nb + 32t + row_of(reg, h), column = token (lane)
  const int nb = n0 + 64 * wn;
  if (EPI != kEpiDGelu && a.bias) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = nb + 32 * t + 8 * g + 4 * h;
        const f32x4 bv = (n < a.N) ? *reinterpret_cast<const f32x4*>(a.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int u = 0; u < UM; ++u) acc[t][u][4 * g + e] += bv[e];
      }
  }
  char* scratch = smem + w * (32 * 64 * 2);   // 4 KiB per wave; the stage buffers are free now
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
#pragma unroll
  for (int u = 0; u < UM; ++u) {
    if constexpr (EPI == kEpiDGelu && UM != 2) load_aux(0, u);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const bf16x4 v = {(__bf16)acc[t][u][4 * g], (__bf16)acc[t][u][4 * g + 1], (__bf16)acc[t][u][4 * g + 2],
                          (__bf16)acc[t][u][4 * g + 3]};
        *reinterpret_cast<bf16x4*>(scratch + r * 128 + 16 * ((4 * t + g) ^ swz<64>(r)) + 8 * h) = v;
      }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int rr = 8 * it + (lane >> 3);
      const int m = m0 + WT * wm + 32 * u + rr;
      const uint4 raw = *reinterpret_cast<const uint4*>(scratch + rr * 128 + 16 * (c8 ^ swz<64>(rr)));
      if (m < a.M && n < a.N) {
        const long long orow = AL::orow(a, m);
        if constexpr (EPI == kEpiNone) {
          *reinterpret_cast<uint4*>(a.c + orow * a.ldc + n) = raw;
        } else if constexpr (EPI == kEpiGelu) {
          gelu_store8(raw, a.gp, a.c + orow * a.ldc + n, a.c2 + orow * a.ldc + n);
        } else {
          *reinterpret_cast<uint4*>(a.c + orow * a.ldc + n) = dgelu8(raw, auxv[UM == 2 ? u : 0][it], a.gp);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// fp32 Dense kernel w [K][N] -> bf16 copies: w16 [K][N] (may be null) and its transpose
// wt16 [N][K] (may be null).  32 x 32 tiles through LDS, 4 elements per thread (many small
// workgroups: the weights are < 10 MB, so this is latency-, not bandwidth-bound).
__global__ __launch_bounds__(256) void weight_cast_kernel(const float* w, __bf16* w16, __bf16* wt16, int K, int N) {
  __shared__ float tile[32][33];
  const int k0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + ty + 8 * i, n = n0 + tx;
    v[i] = (k < K && n < N) ? w[(long long)k * N + n] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + ty + 8 * i, n = n0 + tx;
    if (w16 && k < K && n < N) w16[(long long)k * N + n] = (__bf16)v[i];
    tile[ty + 8 * i][tx] = v[i];
  }
  if (!wt16) return;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + ty + 8 * i, k = k0 + tx;
    if (k < K && n < N) wt16[(long long)n * K + k] = (__bf16)tile[tx][ty + 8 * i];
  }
}

// Every Dense kernel of a model cast in ONE launch (the per-weight casts are ~4 us each, almost
// all launch / ramp latency): item i casts w_i [K][N] into columns col0 .. col0 + N of
// w16 [K][ld16] and rows col0 .. col0 + N of wt16 [*][ldT]; items located by a prefix sum over
// their tile counts.  Items whose sizes, offsets and pointers allow it (vec) take 64 x 64 tiles
// with 16-byte loads and 8-byte bf16x4 stores both ways (HBM-bound: 4 B read + 2 x 2 B written
// per element); the others 32 x 32 tiles element by element.
constexpr int kCastMax = 48;
struct CastItem {
  const float* w;
  __bf16* w16;
  __bf16* wt16;
  int K, N, ld16, ldT, col0, tiles, vec;
};
struct CastList {
  CastItem it[kCastMax];
  int n;
};

__device__ __forceinline__ void cast_tile_vec(const CastItem& c, int b, float (*tile)[65]) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  const int tn = (c.N + 63) / 64;
  const int k0 = (b / tn) * 64, n0 = (b % tn) * 64;
  const int t = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = t + 256 * q, row = i >> 4, c4 = i & 15;
    const int k = k0 + row, n = n0 + 4 * c4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (k < c.K && n < c.N) {
      v = *reinterpret_cast<const f32x4*>(c.w + (long long)k * c.N + n);
      if (c.w16)
        *reinterpret_cast<bf16x4*>(c.w16 + (long long)k * c.ld16 + c.col0 + n) =
            bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) tile[row][4 * c4 + e] = v[e];
  }
  if (!c.wt16) return;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = t + 256 * q, nn = i >> 4, kk = i & 15;
    const int n = n0 + nn, k = k0 + 4 * kk;
    if (n < c.N && k < c.K)
      *reinterpret_cast<bf16x4*>(c.wt16 + (long long)(c.col0 + n) * c.ldT + k) =
          bf16x4{(__bf16)tile[4 * kk][nn], (__bf16)tile[4 * kk + 1][nn], (__bf16)tile[4 * kk + 2][nn],
                 (__bf16)tile[4 * kk + 3][nn]};
  }
}

__global__ __launch_bounds__(256) void weight_cast_multi_kernel(CastList L) {
  __shared__ float tile[64][65];
  int b = blockIdx.x, i = 0;
  while (i + 1 < L.n && b >= L.it[i].tiles) b -= L.it[i++].tiles;
  const CastItem& c = L.it[i];
  if (c.vec) {
    cast_tile_vec(c, b, tile);
    return;
  }
  const int tn = (c.N + 31) / 32;
  const int k0 = (b / tn) * 32, n0 = (b % tn) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = k0 + ty + 8 * r, n = n0 + tx;
    v[r] = (k < c.K && n < c.N) ? c.w[(long long)k * c.N + n] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = k0 + ty + 8 * r, n = n0 + tx;
    if (c.w16 && k < c.K && n < c.N) c.w16[(long long)k * c.ld16 + c.col0 + n] = (__bf16)v[r];
    tile[ty + 8 * r][tx] = v[r];
  }
  if (!c.wt16) return;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int n = n0 + ty + 8 * r, k = k0 + tx;
    if (k < c.K && n < c.N) c.wt16[(long long)(c.col0 + n) * c.ldT + k] = (__bf16)tile[tx][ty + 8 * r];
  }
}

}  // namespace sae
