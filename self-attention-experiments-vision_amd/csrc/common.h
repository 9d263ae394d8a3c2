// common.h -- shared CDNA4 (gfx950) building blocks for the attention kernels.
//
// MFMA engine abstraction.  Every product in the kernels is a 32x32 MFMA tile:
//   bf16: v_mfma_f32_32x32x16_bf16   (K = 16 per instruction, 8 elements per lane)
//   f32 : v_mfma_f32_32x32x2_f32     (K = 2  per instruction, 1 element per lane; exact f32)
// Operand maps (cdna_hip_programming.md §3): lane l = 32*h + r holds A[row r][k] and
// B[k][col r] for k = KSTEP*s + KH*h + j (j < KH).  The accumulator has col = lane & 31 and
// row = row_of(reg, h) = (reg & 3) + 8*(reg >> 2) + 4*h.
//
// "Accumulator as operand": a 32x32 accumulator X (col on the lane, rows in registers) is fed
// to the next MFMA as the operand whose K index runs over X's rows without any lane movement.
// K-step s, element j then carries X row row_of(KH*s + j, h); the other operand must supply the
// same permuted K order -- colfrag() below reads it that way.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sae {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kInf = __builtin_huge_valf();

__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float lg2(float x) { return __builtin_amdgcn_logf(x); }

__device__ __forceinline__ int row_of(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

template <typename T> struct MF;

template <> struct MF<__bf16> {
  static constexpr int KSTEP = 16;
  static constexpr int KH = 8;
  using frag = bf16x8;
  static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ frag zero() { return frag{}; }
};

template <> struct MF<float> {
  static constexpr int KSTEP = 2;
  static constexpr int KH = 1;
  using frag = float;
  static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ frag zero() { return 0.f; }
};

__device__ __forceinline__ f32x16 zero16() { return f32x16{}; }

// In-kernel cycle stamps (diagnostic build only: build.py --stamps defines SAE_STAMPS; the
// release library compiles SAE_STAMP to nothing).  Lane 0 of every wave records the shader clock
// (s_memtime) at slot `slot` of its (block, wave) record with a plain vector store; the host reads
// the table back through sae_dev_stamps (capi.hip).  cdna_hip_programming.md §7 "In-kernel stamps".
#ifdef SAE_STAMPS
constexpr int kStampSlots = 32, kStampWaves = 16, kStampRecs = 1 << 22;
__device__ unsigned long long g_sae_stamps[kStampRecs];
// slot 0 (entry) and 31 (exit) also record the 100 MHz real-time clock in slots 28 / 29
#define SAE_STAMPO(boff, slot)                                                                       \
  do {                                                                                               \
    if ((threadIdx.x & 63) == 0) {                                                                   \
      const size_t i_ = ((size_t)(blockIdx.x + (boff)) * kStampWaves + (threadIdx.x >> 6)) * kStampSlots; \
      if (i_ + kStampSlots <= (size_t)kStampRecs) {                                                   \
        g_sae_stamps[i_ + (slot)] = __builtin_amdgcn_s_memtime();                                    \
        if ((slot) == 0) g_sae_stamps[i_ + 28] = __builtin_amdgcn_s_memrealtime();                   \
        if ((slot) == 31) g_sae_stamps[i_ + 29] = __builtin_amdgcn_s_memrealtime();                  \
      }                                                                                              \
    }                                                                                                \
  } while (0)
#else
#define SAE_STAMPO(boff, slot) \
  do {                         \
  } while (0)
#endif
#define SAE_STAMP(slot) SAE_STAMPO(0, slot)

// s_waitcnt vmcnt(0) as a real S_WAITCNT (gfx9 encoding: expcnt 7, lgkmcnt 15 = no wait).  Put it
// after prologue loads whose registers stay live through a loop: otherwise the waitcnt pass,
// seeing them possibly outstanding at the loop header, waits at their first use INSIDE the loop
// with counts that, from the second trip on, drain the loop's own prefetch every iteration.
__device__ __forceinline__ void vm_wait_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// ------------------------------------------------------------------------------ LDS images
// bf16 tiles are [rows][DP] with 16-byte chunks XOR-swizzled per row so that both the
// ds_read_b128 row reads (MFMA row operand) and the ds_read_b64_tr_b16 column reads
// (accumulator-as-operand partner) are bank-conflict free:
//   DP=32  (64-B rows) : swz = (r>>2)&3
//   DP=64  (128-B rows): swz = bitreverse3((r>>1)&7)  -- rows r, r+2 land in opposite 64-B halves
//   DP=128 (256-B rows): swz = ((r&3)<<2) | ((r>>2)&3)
// f32 tiles are [rows][DP+1] floats (odd stride: conflict-free scalar row and column reads).
template <int DP> __device__ __forceinline__ int swz(int r) {
  if constexpr (DP == 32) return (r >> 2) & 3;
  else if constexpr (DP == 64) return (((r >> 1) & 1) << 2) | (((r >> 2) & 1) << 1) | ((r >> 3) & 1);
  else return ((r & 3) << 2) | ((r >> 2) & 3);
}

template <typename T, int DP> struct Img {
  static constexpr int bytes(int rows) {
    return sizeof(T) == 2 ? rows * DP * 2 : rows * (DP + 1) * 4;
  }
  // operand with the tile row on the lane and K over the head dim: element (r, KSTEP*s + KH*h + j)
  static __device__ __forceinline__ typename MF<T>::frag rowfrag(const char* lds, int r, int s, int h) {
    if constexpr (sizeof(T) == 2) {
      const int c = 2 * s + h;
      return *reinterpret_cast<const bf16x8*>(lds + r * (DP * 2) + 16 * (c ^ swz<DP>(r)));
    } else {
      return reinterpret_cast<const float*>(lds)[r * (DP + 1) + 2 * s + h];
    }
  }
  // operand with the head-dim column (col0 + (lane&31)) on the lane and K over tile rows
  // rowbase + row_of(KH*s + j, h): the partner of an accumulator fed as an operand.
  static __device__ __forceinline__ typename MF<T>::frag colfrag(const char* lds, int rowbase, int s,
                                                                   int col0, int lane) {
    if constexpr (sizeof(T) == 2) {
      const int li = lane & 15, g = lane >> 4, h = lane >> 5;
      const int colb = col0 + 16 * (g & 1) + 4 * (li & 3);
      const int chunk = colb >> 3, half = (colb >> 2) & 1;
      const int r1 = rowbase + 16 * s + 4 * h + (li >> 2);
      const int r2 = r1 + 8;
      const char* p1 = lds + r1 * (DP * 2) + 16 * (chunk ^ swz<DP>(r1)) + 8 * half;
      const char* p2 = lds + r2 * (DP * 2) + 16 * (chunk ^ swz<DP>(r2)) + 8 * half;
      s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
      s16x4 x2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p2));
      typedef __attribute__((ext_vector_type(8))) short s16x8;
      s16x8 v = {x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
      return __builtin_bit_cast(bf16x8, v);
    } else {
      const int h = lane >> 5;
      return reinterpret_cast<const float*>(lds)[(rowbase + row_of(s, h)) * (DP + 1) + col0 + (lane & 31)];
    }
  }
};

typedef __attribute__((ext_vector_type(8))) short s16x8;

// two ds_read_b64_tr_b16 (4 x 16 blocks at p1 and p2) as one 8-element bf16 MFMA operand
__device__ __forceinline__ bf16x8 tr2(const char* p1, const char* p2) {
  const s16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
  const s16x4 x2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p2));
  const s16x8 v = {x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// accumulator registers KH*s .. KH*s+KH-1 as an operand fragment
template <typename T> __device__ __forceinline__ typename MF<T>::frag acc_frag(const f32x16& acc, int s) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (__bf16)acc[8 * s + j];
    return f;
  } else {
    return acc[s];
  }
}

// ------------------------------------------------------------------ global -> LDS staging
// A ROWS x DP tile of a token-major tensor (row stride `rs` elements), staged through
// registers (issue early, write late).  VEC: 16-byte loads (D % (16/sizeof(T)) == 0 and
// aligned strides); otherwise element loads.  Rows >= nrows and columns >= D are zero.
template <typename T, int DP, int ROWS, bool VEC> struct Stage {
  static constexpr int EPC = 16 / sizeof(T);
  static constexpr int CPR = DP / EPC;
  static constexpr int NCH = (ROWS * CPR + 255) / 256;
  uint4 v[NCH];

  __device__ __forceinline__ void load(const T* base, int row0, int nrows, long long rs, int D, int tid) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int id = tid + 256 * i;
      const int r = id / CPR, c = id % CPR;
      const int row = row0 + r;
      if (id >= ROWS * CPR) { v[i] = uint4{0, 0, 0, 0}; continue; }
      if constexpr (VEC) {
        if (row < nrows && c * EPC < D)
          v[i] = *reinterpret_cast<const uint4*>(base + (long long)row * rs + c * EPC);
        else
          v[i] = uint4{0, 0, 0, 0};
      } else {
        T tmp[EPC];
#pragma unroll
        for (int e = 0; e < EPC; ++e) {
          const int d = c * EPC + e;
          tmp[e] = (row < nrows && d < D) ? base[(long long)row * rs + d] : (T)0.f;
        }
        v[i] = *reinterpret_cast<const uint4*>(tmp);
      }
    }
  }
  // VEC path through a buffer descriptor whose range ends at row `nrows`: rows past the end and
  // columns >= D read as zero from the hardware range check -- no branches (T8/T20).
  __device__ __forceinline__ void load_buf(__amdgpu_buffer_rsrc_t rsrc, int row0, long long rs, int D, int tid) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int id = tid + 256 * i;
      const int r = id / CPR, c = id % CPR;
      unsigned off = (unsigned)(((long long)(row0 + r) * rs + c * EPC) * (long long)sizeof(T));
      off = (c * EPC < D && id < ROWS * CPR) ? off : 0x80000000u;
      v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
    }
  }
  __device__ __forceinline__ void write(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int id = tid + 256 * i;
      if (id >= ROWS * CPR) continue;
      const int r = id / CPR, c = id % CPR;
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<uint4*>(lds + r * (DP * 2) + 16 * (c ^ swz<DP>(r))) = v[i];
      } else {
        float* f = reinterpret_cast<float*>(lds) + r * (DP + 1) + c * 4;
        f[0] = __uint_as_float(v[i].x);
        f[1] = __uint_as_float(v[i].y);
        f[2] = __uint_as_float(v[i].z);
        f[3] = __uint_as_float(v[i].w);
      }
    }
  }
};

// Buffer descriptor over rows [0, nrows) of a token-major tensor (row stride rs elements),
// built from wave-uniform values only.
// The inputs are passed through readfirstlane so that the compiler can PROVE the descriptor
// wave-uniform and keep it in SGPRs (otherwise it wraps every buffer op in a waterfall loop,
// cdna_hip_programming.md T20).
template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const T* base, int nrows, long long rs) {
  const unsigned long long p = reinterpret_cast<unsigned long long>(base);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)p);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32));
  const int nbytes = __builtin_amdgcn_readfirstlane((int)((long long)nrows * rs * sizeof(T)));
  void* pu = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pu, (short)0, nbytes, 0x00020000);
}

// Operand fragment read straight from global memory: row `row` of a token-major tensor,
// elements d = KSTEP*s + KH*h + j.
template <typename T, bool VEC>
__device__ __forceinline__ typename MF<T>::frag gfrag(const T* base, int row, int nrows, long long rs,
                                                      int D, int s, int h) {
  const int d0 = MF<T>::KSTEP * s + MF<T>::KH * h;
  if constexpr (sizeof(T) == 2) {
    if (row >= nrows) return bf16x8{};
    const T* p = base + (long long)row * rs + d0;
    if constexpr (VEC) {
      if (d0 < D) return *reinterpret_cast<const bf16x8*>(p);
      return bf16x8{};
    } else {
      bf16x8 f;
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = (d0 + j < D) ? p[j] : (__bf16)0.f;
      return f;
    }
  } else {
    if (row >= nrows || d0 >= D) return 0.f;
    return base[(long long)row * rs + d0];
  }
}

// Store 4 consecutive head-dim values (d0..d0+3) of one row.
template <typename T, bool VEC>
__device__ __forceinline__ void store4(T* rowp, int d0, int D, float a, float b, float c, float d) {
  if constexpr (VEC) {
    if (d0 >= D) return;
    if constexpr (sizeof(T) == 2) {
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      bf16x4 v = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
      *reinterpret_cast<bf16x4*>(rowp + d0) = v;
    } else {
      *reinterpret_cast<f32x4*>(rowp + d0) = f32x4{a, b, c, d};
    }
  } else {
    const float x[4] = {a, b, c, d};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (d0 + e < D) rowp[d0 + e] = (T)x[e];
  }
}

// ------------------------------------------------------------------------------- rotary
// GPT-J interleaved rotary (models/layers/position_embed.py:8-20) applied while q / k are staged
// and undone on dq / dk as they are stored (the attention kernels' ROT instances): pairs
// (2i, 2i+1) of the head dim at position pos, fp32 tables sin / cos [n][P = D / 2]:
//   y[2i] = x[2i] cos - x[2i+1] sin,  y[2i+1] = x[2i+1] cos + x[2i] sin   (SGN = -1: by -theta)
// with explicit FMAs, so the fused path and the standalone rotary_kernel round identically.
struct RopeTab {
  const float* sin;
  const float* cos;
  int P, n;
};
template <int NP, int SGN>
__device__ __forceinline__ void rope_pairs(float* x, const RopeTab& t, int pos, int i0) {
  const float* sp = t.sin + (long long)pos * t.P + i0;
  const float* cp = t.cos + (long long)pos * t.P + i0;
  float sv[NP], cv[NP];
  if constexpr (NP == 4) {
    const f32x4 s4 = *reinterpret_cast<const f32x4*>(sp), c4 = *reinterpret_cast<const f32x4*>(cp);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sv[j] = s4[j];
      cv[j] = c4[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      sv[j] = sp[j];
      cv[j] = cp[j];
    }
  }
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const float sn = SGN > 0 ? sv[j] : -sv[j];
    const float x0 = x[2 * j], x1 = x[2 * j + 1];
    x[2 * j] = __builtin_fmaf(x0, cv[j], -(x1 * sn));
    x[2 * j + 1] = __builtin_fmaf(x1, cv[j], x0 * sn);
  }
}
// one 16-byte chunk = head-dim elements d0 .. d0 + 7 (d0 % 8 == 0) of position pos; chunks past the
// head dim (zero padding) or past the table pass through
template <int SGN>
__device__ __forceinline__ uint4 rope8(uint4 v, const RopeTab& t, int pos, int d0) {
  if (pos >= t.n || d0 >= 2 * t.P) return v;
  const bf16x8 b = __builtin_bit_cast(bf16x8, v);
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (float)b[j];
  rope_pairs<4, SGN>(x, t, pos, d0 / 2);
  bf16x8 y;
#pragma unroll
  for (int j = 0; j < 8; ++j) y[j] = (__bf16)x[j];
  return __builtin_bit_cast(uint4, y);
}
template <int SGN>
__device__ __forceinline__ bf16x8 rope8(bf16x8 v, const RopeTab& t, int pos, int d0) {
  return __builtin_bit_cast(bf16x8, rope8<SGN>(__builtin_bit_cast(uint4, v), t, pos, d0));
}

// ------------------------------------------------------------------------ epilogue stores
// A wave's 32 output rows held as NT accumulator tiles acc[t] = X^T (accumulator row = head-dim
// column 32t + row_of(r, h), accumulator column = the wave's output row lane & 31), scaled by sc,
// are written as bf16 rows into a per-wave LDS scratch of 32 x DP (XOR-swizzled like the tile
// images: conflict-free 8-byte writes and 16-byte reads) and stored as whole 16-byte row chunks:
// one wave-instruction covers 64 x 16 B = complete rows (8 rows of 128 B at DP = 64) instead of
// 16 B slivers of 32 rows, so no partial cache lines are written at the row stride
// (MI355X_MICROARCH.md "attention epilogue store tail").  Rows >= nrows and columns >= D are not
// stored.  Wave-local: the scratch must not be in use by other waves.
// RSGN != 0: the rows are positions pos0 .. pos0 + 31 and each chunk is rotated by RSGN theta
// (rope8) on its way out (dq / dk of the rotary instances: the gradient of the un-rotated input).
template <int DP, int RSGN = 0>
__device__ __forceinline__ void wave_store_rows(const f32x16* acc, float sc, char* scratch, __bf16* dst,
                                                long long rs, int nrows, int D, int lane,
                                                const RopeTab* rope = nullptr, int pos0 = 0) {
  constexpr int NT = DP / 32, CPR = DP / 8, RPI = 64 / CPR;
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  const int h = lane >> 5, r = lane & 31;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const bf16x4 v = {(__bf16)(acc[t][4 * g] * sc), (__bf16)(acc[t][4 * g + 1] * sc),
                        (__bf16)(acc[t][4 * g + 2] * sc), (__bf16)(acc[t][4 * g + 3] * sc)};
      *reinterpret_cast<bf16x4*>(scratch + r * DP * 2 + 16 * ((4 * t + g) ^ swz<DP>(r)) + 8 * h) = v;
    }
  __builtin_amdgcn_wave_barrier();
  const int c = lane % CPR;
#pragma unroll
  for (int it = 0; it < 32 / RPI; ++it) {
    const int rr = it * RPI + lane / CPR;
    uint4 v = *reinterpret_cast<const uint4*>(scratch + rr * DP * 2 + 16 * (c ^ swz<DP>(rr)));
    if constexpr (RSGN != 0) {
      if (rr < nrows) v = rope8<RSGN>(v, *rope, pos0 + rr, c * 8);
    }
    if (rr < nrows && c * 8 < D) *reinterpret_cast<uint4*>(dst + (long long)rr * rs + c * 8) = v;
  }
  __builtin_amdgcn_wave_barrier();
}

// XCD-aware block order (cdna_hip_programming.md T1, bijective form): hardware block `bid` of a
// G-block grid runs on XCD bid % 8; returning logical ids so that consecutive logical blocks
// (which share K/V or Q/dO of one (batch, head)) land on the same XCD and its L2.
__device__ __forceinline__ int xcd_remap(int bid, int G) {
  const int x = bid & 7, j = bid >> 3;
  const int q = G >> 3, r = G & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + j;
}

// exact integer key -> (row, col) split for key < 4096, width <= 64: (key * magic) >> 20
__host__ __device__ inline int div_magic(int w) { return (int)((1u << 20) / (unsigned)w + 1u); }

// Division by a run-time constant d >= 1 for 0 <= n < 2^31 (round-up multiplier, one mul_hi and a
// shift): q = (mulhi(n, mul) + n) >> sh with sh = ceil(log2 d), mul = floor(2^32 (2^sh - d) / d) + 1.
struct FDiv {
  unsigned mul;
  int sh;
  __host__ static FDiv make(unsigned d) {
    int l = 0;
    while ((1ull << l) < d) ++l;
    FDiv f;
    f.mul = (unsigned)((((1ull << l) - d) << 32) / d + 1);
    f.sh = l;
    return f;
  }
  __device__ __forceinline__ int div(int n) const { return (int)((__umulhi((unsigned)n, mul) + (unsigned)n) >> sh); }
};

// Patch-embedding geometry (models/layers/stems/patch_embed.py:15-26): the GEMM operand
// A[m][k] = image[n][py * Ph + ky][px * Pw + kx][c] with k = (ky * Pw + kx) * C + c and token
// m = (n, p = py * gw + px); `hwcn` selects the train-step feed layout [H, W, C, N]
// (train.py:80, input_pipeline.py:187-191), whose GEMM row order is m = p * Nb + n (the batch
// index is the contiguous one there) with output row n * L + p.
struct PatchGeom {
  const void* x;                 // images, bf16 or fp32
  int Nb, Himg, Wimg, C, Ph, Pw;
  int gw, L;                     // patches per image row, patches per image
  int PwC, WC;                   // Pw * C (one patch row), Wimg * C (one image row)
  FDiv dL, dNb, dgw, dPwC;
};

}  // namespace sae
