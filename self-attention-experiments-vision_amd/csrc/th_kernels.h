// th_kernels.h -- fused talking-heads attention (CaiT trunk) for gfx950.
//
// Reference: models/layers/attentions/attention.py:41-58 with talking_heads=True and
// models/layers/attentions/talking_heads.py:9-14 (T is [h_in, h_out]):
//   S_h = scale Q_h K_h^T ; S1_i = sum_h T1[h,i] S_h ; P_i = softmax_k(S1_i) ;
//   P2_i = sum_h T2[h,i] P_h ; O_i = P2_i V_i
// The head mix breaks per-head independence, so a workgroup holds one 32-row query block
// (or 32-key block) for ALL heads: wave w computes head w's 32x32 score tile on MFMA and
// the tiles are exchanged through LDS in accumulator order ([reg/4][lane][4] fp32, 4 KB per
// head) so that each wave mixes its output head with ds_read_b128s.  Nothing N^2 reaches HBM.
//
//   th_fwd    : pass 0 = online max/sum of the mixed logits; pass 1 = normalised P, mix,
//               O_i += P2_i V_i.  lse of S1 kept for the backward.
//   th_bwd_q  : query-major.  pass A: delta_i = rowsum(dP_i o P_i) with
//               dP_h = sum_i T2[h,i] dP2_i, dP2_i = dO_i V_i^T, plus dT2 partials;
//               pass B: dS1 = P (dP - delta), dS_h = sum_i T1[h,i] dS1_i, dQ, dT1 partials.
//   th_bwd_kv : key-major.  dV_h += P2_h^T dO_h, dK_h += scale dS_h^T Q_h.
//   th_reduce : fixed-order sum of the per-workgroup dT partials (deterministic).
#pragma once
#include "common.h"

namespace sae {

constexpr int kThMaxH = 8;

struct ThArgs {
  const void* q;
  const void* k;
  const void* v;
  void* o;
  float* lse;
  const void* dout;
  void* dq;
  void* dk;
  void* dv;
  const float* th1;
  const float* th2;
  float* delta;
  float* part;
  float* dth1;
  float* dth2;
  int B, H, Nq, Nk, D, nblk;
  long long qs[3], ks[3], vs[3], os[3], dos[3], dqs[3], dks[3], dvs[3];
  float scale;
  RopeTab rope;     // rotary tables (th2 kernels rotate q / k when rope.sin != nullptr)
};

// ---- exchange buffer: one 32x32 fp32 accumulator per head, [reg>>2][lane][reg&3]
__device__ __forceinline__ void xput(float* X, int head, int lane, const f32x16& v) {
  f32x4* p = reinterpret_cast<f32x4*>(X + head * 1024);
#pragma unroll
  for (int g = 0; g < 4; ++g) p[g * 64 + lane] = f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
}
__device__ __forceinline__ f32x16 xget(const float* X, int head, int lane) {
  const f32x4* p = reinterpret_cast<const f32x4*>(X + head * 1024);
  f32x16 v;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 t = p[g * 64 + lane];
    v[4 * g] = t[0];
    v[4 * g + 1] = t[1];
    v[4 * g + 2] = t[2];
    v[4 * g + 3] = t[3];
  }
  return v;
}
// out = sum_i tab[i*st] X[i]   (coefficients from an LDS table: wave-uniform broadcast reads;
// a rolled loop keeps the register footprint at two tiles)
__device__ __forceinline__ f32x16 xmix(const float* X, const float* tab, int st, int H, int lane) {
  f32x16 acc = zero16();
#pragma unroll 2
  for (int i = 0; i < H; ++i) {
    const float c = tab[i * st];
    const f32x16 x = xget(X, i, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += c * x[r];
  }
  return acc;
}

// stage th1 / th2 ([H][H] fp32) into LDS (call before the first __syncthreads)
__device__ __forceinline__ void load_tabs(float* tabs, const float* th1, const float* th2, int H, int tid) {
  for (int i = tid; i < 2 * H * H; i += blockDim.x) tabs[i] = i < H * H ? th1[i] : th2[i - H * H];
}

// wave-private staging of 32 rows x DP (bf16 images only)
template <typename T, int DP, bool VEC> struct WStage {
  static constexpr int EPC = 16 / sizeof(T);
  static constexpr int CPR = DP / EPC;
  static constexpr int NCH = (32 * CPR + 63) / 64;
  uint4 v[NCH];
  __device__ __forceinline__ void load(const T* base, int row0, int nrows, long long rs, int D, int lane) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int id = lane + 64 * i;
      const int r = id / CPR, c = id % CPR;
      const int row = row0 + r;
      if constexpr (VEC) {
        v[i] = (row < nrows && c * EPC < D) ? *reinterpret_cast<const uint4*>(base + (long long)row * rs + c * EPC)
                                            : uint4{0, 0, 0, 0};
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
  // VEC bf16 path through a buffer descriptor over the valid rows (row_rsrc): rows past the end
  // and columns >= D read as zero from the hardware range check.  The select-based load above
  // makes hipcc branch around every load and wait vmcnt(0) after it, which turned the next
  // tile's prefetch into a synchronous load (cdna_hip_programming.md §5, "three .s-level traps" (c)).
  __device__ __forceinline__ void load_buf(__amdgpu_buffer_rsrc_t rsrc, int row0, long long rs, int D, int lane) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int id = lane + 64 * i;
      const int r = id / CPR, c = id % CPR;
      const unsigned off = (c * EPC < D && id < 32 * CPR)
                               ? (unsigned)(((long long)(row0 + r) * rs + c * EPC) * (long long)sizeof(T))
                               : 0x80000000u;
      v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0));
    }
  }
  __device__ __forceinline__ void write(char* lds, int lane) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int id = lane + 64 * i;
      const int r = id / CPR, c = id % CPR;
      *reinterpret_cast<uint4*>(lds + r * (DP * 2) + 16 * (c ^ swz<DP>(r))) = v[i];
    }
  }
  // rotary on the staged rows row0 .. row0 + 31 (bf16), before write()
  __device__ __forceinline__ void rope(const RopeTab& t, int row0, int lane) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int id = lane + 64 * i;
      v[i] = rope8<1>(v[i], t, row0 + id / CPR, (id % CPR) * EPC);
    }
  }
};

// colfrag straight from global memory (f32 path: 32 lanes read one 128-B row, coalesced)
template <typename T>
__device__ __forceinline__ float colfrag_g(const T* base, int row0, int nrows, long long rs, int D, int s, int col0,
                                           int lane) {
  const int row = row0 + row_of(s, lane >> 5);
  const int col = col0 + (lane & 31);
  return (row < nrows && col < D) ? (float)base[(long long)row * rs + col] : 0.f;
}

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// LDS map shared by the three kernels: [tabs 512 B][XA H*4 KB][XB H*4 KB][kernel-specific]
constexpr int kTabBytes = 2 * kThMaxH * kThMaxH * 4;

// =================================================================================== fwd
template <typename T, int DP, bool VEC>
__global__ __launch_bounds__(512) void th_fwd_kernel(ThArgs a) {
  using M = MF<T>;
  using I = Img<T, DP>;
  constexpr bool BF = sizeof(T) == 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r32 = lane & 31;
  float* tabs = reinterpret_cast<float*>(smem);
  float* XA = reinterpret_cast<float*>(smem + kTabBytes);
  float* XB = XA + H * 1024;
  char* ldsV = reinterpret_cast<char*>(XB + H * 1024) + w * I::bytes(32);
  const float* c1 = tabs + w;              // T1[i][w], stride H
  const float* c2 = tabs + H * H + w;      // T2[i][w], stride H
  load_tabs(tabs, a.th1, a.th2, H, tid);

  const int nqb = (a.Nq + 31) / 32;
  const int qb = blockIdx.x % nqb, b = blockIdx.x / nqb;
  const int q = qb * 32 + r32;
  const T* Q = reinterpret_cast<const T*>(a.q) + b * a.qs[0] + w * a.qs[2];
  const T* K = reinterpret_cast<const T*>(a.k) + b * a.ks[0] + w * a.ks[2];
  const T* V = reinterpret_cast<const T*>(a.v) + b * a.vs[0] + w * a.vs[2];

  constexpr int NS = DP / M::KSTEP, NP = 32 / M::KSTEP, NT = DP / 32;
  typename M::frag qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) qf[s] = gfrag<T, VEC>(Q, q, a.Nq, a.qs[1], a.D, s, h);
  const float sl2 = a.scale * kLog2e;
  const int nkt = (a.Nk + 31) / 32;

  // ---- pass 0: row statistics of the mixed logits
  float m = -kInf, l = 0.f;
  for (int kt = 0; kt < nkt; ++kt) {
    f32x16 s = zero16();
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) s = M::mma(gfrag<T, VEC>(K, kt * 32 + r32, a.Nk, a.ks[1], a.D, s_, h), qf[s_], s);
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] *= sl2;
    xput(XA, w, lane, s);
    __syncthreads();
    f32x16 s1 = xmix(XA, c1, H, H, lane);
    float mx = -kInf;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kt * 32 + row_of(r, h);
      s1[r] = key < a.Nk ? s1[r] : -kInf;
      mx = fmaxf(mx, s1[r]);
    }
    const float mn = fmaxf(m, mx);
    float ls = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) ls += ex2(s1[r] - mn);
    l = l * ex2(m - mn) + ls;
    m = mn;
    __syncthreads();
  }
  {
    const float mo = __shfl_xor(m, 32), lo = __shfl_xor(l, 32);
    const float mn = fmaxf(m, mo);
    l = l * ex2(m - mn) + lo * ex2(mo - mn);
    m = mn;
  }
  const float il = 1.f / l;

  // ---- pass 1: normalised P, mix, O += P2 V
  f32x16 acco[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acco[t] = zero16();
  WStage<T, DP, VEC> vst;
  for (int kt = 0; kt < nkt; ++kt) {
    f32x16 s = zero16();
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) s = M::mma(gfrag<T, VEC>(K, kt * 32 + r32, a.Nk, a.ks[1], a.D, s_, h), qf[s_], s);
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] *= sl2;
    if constexpr (BF) vst.load(V, kt * 32, a.Nk, a.vs[1], a.D, lane);
    xput(XA, w, lane, s);
    __syncthreads();
    f32x16 p = xmix(XA, c1, H, H, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kt * 32 + row_of(r, h);
      p[r] = key < a.Nk ? ex2(p[r] - m) * il : 0.f;
    }
    xput(XB, w, lane, p);
    if constexpr (BF) vst.write(ldsV, lane);
    __syncthreads();
    const f32x16 p2 = xmix(XB, c2, H, H, lane);
#pragma unroll
    for (int s2 = 0; s2 < NP; ++s2) {
      const typename M::frag pf = acc_frag<T>(p2, s2);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        typename M::frag vf;
        if constexpr (BF) vf = I::colfrag(ldsV, 0, s2, 32 * t, lane);
        else vf = colfrag_g<T>(V, kt * 32, a.Nk, a.vs[1], a.D, s2, 32 * t, lane);
        acco[t] = M::mma(vf, pf, acco[t]);
      }
    }
  }
  if (q < a.Nq) {
    T* O = reinterpret_cast<T*>(a.o) + b * a.os[0] + w * a.os[2] + (long long)q * a.os[1];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        store4<T, VEC>(O, 32 * t + 8 * g + 4 * h, a.D, acco[t][4 * g], acco[t][4 * g + 1], acco[t][4 * g + 2],
                       acco[t][4 * g + 3]);
    if (h == 0) a.lse[((size_t)b * H + w) * a.Nq + q] = (m + lg2(l)) * kLn2;
  }
}

// ============================================================================ bwd: query
template <typename T, int DP, bool VEC>
__global__ __launch_bounds__(512) void th_bwd_q_kernel(ThArgs a) {
  using M = MF<T>;
  using I = Img<T, DP>;
  constexpr bool BF = sizeof(T) == 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r32 = lane & 31;
  float* tabs = reinterpret_cast<float*>(smem);
  float* XA = reinterpret_cast<float*>(smem + kTabBytes);
  float* XB = XA + H * 1024;
  float* dtacc = XB + H * 1024 + w * 2 * H * 64;         // this wave's [2][H][64] lane partials
  char* ldsK = reinterpret_cast<char*>(XB + H * 1024 + H * 2 * H * 64) + w * I::bytes(32);
  const float* c1 = tabs + w;              // T1[i][w]
  const float* t1r = tabs + w * H;         // T1[w][i]
  const float* t2r = tabs + H * H + w * H; // T2[w][i]
  load_tabs(tabs, a.th1, a.th2, H, tid);
  for (int i = lane; i < 2 * H * 64; i += 64) dtacc[i] = 0.f;

  const int nqb = (a.Nq + 31) / 32;
  const int qb = blockIdx.x % nqb, b = blockIdx.x / nqb;
  const int q = qb * 32 + r32;
  const T* Q = reinterpret_cast<const T*>(a.q) + b * a.qs[0] + w * a.qs[2];
  const T* K = reinterpret_cast<const T*>(a.k) + b * a.ks[0] + w * a.ks[2];
  const T* V = reinterpret_cast<const T*>(a.v) + b * a.vs[0] + w * a.vs[2];
  const T* G = reinterpret_cast<const T*>(a.dout) + b * a.dos[0] + w * a.dos[2];

  constexpr int NS = DP / M::KSTEP, NP = 32 / M::KSTEP, NT = DP / 32;
  typename M::frag qf[NS], gf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    qf[s] = gfrag<T, VEC>(Q, q, a.Nq, a.qs[1], a.D, s, h);
    gf[s] = gfrag<T, VEC>(G, q, a.Nq, a.dos[1], a.D, s, h);
  }
  const bool qok = q < a.Nq;
  const size_t rowoff = ((size_t)b * H + w) * a.Nq;
  const float lse2 = qok ? a.lse[rowoff + q] * kLog2e : kInf;
  const float sl2 = a.scale * kLog2e;
  const int nkt = (a.Nk + 31) / 32;

  // ---- pass A: delta_w = rowsum(dP_w o P_w);  dT2[w][i] lane partials = sum P_w o dP2_i
  float dlt = 0.f;
  for (int kt = 0; kt < nkt; ++kt) {
    f32x16 s = zero16(), g = zero16();
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
      s = M::mma(gfrag<T, VEC>(K, kt * 32 + r32, a.Nk, a.ks[1], a.D, s_, h), qf[s_], s);
      g = M::mma(gfrag<T, VEC>(V, kt * 32 + r32, a.Nk, a.vs[1], a.D, s_, h), gf[s_], g);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] *= sl2;
    xput(XA, w, lane, s);
    xput(XB, w, lane, g);
    __syncthreads();
    f32x16 p = xmix(XA, c1, H, H, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kt * 32 + row_of(r, h);
      p[r] = key < a.Nk ? ex2(p[r] - lse2) : 0.f;
    }
    f32x16 dp = zero16();
#pragma unroll 2
    for (int i = 0; i < H; ++i) {
      const float c = t2r[i];
      const f32x16 x = xget(XB, i, lane);
      float acc = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dp[r] += c * x[r];
        acc += p[r] * x[r];
      }
      dtacc[(H + i) * 64 + lane] += acc;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) dlt += p[r] * dp[r];
    __syncthreads();
  }
  dlt += __shfl_xor(dlt, 32);

  // ---- pass B: dS1 = P (dP - delta); dS_w = sum_i T1[w][i] dS1_i; dQ; dT1[h][w] partials
  f32x16 adq[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) adq[t] = zero16();
  WStage<T, DP, VEC> kst;
  for (int kt = 0; kt < nkt; ++kt) {
    f32x16 s = zero16(), g = zero16();
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
      s = M::mma(gfrag<T, VEC>(K, kt * 32 + r32, a.Nk, a.ks[1], a.D, s_, h), qf[s_], s);
      g = M::mma(gfrag<T, VEC>(V, kt * 32 + r32, a.Nk, a.vs[1], a.D, s_, h), gf[s_], g);
    }
    if constexpr (BF) kst.load(K, kt * 32, a.Nk, a.ks[1], a.D, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] *= sl2;
    xput(XA, w, lane, s);
    xput(XB, w, lane, g);
    __syncthreads();                                     // B1
    f32x16 ds1 = xmix(XA, c1, H, H, lane);
    {
      const f32x16 dp = xmix(XB, t2r, 1, H, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + row_of(r, h);
        const float p = key < a.Nk ? ex2(ds1[r] - lse2) : 0.f;
        ds1[r] = p * (dp[r] - dlt);
      }
    }
#pragma unroll 2
    for (int i = 0; i < H; ++i) {
      const f32x16 x = xget(XA, i, lane);
      float acc = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc += x[r] * ds1[r];
      dtacc[i * 64 + lane] += acc;
    }
    if constexpr (BF) kst.write(ldsK, lane);
    __syncthreads();                                     // B2
    xput(XA, w, lane, ds1);
    __syncthreads();                                     // B3
    const f32x16 ds = xmix(XA, t1r, 1, H, lane);
#pragma unroll
    for (int s2 = 0; s2 < NP; ++s2) {
      const typename M::frag sf = acc_frag<T>(ds, s2);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        typename M::frag kf;
        if constexpr (BF) kf = I::colfrag(ldsK, 0, s2, 32 * t, lane);
        else kf = colfrag_g<T>(K, kt * 32, a.Nk, a.ks[1], a.D, s2, 32 * t, lane);
        adq[t] = M::mma(kf, sf, adq[t]);
      }
    }
    __syncthreads();                                     // B4
  }

  if (qok) {
    T* DQ = reinterpret_cast<T*>(a.dq) + b * a.dqs[0] + w * a.dqs[2] + (long long)q * a.dqs[1];
    const float sc = a.scale;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        store4<T, VEC>(DQ, 32 * t + 8 * g4 + 4 * h, a.D, adq[t][4 * g4] * sc, adq[t][4 * g4 + 1] * sc,
                       adq[t][4 * g4 + 2] * sc, adq[t][4 * g4 + 3] * sc);
    if (h == 0) a.delta[rowoff + q] = dlt;
  }
  // per-workgroup transform-gradient partials: part[blk][0][h][i] = dT1, part[blk][1][h][i] = dT2
  float* pb = a.part + (size_t)blockIdx.x * 2 * H * H;
  for (int i = 0; i < H; ++i) {
    const float v1 = wave_sum(dtacc[i * 64 + lane]) * (1.f / kLog2e);   // XA held S * log2(e)
    const float v2 = wave_sum(dtacc[(H + i) * 64 + lane]);
    if (lane == 0) {
      pb[i * H + w] = v1;           // dT1[i][w]
      pb[H * H + w * H + i] = v2;   // dT2[w][i]
    }
  }
}

// =============================================================================== bwd: kv
template <typename T, int DP, bool VEC>
__global__ __launch_bounds__(512) void th_bwd_kv_kernel(ThArgs a) {
  using M = MF<T>;
  using I = Img<T, DP>;
  constexpr bool BF = sizeof(T) == 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = a.H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, r32 = lane & 31;
  float* tabs = reinterpret_cast<float*>(smem);
  float* XA = reinterpret_cast<float*>(smem + kTabBytes);
  float* XB = XA + H * 1024;
  float* rowc = XB + H * 1024;                       // [H][2][32]: lse2, delta of this q tile
  char* ldsQ = reinterpret_cast<char*>(rowc + H * 64) + w * 2 * I::bytes(32);
  char* ldsG = ldsQ + I::bytes(32);
  const float* c1 = tabs + w;              // T1[i][w]
  const float* c2 = tabs + H * H + w;      // T2[i][w]
  const float* t1r = tabs + w * H;         // T1[w][i]
  const float* t2r = tabs + H * H + w * H; // T2[w][i]
  load_tabs(tabs, a.th1, a.th2, H, tid);

  const int nkb = (a.Nk + 31) / 32;
  const int kb = blockIdx.x % nkb, b = blockIdx.x / nkb;
  const int key = kb * 32 + r32;
  const T* Q = reinterpret_cast<const T*>(a.q) + b * a.qs[0] + w * a.qs[2];
  const T* K = reinterpret_cast<const T*>(a.k) + b * a.ks[0] + w * a.ks[2];
  const T* V = reinterpret_cast<const T*>(a.v) + b * a.vs[0] + w * a.vs[2];
  const T* G = reinterpret_cast<const T*>(a.dout) + b * a.dos[0] + w * a.dos[2];

  constexpr int NS = DP / M::KSTEP, NP = 32 / M::KSTEP, NT = DP / 32;
  typename M::frag kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    kf[s] = gfrag<T, VEC>(K, key, a.Nk, a.ks[1], a.D, s, h);
    vf[s] = gfrag<T, VEC>(V, key, a.Nk, a.vs[1], a.D, s, h);
  }
  const size_t rowoff = ((size_t)b * H + w) * a.Nq;
  const float sl2 = a.scale * kLog2e;
  float* myc = rowc + w * 64;
  f32x16 adk[NT], adv[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) { adk[t] = zero16(); adv[t] = zero16(); }
  WStage<T, DP, VEC> qst, gst;
  const int nqt = (a.Nq + 31) / 32;
  for (int qt = 0; qt < nqt; ++qt) {
    __syncthreads();                                     // B0: previous tile's readers done
    if (lane < 32) {
      const int qq = qt * 32 + lane;
      myc[lane] = qq < a.Nq ? a.lse[rowoff + qq] * kLog2e : kInf;
      myc[32 + lane] = qq < a.Nq ? a.delta[rowoff + qq] : 0.f;
    }
    if constexpr (BF) {
      qst.load(Q, qt * 32, a.Nq, a.qs[1], a.D, lane);
      gst.load(G, qt * 32, a.Nq, a.dos[1], a.D, lane);
      qst.write(ldsQ, lane);
      gst.write(ldsG, lane);
    }
    f32x16 s = zero16(), g = zero16();
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
      typename M::frag qa, ga;
      if constexpr (BF) {
        qa = I::rowfrag(ldsQ, r32, s_, h);
        ga = I::rowfrag(ldsG, r32, s_, h);
      } else {
        qa = gfrag<T, VEC>(Q, qt * 32 + r32, a.Nq, a.qs[1], a.D, s_, h);
        ga = gfrag<T, VEC>(G, qt * 32 + r32, a.Nq, a.dos[1], a.D, s_, h);
      }
      s = M::mma(qa, kf[s_], s);
      g = M::mma(ga, vf[s_], g);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] *= sl2;
    xput(XA, w, lane, s);
    xput(XB, w, lane, g);
    __syncthreads();                                     // B1
    f32x16 p = xmix(XA, c1, H, H, lane);
    f32x16 ds1 = xmix(XB, t2r, 1, H, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ql = row_of(r, h);
      p[r] = ex2(p[r] - myc[ql]);
      ds1[r] = p[r] * (ds1[r] - myc[32 + ql]);
    }
    __syncthreads();                                     // B2
    xput(XA, w, lane, p);
    xput(XB, w, lane, ds1);
    __syncthreads();                                     // B3
    const f32x16 p2 = xmix(XA, c2, H, H, lane);
    const f32x16 ds = xmix(XB, t1r, 1, H, lane);
#pragma unroll
    for (int s2 = 0; s2 < NP; ++s2) {
      const typename M::frag pf = acc_frag<T>(p2, s2);
      const typename M::frag sf = acc_frag<T>(ds, s2);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        typename M::frag gq, qq;
        if constexpr (BF) {
          gq = I::colfrag(ldsG, 0, s2, 32 * t, lane);
          qq = I::colfrag(ldsQ, 0, s2, 32 * t, lane);
        } else {
          gq = colfrag_g<T>(G, qt * 32, a.Nq, a.dos[1], a.D, s2, 32 * t, lane);
          qq = colfrag_g<T>(Q, qt * 32, a.Nq, a.qs[1], a.D, s2, 32 * t, lane);
        }
        adv[t] = M::mma(gq, pf, adv[t]);
        adk[t] = M::mma(qq, sf, adk[t]);
      }
    }
  }
  if (key < a.Nk) {
    T* DK = reinterpret_cast<T*>(a.dk) + b * a.dks[0] + w * a.dks[2] + (long long)key * a.dks[1];
    T* DV = reinterpret_cast<T*>(a.dv) + b * a.dvs[0] + w * a.dvs[2] + (long long)key * a.dvs[1];
    const float sc = a.scale;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * t + 8 * g4 + 4 * h;
        store4<T, VEC>(DK, d0, a.D, adk[t][4 * g4] * sc, adk[t][4 * g4 + 1] * sc, adk[t][4 * g4 + 2] * sc,
                       adk[t][4 * g4 + 3] * sc);
        store4<T, VEC>(DV, d0, a.D, adv[t][4 * g4], adv[t][4 * g4 + 1], adv[t][4 * g4 + 2], adv[t][4 * g4 + 3]);
      }
  }
}

// fixed-order reduction of the per-workgroup dT partials: one workgroup per dT element; thread t
// sums partials t, t + 256, ... in order, then a fixed-shape LDS tree (deterministic, and ~40x
// faster than one thread walking all nblk partials serially: 206 -> ~5 us at CaiT-S24 shapes)
__global__ __launch_bounds__(256) void th_reduce_kernel(ThArgs a) {
  __shared__ float red[256];
  const int HH = a.H * a.H;
  const int i = blockIdx.x;   // dT element (th1: i < HH, th2: HH <= i < 2 HH)
  const int t = threadIdx.x;
  float acc = 0.f;
  for (int blk = t; blk < a.nblk; blk += 256) acc += a.part[(size_t)blk * 2 * HH + i];
  red[t] = acc;
  __syncthreads();
#pragma unroll
  for (int off = 128; off > 0; off >>= 1) {
    if (t < off) red[t] += red[t + off];
    __syncthreads();
  }
  if (t == 0) {
    if (i < HH) a.dth1[i] = red[0];
    else a.dth2[i - HH] = red[0];
  }
}

}  // namespace sae

// ---------------------------------------------------------------- launchers (capi.hip)
struct sae_attn_desc;
int th_fwd(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v, const float* th1,
           const float* th2, void* o, float* lse, const sae::RopeTab* rope = nullptr);
size_t th_bwd_workspace_bytes(const sae_attn_desc* d);
int th_bwd(void* stream, const sae_attn_desc* d, const void* q, const void* k, const void* v, const float* th1,
           const float* th2, const float* lse, const void* dout, void* dq, void* dk, void* dv, float* dth1,
           float* dth2, void* workspace, const sae::RopeTab* rope = nullptr);
