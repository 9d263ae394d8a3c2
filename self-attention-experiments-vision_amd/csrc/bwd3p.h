// bwd3p.h -- persistent form of the single-pass bf16 attention backward (bwd3.h).
//
// Same algorithm, layout and arithmetic as attn_bwd3_kernel (the JAX autodiff of
// models/layers/attentions/attention.py:39-58: dV = P^T dO, dP = dO V^T, dS = P o (dP - delta),
// dK = scale dS^T Q, dQ = scale dS K; bit-identical results), with the launch shaped around what
// the in-kernel stamps of that kernel showed (tools/stamps.py, profiles/r03_stamps_*.txt): at
// DeiT-S its 768 workgroups run as three synchronous rounds of 256, and every round opens with
// ~9k cycles of K / V / first-tile loads that all 256 CUs issue at once (an HBM-bound burst, 25 %
// of a workgroup's life) before any MFMA runs.  Here one workgroup per CU walks its (batch, head)
// units u = blockIdx.x, blockIdx.x + gridDim.x, ...:
//   * the NEXT unit's K and V rows are copied into LDS images by buffer_load ... lds (LDS-DMA:
//     no registers, hardware range check = zero rows past Nk and zero head-dim padding) during the
//     current unit's last two query tiles, so the unit prologue reads its K / V fragments from LDS;
//     the K image (double-buffered across units) is also the dQ product's K^T operand, read per
//     tile instead of held in 32 registers (the persistent loop's extra state would spill);
//   * the current unit's last step stages the next unit's first Q / dO / O tile in registers,
//     so only the very first unit of a workgroup waits for global memory.
// The K / V image uses the tile images' XOR swizzle: LDS-DMA writes each wave-instruction's 64 x
// 16 bytes linearly, so the swizzle is applied to the per-lane SOURCE address (row r, slot c' of
// the image holds chunk c' ^ swz(r)) and the fragment reads use the same swizzled addresses.
#pragma once
#include "bwd3.h"

namespace sae {

template <int DP, int NW> struct B3P {
  using C = B3<DP, NW, 1>;
  static constexpr int KVIMG = C::BK * DP * 2;             // one [BK keys][DP] bf16 image
  static constexpr int PF = C::LDS;                        // prefetch images after bwd3's LDS
  static constexpr int LDS = PF + 3 * KVIMG;               // [... | K image x 2 | V image]
  static constexpr int RPI = 1024 / (DP * 2);              // image rows per 1 KiB DMA piece
  static constexpr int PIECES = KVIMG / 1024;              // pieces per image
  static_assert(PIECES % NW == 0, "DMA pieces split evenly over the waves");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// One 16-byte-per-lane LDS-DMA piece (1 KiB at the wave-uniform LDS byte address `lds`).  Inline
// asm on purpose: issued through the builtin, the LDS-DMA makes hipcc put an s_waitcnt vmcnt(0)
// in front of the first LDS read of every later tile (it cannot tell that the DMA's image is not
// the one read), which drained the register prefetch of the next Q / dO tile in every iteration
// (measured: 70 vs 55 us at DeiT-S).  Counted by hand instead: the unit's last wait (vm_wait_all +
// barrier) retires it before any read of the image.  M0 is compiler-reserved: saved and restored
// inside the statement (cdna_hip_programming.md §5.7: s_nop 4 for a fresh descriptor, s_nop 0
// after the M0 write).
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
__device__ __forceinline__ void dma16(u32x4 rs, unsigned voff, unsigned lds) {
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
__device__ __forceinline__ u32x4 row_rsrc_words(const T* base, int nrows, long long rs) {
  const unsigned long long p = reinterpret_cast<unsigned long long>(base);
  u32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((unsigned)p);
  r[1] = __builtin_amdgcn_readfirstlane((unsigned)(p >> 32)) & 0xffffu;   // stride 0
  r[2] = __builtin_amdgcn_readfirstlane((unsigned)((long long)nrows * rs * sizeof(T)));
  r[3] = 0x00020000u;
  return r;
}

// rows past Nk and columns past D read as zero through the buffer descriptor's range check
template <int DP, int NW>
__device__ __forceinline__ void b3p_dma_image(u32x4 rsw, long long rowstride, int D, char* img, int w, int lane) {
  using P = B3P<DP, NW>;
  constexpr int CPR = DP / 8;
  const unsigned base = __builtin_amdgcn_readfirstlane(
      (unsigned)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) char*)img));
#pragma unroll
  for (int i = 0; i < P::PIECES / NW; ++i) {
    const int piece = i * NW + w;
    const int r = piece * P::RPI + lane / CPR;
    const int c = (lane % CPR) ^ swz<DP>(r);   // the chunk this lane's 16 LDS bytes hold
    const unsigned off = (c * 8 < D) ? (unsigned)(((long long)r * rowstride + c * 8) * 2) : 0x80000000u;
    dma16(rsw, off, base + (unsigned)(piece * 1024));
  }
}

template <int DP, int NW, int NSU = DP / 16>
__global__ __launch_bounds__(64 * NW, 2) void attn_bwd3p_kernel(AttnArgs a) {
  using C = B3<DP, NW, 1>;
  using P = B3P<DP, NW>;
  constexpr int NS = NSU, NT = C::NT, TB = C::TB, KS = C::KS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const dsb = smem + 2 * TB;   // two dS^T images
  char* const kimg0 = smem + P::PF;           // K rows: this unit's / the next unit's (alternating)
  char* const pfv = kimg0 + 2 * P::KVIMG;     // next unit's V rows

  const int nunits = a.B * a.H;
  int u = blockIdx.x;
  if (u >= nunits) return;   // (uniform)
  const int G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wrow = w * 32;                    // first key (image row) of this wave
  const bool active = wrow < a.Nk;            // wave-uniform: this wave holds at least one key
  const int nqt = (a.Nq + 31) / 32;
  const float sl2 = a.scale * kLog2e;

  // per-unit buffer descriptors, rebuilt where they are used (SALU work) from kernel arguments
  // re-read through an opaque kernarg pointer: held across the unit loop, the descriptors and the
  // argument words they come from spilled SGPRs into VGPRs (and those into scratch)
  typedef const AttnArgs __attribute__((address_space(4))) KArgs;   // scalar (s_load) reads
  auto arg = [&]() -> KArgs& {
    KArgs* p = (KArgs*)(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(p));
    return *p;
  };
  auto rsq = [&](int uu) {
    KArgs& a = arg();
    const int b = uu / a.H, hh = uu - b * a.H;
    return row_rsrc(reinterpret_cast<const __bf16*>(a.q) + b * a.qs[0] + hh * a.qs[2], a.Nq, a.qs[1]);
  };
  auto rsg = [&](int uu) {
    KArgs& a = arg();
    const int b = uu / a.H, hh = uu - b * a.H;
    return row_rsrc(reinterpret_cast<const __bf16*>(a.dout) + b * a.dos[0] + hh * a.dos[2], a.Nq, a.dos[1]);
  };
  auto rso = [&](int uu) {
    KArgs& a = arg();
    const int b = uu / a.H, hh = uu - b * a.H;
    return row_rsrc(reinterpret_cast<const __bf16*>(a.o) + b * a.os[0] + hh * a.os[2], a.Nq, a.os[1]);
  };
  auto rsk = [&](int uu) {
    KArgs& a = arg();
    const int b = uu / a.H, hh = uu - b * a.H;
    return row_rsrc_words(reinterpret_cast<const __bf16*>(a.k) + b * a.ks[0] + hh * a.ks[2], a.Nk, a.ks[1]);
  };
  auto rsv = [&](int uu) {
    KArgs& a = arg();
    const int b = uu / a.H, hh = uu - b * a.H;
    return row_rsrc_words(reinterpret_cast<const __bf16*>(a.v) + b * a.vs[0] + hh * a.vs[2], a.Nk, a.vs[1]);
  };
  auto stage = [&](B3Stage<DP, NW>& st_, int uu, int qt) {
    st_.load(rsq(uu), rsg(uu), rso(uu), a, qt, (size_t)uu * a.Nq, tid);   // rowoff = (b H + hh) Nq
  };

  B3Stage<DP, NW> st;
  st.init(tid, a);
  // first unit: its K / V rows by DMA and its first tile in registers
  b3p_dma_image<DP, NW>(rsk(u), a.ks[1], a.D, kimg0, w, lane);
  b3p_dma_image<DP, NW>(rsv(u), a.vs[1], a.D, pfv, w, lane);
  stage(st, u, 0);
  vm_wait_all();
  __syncthreads();

  // loop-invariant LDS addresses (as attn_bwd3_kernel)
  const int db = w % C::NDB;
  const bool dqw = w < C::NDQ;
  const int li = lane & 15, gq = lane >> 4;
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
  unsigned wa[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) wa[g] = (unsigned)ds_off(wrow + r32, 2 * g + h);
  bf16x8 one01;
#pragma unroll
  for (int j = 0; j < 8; ++j) one01[j] = (__bf16)((h == 0 && j < 2) ? 1.f : 0.f);
  const int rr = wrow + r32;   // this lane's key row in the images

  for (int par = 0; u < nunits; u += G, par ^= 1) {
    const int un = u + G;
    // this unit's K image (the dQ product's K^T operand for the whole sweep) and the next unit's
    const char* const kimg = kimg0 + par * P::KVIMG;
    char* const pfk = kimg0 + (par ^ 1) * P::KVIMG;
    const bool has_next = un < nunits;
    const int cb = u / a.H, ch = u - cb * a.H;   // this unit's (batch, head)

    // ---- unit prologue: K / V fragments from the prefetched images (the K image stays: it is the
    //      dQ product's K^T operand, read by every tile instead of held in registers)
    bf16x8 kf[NS], vf[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const unsigned o = rr * DP * 2 + 16 * ((2 * s + h) ^ swz<DP>(rr));
      kf[s] = *reinterpret_cast<const bf16x8*>(kimg + o);
      vf[s] = *reinterpret_cast<const bf16x8*>(pfv + o);
    }
    st.write(smem, tid);
    f32x16 adk[NT], adv[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      adk[t] = zero16();
      adv[t] = zero16();
    }
    __syncthreads();   // tile 0 staged; every wave holds its K / V fragments: the V image is free
    if (!active) {     // a wave past the last key writes zero dS once (its K rows are zero)
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      const bf16x4 z = {};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        *reinterpret_cast<bf16x4*>(dsb + wa[g]) = z;
        *reinterpret_cast<bf16x4*>(dsb + C::DSIMG + wa[g]) = z;
      }
    }

    auto dq_tile = [&](const char* img, int qt) {
      if (!dqw) return;
#pragma unroll
      for (int t = 0; t < C::TPW; ++t) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int r1 = 32 * ks + 8 * gq + (li >> 2), r2 = r1 + 4;
          const int col = 16 * db + 4 * (li & 3);
          const int chk = col >> 3, hf = (col >> 2) & 1;
          const bf16x8 aq = tr2(kimg + r1 * DP * 2 + 16 * (chk ^ swz<DP>(r1)) + 8 * hf,
                                kimg + r2 * DP * 2 + 16 * (chk ^ swz<DP>(r2)) + 8 * hf);
          const bf16x8 bq = tr2(img + da[t][0] + ks * 32 * 64, img + da[t][1] + ks * 32 * 64);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq, bq, acc, 0, 0, 0);
        }
        const int qq = qt * 32 + 16 * qhs[t] + li;
        const int d0 = 16 * db + 4 * gq;
        if (qq < a.Nq && d0 < a.D) {
          typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
          const bf16x4 v = {(__bf16)(acc[0] * a.scale), (__bf16)(acc[1] * a.scale), (__bf16)(acc[2] * a.scale),
                            (__bf16)(acc[3] * a.scale)};
          __bf16* DQ = reinterpret_cast<__bf16*>(a.dq) + cb * a.dqs[0] + ch * a.dqs[2] + (long long)qq * a.dqs[1];
          *reinterpret_cast<bf16x4*>(DQ + d0) = v;
        }
      }
    };

    // one query tile (as attn_bwd3_kernel), plus: the last step stages the next unit's first tile,
    // the last two steps copy the next unit's K (then V) rows into the prefetch images
    auto step = [&](int qt, auto bsel_c) {
      constexpr int bsel = decltype(bsel_c)::value;
      const char* ldsQ = smem + bsel * TB;
      const char* ldsG = ldsQ + C::QIMG;
      const float* ldsL = reinterpret_cast<const float*>(ldsQ + 2 * C::QIMG);
      const float* ldsD = ldsL + 32;
      char* img = dsb + bsel * C::DSIMG;
      if (qt + 1 < nqt) stage(st, u, qt + 1);
      else if (has_next) stage(st, un, 0);
      if (has_next) {
        if (qt == (nqt >= 2 ? nqt - 2 : 0)) b3p_dma_image<DP, NW>(rsk(un), a.ks[1], a.D, pfk, w, lane);
        if (qt == nqt - 1) b3p_dma_image<DP, NW>(rsv(un), a.vs[1], a.D, pfv, w, lane);
      }
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
        f32x16 sp = zero16();
        f32x16 dp = MF<__bf16>::mma(dla, one01, zero16());
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          sp = MF<__bf16>::mma(qr[s], kf[s], sp);
          dp = MF<__bf16>::mma(gr[s], vf[s], dp);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float p = __builtin_amdgcn_fmed3f(ex2(__builtin_fmaf(sp[4 * g + i], sl2, -l4[g][i])), 0.f, 1.f);
            sp[4 * g + i] = p;
            dp[4 * g + i] *= p;
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
          const bf16x8 pf = acc_frag<__bf16>(sp, s2);
          const bf16x8 sf = acc_frag<__bf16>(dp, s2);
          const uint4 su = __builtin_bit_cast(uint4, sf);
          *reinterpret_cast<uint2*>(img + wa[2 * s2]) = make_uint2(su.x, su.y);
          *reinterpret_cast<uint2*>(img + wa[2 * s2 + 1]) = make_uint2(su.z, su.w);
#pragma unroll
          for (int tt = 0; tt < NT; ++tt) {
            adv[tt] = MF<__bf16>::mma(gt[tt], pf, adv[tt]);
            adk[tt] = MF<__bf16>::mma(qt_[tt], sf, adk[tt]);
          }
        }
      }
      if (qt > 0) dq_tile(dsb + (bsel ^ 1) * C::DSIMG, qt - 1);
      if (qt + 1 < nqt) st.write(smem + (bsel ^ 1) * TB, tid);
      __syncthreads();
    };
    {
      using B0 = std::integral_constant<int, 0>;
      using B1 = std::integral_constant<int, 1>;
      for (int qt = 0; qt < nqt; qt += 2) {
        step(qt, B0{});
        if (qt + 1 < nqt) step(qt + 1, B1{});
      }
    }
    dq_tile(dsb + ((nqt - 1) & 1) * C::DSIMG, nqt - 1);
    vm_wait_all();     // the next unit's DMA (issued in the last two steps) has landed ...
    __syncthreads();   // ... for every wave; every image read: the LDS below the prefetch images
                       // becomes the store scratch
    if (active) {
      char* scr = smem + w * 32 * DP * 2;
      __bf16* DK = reinterpret_cast<__bf16*>(a.dk) + cb * a.dks[0] + ch * a.dks[2] + (long long)wrow * a.dks[1];
      __bf16* DV = reinterpret_cast<__bf16*>(a.dv) + cb * a.dvs[0] + ch * a.dvs[2] + (long long)wrow * a.dvs[1];
      wave_store_rows<DP>(adk, a.scale, scr, DK, a.dks[1], a.Nk - wrow, a.D, lane);
      wave_store_rows<DP>(adv, 1.f, scr, DV, a.dvs[1], a.Nk - wrow, a.D, lane);
    }
    __syncthreads();   // the scratch is free again (the stores need not have left)
  }
}

}  // namespace sae
