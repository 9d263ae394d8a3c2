// Probe build of gemm8.h variants (dev only: tools/probe/gemm8_probe.py loads it by ctypes).
#include <cstring>
#include <algorithm>
#include "../../self-attention-experiments-vision_amd/csrc/gemm8.h"

using namespace sae;
static int g_persist = 0;   // > 0: persistent grid of at most that many workgroups

template <int EPI, int BN, int BK, int NS, int MODE = 0, int BM = 256>
static int launch(const NtArgs& g, hipStream_t st) {
  constexpr int lds = g8_lds_bytes<BN, BK, NS>();
  const void* fn = (const void*)gemm8_nt_kernel<EPI, BN, BK, NS, MODE, BM>;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return 2;
  const long long tiles = (long long)((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  const long long grid = g_persist ? std::min<long long>(tiles, g_persist) : tiles;
  hipLaunchKernelGGL((gemm8_nt_kernel<EPI, BN, BK, NS, MODE, BM>), dim3((unsigned)grid), dim3(512), lds, st, g);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

template <int BN, int BK, int NS, int BM = 256>
static int launch_epi(const NtArgs& g, int epi, hipStream_t st) {
  if (epi == 0) return launch<kEpiNone, BN, BK, NS, 0, BM>(g, st);
  if (epi == 1) return launch<kEpiGelu, BN, BK, NS, 0, BM>(g, st);
  return launch<kEpiDGelu, BN, BK, NS, 0, BM>(g, st);
}

template <int EPI, int BN, bool BAL = false, int BM = 256>
static int launchx(const NtArgs& g, hipStream_t st) {
  constexpr int lds = g8x_lds_bytes<BN, BM>();
  const void* fn = (const void*)gemm8x_nt_kernel<EPI, BN, BAL, BM>;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return 2;
  if (g.K % 32) return 4;
  const long long tiles = (long long)((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm8x_nt_kernel<EPI, BN, BAL, BM>), dim3((unsigned)tiles), dim3(512), lds, st, g);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// stream-K ping-pong (gemm8s): one workgroup per CU, workspace kept across calls, flags zeroed
// before each launch
static float* g_skpart = nullptr;
static int* g_skflag = nullptr;
static int launchs(NtArgs g, hipStream_t st) {
  constexpr int lds = g8x_lds_bytes<256>();
  const void* fn = (const void*)gemm8s_nt_kernel<256>;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return 2;
  if (g.K % 32) return 4;
  const int G = 256;
  if (!g_skpart) {
    if (hipMalloc(&g_skpart, (size_t)G * 256 * 256 * 4) != hipSuccess) return 6;
    if (hipMalloc(&g_skflag, (size_t)G * 4) != hipSuccess) return 6;
  }
  if (hipMemsetAsync(g_skflag, 0, (size_t)G * 4, st) != hipSuccess) return 7;
  g.skpart = g_skpart;
  g.skflag = g_skflag;
  hipLaunchKernelGGL((gemm8s_nt_kernel<256>), dim3(G), dim3(512), lds, st, g);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

extern "C" int g8_run(int variant, void* stream, int M, int N, int K, const void* a, long long lda, const void* bt,
                      long long ldb, const float* bias, void* c, long long ldc, int epi, const void* aux,
                      long long ldaux, void* c2) {
  NtArgs g;
  memset(&g, 0, sizeof g);
  g.a = (const __bf16*)a;
  g.bt = (const __bf16*)bt;
  g.bias = bias;
  g.aux = (const __bf16*)aux;
  g.c = (__bf16*)c;
  g.c2 = (__bf16*)c2;
  g.M = M;
  g.N = N;
  g.K = K;
  g.lda = lda;
  g.ldb = ldb;
  g.ldc = ldc;
  g.ldaux = ldaux;
  hipStream_t st = (hipStream_t)stream;
  g_persist = variant >= 10 ? 256 : 0;
  if (variant == 40) return epi == 0 ? launchx<kEpiNone, 256>(g, st) : epi == 1 ? launchx<kEpiGelu, 256>(g, st) : 5;
  if (variant == 41) return epi == 0 ? launchx<kEpiNone, 192>(g, st) : epi == 1 ? launchx<kEpiGelu, 192>(g, st) : 5;
  if (variant == 43) return epi == 0 ? launchx<kEpiNone, 256, true>(g, st) : epi == 1 ? launchx<kEpiGelu, 256, true>(g, st) : 5;
  if (variant == 44) return epi == 0 ? launchx<kEpiNone, 192, true>(g, st) : epi == 1 ? launchx<kEpiGelu, 192, true>(g, st) : 5;
  if (variant == 46) return epi == 0 ? launchs(g, st) : 5;
  if (variant == 45) return epi == 0 ? launchx<kEpiNone, 256, true, 224>(g, st) : epi == 1 ? launchx<kEpiGelu, 256, true, 224>(g, st) : 5;
  if (variant == 55) { g_persist = 256; return launch_epi<128, 64, 2, 224>(g, epi, st); }
  if (variant == 53) { g_persist = 256; return launch_epi<192, 64, 2, 224>(g, epi, st); }
  if (variant == 50) { g_persist = 256; return launch_epi<256, 32, 3, 224>(g, epi, st); }
  if (variant == 51) { g_persist = 256; return launch_epi<192, 64, 2, 192>(g, epi, st); }
  if (variant == 42) return epi == 0 ? launchx<kEpiNone, 128>(g, st) : epi == 1 ? launchx<kEpiGelu, 128>(g, st) : 5;
  if (variant >= 20) {   // staging / store experiments on the persistent 256 x 192 bk64 ns2 tile
    g_persist = 256;
    if (variant == 21) return epi == 0 ? launch<kEpiNone, 192, 64, 2, 1>(g, st) : 1;
    if (variant == 22) return epi == 0 ? launch<kEpiNone, 192, 64, 2, 2>(g, st) : 1;
    if (variant == 23) return epi == 0 ? launch<kEpiNone, 256, 32, 3, 1>(g, st) : 1;
    if (variant == 24) return epi == 0 ? launch<kEpiNone, 256, 32, 3, 2>(g, st) : 1;
    return 1;
  }
  switch (variant % 10) {
    case 0: return launch_epi<256, 32, 3>(g, epi, st);
    case 1: return launch_epi<192, 32, 3>(g, epi, st);
    case 2: return launch_epi<192, 32, 4>(g, epi, st);
    case 3: return launch_epi<192, 64, 2>(g, epi, st);
    case 4: return launch_epi<128, 32, 4>(g, epi, st);
    case 5: return launch_epi<128, 64, 2>(g, epi, st);
  }
  return 1;
}
