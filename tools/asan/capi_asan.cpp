// Host-side AddressSanitizer run of the C ABI ("race detection / sanitizers":
// the reference has none; this is the host half of the plan -- GPU ASan is not available on the
// MI355X pool).  Built by tools/asan/build.sh with the host code of capi.hip instrumented
// (-Xarch_host -fsanitize=address); needs no GPU.  It drives every host-only code path of the ABI
// with exact-capacity heap tables, so any overrun of a caller buffer or a descriptor is caught:
//   * the AdamW chunk / tile planners (host only: they write the tables the caller allocated), on
//     random item lists, at exact capacity and one short (must refuse, not overrun);
//   * every workspace-size function over a sweep of shapes (no overflow, no negative sizes);
//   * the validation of every launcher (bad shapes, strides, alignment, NULLs): the error code and
//     sae_last_error() text, read back each time.
// Launchers whose arguments pass validation would launch: with no GPU the HIP launch fails and
// the ABI reports SAE_EHIP, which is the expected outcome here (no device memory is touched).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "sae_attn.h"

static int g_checks = 0, g_fail = 0;

static void expect(bool ok, const char* what) {
  ++g_checks;
  if (!ok) {
    ++g_fail;
    std::printf("FAIL %s (last error: %s)\n", what, sae_last_error());
  }
}

// a heap block per fake pointer, so a host-side dereference would be an ASan report
static void* fake(size_t bytes = 4096) {
  void* p = nullptr;
  if (posix_memalign(&p, 256, bytes)) std::abort();
  std::memset(p, 0, bytes);
  return p;
}

static void adamw_plans(std::mt19937& rng) {
  for (int trial = 0; trial < 200; ++trial) {
    const int n = 1 + rng() % 40;
    std::vector<float*> p(n), m(n), v(n);
    std::vector<const float*> g(n);
    std::vector<int64_t> sz(n);
    int64_t need = 0;
    for (int i = 0; i < n; ++i) {
      sz[i] = 1 + rng() % 20000;
      // misaligned starts on purpose (the plan marks those chunks scalar)
      p[i] = reinterpret_cast<float*>(0x100000 + 4 * (rng() % 7) + 0x1000000LL * i);
      g[i] = p[i] + 1;
      m[i] = p[i] + 2;
      v[i] = p[i] + 3;
      need += (sz[i] + SAE_ADAMW_CHUNK - 1) / SAE_ADAMW_CHUNK;
    }
    sae_adamw_chunk* exact = new sae_adamw_chunk[need];
    int64_t got = -1;
    expect(sae_adamw_plan(n, p.data(), g.data(), m.data(), v.data(), sz.data(), exact, need, &got) == SAE_OK &&
               got == need,
           "adamw_plan at exact capacity");
    int64_t total = 0;
    for (int64_t c = 0; c < got; ++c) total += exact[c].n;
    int64_t want = 0;
    for (int i = 0; i < n; ++i) want += sz[i];
    expect(total == want, "adamw_plan covers every element once");
    delete[] exact;
    if (need > 1) {
      sae_adamw_chunk* shrt = new sae_adamw_chunk[need - 1];
      expect(sae_adamw_plan(n, p.data(), g.data(), m.data(), v.data(), sz.data(), shrt, need - 1, &got) != SAE_OK,
             "adamw_plan refuses a short table");
      delete[] shrt;
    }
  }
  for (int trial = 0; trial < 200; ++trial) {
    const int n = 1 + rng() % 12;
    std::vector<float*> p(n), m(n), v(n);
    std::vector<const float*> g(n);
    std::vector<int32_t> K(n), N(n), ld16(n), ldT(n), col0(n);
    std::vector<void*> w16(n), wt16(n);
    int64_t need = 0;
    for (int i = 0; i < n; ++i) {
      K[i] = 4 * (1 + rng() % 300);
      N[i] = 4 * (1 + rng() % 300);
      col0[i] = 4 * (rng() % 8);
      ld16[i] = N[i] + col0[i] + 4 * (rng() % 3);
      ldT[i] = K[i] + 4 * (rng() % 3);
      p[i] = reinterpret_cast<float*>(0x200000LL + 0x10000000LL * i);
      g[i] = p[i] + 0x1000000;
      m[i] = p[i] + 0x2000000;
      v[i] = p[i] + 0x3000000;
      w16[i] = rng() % 4 ? reinterpret_cast<void*>(p[i] + 0x4000000) : nullptr;
      wt16[i] = (rng() % 4 || !w16[i]) ? reinterpret_cast<void*>(p[i] + 0x5000000) : nullptr;   // >= 1 copy
      need += (int64_t)((K[i] + 63) / 64) * ((N[i] + 63) / 64);
    }
    sae_adamw_cast_tile* exact = new sae_adamw_cast_tile[need];
    int64_t got = -1;
    expect(sae_adamw_cast_plan(n, p.data(), g.data(), m.data(), v.data(), K.data(), N.data(), w16.data(),
                               ld16.data(), wt16.data(), ldT.data(), col0.data(), exact, need, &got) == SAE_OK &&
               got == need,
           "adamw_cast_plan at exact capacity");
    delete[] exact;
    sae_adamw_cast_tile* shrt = new sae_adamw_cast_tile[need - 1 > 0 ? need - 1 : 1];
    if (need > 1)
      expect(sae_adamw_cast_plan(n, p.data(), g.data(), m.data(), v.data(), K.data(), N.data(), w16.data(),
                                 ld16.data(), wt16.data(), ldT.data(), col0.data(), shrt, need - 1, &got) != SAE_OK,
             "adamw_cast_plan refuses a short table");
    delete[] shrt;
  }
  {   // an item with neither copy is refused
    float* p = reinterpret_cast<float*>(0x400000);
    const float* g = p + 4096;
    float *m = p + 8192, *v = p + 12288;
    void* none = nullptr;
    const int32_t K = 64, N = 64, ld = 64, col0 = 0;
    sae_adamw_cast_tile t[1];
    int64_t got = -1;
    expect(sae_adamw_cast_plan(1, &p, &g, &m, &v, &K, &N, &none, &ld, &none, &ld, &col0, t, 1, &got) == SAE_EINVAL,
           "adamw_cast_plan refuses an item with no bf16 copy");
  }
}

static void workspace_sizes() {
  const int dims[] = {1, 7, 64, 197, 384, 577, 1152, 3072, 25216, 100000};
  for (int a : dims)
    for (int b : dims)
      for (int c : dims) {
        expect(sae_gemm_dw_workspace_bytes(a, b, c) < ((size_t)1 << 44), "gemm_dw workspace bounded");
        expect(sae_gemm_f32_workspace_bytes(a, b, c) < ((size_t)1 << 44), "gemm_f32 workspace bounded");
        expect(sae_layernorm_bwd_workspace_bytes(a, b % 4097 + 4) < ((size_t)1 << 40), "ln workspace bounded");
      }
  sae_attn_desc d;
  for (int n : {1, 17, 197, 577, 3136})
    for (int h : {1, 6, 12, 16})
      for (int dd : {6, 10, 32, 48, 64, 128}) {
        sae_attn_desc_init(&d, 3, h, n, n, dd, SAE_DTYPE_BF16, 0.125f);
        expect(sae_attn_bwd_workspace_bytes(&d) < ((size_t)1 << 40), "attn bwd workspace bounded");
        expect(sae_th_attn_bwd_workspace_bytes(&d) < ((size_t)1 << 40), "th bwd workspace bounded");
      }
  sae_patch_desc pd = {8, 224, 224, 3, 16, 16, 384, SAE_LAYOUT_HWCN, SAE_DTYPE_F32};
  expect(sae_patch_embed_bwd_workspace_bytes(&pd) > 0, "patch workspace");
}

static void validation() {
  void *q = fake(), *k = fake(), *v = fake(), *o = fake();
  float* lse = static_cast<float*>(fake());
  sae_attn_desc d;
  sae_attn_desc_init(&d, 2, 4, 64, 64, 64, SAE_DTYPE_BF16, 0.125f);
  d.head_dim = 0;
  expect(sae_attn_fwd(nullptr, &d, q, k, v, nullptr, nullptr, o, lse) == SAE_EINVAL, "head_dim 0");
  expect(std::strlen(sae_last_error()) > 0, "error text");
  sae_attn_desc_init(&d, 2, 4, 64, 64, 256, SAE_DTYPE_BF16, 0.125f);
  expect(sae_attn_fwd(nullptr, &d, q, k, v, nullptr, nullptr, o, lse) == SAE_EUNSUPPORTED, "head_dim 256");
  sae_attn_desc_init(&d, 2, 4, 64, 64, 64, 7, 0.125f);
  expect(sae_attn_fwd(nullptr, &d, q, k, v, nullptr, nullptr, o, lse) != SAE_OK, "bad dtype");
  sae_attn_desc_init(&d, 2, 4, 64, 64, 64, SAE_DTYPE_BF16, 0.125f);
  expect(sae_attn_fwd(nullptr, &d, nullptr, k, v, nullptr, nullptr, o, lse) == SAE_EINVAL, "null q");
  expect(sae_attn_fwd(nullptr, nullptr, q, k, v, nullptr, nullptr, o, lse) == SAE_EINVAL, "null desc");
  d.flags = SAE_FLAG_RELPOS;
  d.rel_h = 3;
  d.rel_w = 5;   // 15 != seq_k
  expect(sae_attn_fwd(nullptr, &d, q, k, v, lse, lse, o, lse) != SAE_OK, "relpos grid != seq_k");
  // launches that pass validation: no GPU here, so the HIP launch must fail cleanly
  sae_attn_desc_init(&d, 1, 1, 16, 16, 64, SAE_DTYPE_BF16, 0.125f);
  const int rc = sae_attn_fwd(nullptr, &d, q, k, v, nullptr, nullptr, o, lse);
  expect(rc == SAE_OK || rc == SAE_EHIP, "valid launch without a GPU: SAE_EHIP");

  expect(sae_gemm_nt(nullptr, 128, 128, 60, q, 64, k, 64, nullptr, o, 128, SAE_EPI_NONE, nullptr, 0, nullptr) ==
             SAE_EUNSUPPORTED,
         "gemm_nt K % 64");
  expect(sae_gemm_nt(nullptr, 0, 128, 64, q, 64, k, 64, nullptr, o, 128, SAE_EPI_NONE, nullptr, 0, nullptr) ==
             SAE_EINVAL,
         "gemm_nt M 0");
  float* fa = static_cast<float*>(fake());
  expect(sae_gemm_f32(nullptr, 64, 64, 30, fa, 30, 1, fa, 64, 1, nullptr, fa, 64, nullptr, 0, nullptr) ==
             SAE_EUNSUPPORTED,
         "gemm_f32 K % 4 (k-contiguous A)");
  expect(sae_gemm_f32(nullptr, 64, 64, 32, fa, 3, 2, fa, 64, 1, nullptr, fa, 64, nullptr, 0, nullptr) ==
             SAE_EUNSUPPORTED,
         "gemm_f32 no unit stride");
  expect(sae_gemm_f32(nullptr, 64, 64, 32, fa + 1, 32, 1, fa, 64, 1, nullptr, fa, 64, nullptr, 0, nullptr) ==
             SAE_EINVAL,
         "gemm_f32 misaligned a");
  expect(sae_gemm_f32(nullptr, 64, 64, 100000, fa, 100000, 1, fa, 64, 1, nullptr, fa, 64, nullptr, 0, nullptr) ==
             SAE_EINVAL,
         "gemm_f32 split without workspace");
  expect(sae_gemm_dw(nullptr, 64, 12, 16, q, 12, k, 16, fa, 16, nullptr, 0, fake()) == SAE_EUNSUPPORTED,
         "gemm_dw I % 8");
  expect(sae_gemm_dw_blocked(nullptr, 64, 16, 24, 5, q, 16, k, 24, fa, nullptr, 0, fake()) == SAE_EINVAL,
         "gemm_dw_blocked jblock");
  std::vector<sae_weight_cast_item> items(100);
  expect(sae_weight_cast_multi(nullptr, 100, items.data()) != SAE_OK, "weight_cast_multi too many items");
  expect(sae_layernorm_fwd(nullptr, 16, 6, fa, nullptr, fa, fa, fa, q, fa, fa, 1e-6f) != SAE_OK, "layernorm C % 4");
  sae_patch_desc pd = {8, 224, 224, 3, 16, 16, 384, SAE_LAYOUT_HWCN, SAE_DTYPE_F32};
  pd.patch_h = 15;
  expect(sae_patch_embed_fwd(nullptr, &pd, q, k, nullptr, o) != SAE_OK, "patch not dividing the image");
  expect(sae_tokens_fwd(nullptr, 2, 196, 6, q, fa, fa, fa) != SAE_OK, "tokens E % 4");
  expect(sae_smoothed_ce_fwd(nullptr, 0, 1000, q, 1000, SAE_DTYPE_BF16, static_cast<const int64_t*>(fake()), 0.1f,
                             fa, fa, fa) != SAE_OK,
         "ce zero rows");
  expect(sae_abi_version() == SAE_ABI_VERSION, "abi version");
  expect(std::strlen(sae_build_info()) > 0, "build info");
}

int main() {
  std::mt19937 rng(1234);
  adamw_plans(rng);
  workspace_sizes();
  validation();
  std::printf("capi_asan: %d checks, %d failed\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
