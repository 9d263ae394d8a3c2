/* attn_cpu.c -- CPU restatement of the reference's UNFUSED attention core, fp32, OpenMP.
 *
 * TEST INFRASTRUCTURE / CPU BASELINE ONLY (see attention_ref.py's header): only tests/ and the
 * cpu_baseline leg of bench.py load libattn_cpu.so.  The product path (libsae_attn.so) never links
 * or calls it.  Parity status: as oracle/attention_ref.py (unpinned by the reference, which holds
 * no vectors); tests/test_cpu_attn.py pins this file to that float64 restatement.
 *
 * The algorithm is the reference's, op for op, not a fused kernel: per (batch, head) it
 * materialises the [Nq, Nk] logits S, the probabilities P and, in the backward, dP and dS, as
 * XLA does for models/layers/attentions/attention.py:39-58:
 *   S = (q * scale) k^T (+ relative logits, botnet.py:191-192 in the index-map form of
 *       sae_attn.h: bias_h[q, k / rel_w] + bias_w[q, k % rel_w])       attention.py:39-42
 *   P = softmax(S) over keys (exp(S - max) / sum)                       attention.py:48
 *   O = P V, lse = max + log(sum)                                       attention.py:57-58
 * backward (JAX autodiff of the same, survey A18):
 *   dV = P^T dO, dP = dO V^T, dS = P o (dP - rowsum(dO o O)), dQ = scale dS K, dK = scale dS^T q,
 *   dbias_h[q, r] = sum_c dS[q, r * rel_w + c], dbias_w[q, c] = sum_r dS[q, r * rel_w + c].
 * Entry points mirror sae_attn_fwd / sae_attn_bwd (include/sae_attn.h) with fp32 host pointers;
 * the stream argument is ignored.  OpenMP over (batch, head), one S / P scratch per thread.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "sae_attn.h"

#define AT(p, s, b, n, h) ((p) + (b) * (s)[0] + (n) * (s)[1] + (h) * (s)[2])

static int check(const sae_attn_desc* d) {
  if (!d || d->dtype != SAE_DTYPE_F32 || d->batch < 1 || d->heads < 1 || d->seq_q < 1 || d->seq_k < 1 ||
      d->head_dim < 1)
    return SAE_EINVAL;
  if ((d->flags & SAE_FLAG_RELPOS) && d->rel_h * d->rel_w != d->seq_k) return SAE_EINVAL;
  return SAE_OK;
}

/* S[i][j] for one (b, h): scale <q_i, k_j> (+ relative logits) */
static void logits(const sae_attn_desc* d, const float* q, const float* k, const float* bias_h,
                   const float* bias_w, int b, int h, float* S) {
  const int Nq = d->seq_q, Nk = d->seq_k, D = d->head_dim;
  const int rel = d->flags & SAE_FLAG_RELPOS;
  const size_t row = ((size_t)b * d->heads + h) * Nq;
  for (int i = 0; i < Nq; ++i) {
    const float* qi = AT(q, d->q_stride, b, i, h);
    for (int j = 0; j < Nk; ++j) {
      const float* kj = AT(k, d->k_stride, b, j, h);
      float acc = 0.f;
      for (int e = 0; e < D; ++e) acc += qi[e] * kj[e];
      float s = acc * d->scale;
      if (rel) s += bias_h[(row + i) * d->rel_h + j / d->rel_w] + bias_w[(row + i) * d->rel_w + j % d->rel_w];
      S[(size_t)i * Nk + j] = s;
    }
  }
}

int sae_cpu_attn_fwd(void* stream, const sae_attn_desc* d, const float* q, const float* k, const float* v,
                     const float* bias_h, const float* bias_w, float* o, float* lse) {
  (void)stream;
  if (check(d)) return SAE_EINVAL;
  const int B = d->batch, H = d->heads, Nq = d->seq_q, Nk = d->seq_k, D = d->head_dim;
  int rc = SAE_OK;
#pragma omp parallel
  {
    float* S = (float*)malloc(sizeof(float) * (size_t)Nq * Nk);
    if (!S) {
#pragma omp atomic write
      rc = SAE_EINVAL;
    }
#pragma omp for schedule(dynamic)
    for (int bh = 0; bh < B * H; ++bh) {
      if (!S) continue;
      const int b = bh / H, h = bh % H;
      logits(d, q, k, bias_h, bias_w, b, h, S);
      for (int i = 0; i < Nq; ++i) {
        float* Si = S + (size_t)i * Nk;
        float m = -INFINITY;
        for (int j = 0; j < Nk; ++j) m = Si[j] > m ? Si[j] : m;
        float l = 0.f;
        for (int j = 0; j < Nk; ++j) {
          Si[j] = expf(Si[j] - m);
          l += Si[j];
        }
        const float inv = 1.f / l;
        float* oi = AT(o, d->o_stride, b, i, h);
        for (int e = 0; e < D; ++e) oi[e] = 0.f;
        for (int j = 0; j < Nk; ++j) {
          const float p = Si[j] * inv;
          const float* vj = AT(v, d->v_stride, b, j, h);
          for (int e = 0; e < D; ++e) oi[e] += p * vj[e];
        }
        if (lse) lse[((size_t)b * H + h) * Nq + i] = m + logf(l);
      }
    }
    free(S);
  }
  return rc;
}

int sae_cpu_attn_bwd(void* stream, const sae_attn_desc* d, const float* q, const float* k, const float* v,
                     const float* o, const float* lse, const float* dout, const float* bias_h,
                     const float* bias_w, float* dq, float* dk, float* dv, float* dbias_h, float* dbias_w) {
  (void)stream;
  if (check(d) || !lse) return SAE_EINVAL;
  const int B = d->batch, H = d->heads, Nq = d->seq_q, Nk = d->seq_k, D = d->head_dim;
  const int rel = d->flags & SAE_FLAG_RELPOS;
  int rc = SAE_OK;
#pragma omp parallel
  {
    float* S = (float*)malloc(sizeof(float) * (size_t)Nq * Nk);
    if (!S) {
#pragma omp atomic write
      rc = SAE_EINVAL;
    }
#pragma omp for schedule(dynamic)
    for (int bh = 0; bh < B * H; ++bh) {
      if (!S) continue;
      const int b = bh / H, h = bh % H;
      const size_t row = ((size_t)b * H + h) * Nq;
      logits(d, q, k, bias_h, bias_w, b, h, S);
      for (int j = 0; j < Nk; ++j) {
        float* dkj = AT(dk, d->dk_stride, b, j, h);
        float* dvj = AT(dv, d->dv_stride, b, j, h);
        for (int e = 0; e < D; ++e) dkj[e] = dvj[e] = 0.f;
      }
      for (int i = 0; i < Nq; ++i) {
        float* Si = S + (size_t)i * Nk;   /* P, then dS, in place */
        const float* gi = AT(dout, d->do_stride, b, i, h);
        const float* oi = AT(o, d->o_stride, b, i, h);
        float delta = 0.f;
        for (int e = 0; e < D; ++e) delta += gi[e] * oi[e];
        const float l = lse[row + i];
        for (int j = 0; j < Nk; ++j) {
          const float p = expf(Si[j] - l);
          const float* vj = AT(v, d->v_stride, b, j, h);
          float* dvj = AT(dv, d->dv_stride, b, j, h);
          float dp = 0.f;
          for (int e = 0; e < D; ++e) {
            dp += gi[e] * vj[e];
            dvj[e] += p * gi[e];
          }
          Si[j] = p * (dp - delta);
        }
        const float* qi = AT(q, d->q_stride, b, i, h);
        float* dqi = AT(dq, d->dq_stride, b, i, h);
        for (int e = 0; e < D; ++e) dqi[e] = 0.f;
        for (int j = 0; j < Nk; ++j) {
          const float ds = Si[j] * d->scale;
          const float* kj = AT(k, d->k_stride, b, j, h);
          float* dkj = AT(dk, d->dk_stride, b, j, h);
          for (int e = 0; e < D; ++e) {
            dqi[e] += ds * kj[e];
            dkj[e] += ds * qi[e];
          }
        }
        if (rel) {
          for (int r = 0; r < d->rel_h; ++r) {
            float acc = 0.f;
            for (int c = 0; c < d->rel_w; ++c) acc += Si[r * d->rel_w + c];
            dbias_h[(row + i) * d->rel_h + r] = acc;
          }
          for (int c = 0; c < d->rel_w; ++c) {
            float acc = 0.f;
            for (int r = 0; r < d->rel_h; ++r) acc += Si[r * d->rel_w + c];
            dbias_w[(row + i) * d->rel_w + c] = acc;
          }
        }
      }
    }
    free(S);
  }
  return rc;
}

/* threads the OpenMP runtime will use (for the baseline's "cores" field) */
#ifdef _OPENMP
#include <omp.h>
int sae_cpu_threads(void) { return omp_get_max_threads(); }
#else
int sae_cpu_threads(void) { return 1; }
#endif
