/*
 * sae_attn.h -- C ABI of the MI355X (gfx950) multi-head self-attention hot path.
 *
 * This is the drop-in boundary of the build: every entry point takes plain device
 * pointers, sizes and a HIP stream (as void*), never a framework type.  It replaces the
 * XLA-lowered einsum / softmax chains of the reference's Flax attention modules
 * (cfoster0/self-attention-experiments-vision):
 *
 *   sae_attn_fwd / sae_attn_bwd
 *       AttentionBlock core, models/layers/attentions/attention.py:39-58
 *       (q/sqrt(D) :39, QK^T einsum :41-42, softmax :48, AV einsum :57-58) and its JAX
 *       autodiff backward.  Also the core of CvTAttentionBlock
 *       (models/layers/attentions/cvt_attention.py:85-104, Nq != Nk), of
 *       ClassSelfAttentionBlock (models/cait.py:10-15, Nq = 1) and of
 *       LCSelfAttentionBlock (models/ceit.py:11-16, Nq = 1).
 *   SAE_FLAG_RELPOS (bias_h / bias_w in sae_attn_fwd/bwd) + sae_relpos_bias_fwd/bwd
 *       BoTNet RelativeLogits added to the score tile, models/botnet.py:70-141,191-192.
 *   sae_th_attn_fwd / sae_th_attn_bwd
 *       talking-heads attention, attention.py:44-52 + talking_heads.py:9-14.
 *   sae_rotary
 *       rotary position embedding, models/layers/position_embed.py:8-20 (README to-do).
 *
 * Conventions
 *   - Activations are token-major [B, N, H, D] (the reference einsum layout), addressed by
 *     element strides (batch, token, head); the head_dim stride is 1.
 *   - Scores are scale * <q, k> (+ bias); the reference's scale is 1/sqrt(head_ch).
 *   - lse is float32 [B, H, Nq], the natural-log log-sum-exp of each score row.
 *   - dtype is SAE_DTYPE_BF16 (compute: bf16 MFMA, fp32 accumulate / softmax) or
 *     SAE_DTYPE_F32 (exact fp32 MFMA).
 *   - All buffers are caller-owned; nothing is allocated or retained; every launch is
 *     ordered on `stream`; no host synchronisation (graph-capturable); re-entrant.
 *   - Return 0 on success, a negative SAE_E* code otherwise; sae_last_error() returns a
 *     thread-local message for the last failure on the calling thread.
 */
#ifndef SAE_ATTN_H
#define SAE_ATTN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SAE_ABI_VERSION 1

enum {
  SAE_OK = 0,
  SAE_EINVAL = -1,        /* descriptor / argument validation failed */
  SAE_EUNSUPPORTED = -2,  /* valid but outside the implemented envelope (e.g. D > 128) */
  SAE_EHIP = -3           /* a HIP runtime call failed */
};

enum { SAE_DTYPE_F32 = 0, SAE_DTYPE_BF16 = 1 };

enum { SAE_FLAG_RELPOS = 1 };

typedef struct sae_attn_desc {
  int32_t batch, heads, seq_q, seq_k, head_dim;
  int32_t dtype;          /* SAE_DTYPE_* of q, k, v, o, dout, dq, dk, dv */
  int32_t flags;          /* SAE_FLAG_* */
  float scale;            /* score = scale * <q, k> + bias */
  /* element strides (batch, token, head); head_dim stride must be 1 */
  int64_t q_stride[3], k_stride[3], v_stride[3], o_stride[3];
  /* backward only */
  int64_t do_stride[3], dq_stride[3], dk_stride[3], dv_stride[3];
  /* SAE_FLAG_RELPOS: keys form a rel_h x rel_w grid (seq_k == rel_h * rel_w) and
     bias_h [B,H,Nq,rel_h], bias_w [B,H,Nq,rel_w] (fp32) are added to the scores:
     score[q, k] += bias_h[q, k / rel_w] + bias_w[q, k % rel_w]. */
  int32_t rel_h, rel_w;
} sae_attn_desc;

/* Fill `desc` for contiguous [B, N, H, D] tensors (all eight stride triples). */
void sae_attn_desc_init(sae_attn_desc* desc, int32_t batch, int32_t heads, int32_t seq_q,
                        int32_t seq_k, int32_t head_dim, int32_t dtype, float scale);

/* Forward: o = softmax(scale q k^T + bias) v, lse = logsumexp rows.
   bias_h / bias_w may be NULL unless SAE_FLAG_RELPOS.  lse may be NULL (inference). */
int sae_attn_fwd(void* stream, const sae_attn_desc* desc, const void* q, const void* k,
                 const void* v, const float* bias_h, const float* bias_w, void* o,
                 float* lse);

/* Bytes of device workspace sae_attn_bwd needs (float32 delta = rowsum(dout * o)). */
size_t sae_attn_bwd_workspace_bytes(const sae_attn_desc* desc);

/* Backward: writes dq, dk, dv (and dbias_h / dbias_w if SAE_FLAG_RELPOS: the score
   gradient summed over key rows / key columns).  Deterministic: no atomics to HBM. */
int sae_attn_bwd(void* stream, const sae_attn_desc* desc, const void* q, const void* k,
                 const void* v, const void* o, const float* lse, const void* dout,
                 const float* bias_h, const float* bias_w, void* dq, void* dk, void* dv,
                 float* dbias_h, float* dbias_w, void* workspace);

/* BoTNet relative logits (botnet.py:70-141) in index-map form, qhat = scaled query
   [B, N = Hs*Ws, H, D] (dtype), emb_h [2Hs-1, D], emb_w [2Ws-1, D] fp32:
     bias_h[b,h,n,p] = <qhat[b,n,h], emb_h[p - n/Ws + Hs - 1]>
     bias_w[b,h,n,c] = <qhat[b,n,h], emb_w[c - n%Ws + Ws - 1]>                        */
int sae_relpos_bias_fwd(void* stream, int32_t batch, int32_t heads, int32_t rel_h,
                        int32_t rel_w, int32_t head_dim, int32_t dtype, const void* qhat,
                        const int64_t qhat_stride[3], const float* emb_h,
                        const float* emb_w, float* bias_h, float* bias_w);

size_t sae_relpos_bias_bwd_workspace_bytes(int32_t batch, int32_t rel_h, int32_t rel_w,
                                           int32_t head_dim);

/* Backward of sae_relpos_bias_fwd.  dqhat_out = dqhat_in + d(bias)/d(qhat)
   (dqhat_in may equal dqhat_out, or be NULL for zero), demb_h / demb_w overwritten. */
int sae_relpos_bias_bwd(void* stream, int32_t batch, int32_t heads, int32_t rel_h,
                        int32_t rel_w, int32_t head_dim, int32_t dtype, const void* qhat,
                        const int64_t qhat_stride[3], const float* emb_h,
                        const float* emb_w, const float* dbias_h, const float* dbias_w,
                        const void* dqhat_in, void* dqhat_out, const int64_t dq_stride[3],
                        float* demb_h, float* demb_w, void* workspace);

/* Rotary embedding (position_embed.py:8-20, GPT-J interleaved pairs) on x [B,N,H,D]:
     y[2i]   = x[2i] cos[n,i] - x[2i+1] sin[n,i]
     y[2i+1] = x[2i+1] cos[n,i] + x[2i] sin[n,i]
   sin/cos are fp32 [N, D/2] tables.  inverse != 0 rotates by -theta (the backward).
   y may alias x. */
int sae_rotary(void* stream, int32_t batch, int32_t seq, int32_t heads, int32_t head_dim,
               int32_t dtype, const void* x, const int64_t x_stride[3], void* y,
               const int64_t y_stride[3], const float* sin_tab, const float* cos_tab,
               int32_t inverse);

/* Attention with the rotary embedding fused (position_embed.py:8-20 applied to q and k before
   the scores): q and k are passed UN-rotated and rotated by the kernels as they are staged
   (sin/cos fp32 [max(seq_q, seq_k)][head_dim / 2], row = position), so the rotated tensors
   never exist in memory; the backward returns dq / dk for the un-rotated q / k (rotated back
   as they are stored).  Bit-identical to sae_rotary + sae_attn_fwd / sae_attn_bwd + sae_rotary
   (inverse).  bf16, 16-byte aligned strides, head_dim % 8 == 0 and head_dim <= 64 (forward
   and backward alike, so a forward that runs always has its backward), no flags; otherwise
   SAE_EUNSUPPORTED (use sae_rotary + the plain entry points). */
int sae_attn_fwd_rotary(void* stream, const sae_attn_desc* desc, const void* q, const void* k,
                        const void* v, const float* sin_tab, const float* cos_tab, void* o,
                        float* lse);
int sae_attn_bwd_rotary(void* stream, const sae_attn_desc* desc, const void* q, const void* k,
                        const void* v, const void* o, const float* lse, const void* dout,
                        const float* sin_tab, const float* cos_tab, void* dq, void* dk, void* dv,
                        void* workspace);

/* Talking-heads attention (attention.py:41-58 with talking_heads=True):
     S = scale q k^T ; S1[i] = sum_h th1[h,i] S[h] ; P = softmax(S1) ;
     P2[i] = sum_h th2[h,i] P[h] ; o = P2 v
   th1/th2 are fp32 [H, H] ([h_in, h_out], talking_heads.py:13).  One workgroup holds one
   query (or key) block for all heads, so heads <= SAE_TH_MAX_HEADS and head_dim <=
   SAE_TH_MAX_HEAD_DIM: bf16 (16-byte aligned strides) takes up to 16 heads -- every CaiT config
   of models/create_model.py:79-168, cait_m_24/36/48 included (16 heads, head_dim 48); the fp32
   (exact) and unaligned paths take up to 8 heads.
   lse: fp32 [B, H, Nq] log-sum-exp of the mixed logits S1 (for the backward). */
#define SAE_TH_MAX_HEADS 16
#define SAE_TH_MAX_HEAD_DIM 64
int sae_th_attn_fwd(void* stream, const sae_attn_desc* desc, const void* q, const void* k,
                    const void* v, const float* th1, const float* th2, void* o, float* lse);

size_t sae_th_attn_bwd_workspace_bytes(const sae_attn_desc* desc);

/* Backward of sae_th_attn_fwd: dq, dk, dv and the transform gradients dth1, dth2
   (fp32 [H, H], overwritten; reduced deterministically through the workspace). */
int sae_th_attn_bwd(void* stream, const sae_attn_desc* desc, const void* q, const void* k,
                    const void* v, const float* th1, const float* th2, const float* lse,
                    const void* dout, void* dq, void* dk, void* dv, float* dth1,
                    float* dth2, void* workspace);

/* Talking heads with the rotary embedding fused (as sae_attn_fwd_rotary; bf16, aligned). */
int sae_th_attn_fwd_rotary(void* stream, const sae_attn_desc* desc, const void* q, const void* k,
                           const void* v, const float* th1, const float* th2,
                           const float* sin_tab, const float* cos_tab, void* o, float* lse);
int sae_th_attn_bwd_rotary(void* stream, const sae_attn_desc* desc, const void* q, const void* k,
                           const void* v, const float* th1, const float* th2, const float* lse,
                           const void* dout, const float* sin_tab, const float* cos_tab, void* dq,
                           void* dk, void* dv, float* dth1, float* dth2, void* workspace);

/* Weight / bias gradients of a projection on the path (the Dense / DenseGeneral kernels of
   attention.py:29-37,60-63 and ff.py:8-34, whose JAX autodiff computes them):
     dw[i][j] (+)= sum_m x[m][i] * dy[m][j]      dw fp32 [I][J] (row stride ldw)
     db[j]    (+)= sum_m dy[m][j]                db fp32 [J] (may be NULL)
   x bf16 [M][I] (row stride ldx), dy bf16 [M][J] (row stride ldy); I, J, ldx, ldy multiples
   of 8, pointers 16-byte aligned.  accumulate != 0 adds into dw / db.  Split over m with a
   fixed-order reduction of the splits: deterministic, no atomics. */
size_t sae_gemm_dw_workspace_bytes(int32_t M, int32_t I, int32_t J);
int sae_gemm_dw(void* stream, int32_t M, int32_t I, int32_t J, const void* x, int64_t ldx,
                const void* dy, int64_t ldy, float* dw, int64_t ldw, float* db,
                int32_t accumulate, void* workspace);
/* Same, with dw laid out as J / jblock contiguous column blocks [J/jblock][I][jblock] (the
   separate queries / keys / values kernel gradients of one stacked projection); jblock a
   multiple of 4 dividing J.  Workspace: sae_gemm_dw_workspace_bytes(M, I, J). */
int sae_gemm_dw_blocked(void* stream, int32_t M, int32_t I, int32_t J, int32_t jblock,
                        const void* x, int64_t ldx, const void* dy, int64_t ldy, float* dw,
                        float* db, int32_t accumulate, void* workspace);

/* Forward and input-gradient GEMMs of the projections and the FF block (the dot_generals of
   Flax Dense / DenseGeneral, attention.py:29-37,60-63 and ff.py:8-34), with the FF block's
   nn.gelu (tanh form, ff.py:27) and its derivative fused into the epilogue:
     acc[m][n] = sum_k a[m][k] * bt[n][k]      a bf16 [M][K] (lda), bt bf16 [N][K] (ldb)
     SAE_EPI_NONE : c = bf16(acc + bias)
     SAE_EPI_GELU : c2 = h = bf16(acc + bias), c = bf16(gelu(h))
     SAE_EPI_DGELU: c = bf16(bf16(acc) * gelu'(aux))   (aux bf16 [M][N], ldaux; bias NULL)
     SAE_EPI_GELU_GRAD: c2 = g = bf16(gelu'(bf16(acc + bias))), c = bf16(gelu(bf16(acc + bias)))
     SAE_EPI_MUL_AUX  : c = bf16(bf16(acc) * aux)       (aux = the g above; bias NULL)
   (the FF block's pair: the forward saves gelu'(h) instead of h, so the input-gradient GEMM's
   epilogue is one multiply instead of the sigmoid algebra -- gelu' rounded to bf16 once, the
   rounding the reference's bf16 derivative carries anyway)
   c, c2 bf16 [M][N] (ldc); bias fp32 [N] or NULL.  K a multiple of 8; N, lda, ldb, ldc
   multiples of 8; pointers 16-byte aligned.  A Dense forward passes the transposed bf16
   kernel as bt (see sae_weight_cast); its input gradient passes the kernel itself. */
#define SAE_EPI_NONE 0
#define SAE_EPI_GELU 1
#define SAE_EPI_DGELU 2
#define SAE_EPI_GELU_GRAD 3
#define SAE_EPI_MUL_AUX 4
int sae_gemm_nt(void* stream, int32_t M, int32_t N, int32_t K, const void* a, int64_t lda,
                const void* bt, int64_t ldb, const float* bias, void* c, int64_t ldc,
                int32_t epilogue, const void* aux, int64_t ldaux, void* c2);
/* Which kernel sae_gemm_nt runs for a shape (host-only, no device needed): the round-5 routing
   rule by tile fill and reduction depth (capi.hip, g8x_route / g8_route). */
#define SAE_NT_ROUTE_NONE 0           /* shape not supported: sae_gemm_nt returns SAE_EUNSUPPORTED */
#define SAE_NT_ROUTE_TILE128 1        /* 128-row tiles (gemm_nt_kernel), K % 64 == 0 */
#define SAE_NT_ROUTE_TILE128_KTAIL 2  /* 128-row tiles, K % 8 == 0 with a partial last K stage */
#define SAE_NT_ROUTE_GEMM8 3          /* persistent 224/256 x 192 tiles (GELU forward at K < 768: 256 x 128 where that loads the CUs more evenly), LDS-DMA (gemm8_nt_kernel) */
#define SAE_NT_ROUTE_GEMM8X 4         /* ping-pong 256 x 256 tiles, LDS-DMA (gemm8x_nt_kernel) */
int sae_gemm_nt_route(int32_t M, int32_t N, int32_t K, int32_t epilogue);
/* The same projections at compute dtype float32 (the reference's fp32 trunks, cait.py:147-154,
   and every fp32 run), on the exact-f32 MFMA:
     c[m][n] = (accumulate ? c[m][n] : 0) + sum_k A(m,k) B(k,n) (+ bias[n])
     A(m,k) = a[m*sam + k*sak], B(k,n) = b[k*sbk + n*sbn]
   One stride of each operand must be 1 (sak == 1: k-contiguous, else sam == 1), the other a
   multiple of 4 covering the contiguous extent, that extent (K, M or N) a multiple of 4; a and b
   16-byte aligned; c fp32 [M][ldc]; bias fp32 [N] or NULL.  colsum != NULL also writes
   colsum[n] (+)= sum_k B(k,n) (a weight gradient's db beside its dW, one pass).  Deep, narrow
   shapes split K over sae_gemm_f32_workspace_bytes(M, N, K) bytes of workspace (0: none
   needed) with a fixed-order reduction: deterministic, no atomics.
     forward  y = x W:      a = x, sam = I, sak = 1;   b = W, sbk = J, sbn = 1
     input    dx = dy W^T:  a = dy, sam = J, sak = 1;  b = W, sbk = 1, sbn = J
     weight   dW = x^T dy:  a = x, sam = 1, sak = I;   b = dy, sbk = J, sbn = 1, colsum = db */
size_t sae_gemm_f32_workspace_bytes(int32_t M, int32_t N, int32_t K);
int sae_gemm_f32(void* stream, int32_t M, int32_t N, int32_t K, const float* a, int64_t sam,
                 int64_t sak, const float* b, int64_t sbk, int64_t sbn, const float* bias, float* c,
                 int64_t ldc, float* colsum, int32_t accumulate, void* workspace);
/* fp32 Dense kernel w [K][N] -> bf16 w16 [K][N] and/or its transpose wt16 [N][K] (either may
   be NULL): the compute-dtype casts of Flax Dense (kernel cast to dtype). */
int sae_weight_cast(void* stream, int32_t K, int32_t N, const float* w, void* w16, void* wt16);
/* Many casts in one launch (every Dense kernel of a model once per step): item i casts
   w [K][N] (contiguous fp32) into columns col0 .. col0+N-1 of w16 [K][ld16] and rows
   col0 .. col0+N-1 of wt16 [*][ldT] (either may be NULL) -- e.g. the queries / keys / values
   kernels into one stacked [C][3HD] projection and its transpose. */
typedef struct sae_weight_cast_item {
  const float* w;
  void* w16;
  void* wt16;
  int32_t K, N, ld16, ldT, col0;
} sae_weight_cast_item;
int sae_weight_cast_multi(void* stream, int32_t n, const sae_weight_cast_item* items);

/* Patch embedding (models/layers/stems/patch_embed.py:15-26: einops
   'b (h ph) (w pw) c -> b (h w) (ph pw c)' then Dense) as one GEMM whose A operand is gathered
   from the images while it is staged (no patchified copy):
     out[n][p][e] = sum_k image[n][py*ph + ky][px*pw + kx][c] * wt[e][k] (+ bias[e])
   with p = py * (width / pw) + px, k = (ky * pw + kx) * channels + c.  images bf16 or fp32
   (rounded to bf16, train.py:81) in layout SAE_LAYOUT_NHWC [batch][height][width][channels]
   (the model call) or SAE_LAYOUT_HWCN [height][width][channels][batch] (the train-step feed,
   train.py:80); wt bf16 [embed][K] (the transposed bf16 kernel, sae_weight_cast), bias fp32
   [embed] or NULL, out bf16 [batch][L][embed] (L = patches per image).  Requirements:
   height % ph == width % pw == 0, K = ph*pw*channels a multiple of 64, pw*channels and embed
   multiples of 8, HWCN batch a multiple of 8, image elements < 2^31, 16-byte aligned pointers. */
#define SAE_LAYOUT_NHWC 0
#define SAE_LAYOUT_HWCN 1
typedef struct sae_patch_desc {
  int32_t batch, height, width, channels;
  int32_t patch_h, patch_w, embed;
  int32_t layout;   /* SAE_LAYOUT_* */
  int32_t dtype;    /* SAE_DTYPE_BF16 / SAE_DTYPE_F32: the images' element type */
} sae_patch_desc;
int sae_patch_embed_fwd(void* stream, const sae_patch_desc* desc, const void* images,
                        const void* wt, const float* bias, void* out);
/* Weight / bias gradients of the patch embedding: dw fp32 [K][embed] (+)= sum over tokens of
   patch[m][k] * dout[m][e], db fp32 [embed] (may be NULL); dout bf16 [batch][L][embed];
   deterministic split-token reduction through the workspace. */
size_t sae_patch_embed_bwd_workspace_bytes(const sae_patch_desc* desc);
int sae_patch_embed_bwd(void* stream, const sae_patch_desc* desc, const void* images,
                        const void* dout, float* dw, float* db, int32_t accumulate, void* workspace);
/* The patch matrix of HWCN images as bf16 rows: patches[n * L + p][k], k = (ky * Pw + kx) * C + c
   (the einops order of patch_embed.py:21), L = (H / Ph) * (W / Pw), K = Ph * Pw * C; fp32 images
   are rounded to bf16 (the same operand bits as sae_patch_embed_fwd's loaders).  The train step
   writes it once and runs the embedding as sae_gemm_nt(patches, W^T) and its weight gradient as
   sae_gemm_dw(patches, dY): the LDS-DMA GEMM kernels instead of the per-chunk eight-image scatter of
   the fused HWCN loaders.  desc as sae_patch_embed_fwd, layout SAE_LAYOUT_HWCN. */
int sae_patch_gather(void* stream, const sae_patch_desc* desc, const void* images, void* patches);

/* Residual add + LayerNorm of the encoder blocks around the path (models/vit.py:19-31,57;
   Flax nn.LayerNorm: fp32 statistics, eps, output in the compute dtype):
     xout = x + delta (fp32; when delta != NULL), y = LN(xout) * gamma + beta in bf16,
     mean / rstd fp32 [M] saved for the backward.  x, xout fp32 [M][C]; delta, y bf16 [M][C];
     C a multiple of 4, <= 1024. */
int sae_layernorm_fwd(void* stream, int32_t M, int32_t C, const float* x, const void* delta,
                      float* xout, const float* gamma, const float* beta, void* y, float* mean,
                      float* rstd, float eps);
/* CaiT form (layerscale.py:21-23, stochastic_depth.py:19-28 folded into the residual add):
     xout = x + delta * bf16(layerscale[c]) * rowscale[row / rows_per_sample]   (rowscale may be NULL)
   layerscale fp32 [C] (16-byte aligned; the parameter as stored -- the kernels round it to bf16,
   the compute-dtype cast of layerscale.py:22), rowscale fp32 [M / rows_per_sample]. */
int sae_layernorm_fwd_scaled(void* stream, int32_t M, int32_t C, const float* x, const void* delta,
                             float* xout, const float* gamma, const float* beta, void* y,
                             float* mean, float* rstd, float eps, const float* layerscale,
                             const float* rowscale, int32_t rows_per_sample);
size_t sae_layernorm_bwd_workspace_bytes(int32_t M, int32_t C);
/* dx = dxin + dLN/dx(dy) (fp32; dxin may be NULL), ddelta = bf16(dx) (may be NULL),
   dgamma / dbeta fp32 [C] overwritten (fixed-order reduction, deterministic). */
int sae_layernorm_bwd(void* stream, int32_t M, int32_t C, const float* x, const float* mean,
                      const float* rstd, const float* gamma, const void* dy, const float* dxin,
                      float* dx, void* ddelta, float* dgamma, float* dbeta, void* workspace);
/* Backward of the scaled form: ddelta = bf16(dx * layerscale * rowscale), dlayerscale[c] =
   sum over rows of dx * delta * rowscale (fixed order, with dgamma / dbeta); delta is the bf16
   addend of the forward. */
int sae_layernorm_bwd_scaled(void* stream, int32_t M, int32_t C, const float* x, const float* mean,
                             const float* rstd, const float* gamma, const void* dy, const float* dxin,
                             float* dx, void* ddelta, float* dgamma, float* dbeta, void* workspace,
                             const void* delta, const float* layerscale, const float* rowscale,
                             int32_t rows_per_sample, float* dlayerscale);

/* Optimizer update of the data-parallel training step (train.py:25-27,229-233: optax.adamw,
   survey D9 descent), every parameter in ONE launch.  The parameters are cut into chunks of
   SAE_ADAMW_CHUNK elements; sae_adamw_plan (host only, no GPU call) fills that chunk table for
   n_items fp32 tensors (item i: parameter p[i], gradient g[i], moments m[i], v[i], n[i] elements,
   contiguous) into `chunks` (capacity max_chunks) and returns the count in *n_chunks.  The caller
   copies the table to device memory once; sae_adamw_step then increments the device-resident
   step counter *step (int32) and applies, with t = the new *step (torch.optim.AdamW order):
     p *= 1 - lr*wd;  m = m + (1-b1)(g - m);  v = b2 v + (1-b2) g^2;
     p -= lr/(1 - b1^t) * m / (sqrt(v)/sqrt(1 - b2^t) + eps)
   Both launches are stream-ordered, so a captured graph replays with the right t. */
#define SAE_ADAMW_CHUNK 2048
typedef struct sae_adamw_chunk {
  float* p;
  const float* g;
  float* m;
  float* v;
  int32_t n;     /* elements of this chunk, <= SAE_ADAMW_CHUNK */
  int32_t vec;   /* set by the plan: 16-byte aligned full chunk (vector path) */
} sae_adamw_chunk;
int sae_adamw_plan(int32_t n_items, float* const* p, const float* const* g, float* const* m,
                   float* const* v, const int64_t* n, sae_adamw_chunk* chunks, int64_t max_chunks,
                   int64_t* n_chunks);
int sae_adamw_step(void* stream, int64_t n_chunks, const sae_adamw_chunk* chunks, int32_t* step,
                   float lr, float beta1, float beta2, float eps, float weight_decay);

/* The same update with the bf16 compute copies of the Dense kernels written by the optimizer pass
   (the per-forward fp32 -> bf16 casts of Flax Dense, sae_weight_cast_multi, move into the
   update): item i is a Dense kernel p[i] fp32 [K[i]][N[i]] (contiguous, gradient and moments laid
   out alike) whose updated values are also stored as bf16 into columns col0[i] .. col0[i] + N[i]
   of w16[i] [K][ld16[i]] and rows col0[i] .. of wt16[i] [*][ldT[i]] (either may be NULL).
   sae_adamw_cast_plan (host only) cuts the items into 64 x 64 tiles (K, N, col0, ld16, ldT
   multiples of 4; p / g / m / v 16-byte, w16 / wt16 8-byte aligned: SAE_EUNSUPPORTED otherwise);
   sae_adamw_step_cast runs the chunk table (the other parameters) and the tile table in ONE launch
   after the step-counter tick.  The parameter values are bit-identical to sae_adamw_step's. */
typedef struct sae_adamw_cast_tile {
  float* p;
  const float* g;
  float* m;
  float* v;
  void* w16;
  void* wt16;
  int32_t K, N, ld16, ldT, col0, k0, n0, pad;
} sae_adamw_cast_tile;
int sae_adamw_cast_plan(int32_t n_items, float* const* p, const float* const* g, float* const* m,
                        float* const* v, const int32_t* K, const int32_t* N, void* const* w16,
                        const int32_t* ld16, void* const* wt16, const int32_t* ldT, const int32_t* col0,
                        sae_adamw_cast_tile* tiles, int64_t max_tiles, int64_t* n_tiles);
int sae_adamw_step_cast(void* stream, int64_t n_chunks, const sae_adamw_chunk* chunks, int64_t n_tiles,
                        const sae_adamw_cast_tile* tiles, int32_t* step, float lr, float beta1, float beta2,
                        float eps, float weight_decay);

/* Encoder input of ViT / DeiT (models/vit.py:82-85 class-token concatenate, vit.py:46 +
   position_embed.py:48 AddAbsPosEmbed), tokens bf16 [B][L][E] from the patch embedding, cls fp32
   [E], pos fp32 [L+1][E]:  x fp32 [B][L+1][E] = concat(cls, float(tokens)) + pos.  Backward:
   dtokens bf16 [B][L][E] = bf16(dx[:, 1:]), dpos [L+1][E] = sum_b dx[b], dcls [E] = dpos[0] (may be
   NULL); batch sums in a fixed order.  E % 4 == 0, E <= 4096; x / dx / cls / pos / dpos / dcls
   16-byte and tokens / dtokens 8-byte aligned. */
int sae_tokens_fwd(void* stream, int32_t B, int32_t L, int32_t E, const void* tokens, const float* cls,
                   const float* pos, float* x);
int sae_tokens_bwd(void* stream, int32_t B, int32_t L, int32_t E, const float* dx, void* dtokens, float* dcls,
                   float* dpos);

/* Label-smoothed softmax cross entropy of the training step (replaces train.py:77-90:
   optax.smooth_labels(one_hot(labels), alpha) + jnp.mean(optax.softmax_cross_entropy)):
     loss = mean_r [ lse_r - (1 - alpha) x[r, labels[r]] - (alpha / classes) sum_c x[r, c] ]
   logits x [rows][classes] (row stride ld elements, dtype SAE_DTYPE_BF16 or SAE_DTYPE_F32),
   labels int64 [rows] (a label outside [0, classes) contributes no target term).  fwd writes
   lse [rows] (fp32, for the backward), row_loss [rows] (fp32) and *loss (fp32, device memory);
   the row losses are summed in a fixed order (deterministic).  bwd writes dlogits [rows][classes] (row stride ldd, the logits'
   dtype) = (*grad_loss / rows) (softmax(x_r) - (1 - alpha) onehot - alpha / classes).
   rows <= SAE_CE_MAX_ROWS. */
#define SAE_CE_MAX_ROWS 16384
int sae_smoothed_ce_fwd(void* stream, int32_t rows, int32_t classes, const void* logits, int64_t ld,
                        int32_t dtype, const int64_t* labels, float alpha, float* lse, float* row_loss,
                        float* loss);
int sae_smoothed_ce_bwd(void* stream, int32_t rows, int32_t classes, const void* logits, int64_t ld,
                        int32_t dtype, const int64_t* labels, float alpha, const float* lse,
                        const float* grad_loss, void* dlogits, int64_t ldd);

/* Diagnostic: occupy `workgroups` workgroups of `threads` threads, each holding `lds_bytes` of LDS,
   for `usec` microseconds (a timed s_sleep loop, no memory traffic), on `stream`.  Used by
   bench.py --emulate-rccl to stand in, on one GPU, for the RCCL all-reduce kernels that share the
   CUs with the backward on an 8-GPU node (one workgroup per ring channel, busy for the bucket's
   ring time).  threads in [64, 1024], lds_bytes <= 160 KiB. */
int sae_occupy_cus(void* stream, int32_t workgroups, int32_t threads, int32_t lds_bytes, float usec);

/* Stream-ordered flags for collectives gated outside a HIP graph (train.py, the data-parallel step):
   sae_flag_bump adds 1 to flags[index] (a one-thread kernel; system-scope atomic after the stream's
   earlier kernels, whose writes the kernel boundary has made visible), so a graph can mark points of
   its kernel chain without forking a branch; sae_stream_wait_flag makes `stream` wait until
   *flag >= value (hipStreamWaitValue32, greater-or-equal) before its later work starts. */
int sae_flag_bump(void* stream, uint32_t* flags, int32_t index);
int sae_stream_wait_flag(void* stream, const uint32_t* flag, uint32_t value);

/* Thread-local message describing the last failure on this thread ("" if none). */
const char* sae_last_error(void);

/* ABI version (SAE_ABI_VERSION) and a build string. */
int32_t sae_abi_version(void);
const char* sae_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* SAE_ATTN_H */
