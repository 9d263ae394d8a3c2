"""CPU oracle for the ViT/DeiT training step (numpy restatement, float32 or float64).

TEST INFRASTRUCTURE ONLY (see attention_ref.py header): used by ``tests/`` as the e2e checker
of ``sae_vision_amd.vit`` and by ``bench.py``'s ``cpu_baseline`` leg as the timed CPU port of
the reference's training step.  Parity unpinned by the reference (shape-only tests, no JAX).

Restates models/vit.py:9-99 (EncoderBlock / Encoder / ViT), patch_embed.py:15-26,
ff.py:17-34 (Dense -> tanh-GELU -> Dense), position_embed.py:48-57 (AddAbsPosEmbed),
attention.py:20-67 (the attention block, same algorithm as attention_ref.attention_block_fwd but
written with batched matmuls so the CPU baseline runs on BLAS), and train.py:79-92 (softmax
cross-entropy with optax.smooth_labels, mean over the batch).  Backward is hand-derived.
Parameters are a flat dict keyed by the torch module's parameter names (Flax tree paths with
'.' separators), e.g. ``Encoder_0.EncoderBlock_3.SelfAttentionBlock_0.queries.kernel``.
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np

EPS = 1e-6
_C = math.sqrt(2.0 / math.pi)


def gelu_tanh(x):
    """Flax nn.gelu(approximate=True)."""
    return 0.5 * x * (1.0 + np.tanh(_C * (x + 0.044715 * x ** 3)))


def gelu_tanh_grad(x):
    u = _C * (x + 0.044715 * x ** 3)
    t = np.tanh(u)
    return 0.5 * (1.0 + t) + 0.5 * x * (1.0 - t * t) * _C * (1.0 + 3 * 0.044715 * x * x)


def layer_norm(x, s, b):
    mu = x.mean(-1, keepdims=True)
    xc = x - mu
    var = (xc * xc).mean(-1, keepdims=True)
    rstd = 1.0 / np.sqrt(var + EPS)
    xh = xc * rstd
    return xh * s + b, (xh, rstd)


def layer_norm_bwd(dy, s, cache):
    xh, rstd = cache
    g = dy * s
    n = xh.shape[-1]
    dx = rstd * (g - g.mean(-1, keepdims=True) - xh * (g * xh).mean(-1, keepdims=True))
    ds = (dy * xh).reshape(-1, n).sum(0)
    db = dy.reshape(-1, n).sum(0)
    return dx, ds, db


def attn_fwd(x, Wq, Wk, Wv, Wo):
    """x [B,N,C]; W* [C,H,D], Wo [H,D,C] -> y, cache (token-major like attention.py)."""
    B, N, C = x.shape
    _, H, D = Wq.shape
    q = (x @ Wq.reshape(C, H * D)).reshape(B, N, H, D).transpose(0, 2, 1, 3)   # [B,H,N,D]
    k = (x @ Wk.reshape(C, H * D)).reshape(B, N, H, D).transpose(0, 2, 1, 3)
    v = (x @ Wv.reshape(C, H * D)).reshape(B, N, H, D).transpose(0, 2, 1, 3)
    qh = q / np.sqrt(D).astype(x.dtype)
    s = qh @ k.transpose(0, 1, 3, 2)
    s = s - s.max(-1, keepdims=True)
    p = np.exp(s)
    p /= p.sum(-1, keepdims=True)
    o = (p @ v).transpose(0, 2, 1, 3).reshape(B, N, H * D)
    y = o @ Wo.reshape(H * D, -1)
    return y, (x, qh, k, v, p, o)


def attn_bwd(dy, Wq, Wk, Wv, Wo, cache):
    x, qh, k, v, p, o = cache
    B, N, C = x.shape
    _, H, D = Wq.shape
    dWo = (o.reshape(-1, H * D).T @ dy.reshape(-1, dy.shape[-1])).reshape(H, D, -1)
    do = (dy @ Wo.reshape(H * D, -1).T).reshape(B, N, H, D).transpose(0, 2, 1, 3)
    dv = p.transpose(0, 1, 3, 2) @ do
    dp = do @ v.transpose(0, 1, 3, 2)
    ds = p * (dp - (dp * p).sum(-1, keepdims=True))
    dqh = ds @ k
    dk = ds.transpose(0, 1, 3, 2) @ qh
    dq = dqh / np.sqrt(D).astype(x.dtype)
    tok = lambda t: t.transpose(0, 2, 1, 3).reshape(B * N, H * D)
    x2 = x.reshape(B * N, C)
    dWq = (x2.T @ tok(dq)).reshape(C, H, D)
    dWk = (x2.T @ tok(dk)).reshape(C, H, D)
    dWv = (x2.T @ tok(dv)).reshape(C, H, D)
    dx = (tok(dq) @ Wq.reshape(C, H * D).T + tok(dk) @ Wk.reshape(C, H * D).T +
          tok(dv) @ Wv.reshape(C, H * D).T).reshape(B, N, C)
    return dx, dWq, dWk, dWv, dWo


def patchify(images, p):
    """patch_embed.py:19-22, einops 'b (h ph) (w pw) c -> b (h w) (ph pw c)'; p an int or (ph, pw)."""
    ph, pw = (p, p) if np.isscalar(p) else p
    B, Hh, Ww, c = images.shape
    x = images.reshape(B, Hh // ph, ph, Ww // pw, pw, c).transpose(0, 1, 3, 2, 4, 5)
    return x.reshape(B, (Hh // ph) * (Ww // pw), ph * pw * c)


def hwcn_to_nhwc(images):
    """train.py:80, einops 'H W C N -> N H W C' (the feed's double-transpose layout)."""
    return np.transpose(images, (3, 0, 1, 2))


def smoothed_ce(logits, labels, smoothing, num_classes):
    """train.py:83-90: one_hot -> optax.smooth_labels -> softmax_cross_entropy, mean."""
    y = np.eye(num_classes, dtype=logits.dtype)[labels]
    y = y * (1.0 - smoothing) + smoothing / num_classes
    m = logits.max(-1, keepdims=True)
    lse = m + np.log(np.exp(logits - m).sum(-1, keepdims=True))
    logp = logits - lse
    loss = -(y * logp).sum(-1).mean()
    dlogits = (np.exp(logp) - y) / logits.shape[0]
    return loss, dlogits


def _vit_forward(P, images, num_layers, patch, keep=True):
    """models/vit.py:61-99 forward (fp32 numpy): patch embed, [cls] + pos-embed, encoder blocks,
    final LayerNorm, CLS head.  keep=False drops the backward caches (forward-only timing)."""
    dt = P["cls"].dtype
    B = images.shape[0]
    pe_in = patchify(images.astype(dt), patch)
    pe = pe_in @ P["PatchEmbedBlock_0.Dense_0.kernel"]
    C = pe.shape[-1]
    x = np.concatenate([np.broadcast_to(P["cls"], (B, 1, C)), pe], 1) + P["Encoder_0.AddAbsPosEmbed_0.pos_embed"]
    caches = []
    for i in range(num_layers):
        pre = f"Encoder_0.EncoderBlock_{i}."
        h1, c1 = layer_norm(x, P[pre + "LayerNorm_0.scale"], P[pre + "LayerNorm_0.bias"])
        a, ca = attn_fwd(h1, *(P[pre + f"SelfAttentionBlock_0.{n}.kernel"]
                               for n in ("queries", "keys", "values", "DenseGeneral_0")))
        x = x + a
        h2, c2 = layer_norm(x, P[pre + "LayerNorm_1.scale"], P[pre + "LayerNorm_1.bias"])
        u = h2 @ P[pre + "FFBlock_0.Dense_0.kernel"] + P[pre + "FFBlock_0.Dense_0.bias"]
        g = gelu_tanh(u)
        f = g @ P[pre + "FFBlock_0.Dense_1.kernel"] + P[pre + "FFBlock_0.Dense_1.bias"]
        x = x + f
        if keep:
            caches.append((c1, ca, h2, c2, u, g))
    z, cz = layer_norm(x, P["Encoder_0.LayerNorm_0.scale"], P["Encoder_0.LayerNorm_0.bias"])
    logits = z[:, 0] @ P["Dense_0.kernel"] + P["Dense_0.bias"]
    return logits, (pe_in, caches, z, cz)


def vit_loss(params: Dict[str, np.ndarray], images, labels, num_layers: int, patch: int,
             smoothing: float = 0.1) -> float:
    """Forward + loss only (BASELINE configs[0]: DeiT-Ti forward+loss on the CPU path)."""
    logits, _ = _vit_forward(params, images, num_layers, patch, keep=False)
    return float(smoothed_ce(logits, labels, smoothing, logits.shape[-1])[0])


def vit_loss_and_grads(params: Dict[str, np.ndarray], images, labels, num_layers: int, num_heads: int,
                       patch: int, smoothing: float = 0.1) -> Tuple[float, np.ndarray, Dict[str, np.ndarray]]:
    """Forward + loss + full backward of ViT (all params).  Returns (loss, logits, grads)."""
    P = params
    logits, (pe_in, caches, z, cz) = _vit_forward(P, images, num_layers, patch)
    C = z.shape[-1]
    num_classes = logits.shape[-1]
    loss, dlogits = smoothed_ce(logits, labels, smoothing, num_classes)

    G = {}
    G["Dense_0.kernel"] = z[:, 0].T @ dlogits
    G["Dense_0.bias"] = dlogits.sum(0)
    dz = np.zeros_like(z)
    dz[:, 0] = dlogits @ P["Dense_0.kernel"].T
    dx, G["Encoder_0.LayerNorm_0.scale"], G["Encoder_0.LayerNorm_0.bias"] = layer_norm_bwd(
        dz, P["Encoder_0.LayerNorm_0.scale"], cz)
    for i in reversed(range(num_layers)):
        pre = f"Encoder_0.EncoderBlock_{i}."
        c1, ca, h2, c2, u, g = caches[i]
        W1, W2 = P[pre + "FFBlock_0.Dense_0.kernel"], P[pre + "FFBlock_0.Dense_1.kernel"]
        G[pre + "FFBlock_0.Dense_1.kernel"] = g.reshape(-1, g.shape[-1]).T @ dx.reshape(-1, C)
        G[pre + "FFBlock_0.Dense_1.bias"] = dx.reshape(-1, C).sum(0)
        du = (dx @ W2.T) * gelu_tanh_grad(u)
        G[pre + "FFBlock_0.Dense_0.kernel"] = h2.reshape(-1, C).T @ du.reshape(-1, du.shape[-1])
        G[pre + "FFBlock_0.Dense_0.bias"] = du.reshape(-1, du.shape[-1]).sum(0)
        dh2 = du @ W1.T
        dxx, G[pre + "LayerNorm_1.scale"], G[pre + "LayerNorm_1.bias"] = layer_norm_bwd(
            dh2, P[pre + "LayerNorm_1.scale"], c2)
        dx = dx + dxx
        Ws = [P[pre + f"SelfAttentionBlock_0.{n}.kernel"] for n in ("queries", "keys", "values", "DenseGeneral_0")]
        dh1, dWq, dWk, dWv, dWo = attn_bwd(dx, *Ws, ca)
        for n, gW in zip(("queries", "keys", "values", "DenseGeneral_0"), (dWq, dWk, dWv, dWo)):
            G[pre + f"SelfAttentionBlock_0.{n}.kernel"] = gW
        dxx, G[pre + "LayerNorm_0.scale"], G[pre + "LayerNorm_0.bias"] = layer_norm_bwd(
            dh1, P[pre + "LayerNorm_0.scale"], c1)
        dx = dx + dxx
    G["Encoder_0.AddAbsPosEmbed_0.pos_embed"] = dx.sum(0, keepdims=True)
    G["cls"] = dx[:, 0:1].sum(0, keepdims=True)
    G["PatchEmbedBlock_0.Dense_0.kernel"] = pe_in.reshape(-1, pe_in.shape[-1]).T @ dx[:, 1:].reshape(-1, C)
    return float(loss), logits, G


def adam_update(params, grads, state, lr=5e-4, b1=0.9, b2=0.999, eps=1e-8, wd=1e-4):
    """Decoupled-weight-decay Adam step (train.py:25-27 optax chain, descending; survey D9)."""
    t = state.get("t", 0) + 1
    state["t"] = t
    for k, g in grads.items():
        m = state.setdefault("m_" + k, np.zeros_like(g))
        v = state.setdefault("v_" + k, np.zeros_like(g))
        m *= b1
        m += (1 - b1) * g
        v *= b2
        v += (1 - b2) * g * g
        mh = m / (1 - b1 ** t)
        vh = v / (1 - b2 ** t)
        params[k] -= lr * (mh / (np.sqrt(vh) + eps) + wd * params[k])


# ------------------------------------------------------------------ bf16-emulated training step
def _rb(x):
    """Round to bfloat16 (ties to even), kept in float64: the emulated dot products accumulate wide
    and round their outputs, as XLA does for bf16 dot_general."""
    a = np.ascontiguousarray(np.asarray(x, np.float32))
    u = a.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32).astype(np.float64)


def _softmax_bf16(s):
    m = s.max(-1, keepdims=True)
    e = _rb(np.exp(_rb(s - m)))
    return _rb(e / _rb(e.sum(-1, keepdims=True)))


def vit_loss_and_grads_bf16(params: Dict[str, np.ndarray], images, labels, num_layers: int, num_heads: int,
                            patch: int, smoothing: float = 0.1):
    """The training step of ``create_model(..., dtype=jnp.bfloat16)`` (train.py:222-224) with the
    reference's bf16 rounding points: every Dense / DenseGeneral casts input and kernel to bf16 and
    returns bf16 (bias cast to bf16 and added in bf16), LayerNorm computes in fp32 and returns bf16,
    the attention internals are bf16 (attention.py:29-63), GELU returns bf16, the residual stream is
    fp32 (promoted by the fp32 cls / pos-embed params, vit.py:46,85).  Backward is JAX autodiff of
    that program: the cotangent of every bf16 value is bf16, a bf16-cast fp32 parameter receives its
    bf16 cotangent cast to fp32.  Returns (loss, logits, grads) like :func:`vit_loss_and_grads`."""
    P = {k: np.asarray(v, np.float64) for k, v in params.items()}
    r = _rb
    B = images.shape[0]
    pe_in = r(patchify(np.asarray(images, np.float64), patch))
    Wp = r(P["PatchEmbedBlock_0.Dense_0.kernel"])
    pe = r(pe_in @ Wp)
    C = pe.shape[-1]
    x = np.concatenate([np.broadcast_to(P["cls"], (B, 1, C)), pe], 1) + P["Encoder_0.AddAbsPosEmbed_0.pos_embed"]
    caches = []
    for i in range(num_layers):
        pre = f"Encoder_0.EncoderBlock_{i}."
        h1f, c1 = layer_norm(x, P[pre + "LayerNorm_0.scale"], P[pre + "LayerNorm_0.bias"])
        h1 = r(h1f)
        W = [r(P[pre + f"SelfAttentionBlock_0.{n}.kernel"]) for n in ("queries", "keys", "values", "DenseGeneral_0")]
        Hh, D = W[0].shape[1], W[0].shape[2]
        N = h1.shape[1]
        q, k, v = (r(h1 @ w.reshape(C, Hh * D)).reshape(B, N, Hh, D).transpose(0, 2, 1, 3) for w in W[:3])
        qh = r(q / np.sqrt(D))
        p = _softmax_bf16(r(qh @ k.transpose(0, 1, 3, 2)))
        o = r(p @ v).transpose(0, 2, 1, 3).reshape(B, N, Hh * D)
        a = r(o @ W[3].reshape(Hh * D, C))
        x = x + a
        h2f, c2 = layer_norm(x, P[pre + "LayerNorm_1.scale"], P[pre + "LayerNorm_1.bias"])
        h2 = r(h2f)
        W1, W2 = r(P[pre + "FFBlock_0.Dense_0.kernel"]), r(P[pre + "FFBlock_0.Dense_1.kernel"])
        u = r(r(h2 @ W1) + r(P[pre + "FFBlock_0.Dense_0.bias"]))
        g = r(gelu_tanh(u))
        f = r(r(g @ W2) + r(P[pre + "FFBlock_0.Dense_1.bias"]))
        x = x + f
        caches.append((c1, h1, W, q, k, v, qh, p, o, c2, h2, W1, W2, u, g))
    zf, cz = layer_norm(x, P["Encoder_0.LayerNorm_0.scale"], P["Encoder_0.LayerNorm_0.bias"])
    z = r(zf)
    Wd = r(P["Dense_0.kernel"])
    logits = r(r(z[:, 0] @ Wd) + r(P["Dense_0.bias"]))
    loss, dlogits = smoothed_ce(logits, labels, smoothing, logits.shape[-1])

    G = {}
    dl = r(dlogits)
    G["Dense_0.kernel"] = r(z[:, 0].T @ dl)
    G["Dense_0.bias"] = r(dl.sum(0))
    dz = np.zeros_like(z)
    dz[:, 0] = r(dl @ Wd.T)
    dx, G["Encoder_0.LayerNorm_0.scale"], G["Encoder_0.LayerNorm_0.bias"] = layer_norm_bwd(
        dz, P["Encoder_0.LayerNorm_0.scale"], cz)
    for i in reversed(range(num_layers)):
        pre = f"Encoder_0.EncoderBlock_{i}."
        c1, h1, W, q, k, v, qh, p, o, c2, h2, W1, W2, u, g = caches[i]
        Hh, D = W[0].shape[1], W[0].shape[2]
        N = h1.shape[1]
        df = r(dx)
        G[pre + "FFBlock_0.Dense_1.kernel"] = r(g.reshape(-1, g.shape[-1]).T @ df.reshape(-1, C))
        G[pre + "FFBlock_0.Dense_1.bias"] = r(df.reshape(-1, C).sum(0))
        dg = r(df @ W2.T)
        du = r(dg * gelu_tanh_grad(u))
        G[pre + "FFBlock_0.Dense_0.kernel"] = r(h2.reshape(-1, C).T @ du.reshape(-1, du.shape[-1]))
        G[pre + "FFBlock_0.Dense_0.bias"] = r(du.reshape(-1, du.shape[-1]).sum(0))
        dh2 = r(du @ W1.T)
        dxx, G[pre + "LayerNorm_1.scale"], G[pre + "LayerNorm_1.bias"] = layer_norm_bwd(
            dh2, P[pre + "LayerNorm_1.scale"], c2)
        dx = dx + dxx
        da = r(dx)
        G[pre + "SelfAttentionBlock_0.DenseGeneral_0.kernel"] = r(o.reshape(-1, Hh * D).T @ da.reshape(-1, C)).reshape(Hh, D, C)
        do = r(da @ W[3].reshape(Hh * D, C).T).reshape(B, N, Hh, D).transpose(0, 2, 1, 3)
        dv = r(p.transpose(0, 1, 3, 2) @ do)
        dp = r(do @ v.transpose(0, 1, 3, 2))
        ds = r(p * r(dp - r(r(dp * p).sum(-1, keepdims=True))))
        dq = r(r(ds @ k) / np.sqrt(D))
        dk = r(ds.transpose(0, 1, 3, 2) @ qh)
        tok = lambda t: t.transpose(0, 2, 1, 3).reshape(B * N, Hh * D)
        h1_2 = h1.reshape(B * N, C)
        for n, dd in (("queries", dq), ("keys", dk), ("values", dv)):
            G[pre + f"SelfAttentionBlock_0.{n}.kernel"] = r(h1_2.T @ tok(dd)).reshape(C, Hh, D)
        dh1 = r(r(r(tok(dq) @ W[0].reshape(C, Hh * D).T) + r(tok(dk) @ W[1].reshape(C, Hh * D).T))
                + r(tok(dv) @ W[2].reshape(C, Hh * D).T)).reshape(B, N, C)
        dxx, G[pre + "LayerNorm_0.scale"], G[pre + "LayerNorm_0.bias"] = layer_norm_bwd(
            dh1, P[pre + "LayerNorm_0.scale"], c1)
        dx = dx + dxx
    G["Encoder_0.AddAbsPosEmbed_0.pos_embed"] = dx.sum(0, keepdims=True)
    G["cls"] = dx[:, 0:1].sum(0, keepdims=True)
    dpe = r(dx[:, 1:])
    G["PatchEmbedBlock_0.Dense_0.kernel"] = r(pe_in.reshape(-1, pe_in.shape[-1]).T @ dpe.reshape(-1, C))
    return float(loss), logits, G
