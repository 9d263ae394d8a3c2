"""CPU oracle: a numpy restatement of the reference's multi-head attention hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``sae_vision_amd``) never
imports it and fails loudly when its HIP library is missing.

PARITY STATUS: **parity unpinned by the reference.**  The reference
(cfoster0/self-attention-experiments-vision, JAX/Flax) holds no golden vectors or
numeric known-answer tests -- its seven ``models/*_test.py`` files assert output
shapes only (e.g. ``models/vit_test.py:23-26``) -- and JAX/Flax are not installed
in this image (an ordinary ``ModuleNotFoundError``, not a permission denial), so
the reference cannot be run to produce vectors.  This restatement is therefore
pinned by (a) the reference's shape contracts, (b) an independent torch-CPU
autograd re-derivation of the same forward (``tests/test_oracle.py``), and
(c) exact integer index tests of the BoTNet relative-logit map against a literal
restatement of the reference's pad/reshape algorithm.

Every function cites the reference file:line it restates.  Layout follows the
reference einsums: activations token-major ``[B, N, H, D]``, scores ``[B, H, Nq, Nk]``.

Precision modes (``mode``):
  * ``"f64"``  -- float64 master, used for gradients and as the truth.
  * ``"f32"``  -- float32 arithmetic, the reference's default ``dtype``.
  * ``"bf16"`` -- float32 arithmetic with round-to-nearest-even to bfloat16 at every
    op boundary where the reference's tensors are bf16 (after each DenseGeneral,
    after q/sqrt(D), after QK^T, inside softmax, after AV), reproducing the Flax
    ``dtype=jnp.bfloat16`` semantics (``models/layers/attentions/attention.py:27-63``)
    including the float32 promotion of the talking-heads mix
    (``models/layers/attentions/talking_heads.py:11-13``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

__all__ = [
    "round_bf16", "cast", "dense_general", "dense_general_out", "softmax",
    "talking_heads_mix", "rotary_sincos", "rotate_every_two", "apply_rotary",
    "to_absolute_logits", "relative_logits_1d", "relative_logits",
    "relative_logits_indexed", "relpos_bias_tables", "attention_core_fwd",
    "attention_core_bwd", "AttnParams", "attention_block_fwd",
    "attention_block_bwd", "attention_block_bwd_bf16", "class_query", "lc_query", "logsumexp",
]


# --------------------------------------------------------------------------- dtypes
def round_bf16(x: np.ndarray) -> np.ndarray:
    """Round float32 values to the nearest bfloat16 (ties to even), returned as float32."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    u = a.view(np.uint32).astype(np.uint64)
    nan = np.isnan(a)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    out = r.astype(np.uint32).view(np.float32).copy()
    out[nan] = np.nan
    return out


def cast(x, mode: str) -> np.ndarray:
    """Cast to the arithmetic type of ``mode`` (bf16 is float32 holding bf16 values)."""
    if mode == "f64":
        return np.asarray(x, dtype=np.float64)
    if mode == "f32":
        return np.asarray(x, dtype=np.float32)
    if mode == "bf16":
        return round_bf16(np.asarray(x, dtype=np.float32))
    raise ValueError(f"unknown mode {mode!r}")


def _acc(mode: str):
    return np.float64 if mode == "f64" else np.float32


# ----------------------------------------------------------------- projections (A2, A10)
def dense_general(x, kernel, mode: str, bias=None):
    """``nn.DenseGeneral(axis=-1, features=(H, D))``: attention.py:29-37.

    Flax casts input and kernel to ``dtype`` and runs dot_general; result is in dtype.
    x [..., C], kernel [C, H, D] -> [..., H, D].
    """
    xc, kc = cast(x, mode), cast(kernel, mode)
    y = np.einsum("...c,chd->...hd", xc.astype(_acc(mode)), kc.astype(_acc(mode)))
    if bias is not None:
        y = y + cast(bias, mode)
    return cast(y, mode)


def dense_general_out(o, kernel, mode: str, bias=None):
    """``nn.DenseGeneral(features=C, axis=(-2, -1))`` named DenseGeneral_0: attention.py:60-63.

    o [..., H, D], kernel [H, D, C] -> [..., C].
    """
    oc, kc = cast(o, mode), cast(kernel, mode)
    y = np.einsum("...hd,hdc->...c", oc.astype(_acc(mode)), kc.astype(_acc(mode)))
    if bias is not None:
        y = y + cast(bias, mode)
    return cast(y, mode)


# ------------------------------------------------------------------------- softmax (A6)
def softmax(x, mode: str, axis: int = -1):
    """``flax.linen.softmax`` == ``jax.nn.softmax`` (jax 0.2.x, requirements.txt:7):
    ``exp(x - stop_gradient(max)) / sum``, in the input's dtype (attention.py:48).
    In bf16 mode every intermediate (x - max, exp, sum, quotient) is rounded to bf16."""
    xc = cast(x, mode)
    m = xc.max(axis=axis, keepdims=True)
    if mode == "bf16":
        d = cast(xc - m, mode)
        e = cast(np.exp(d), mode)
        s = cast(e.sum(axis=axis, keepdims=True), mode)
        return cast(e / s, mode)
    e = np.exp(xc - m)
    return e / e.sum(axis=axis, keepdims=True)


def logsumexp(x, axis=-1):
    x = np.asarray(x, dtype=np.float64)
    m = x.max(axis=axis, keepdims=True)
    return (m + np.log(np.exp(x - m).sum(axis=axis, keepdims=True))).squeeze(axis)


# -------------------------------------------------------------------- talking heads (A5/A7)
def talking_heads_mix(transform, x):
    """``TalkingHeadsBlock``: ``einsum('h i, b h ... -> b i ...', T, x)``
    (models/layers/attentions/talking_heads.py:9-14).  T is [h_in, h_out]; the fp32
    parameter promotes a bf16 ``x`` to fp32 (survey D8), so no rounding is applied."""
    t = np.asarray(transform)
    dt = np.float64 if (t.dtype == np.float64 or np.asarray(x).dtype == np.float64) else np.float32
    return np.einsum("hi,bh...->bi...", t.astype(dt), np.asarray(x).astype(dt))


# ---------------------------------------------------------------------------- rotary (A17)
def rotary_sincos(n: int, dim: int, base: float = 10000.0, dtype=np.float64):
    """Build-defined rotary tables (survey D6): ``inv_freq[i] = base^(-2i/dim)``, positions
    0..n-1.  The reference's ``FixedPositionalEmbedding`` (position_embed.py:23-34) is
    broken (undefined fields, ``10e4**intervals/dim`` precedence), so base 10000 is fixed."""
    i = np.arange(dim // 2, dtype=np.float64)
    inv_freq = base ** (-2.0 * i / dim)
    t = np.arange(n, dtype=np.float64)
    freqs = np.einsum("i,j->ij", t, inv_freq)          # [n, dim/2]
    return np.sin(freqs).astype(dtype), np.cos(freqs).astype(dtype)


def rotate_every_two(x):
    """position_embed.py:8-14: ``stack((-x[..., 1::2], x[..., ::2]), -1)`` interleaved."""
    x1 = x[..., ::2]
    x2 = x[..., 1::2]
    return np.stack((-x2, x1), axis=-1).reshape(x.shape)


def apply_rotary(x, sin, cos):
    """position_embed.py:17-20: ``x*cos + rotate_every_two(x)*sin`` with sin/cos repeated
    per pair (``'b n -> b (n j)', j=2``).  x is [B, N, H, D]; sin/cos are [N, D/2]."""
    s = np.repeat(sin, 2, axis=-1)[None, :, None, :]
    c = np.repeat(cos, 2, axis=-1)[None, :, None, :]
    return x * c + rotate_every_two(x) * s


# ------------------------------------------------------------------- BoTNet rel-pos (A15)
def to_absolute_logits(rel):
    """Literal restatement of ``RelativeLogits._to_absolute_logits`` (botnet.py:77-93):
    pad a zero column, flatten, pad l-1 zeros, reshape to (l+1, 2l-1), slice."""
    b, h, l, _ = rel.shape
    x = np.concatenate((rel, np.zeros((b, h, l, 1), rel.dtype)), axis=3)
    x = x.reshape(b, h, l * 2 * l)
    x = np.concatenate((x, np.zeros((b, h, l - 1), rel.dtype)), axis=2)
    x = x.reshape(b, h, l + 1, 2 * l - 1)
    return x[:, :, :l, l - 1:]


def relative_logits_1d(query, rel_pos_emb):
    """Literal restatement of ``RelativeLogits._relative_logits_1d`` (botnet.py:95-111).
    query [b,h,H,W,d], rel_pos_emb [2W-1,d] -> [b,h,H,H,W,W]."""
    b, h, H, W, _ = query.shape
    x = np.einsum("bhHWd,md->bhHWm", query, rel_pos_emb)
    x = x.reshape(b, h * H, W, 2 * W - 1)
    x = to_absolute_logits(x)
    x = x.reshape(b, h, H, W, W)
    x = np.expand_dims(x, axis=3)
    return np.tile(x, (1, 1, 1, H, 1, 1))


def relative_logits(query, rel_pos_emb_h, rel_pos_emb_w):
    """Literal restatement of ``RelativeLogits.__call__`` (botnet.py:113-141).
    query [b,h,H,W,d] (the *scaled* query, botnet.py:185,191) -> [b,h,H,W,H,W]."""
    rel_w = relative_logits_1d(query, rel_pos_emb_w)
    rel_w = rel_w.transpose(0, 1, 2, 4, 3, 5)                       # b h H I W V -> b h H W I V
    rel_h = relative_logits_1d(query.transpose(0, 1, 3, 2, 4), rel_pos_emb_h)
    rel_h = rel_h.transpose(0, 1, 4, 2, 5, 3)                       # b h W V H I -> b h H W I V
    return rel_h + rel_w


def relpos_bias_tables(qhat, rel_pos_emb_h, rel_pos_emb_w, Hs: int, Ws: int):
    """Index-map form used by the kernels: for query token (x, y) and key row p / column c
    ``bias_h[.., (x,y), p] = qhat·E_h[p - x + Hs - 1]``, ``bias_w[.., (x,y), c] = qhat·E_w[c - y + Ws - 1]``.
    qhat [B, N, H, D] token-major -> (bias_h [B,H,N,Hs], bias_w [B,H,N,Ws])."""
    B, N, H, D = qhat.shape
    assert N == Hs * Ws
    qe_h = np.einsum("bnhd,md->bhnm", qhat, rel_pos_emb_h)          # [B,H,N,2Hs-1]
    qe_w = np.einsum("bnhd,md->bhnm", qhat, rel_pos_emb_w)          # [B,H,N,2Ws-1]
    xs = np.arange(N) // Ws
    ys = np.arange(N) % Ws
    idx_h = np.arange(Hs)[None, :] - xs[:, None] + Hs - 1            # [N, Hs]
    idx_w = np.arange(Ws)[None, :] - ys[:, None] + Ws - 1            # [N, Ws]
    bh = np.take_along_axis(qe_h, np.broadcast_to(idx_h, (B, H, N, Hs)), axis=3)
    bw = np.take_along_axis(qe_w, np.broadcast_to(idx_w, (B, H, N, Ws)), axis=3)
    return bh, bw


def relative_logits_indexed(qhat, rel_pos_emb_h, rel_pos_emb_w, Hs: int, Ws: int):
    """Full [B,H,N,N] relative logits from the bias tables: R[q, k] = bh[q, k//Ws] + bw[q, k%Ws]."""
    bh, bw = relpos_bias_tables(qhat, rel_pos_emb_h, rel_pos_emb_w, Hs, Ws)
    N = Hs * Ws
    kx = np.arange(N) // Ws
    ky = np.arange(N) % Ws
    return bh[..., kx] + bw[..., ky]


# ----------------------------------------------------------------- attention core (A3-A9)
def attention_core_fwd(q, k, v, mode: str = "f64", scale: Optional[float] = None,
                       th1=None, th2=None, bias=None, return_aux=False, round_scores: bool = True):
    """Core of ``AttentionBlock.__call__`` after the projections (attention.py:39-58).

    q [B,Nq,H,D], k/v [B,Nk,H,D] token-major.  ``scale`` defaults to the reference's
    division by sqrt(head_ch) (attention.py:39), applied to q **in dtype**.  Optional
    ``bias`` [B,H,Nq,Nk] is added to the logits (BoTNet relative logits, botnet.py:191).
    Optional talking-heads transforms th1/th2 [H,H] (attention.py:44-52).
    Returns o [B,Nq,H,D] (and an aux dict with the logits / probabilities / LSE).

    ``round_scores=False`` (bf16 mode only) keeps the QK^T einsum's output in fp32 instead of
    rounding it to bf16 as the reference's bf16 einsum does (attention.py:41-42): the arithmetic
    of the HIP kernels, which exponentiate the fp32 MFMA accumulator."""
    D = q.shape[-1]
    qc, kc, vc = cast(q, mode), cast(k, mode), cast(v, mode)
    hi = "f64" if mode == "f64" else "f32"          # promoted type of fp32-param mixes
    if scale is None:
        qh = cast(qc / np.sqrt(D).astype(_acc(mode)), mode)
    else:
        qh = cast(qc * _acc(mode)(scale), mode)
    s = np.einsum("bqhd,bkhd->bhqk", qh.astype(_acc(mode)), kc.astype(_acc(mode)))
    s = cast(s, mode) if round_scores else s
    pmode = mode
    s1 = s
    if bias is not None:
        # botnet.py:191-193: fp32 relative logits promote the sum; softmax runs in fp32
        # and ``.astype(self.dtype)`` casts P back before the AV einsum.
        s1 = cast(s1, hi) + cast(bias, hi)
        pmode = hi
    if th1 is not None:
        s1 = talking_heads_mix(th1, s1)      # fp32 param promotes (talking_heads.py:13)
        pmode = hi
    # unrounded scores: the kernels' fp32 softmax (P rounded to bf16 only as the AV operand)
    p = softmax(s1, pmode if round_scores or pmode != "bf16" else "f32")
    p2 = p
    if th2 is not None:
        p2 = talking_heads_mix(th2, p)
        pmode = hi
    elif bias is not None:
        p2 = cast(p, mode)
        pmode = mode
    o = np.einsum("bhqk,bkhd->bqhd", cast(p2, pmode).astype(_acc(pmode)),
                  cast(vc, pmode).astype(_acc(pmode)))
    o = cast(o, pmode)
    if return_aux:
        aux = dict(qhat=qh, s=s, s1=s1, p=p, p2=p2, lse=logsumexp(s1, axis=-1))
        return o, aux
    return o


def attention_core_bwd(q, k, v, do, scale: Optional[float] = None, th1=None, th2=None,
                       bias=None):
    """Hand-derived float64 backward of :func:`attention_core_fwd` (what JAX autodiff
    computes for attention.py:39-58, survey A18).  Returns dict(dq, dk, dv[, dbias, dth1, dth2])."""
    q, k, v, do = (np.asarray(t, np.float64) for t in (q, k, v, do))
    D = q.shape[-1]
    sc = (1.0 / math.sqrt(D)) if scale is None else float(scale)
    qh = q * sc
    s = np.einsum("bqhd,bkhd->bhqk", qh, k)
    if bias is not None:
        s = s + np.asarray(bias, np.float64)
    s1 = talking_heads_mix(np.asarray(th1, np.float64), s) if th1 is not None else s
    m = s1.max(-1, keepdims=True)
    e = np.exp(s1 - m)
    p = e / e.sum(-1, keepdims=True)
    p2 = talking_heads_mix(np.asarray(th2, np.float64), p) if th2 is not None else p
    dv = np.einsum("bhqk,bqhd->bkhd", p2, do)
    dp2 = np.einsum("bqhd,bkhd->bhqk", do, v)
    out = {}
    if th2 is not None:
        out["dth2"] = np.einsum("bhqk,biqk->hi", p, dp2)
        dp = np.einsum("hi,biqk->bhqk", np.asarray(th2, np.float64), dp2)
    else:
        dp = dp2
    ds1 = p * (dp - (dp * p).sum(-1, keepdims=True))
    if th1 is not None:
        out["dth1"] = np.einsum("bhqk,biqk->hi", s, ds1)
        ds = np.einsum("hi,biqk->bhqk", np.asarray(th1, np.float64), ds1)
    else:
        ds = ds1
    if bias is not None:
        out["dbias"] = ds
    dqh = np.einsum("bhqk,bkhd->bqhd", ds, k)
    dk = np.einsum("bhqk,bqhd->bkhd", ds, qh)
    out.update(dq=dqh * sc, dk=dk, dv=dv)
    return out


# ------------------------------------------------------------- whole AttentionBlock (A1)
@dataclass
class AttnParams:
    """Param tree of one ``AttentionBlock`` (survey §8b): names follow Flax's
    auto-naming in attention.py:33-63 and talking_heads.py:11-12."""
    queries: np.ndarray                 # [C, H, D]
    keys: np.ndarray                    # [C, H, D]
    values: np.ndarray                  # [C, H, D]
    out: np.ndarray                     # DenseGeneral_0 kernel [H, D, Cout]
    th1: Optional[np.ndarray] = None    # TalkingHeadsBlock_0 [H, H]
    th2: Optional[np.ndarray] = None    # TalkingHeadsBlock_1 [H, H]
    bq: Optional[np.ndarray] = None     # biases when use_bias=True
    bk: Optional[np.ndarray] = None
    bv: Optional[np.ndarray] = None
    bo: Optional[np.ndarray] = None
    extra: Dict[str, np.ndarray] = field(default_factory=dict)


def class_query(x):
    """``ClassSelfAttentionBlock``: ``inputs[:, 0]`` expanded (models/cait.py:14)."""
    return x[:, 0:1, :]


def lc_query(x):
    """``LCSelfAttentionBlock``: ``inputs[:, -1]`` expanded (models/ceit.py:15)."""
    return x[:, -1:, :]


def attention_block_fwd(x_q, x_kv, p: AttnParams, mode: str = "f64", rotary: bool = False,
                        return_aux: bool = False):
    """``AttentionBlock.__call__`` (attention.py:20-67) with dropout rate 0 (identity, A8).
    ``rotary=True`` applies the build-defined rotary to q and k after projection (A17)."""
    q = dense_general(x_q, p.queries, mode, p.bq)
    k = dense_general(x_kv, p.keys, mode, p.bk)
    v = dense_general(x_kv, p.values, mode, p.bv)
    if rotary:
        D = q.shape[-1]
        sq, cq = rotary_sincos(q.shape[1], D)
        sk, ck = rotary_sincos(k.shape[1], D)
        q = cast(apply_rotary(q.astype(np.float64), sq, cq), mode)
        k = cast(apply_rotary(k.astype(np.float64), sk, ck), mode)
    o, aux = attention_core_fwd(q, k, v, mode, th1=p.th1, th2=p.th2, return_aux=True)
    y = dense_general_out(o, p.out, mode, p.bo)
    if return_aux:
        aux.update(q=q, k=k, v=v, o=o)
        return y, aux
    return y


def attention_block_bwd(x_q, x_kv, p: AttnParams, dy, rotary: bool = False):
    """Float64 backward of :func:`attention_block_fwd` -> dict of input and param grads
    keyed by the Flax names (``queries``, ``keys``, ``values``, ``DenseGeneral_0``,
    ``TalkingHeadsBlock_0``, ``TalkingHeadsBlock_1``) plus ``x_q`` / ``x_kv``."""
    f = lambda t: None if t is None else np.asarray(t, np.float64)
    xq, xkv, dy = f(x_q), f(x_kv), f(dy)
    Wq, Wk, Wv, Wo = f(p.queries), f(p.keys), f(p.values), f(p.out)
    q = np.einsum("bnc,chd->bnhd", xq, Wq) + (0 if p.bq is None else f(p.bq))
    k = np.einsum("bnc,chd->bnhd", xkv, Wk) + (0 if p.bk is None else f(p.bk))
    v = np.einsum("bnc,chd->bnhd", xkv, Wv) + (0 if p.bv is None else f(p.bv))
    if rotary:
        D = q.shape[-1]
        sq, cq = rotary_sincos(q.shape[1], D)
        sk, ck = rotary_sincos(k.shape[1], D)
        qr, kr = apply_rotary(q, sq, cq), apply_rotary(k, sk, ck)
    else:
        qr, kr = q, k
    o = attention_core_fwd(qr, kr, v, "f64", th1=f(p.th1), th2=f(p.th2))
    g = {}
    g["DenseGeneral_0"] = np.einsum("bnhd,bnc->hdc", o, dy)
    if p.bo is not None:
        g["DenseGeneral_0_bias"] = dy.sum(axis=(0, 1))
    do = np.einsum("bnc,hdc->bnhd", dy, Wo)
    cg = attention_core_bwd(qr, kr, v, do, th1=f(p.th1), th2=f(p.th2))
    dq, dk, dv = cg["dq"], cg["dk"], cg["dv"]
    if rotary:   # inverse rotation: the rotary map is orthogonal, its transpose is rotation by -theta
        dq = apply_rotary(dq, -sq, cq)
        dk = apply_rotary(dk, -sk, ck)
    if "dth1" in cg:
        g["TalkingHeadsBlock_0"] = cg["dth1"]
        g["TalkingHeadsBlock_1"] = cg["dth2"]
    g["queries"] = np.einsum("bnc,bnhd->chd", xq, dq)
    g["keys"] = np.einsum("bnc,bnhd->chd", xkv, dk)
    g["values"] = np.einsum("bnc,bnhd->chd", xkv, dv)
    if p.bq is not None:
        g["queries_bias"] = dq.sum(axis=(0, 1))
        g["keys_bias"] = dk.sum(axis=(0, 1))
        g["values_bias"] = dv.sum(axis=(0, 1))
    g["x_q"] = np.einsum("bnhd,chd->bnc", dq, Wq)
    g["x_kv"] = np.einsum("bnhd,chd->bnc", dk, Wk) + np.einsum("bnhd,chd->bnc", dv, Wv)
    g["dq"], g["dk"], g["dv"], g["do"] = dq, dk, dv, do
    return g


def _rb(x):
    """bf16 rounding, kept in float64 (the accumulation type of the emulated dot products)."""
    return round_bf16(np.asarray(x, np.float32)).astype(np.float64)


def attention_block_bwd_bf16(x_q, x_kv, p: AttnParams, dy):
    """bf16-emulated JAX autodiff of ``attention_block_fwd(..., "bf16")`` (no rotary): the
    cotangent of every bf16 value is bf16 (each dot_general / elementwise op of the backward rounds
    its output; products accumulate in wider precision), the gradient of a bf16-cast fp32
    parameter is the bf16 cotangent cast back to fp32.  jax.nn.softmax's VJP (jax 0.2.x) is
    ``p * (g - sum(g * p))`` evaluated in bf16.  Talking heads (attention.py:44-52): the fp32
    transforms promote the scores, so the mixes, the softmax, P V and their cotangents are fp32
    (survey D8) until the bf16 scores' and the bf16-cast output's cotangents.  Returns the same
    keys as :func:`attention_block_bwd`."""
    y, aux = attention_block_fwd(x_q, x_kv, p, "bf16", return_aux=True)
    f = lambda t: np.asarray(t, np.float64)
    xq, xkv = _rb(x_q), _rb(x_kv)
    Wq, Wk, Wv, Wo = (_rb(t) for t in (p.queries, p.keys, p.values, p.out))
    q, k, v, o = (f(aux[n]) for n in ("q", "k", "v", "o"))
    qh, pr = f(aux["qhat"]), f(aux["p"])
    D = q.shape[-1]
    g = {}
    dyb = _rb(dy)
    g["DenseGeneral_0"] = _rb(np.einsum("bnhd,bnc->hdc", _rb(o), dyb))
    do = _rb(np.einsum("bnc,hdc->bnhd", dyb, Wo))
    if p.th1 is None and p.th2 is None:
        dv = _rb(np.einsum("bhqk,bqhd->bkhd", pr, do))
        dp = _rb(np.einsum("bqhd,bkhd->bhqk", do, v))
        t = _rb(dp * pr)
        sm = _rb(t.sum(-1, keepdims=True))
        ds = _rb(pr * _rb(dp - sm))
    else:
        t1, t2 = f(p.th1), f(p.th2)
        p2, s = f(aux["p2"]), f(aux["s"])
        dv = _rb(np.einsum("bhqk,bqhd->bkhd", p2, do))                      # fp32 P V, bf16-cast v
        dp2 = np.einsum("bqhd,bkhd->bhqk", do, v)
        g["TalkingHeadsBlock_1"] = np.einsum("bhqk,biqk->hi", pr, dp2)
        dp = np.einsum("hi,biqk->bhqk", t2, dp2)
        ds1 = pr * (dp - (dp * pr).sum(-1, keepdims=True))                    # fp32 softmax VJP
        g["TalkingHeadsBlock_0"] = np.einsum("bhqk,biqk->hi", s, ds1)
        ds = _rb(np.einsum("hi,biqk->bhqk", t1, ds1))                         # cotangent of bf16 scores
    dqh = _rb(np.einsum("bhqk,bkhd->bqhd", ds, k))
    dk = _rb(np.einsum("bhqk,bqhd->bkhd", ds, qh))
    dq = _rb(dqh / np.sqrt(D))
    g["queries"] = _rb(np.einsum("bnc,bnhd->chd", xq, dq))
    g["keys"] = _rb(np.einsum("bnc,bnhd->chd", xkv, dk))
    g["values"] = _rb(np.einsum("bnc,bnhd->chd", xkv, dv))
    g["x_q"] = _rb(np.einsum("bnhd,chd->bnc", dq, Wq))
    g["x_kv"] = _rb(_rb(np.einsum("bnhd,chd->bnc", dk, Wk)) + _rb(np.einsum("bnhd,chd->bnc", dv, Wv)))
    g["dq"], g["dk"], g["dv"], g["do"] = dq, dk, dv, do
    return g


# ----------------------------------------------------------- BoTNet MHSA core (A15/A16)
def botnet_mhsa_core_fwd(q, k, v, rel_pos_emb_h, rel_pos_emb_w, Hs: int, Ws: int,
                         mode: str = "f64"):
    """Intended ``BoTMHSA`` core (botnet.py:185-198 with survey decisions D1, D3, D4):
    qhat = q / sqrt(d); logits = qhat k^T + RelativeLogits(qhat); softmax over all Hs*Ws
    keys; out = P V.  q/k/v token-major [B, Hs*Ws, h, d]."""
    D = q.shape[-1]
    qh = cast(cast(q, mode) / np.sqrt(D).astype(_acc(mode)), mode)
    bias = relative_logits_indexed(qh.astype(np.float64), np.asarray(rel_pos_emb_h, np.float64),
                                   np.asarray(rel_pos_emb_w, np.float64), Hs, Ws)
    return attention_core_fwd(qh, k, v, mode, scale=1.0, bias=bias)
