"""CPU oracle for the CaiT forward (numpy, float64).

TEST INFRASTRUCTURE ONLY (see attention_ref.py header): used by ``tests/test_gpu_cait.py`` as the
checker of ``sae_vision_amd.cait``.  Parity unpinned by the reference (shape-only tests, no JAX).

Restates models/cait.py:10-186 in evaluation mode (stochastic depth is the identity there,
stochastic_depth.py:19-28): PatchEmbedBlock (patch_embed.py:15-26), Encoder = AddAbsPosEmbed +
EncoderBlock_i (cait.py:18-91: LN -> talking-heads SelfAttentionBlock -> LayerScale -> + ;
LN -> FFBlock -> LayerScale -> +), CAEncoderBlock_i (cait.py:94-129: class attention of the CLS
token over [cls, x] -> LayerScale -> + ; LN -> FFBlock -> LayerScale -> +), final LayerNorm over
[cls, x] and the CLS row's Dense head (cait.py:171-186).  The attention cores come from
attention_ref.attention_core_fwd (talking heads: attention.py:44-52, talking_heads.py:9-14).
Parameters: a flat dict keyed by the torch module's parameter names (Flax tree paths).
"""
from __future__ import annotations

from typing import Dict

import numpy as np

import attention_ref as R
import vit_ref as V


def _attention(P, pre: str, x_q, x_kv, talking: bool):
    """attention.py:20-67 with the block's params under ``pre`` (no bias: use_bias=False)."""
    Wq, Wk, Wv = (P[pre + f"{n}.kernel"] for n in ("queries", "keys", "values"))
    Wo = P[pre + "DenseGeneral_0.kernel"]
    C, H, D = Wq.shape
    B, Nq, _ = x_q.shape
    Nk = x_kv.shape[1]
    q = (x_q @ Wq.reshape(C, H * D)).reshape(B, Nq, H, D)
    k = (x_kv @ Wk.reshape(C, H * D)).reshape(B, Nk, H, D)
    v = (x_kv @ Wv.reshape(C, H * D)).reshape(B, Nk, H, D)
    th1 = P[pre + "TalkingHeadsBlock_0.talking_heads_transform"] if talking else None
    th2 = P[pre + "TalkingHeadsBlock_1.talking_heads_transform"] if talking else None
    o = R.attention_core_fwd(q, k, v, "f64", th1=th1, th2=th2)
    return o.reshape(B, Nq, H * D) @ Wo.reshape(H * D, -1)


def _ff(P, pre: str, x):
    """ff.py:17-34: Dense -> tanh-GELU -> Dense."""
    u = x @ P[pre + "Dense_0.kernel"] + P[pre + "Dense_0.bias"]
    return V.gelu_tanh(u) @ P[pre + "Dense_1.kernel"] + P[pre + "Dense_1.bias"]


def _ln(P, pre: str, x):
    return V.layer_norm(x, P[pre + "scale"], P[pre + "bias"])[0]


def cait_forward(params: Dict[str, np.ndarray], images, num_layers: int, num_layers_token_only: int,
                 patch: int) -> np.ndarray:
    """Logits [B, classes] of CaiT on NHWC ``images`` (evaluation mode)."""
    P = {k: np.asarray(v, np.float64) for k, v in params.items()}
    B = images.shape[0]
    x = V.patchify(np.asarray(images, np.float64), patch) @ P["PatchEmbedBlock_0.Dense_0.kernel"]
    x = x + P["Encoder_0.AddAbsPosEmbed_0.pos_embed"]                       # no CLS in the trunk
    for i in range(num_layers):
        pre = f"Encoder_0.EncoderBlock_{i}."
        a = _attention(P, pre + "SelfAttentionBlock_0.", _ln(P, pre + "LayerNorm_0.", x),
                       _ln(P, pre + "LayerNorm_0.", x), talking=True)
        x = x + a * P[pre + "LayerScaleBlock_0.layerscale"]
        y = _ff(P, pre + "FFBlock_0.", _ln(P, pre + "LayerNorm_1.", x))
        x = x + y * P[pre + "LayerScaleBlock_1.layerscale"]
    cls = np.broadcast_to(P["cls"], (B, 1, x.shape[-1]))
    for i in range(num_layers_token_only):
        pre = f"CAEncoderBlock_{i}."
        z = _ln(P, pre + "LayerNorm_0.", np.concatenate([cls, x], axis=1))
        a = _attention(P, pre + "ClassSelfAttentionBlock_0.", z[:, 0:1], z, talking=False)   # cait.py:14
        cls = cls + a * P[pre + "LayerScaleBlock_0.layerscale"]
        y = _ff(P, pre + "FFBlock_0.", _ln(P, pre + "LayerNorm_1.", cls))
        cls = cls + y * P[pre + "LayerScaleBlock_1.layerscale"]
    z = _ln(P, "LayerNorm_0.", np.concatenate([cls, x], axis=1))
    return z[:, 0] @ P["Dense_0.kernel"] + P["Dense_0.bias"]


# ------------------------------------------------------------ bf16-emulated training chain
def _torch_rb():
    """Round-to-bf16 as an autograd op in float64 torch: forward rounds the value (RNE), backward
    rounds the cotangent -- JAX autodiff's contract for a bf16 value (its cotangent is bf16)."""
    import torch

    def rnd(t):
        return t.float().to(torch.bfloat16).double()

    class RB(torch.autograd.Function):
        @staticmethod
        def forward(ctx, t):
            return rnd(t)

        @staticmethod
        def backward(ctx, g):
            return rnd(g)

    return RB.apply


def cait_logits_bf16(params, images, num_layers: int, num_layers_token_only: int, patch: int):
    """The bf16 CaiT model of this build (``create_cait(..., dtype=bfloat16)``: the trunk in bf16 as
    BASELINE configs[4] runs it, survey D7) as a float64 torch program with the bf16 rounding points
    of the Flax modules: every Dense / DenseGeneral casts input and kernel to bf16 and returns bf16
    (bias cast to bf16 and added), LayerNorm computes in fp32 and returns bf16, q / sqrt(D), the
    scores and the class-attention softmax are bf16, the talking-heads mixes (fp32 params) promote
    the scores, softmax and P V to fp32 (talking_heads.py:13, survey D8), GELU returns bf16,
    LayerScale multiplies in bf16, the residual stream is fp32.  ``params``: dict name -> float64
    torch tensors (leaves with requires_grad for the backward); ``images`` NHWC.  Autograd through
    it is the bf16-emulated JAX-autodiff backward (each bf16 value's cotangent rounded to bf16).
    Evaluation semantics of stochastic depth (rate 0).  Returns logits [B, classes] (bf16 values)."""
    import math as _m

    import torch
    rb = _torch_rb()
    P = params

    def dense(x, pre, bias=True):
        y = rb(rb(x) @ rb(P[pre + "kernel"].reshape(x.shape[-1], -1)))
        if bias and (pre + "bias") in P:
            y = rb(y + rb(P[pre + "bias"]))
        return y

    def ln(x, pre, eps=1e-6):
        mu = x.mean(-1, keepdim=True)
        xc = x - mu
        var = (xc * xc).mean(-1, keepdim=True)
        return rb(xc / torch.sqrt(var + eps) * P[pre + "scale"] + P[pre + "bias"])

    def gelu(u):
        c = _m.sqrt(2.0 / _m.pi)
        return rb(0.5 * u * (1.0 + torch.tanh(c * (u + 0.044715 * u ** 3))))

    def attention(pre, xq, xkv, talking):
        Wq = P[pre + "queries.kernel"]
        C, H, D = Wq.shape
        B, Nq, _ = xq.shape
        Nk = xkv.shape[1]
        q = dense(xq, pre + "queries.", False).reshape(B, Nq, H, D).permute(0, 2, 1, 3)
        k = dense(xkv, pre + "keys.", False).reshape(B, Nk, H, D).permute(0, 2, 1, 3)
        v = dense(xkv, pre + "values.", False).reshape(B, Nk, H, D).permute(0, 2, 1, 3)
        qh = rb(q / _m.sqrt(D))
        s = rb(qh @ k.transpose(-1, -2))                                    # [B, H, Nq, Nk] bf16
        if talking:   # fp32 transforms promote: mix, softmax, mix and P V in fp32
            t1 = P[pre + "TalkingHeadsBlock_0.talking_heads_transform"]
            t2 = P[pre + "TalkingHeadsBlock_1.talking_heads_transform"]
            s1 = torch.einsum("hi,bhqk->biqk", t1, s)
            p = torch.softmax(s1, -1)
            p2 = torch.einsum("hi,bhqk->biqk", t2, p)
            o = p2 @ v
        else:         # jax.nn.softmax in bf16, then P V in bf16
            e = rb(torch.exp(rb(s - s.max(-1, keepdim=True).values.detach())))
            p = rb(e / rb(e.sum(-1, keepdim=True)))
            o = rb(p @ v)
        o = o.permute(0, 2, 1, 3).reshape(B, Nq, H * D)
        return dense(o, pre + "DenseGeneral_0.", False)

    def ff(pre, x):
        return dense(gelu(dense(x, pre + "Dense_0.")), pre + "Dense_1.")

    def scaled(y, pre):
        return rb(y * rb(P[pre + "layerscale"]))

    imgs = torch.as_tensor(images, dtype=torch.float64)
    B, Hh, Ww, c = imgs.shape
    xp = imgs.reshape(B, Hh // patch, patch, Ww // patch, patch, c).permute(0, 1, 3, 2, 4, 5)
    xp = xp.reshape(B, (Hh // patch) * (Ww // patch), patch * patch * c)
    x = dense(xp, "PatchEmbedBlock_0.Dense_0.", False) + P["Encoder_0.AddAbsPosEmbed_0.pos_embed"]
    for i in range(num_layers):
        pre = f"Encoder_0.EncoderBlock_{i}."
        h = ln(x, pre + "LayerNorm_0.")
        x = x + scaled(attention(pre + "SelfAttentionBlock_0.", h, h, True), pre + "LayerScaleBlock_0.")
        x = x + scaled(ff(pre + "FFBlock_0.", ln(x, pre + "LayerNorm_1.")), pre + "LayerScaleBlock_1.")
    cls = P["cls"].expand(B, 1, x.shape[-1])
    for i in range(num_layers_token_only):
        pre = f"CAEncoderBlock_{i}."
        z = ln(torch.cat([cls, x], 1), pre + "LayerNorm_0.")
        cls = cls + scaled(attention(pre + "ClassSelfAttentionBlock_0.", z[:, 0:1], z, False),
                           pre + "LayerScaleBlock_0.")
        cls = cls + scaled(ff(pre + "FFBlock_0.", ln(cls, pre + "LayerNorm_1.")), pre + "LayerScaleBlock_1.")
    return dense(ln(cls[:, 0], "LayerNorm_0."), "Dense_0.")
