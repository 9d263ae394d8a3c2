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
