"""Drop-in attention modules mirroring the reference's Flax API.

Reference: models/layers/attentions/attention.py:10-74 (AttentionBlock, SelfAttentionBlock),
models/layers/attentions/talking_heads.py:5-14 (TalkingHeadsBlock), models/cait.py:10-15
(ClassSelfAttentionBlock), models/ceit.py:11-16 (LCSelfAttentionBlock).

Same dataclass fields, same call signatures (``(inputs_q, inputs_kv, is_training)`` /
``(inputs, is_training)``), same parameter tree (``queries/kernel [C,H,D]``,
``keys/kernel``, ``values/kernel``, ``DenseGeneral_0/kernel [H,D,C]``, optional ``bias``,
``TalkingHeadsBlock_0/talking_heads_transform [H,H]`` and ``_1``), parameters kept in fp32 and
cast to ``dtype`` for compute like Flax's DenseGeneral.  Parameters are created at
construction when ``in_ch`` is given, otherwise at the first call (Flax ``init`` semantics).

Compute path: projections go through ``ops.dense``.  bf16 forward and input gradient run on the
hand-written ``sae_gemm_nt`` for every width that is a multiple of 8 (the C ABI picks the kernel:
the persistent LDS-DMA ``gemm8`` for 192-wide output tiles -- every DeiT-S / CaiT shape and the
ViT-B wide forwards --, the ping-pong ``gemm8x`` for the 768 / 1024-feature outputs at K >= 768,
the 128-row kernel for the rest, K-tail instances included); the fp32 compute dtype runs on the
exact-f32 MFMA GEMM ``sae_gemm_f32``; weight / bias gradients go straight into fp32 through the
split-token MFMA kernels (``sae_gemm_dw``).  The self-attention Q/K/V projection is ONE GEMM
producing a packed [B, N, 3, H, D] buffer that the attention kernel reads in place by strides; the
attention core is the fused HIP kernel (``ops.attention*``).  There is no eager/CPU fallback.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops

# rotary base (position_embed.py: build-defined, survey D6); the standalone ops.rotary default
ROTARY_BASE = 10000.0

__all__ = ["DenseGeneral", "AttentionBlock", "SelfAttentionBlock", "TalkingHeadsBlock",
           "ClassSelfAttentionBlock", "LCSelfAttentionBlock", "lecun_normal_", "flax_params",
           "load_flax_params"]


def lecun_normal_(t: torch.Tensor, fan_in: int) -> torch.Tensor:
    """Flax ``initializers.lecun_normal()``: variance_scaling(1, 'fan_in', 'truncated_normal')."""
    std = math.sqrt(1.0 / fan_in) / 0.87962566103423978
    with torch.no_grad():
        return nn.init.trunc_normal_(t, mean=0.0, std=std, a=-2.0 * std, b=2.0 * std)


class DenseGeneral(nn.Module):
    """Parameter holder named like Flax's ``nn.DenseGeneral`` (kernel [*in, *out], bias [*out])."""

    def __init__(self, in_shape, out_shape, use_bias: bool, device=None):
        super().__init__()
        in_shape, out_shape = tuple(in_shape), tuple(out_shape)
        self.in_shape, self.out_shape = in_shape, out_shape
        fan_in = int(math.prod(in_shape))
        self.kernel = nn.Parameter(lecun_normal_(torch.empty(in_shape + out_shape, device=device), fan_in))
        self.bias = nn.Parameter(torch.zeros(out_shape, device=device)) if use_bias else None


class TalkingHeadsBlock(nn.Module):
    """``TalkingHeadsBlock(num_heads)`` (talking_heads.py:5-14).  Holds the fp32
    ``talking_heads_transform`` [H, H] (orthogonal init, indexed [h_in, h_out]).  Inside
    AttentionBlock the mix is fused into the HIP kernel; calling the block directly applies
    ``einsum('h i, b h ... -> b i ...')`` as the reference does."""

    def __init__(self, num_heads: int, device=None):
        super().__init__()
        self.num_heads = num_heads
        t = torch.empty(num_heads, num_heads, device=device)
        nn.init.orthogonal_(t)
        self.talking_heads_transform = nn.Parameter(t)

    def forward(self, inputs: torch.Tensor) -> torch.Tensor:
        w = self.talking_heads_transform
        return torch.einsum("hi,bh...->bi...", w.to(torch.promote_types(w.dtype, inputs.dtype)),
                            inputs.to(torch.promote_types(w.dtype, inputs.dtype)))


class AttentionBlock(nn.Module):
    """``AttentionBlock`` (attention.py:10-67)."""

    def __init__(self, num_heads: int, head_ch: Optional[int] = None, out_ch: Optional[int] = None,
                 talking_heads: bool = False, attn_dropout_rate: float = 0.0, out_dropout_rate: float = 0.0,
                 use_bias: bool = False, dtype: torch.dtype = torch.float32, *, in_ch: Optional[int] = None,
                 rotary: bool = False, device=None):
        super().__init__()
        self.num_heads = num_heads
        self.head_ch = head_ch
        self.out_ch = out_ch
        self.talking_heads = talking_heads
        self.attn_dropout_rate = attn_dropout_rate
        self.out_dropout_rate = out_dropout_rate
        self.use_bias = use_bias
        self.dtype = dtype
        self.rotary = rotary          # build-defined rotary on q/k (README to-do, survey D6)
        self._in_ch = None
        if in_ch is not None:
            self._build(in_ch, device)

    # -- parameters --------------------------------------------------------------------
    def _build(self, in_ch: int, device=None):
        assert in_ch % self.num_heads == 0
        head_ch = self.head_ch or int(in_ch / self.num_heads)
        out_ch = self.out_ch or in_ch
        H = self.num_heads
        self._in_ch, self._head_ch_eff, self._out_ch_eff = in_ch, head_ch, out_ch
        self.queries = DenseGeneral((in_ch,), (H, head_ch), self.use_bias, device)
        self.keys = DenseGeneral((in_ch,), (H, head_ch), self.use_bias, device)
        self.values = DenseGeneral((in_ch,), (H, head_ch), self.use_bias, device)
        if self.talking_heads:
            self.TalkingHeadsBlock_0 = TalkingHeadsBlock(H, device)
            self.TalkingHeadsBlock_1 = TalkingHeadsBlock(H, device)
        self.DenseGeneral_0 = DenseGeneral((H, head_ch), (out_ch,), self.use_bias, device)

    def weight_groups(self):
        """The fp32 kernels as the 2-D column blocks the projections use (``ops.cast_weights``)."""
        if self._in_ch is None:
            return []
        C, HD = self._in_ch, self.num_heads * self._head_ch_eff
        return [[m.kernel.reshape(C, HD) for m in (self.queries, self.keys, self.values)],
                [self.DenseGeneral_0.kernel.reshape(HD, self._out_ch_eff)]]

    def cross_weight_groups(self):
        """The column blocks the projections use when queries and keys / values come from
        different inputs (class / last-token attention): [queries], [keys | values], [output]."""
        if self._in_ch is None:
            return []
        C, HD = self._in_ch, self.num_heads * self._head_ch_eff
        return [[self.queries.kernel.reshape(C, HD)],
                [m.kernel.reshape(C, HD) for m in (self.keys, self.values)],
                [self.DenseGeneral_0.kernel.reshape(HD, self._out_ch_eff)]]

    # -- forward -----------------------------------------------------------------------
    def forward(self, inputs_q: torch.Tensor, inputs_kv: torch.Tensor, is_training: bool) -> torch.Tensor:
        assert inputs_q.ndim == inputs_kv.ndim == 3
        in_ch = inputs_q.shape[-1]
        assert in_ch % self.num_heads == 0
        if self._in_ch is None:
            self._build(in_ch, inputs_q.device)
        elif self._in_ch != in_ch:
            raise ValueError(f"AttentionBlock built for {self._in_ch} channels, got {in_ch}")
        if is_training and self.attn_dropout_rate > 0.0:
            raise NotImplementedError(
                "attention-probability dropout (attn_dropout_rate > 0 while training) is not fused into the "
                "HIP kernel; every reference config uses rate 0 (vit.py:68, create_model.py)")
        H, D = self.num_heads, self._head_ch_eff
        dt = self.dtype
        B, Nq, C = inputs_q.shape
        Nk = inputs_kv.shape[1]
        xq = inputs_q.to(dt)
        scale = 1.0 / math.sqrt(D)
        HD = H * D
        wq, wk, wv = (m.kernel for m in (self.queries, self.keys, self.values))     # fp32 [C, H, D]
        bias = (lambda *ms: torch.stack([m.bias for m in ms], 0).reshape(-1)) if self.use_bias else None
        self_attn = inputs_q is inputs_kv
        if self_attn:
            # ONE projection GEMM producing the packed [B, N, 3, H, D] buffer the kernels read in place
            w = [wq.reshape(C, HD), wk.reshape(C, HD), wv.reshape(C, HD)]   # = stack(dim=1) columns
            qkv = ops.dense(xq, w, bias(self.queries, self.keys, self.values) if bias else None, dt)
            qkv = qkv.view(B, Nq, 3, H, D)
            q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        else:
            xkv = inputs_kv.to(dt)
            q = ops.dense(xq, wq.reshape(C, HD), self.queries.bias.reshape(-1) if bias else None, dt)
            q = q.view(B, Nq, H, D)
            kv = ops.dense(xkv, [wk.reshape(C, HD), wv.reshape(C, HD)],
                           bias(self.keys, self.values) if bias else None, dt).view(B, Nk, 2, H, D)
            k, v = kv[:, :, 0], kv[:, :, 1]
        # rotary (position_embed.py:8-20) rides inside the attention kernels: q / k stay un-rotated
        rope = ROTARY_BASE if self.rotary else None
        if self.talking_heads and self_attn:
            o = ops.talking_heads_attention_packed(qkv, self.TalkingHeadsBlock_0.talking_heads_transform,
                                                   self.TalkingHeadsBlock_1.talking_heads_transform, scale, rope)
        elif self.talking_heads:
            o = ops.talking_heads_attention(q, k, v, self.TalkingHeadsBlock_0.talking_heads_transform,
                                            self.TalkingHeadsBlock_1.talking_heads_transform, scale, rope)
        elif self_attn:
            o = ops.attention_packed(qkv, scale, rope)
        else:
            o = ops.attention(q, k, v, scale, rotary=rope)
        wo = self.DenseGeneral_0.kernel.reshape(HD, self._out_ch_eff)
        y = ops.dense(o.reshape(B, Nq, HD), wo, self.DenseGeneral_0.bias if self.use_bias else None, dt)
        if self.out_dropout_rate > 0.0:
            y = F.dropout(y, p=self.out_dropout_rate, training=is_training)
        return y


class SelfAttentionBlock(AttentionBlock):
    """``SelfAttentionBlock`` (attention.py:70-74): ``AttentionBlock(inputs, inputs)``."""

    def forward(self, inputs: torch.Tensor, is_training: bool) -> torch.Tensor:  # type: ignore[override]
        return super().forward(inputs, inputs, is_training=is_training)


class ClassSelfAttentionBlock(AttentionBlock):
    """CaiT class attention (models/cait.py:10-15): query = token 0 (CLS), keys = all tokens."""

    def forward(self, inputs: torch.Tensor, is_training: bool) -> torch.Tensor:  # type: ignore[override]
        inputs_q = inputs[:, 0:1, :]
        return super().forward(inputs_q, inputs, is_training=is_training)


class LCSelfAttentionBlock(AttentionBlock):
    """CeiT layer-wise class-token attention (models/ceit.py:11-16): query = last token."""

    def forward(self, inputs: torch.Tensor, is_training: bool) -> torch.Tensor:  # type: ignore[override]
        inputs_q = inputs[:, -1:, :]
        return super().forward(inputs_q, inputs, is_training=is_training)


# ------------------------------------------------------------------ Flax param-tree interop
def flax_params(module: nn.Module) -> Dict:
    """Nested dict of fp32 tensors in the reference's Flax param-tree layout
    (``{'queries': {'kernel': ...}, 'DenseGeneral_0': {...}, ...}``)."""
    tree: Dict = {}
    for name, p in module.named_parameters():
        node = tree
        parts = name.split(".")
        for part in parts[:-1]:
            node = node.setdefault(part, {})
        node[parts[-1]] = p.detach()
    return tree


def load_flax_params(module: nn.Module, tree: Dict) -> None:
    """Copy a Flax-layout param tree (nested dict of arrays / tensors) into ``module``."""
    params = dict(module.named_parameters())

    def walk(node, prefix):
        for k, v in node.items():
            key = f"{prefix}.{k}" if prefix else k
            if isinstance(v, dict):
                walk(v, key)
            else:
                if key not in params:
                    raise KeyError(f"unexpected parameter {key!r}")
                t = torch.as_tensor(v)
                if tuple(t.shape) != tuple(params[key].shape):
                    raise ValueError(f"{key}: shape {tuple(t.shape)} != {tuple(params[key].shape)}")
                with torch.no_grad():
                    params[key].copy_(t.to(params[key].dtype))

    walk(tree, "")
