"""CvT attention modules (models/layers/attentions/cvt_attention.py:12-120), MI355X path.

``CvTAttentionBlock`` keeps the reference's fields, call signature
``(inputs_q [b, H, W, c], inputs_kv [b, H', W', c], is_training)`` and param tree
(``ConvProjectionBlock_{0,1,2}/{Conv_0, BatchNorm_0, Conv_1}``, ``TalkingHeadsBlock_{0,1}``,
``DenseGeneral_0``).  The convolutional projections (depthwise 3x3 + BatchNorm + 1x1,
cvt_attention.py:21-40) are outside the hot path (conv, not attention) and run as
framework convolutions; the attention core with Nq != Nk -- the query keeps the full grid
(stride 1), keys and values are strided (2, 2) -- runs on the fused HIP kernels
(``ops.attention`` / ``ops.talking_heads_attention``), and the output projection on ``ops.dense``.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .attention import DenseGeneral, TalkingHeadsBlock, lecun_normal_

__all__ = ["ConvProjectionBlock", "CvTAttentionBlock", "CvTSelfAttentionBlock"]


class _Conv(nn.Module):
    """Flax ``nn.Conv`` param holder: kernel [kh, kw, in / groups, out] (lecun_normal), bias."""

    def __init__(self, k, cin_per_group, cout, use_bias, device=None):
        super().__init__()
        w = torch.empty(k, k, cin_per_group, cout, device=device)
        self.kernel = nn.Parameter(lecun_normal_(w, k * k * cin_per_group))
        self.bias = nn.Parameter(torch.zeros(cout, device=device)) if use_bias else None


class _BatchNorm(nn.Module):
    """Flax ``nn.BatchNorm`` (cvt_attention.py:33-36): params scale / bias, batch_stats mean / var;
    training normalises with the biased batch statistics and moves the running averages by
    ``momentum`` (Flax convention: ra = momentum * ra + (1 - momentum) * batch)."""

    def __init__(self, ch, momentum, eps, device=None):
        super().__init__()
        self.scale = nn.Parameter(torch.ones(ch, device=device))
        self.bias = nn.Parameter(torch.zeros(ch, device=device))
        self.register_buffer("mean", torch.zeros(ch, device=device))
        self.register_buffer("var", torch.ones(ch, device=device))
        self.momentum, self.eps = momentum, eps

    def forward(self, x, is_training):   # x [b, H, W, c]
        xf = x.float()
        if is_training:
            mean = xf.mean((0, 1, 2))
            var = xf.var((0, 1, 2), unbiased=False)
            with torch.no_grad():
                self.mean.mul_(self.momentum).add_((1 - self.momentum) * mean.detach())
                self.var.mul_(self.momentum).add_((1 - self.momentum) * var.detach())
        else:
            mean, var = self.mean, self.var
        y = (xf - mean) * torch.rsqrt(var + self.eps) * self.scale + self.bias
        return y.to(x.dtype)


class ConvProjectionBlock(nn.Module):
    """cvt_attention.py:12-40: depthwise conv (kernel_size, strides, SAME) -> BatchNorm -> 1x1 conv."""

    def __init__(self, in_ch, out_ch, kernel_size=3, strides=1, use_bias=True, bn_momentum=0.9,
                 bn_epsilon=1e-5, dtype=torch.float32, device=None):
        super().__init__()
        self.kernel_size, self.strides, self.dtype = kernel_size, strides, dtype
        self.Conv_0 = _Conv(kernel_size, 1, in_ch, False, device)
        self.BatchNorm_0 = _BatchNorm(in_ch, bn_momentum, bn_epsilon, device)
        self.Conv_1 = _Conv(1, in_ch, out_ch, use_bias, device)

    def forward(self, x, is_training):   # x [b, H, W, c] -> [b, H', W', out]
        dt, k, s = self.dtype, self.kernel_size, self.strides
        c = x.shape[-1]
        xc = x.to(dt)                                                   # [b, H, W, c]
        H, W = xc.shape[1:3]
        # Flax 'SAME': output ceil(n / s), total padding max((ceil(n/s) - 1) s + k - n, 0), low = total // 2
        Ho, Wo = math.ceil(H / s), math.ceil(W / s)
        ph = max((Ho - 1) * s + k - H, 0)
        pw = max((Wo - 1) * s + k - W, 0)
        xp = F.pad(xc.float(), (0, 0, pw // 2, pw - pw // 2, ph // 2, ph - ph // 2))
        # the depthwise k x k conv as k^2 strided multiply-adds in fp32 (exact fp32 products and a
        # fixed summation order; inputs and kernel cast to the compute dtype first, as Flax's Conv
        # does), output in the compute dtype
        w0 = self.Conv_0.kernel.to(dt).float()                          # [k, k, 1, c]
        y = None
        for i in range(k):
            for j in range(k):
                tap = xp[:, i:i + s * (Ho - 1) + 1:s, j:j + s * (Wo - 1) + 1:s, :] * w0[i, j, 0]
                y = tap if y is None else y + tap
        y = self.BatchNorm_0(y.to(dt), is_training)
        w1 = self.Conv_1.kernel.reshape(c, -1)                          # [c, out]
        b1 = self.Conv_1.bias
        return ops.dense(y, w1, b1, dt)


class CvTAttentionBlock(nn.Module):
    """``CvTAttentionBlock`` (cvt_attention.py:43-113)."""

    def __init__(self, num_heads: int, head_ch: Optional[int] = None, out_ch: Optional[int] = None,
                 talking_heads: bool = False, attn_dropout_rate: float = 0.0, out_dropout_rate: float = 0.0,
                 kernel_size: int = 3, strides: Tuple[int, int, int] = (1, 2, 2), use_bias: bool = False,
                 bn_momentum: float = 0.9, bn_epsilon: float = 1e-5, dtype: torch.dtype = torch.float32, *,
                 in_ch: Optional[int] = None, device=None):
        super().__init__()
        assert len(strides) == 3
        self.num_heads, self.head_ch, self.out_ch = num_heads, head_ch, out_ch
        self.talking_heads = talking_heads
        self.attn_dropout_rate, self.out_dropout_rate = attn_dropout_rate, out_dropout_rate
        self.kernel_size, self.strides, self.use_bias = kernel_size, tuple(strides), use_bias
        self.bn_momentum, self.bn_epsilon, self.dtype = bn_momentum, bn_epsilon, dtype
        self._in_ch = None
        if in_ch is not None:
            self._build(in_ch, device)

    def _build(self, in_ch, device=None):
        assert in_ch % self.num_heads == 0
        H = self.num_heads
        D = self.head_ch or int(in_ch / H)
        out = self.out_ch or in_ch
        self._in_ch, self._D, self._out = in_ch, D, out
        for i, s in enumerate(self.strides):
            setattr(self, f"ConvProjectionBlock_{i}",
                    ConvProjectionBlock(in_ch, H * D, self.kernel_size, s, self.use_bias, self.bn_momentum,
                                        self.bn_epsilon, self.dtype, device))
        if self.talking_heads:
            self.TalkingHeadsBlock_0 = TalkingHeadsBlock(H, device)
            self.TalkingHeadsBlock_1 = TalkingHeadsBlock(H, device)
        self.DenseGeneral_0 = DenseGeneral((H, D), (out,), self.use_bias, device)

    def forward(self, inputs_q, inputs_kv, is_training: bool):
        assert inputs_q.ndim == 4 and inputs_kv.ndim == 4
        in_ch = inputs_q.shape[-1]
        assert in_ch % self.num_heads == 0
        if self._in_ch is None:
            self._build(in_ch, inputs_q.device)
        if is_training and self.attn_dropout_rate > 0.0:
            raise NotImplementedError("attention-probability dropout is not fused into the HIP kernel "
                                      "(no reference config sets attn_dropout_rate)")
        H, D, dt = self.num_heads, self._D, self.dtype
        q = self.ConvProjectionBlock_0(inputs_q, is_training)
        k = self.ConvProjectionBlock_1(inputs_kv, is_training)
        v = self.ConvProjectionBlock_2(inputs_kv, is_training)
        b = q.shape[0]
        q, k, v = (t.reshape(b, -1, H, D) for t in (q, k, v))          # 'b H W (h d) -> b (H W) h d'
        scale = 1.0 / math.sqrt(D)                                      # cvt_attention.py:85
        if self.talking_heads:
            o = ops.talking_heads_attention(q, k, v, self.TalkingHeadsBlock_0.talking_heads_transform,
                                            self.TalkingHeadsBlock_1.talking_heads_transform, scale)
        else:
            o = ops.attention(q, k, v, scale)
        y = ops.dense(o.reshape(b, -1, H * D), self.DenseGeneral_0.kernel.reshape(H * D, self._out),
                      self.DenseGeneral_0.bias if self.use_bias else None, dt)
        if self.out_dropout_rate > 0.0:
            y = F.dropout(y, p=self.out_dropout_rate, training=is_training)
        return y


class CvTSelfAttentionBlock(CvTAttentionBlock):
    """``CvTSelfAttentionBlock`` (cvt_attention.py:116-120)."""

    def forward(self, inputs, is_training: bool):  # type: ignore[override]
        return super().forward(inputs, inputs, is_training=is_training)
