"""BoTNet relative-position attention (models/botnet.py:70-199), MI355X path.

``RelativeLogits(head_ch)`` keeps the reference's params (``rel_pos_emb_w [2W-1, d]``,
``rel_pos_emb_h [2H-1, d]``, normal(stddev = d^-1/2)) and call signature
(query [b, h, H, W, d] -> logits [b, h, H, W, H, W]).  ``BoTMHSA`` is the intended MHSA with
the survey §9 decisions applied (D1 head_ch, D3 softmax over all H*W keys, D4 V indexed by key
position); its relative logits never materialise: the attention kernel adds
``bias_h[q, k // W] + bias_w[q, k % W]`` to the score tile (``ops.relpos_bias``).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops

__all__ = ["RelativeLogits", "BoTMHSA"]


class RelativeLogits(nn.Module):
    """``RelativeLogits`` (botnet.py:70-141).  Parameters are created on the first call
    (their shape depends on the feature map, as in Flax)."""

    def __init__(self, head_ch: int):
        super().__init__()
        self.head_ch = head_ch
        self.rel_pos_emb_w = None
        self.rel_pos_emb_h = None

    def _build(self, Hs: int, Ws: int, device):
        std = self.head_ch ** -0.5
        self.rel_pos_emb_w = nn.Parameter(torch.randn(2 * Ws - 1, self.head_ch, device=device) * std)
        self.rel_pos_emb_h = nn.Parameter(torch.randn(2 * Hs - 1, self.head_ch, device=device) * std)

    def tables(self, qhat_tokens: torch.Tensor, grid):
        """Fused form: qhat [B, Hs*Ws, h, d] -> (bias_h, bias_w, grid) for ``ops.attention``."""
        Hs, Ws = grid
        if self.rel_pos_emb_h is None:
            self._build(Hs, Ws, qhat_tokens.device)
        bh, bw = ops.relpos_bias(qhat_tokens, self.rel_pos_emb_h, self.rel_pos_emb_w, (Hs, Ws))
        return bh, bw, (Hs, Ws)

    def forward(self, query: torch.Tensor) -> torch.Tensor:
        """Reference signature: query [b, h, H, W, d] -> [b, h, H, W, H, W] (materialised;
        the fused BoTMHSA path uses :meth:`tables` instead)."""
        b, h, Hs, Ws, d = query.shape
        q_tok = query.permute(0, 2, 3, 1, 4).reshape(b, Hs * Ws, h, d)
        bh, bw, _ = self.tables(q_tok, (Hs, Ws))
        kx = torch.arange(Hs * Ws, device=query.device) // Ws
        ky = torch.arange(Hs * Ws, device=query.device) % Ws
        full = bh[..., kx] + bw[..., ky]                      # [b, h, N, N]
        return full.reshape(b, h, Hs, Ws, Hs, Ws)


class BoTMHSA(nn.Module):
    """``BoTMHSA(num_heads, head_ch, dtype)`` (botnet.py:144-199): 1x1-conv Q/K/V (``query``,
    ``key``, ``value`` kernels [1, 1, Cin, h*d], he_uniform, no bias), relative logits,
    softmax over all positions, output [b, H, W, h*d] (no output projection)."""

    def __init__(self, num_heads: int, head_ch: int, dtype: torch.dtype = torch.float32, *, in_ch=None,
                 device=None):
        super().__init__()
        self.num_heads, self.head_ch, self.dtype = num_heads, head_ch, dtype
        self.RelativeLogits_0 = RelativeLogits(head_ch)
        self._in_ch = None
        if in_ch is not None:
            self._build(in_ch, device)

    def _build(self, in_ch, device):
        f = self.num_heads * self.head_ch
        bound = math.sqrt(6.0 / in_ch)          # he_uniform: fan_in = 1*1*Cin

        def mk():   # Flax nn.Conv(kernel_size=(1, 1), use_bias=False): param 'kernel' [1, 1, Cin, h*d]
            m = nn.Module()
            m.kernel = nn.Parameter(torch.empty(1, 1, in_ch, f, device=device).uniform_(-bound, bound))
            return m
        self.query, self.key, self.value = mk(), mk(), mk()
        self._in_ch = in_ch

    def forward(self, inputs: torch.Tensor) -> torch.Tensor:
        b, Hs, Ws, cin = inputs.shape
        if self._in_ch is None:
            self._build(cin, inputs.device)
        h, d, dt = self.num_heads, self.head_ch, self.dtype
        x = inputs.to(dt).reshape(b, Hs * Ws, cin)
        w = [m.kernel.reshape(cin, h * d) for m in (self.query, self.key, self.value)]
        qkv = ops.dense(x, w, None, dt).view(b, Hs * Ws, 3, h, d)   # the three 1x1 convs as one GEMM
        qhat = qkv[:, :, 0] / math.sqrt(d)                  # botnet.py:185 (head_ch, D1)
        bias = self.RelativeLogits_0.tables(qhat, (Hs, Ws))
        o = ops.attention(qhat, qkv[:, :, 1], qkv[:, :, 2], scale=1.0, bias=bias)
        return o.reshape(b, Hs, Ws, h * d)
