"""Rotary position embedding (models/layers/position_embed.py:8-45, README to-do item).

The reference's ``RotaryPositionalEmbedding`` cannot run (``self.dim`` / ``self.dtype`` are
undefined in FixedPositionalEmbedding, ``10e4**intervals/dim`` has a precedence bug and it
returns concatenated freqs instead of (sin, cos); survey D6).  This build defines it as the
GPT-J interleaved rotation the reference's helpers describe (``rotate_every_two`` :8-14,
``apply_rotary_pos_emb`` :17-20) with base 10000 and positions 0..N-1, applied by a HIP kernel.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops

__all__ = ["RotaryPositionalEmbedding"]


class RotaryPositionalEmbedding(nn.Module):
    """Rotate ``inputs`` [B, N, D] or [B, N, H, D] along the token axis (seq_dim=1)."""

    def __init__(self, base: float = 10000.0, dtype: torch.dtype = torch.float32):
        super().__init__()
        self.base, self.dtype = base, dtype

    def forward(self, inputs: torch.Tensor) -> torch.Tensor:
        x = inputs.to(self.dtype)
        if x.dim() == 3:
            return ops.rotary(x.unsqueeze(2), self.base).squeeze(2)
        return ops.rotary(x, self.base)
