"""ViT / DeiT -- the caller of the attention hot path used for the end-to-end img/s metric.

Mirrors models/vit.py:9-99 (EncoderBlock, Encoder, ViT), models/layers/stems/patch_embed.py:8-26
(PatchEmbedBlock), models/layers/feedforwards/ff.py:8-34 (FFBlock) and
models/layers/position_embed.py:48-57 (AddAbsPosEmbed), with Flax-style submodule names so
the parameter tree matches (``PatchEmbedBlock_0/Dense_0/kernel``, ``cls``,
``Encoder_0/EncoderBlock_i/SelfAttentionBlock_0/queries/kernel``, ...).  Numerics follow the
reference's mixed precision: fp32 params, ``dtype`` compute, fp32 residual stream (the fp32
cls / pos-embed params promote it, vit.py:46,85), LayerNorm eps 1e-6, tanh-GELU (Flax
``nn.gelu`` default).

The attention is ``layers.SelfAttentionBlock`` (fused HIP kernels).  Around it (survey §8f
"next"): Dense / DenseGeneral go through ``ops.dense`` (library GEMM forward and input gradient,
HIP split-token weight/bias gradients), and with a bf16 compute dtype every residual add is fused
with the LayerNorm that follows it (``ops.add_layer_norm``, HIP) and the FF block runs as
``ops.ff_block`` (HIP GEMMs with the tanh-GELU and its derivative fused into their epilogues).
"""
from __future__ import annotations

import math
from typing import Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .layers.attention import DenseGeneral, SelfAttentionBlock, lecun_normal_

__all__ = ["ViT", "create_model", "MODEL_CONFIGS", "vit_flops_per_image"]


class Dense(nn.Module):
    """Flax ``nn.Dense`` param holder (kernel [in, out] lecun_normal, bias zeros)."""

    def __init__(self, in_features, features, use_bias=True, zero_init=False, device=None):
        super().__init__()
        k = torch.zeros(in_features, features, device=device)
        if not zero_init:
            lecun_normal_(k, in_features)
        self.kernel = nn.Parameter(k)
        self.bias = nn.Parameter(torch.zeros(features, device=device)) if use_bias else None

    def forward(self, x, dtype):
        return ops.dense(x, self.kernel, self.bias, dtype)


class LayerNorm(nn.Module):
    """Flax ``nn.LayerNorm(dtype)``: params ``scale`` / ``bias``, eps 1e-6, output in dtype."""

    def __init__(self, dim, device=None):
        super().__init__()
        self.scale = nn.Parameter(torch.ones(dim, device=device))
        self.bias = nn.Parameter(torch.zeros(dim, device=device))

    def forward(self, x, dtype):
        return F.layer_norm(x.float(), (x.shape[-1],), self.scale, self.bias, 1e-6).to(dtype)


class FFBlock(nn.Module):
    """ff.py:8-34 (expand_ratio, Dense -> GELU -> Dense, dropout 0)."""

    def __init__(self, dim, expand_ratio=4, device=None):
        super().__init__()
        hid = max(1, int(expand_ratio * dim))
        self.Dense_0 = Dense(dim, hid, device=device)
        self.Dense_1 = Dense(hid, dim, device=device)

    def forward(self, x, dtype):
        d0, d1 = self.Dense_0, self.Dense_1
        if dtype == torch.bfloat16 and ops.ff_block_ok(x, d0.kernel, d1.kernel):
            # GELU fused into Dense_0's GEMM epilogue, its derivative into Dense_1's dX GEMM
            return ops.ff_block(x, d0.kernel, d0.bias, d1.kernel, d1.bias)
        return d1(F.gelu(d0(x, dtype), approximate="tanh"), dtype)


class EncoderBlock(nn.Module):
    """vit.py:9-32."""

    def __init__(self, dim, num_heads, expand_ratio, dtype, device=None):
        super().__init__()
        self.dtype = dtype
        self.LayerNorm_0 = LayerNorm(dim, device)
        self.SelfAttentionBlock_0 = SelfAttentionBlock(num_heads=num_heads, dtype=dtype, in_ch=dim, device=device)
        self.LayerNorm_1 = LayerNorm(dim, device)
        self.FFBlock_0 = FFBlock(dim, expand_ratio, device)

    def forward(self, inputs, is_training):
        x = self.SelfAttentionBlock_0(self.LayerNorm_0(inputs, self.dtype), is_training=is_training)
        x = x + inputs
        y = self.FFBlock_0(self.LayerNorm_1(x, self.dtype), self.dtype)
        return x + y


def encoder_weight_groups(blocks):
    """Column-block groups of every Dense kernel of the blocks (attention QKV / output projection,
    FF Dense_0 / Dense_1) for ``ops.cast_weights``."""
    groups = []
    for blk in blocks:
        groups += blk.SelfAttentionBlock_0.weight_groups()
        groups += [[blk.FFBlock_0.Dense_0.kernel], [blk.FFBlock_0.Dense_1.kernel]]
    return groups


class Encoder(nn.Module):
    """vit.py:35-58 (AddAbsPosEmbed_0 + EncoderBlock_i + LayerNorm_0)."""

    def __init__(self, num_tokens, dim, num_layers, num_heads, expand_ratio, dtype, device=None):
        super().__init__()
        self.dtype = dtype
        self.AddAbsPosEmbed_0 = nn.Module()
        self.AddAbsPosEmbed_0.pos_embed = nn.Parameter(torch.randn(1, num_tokens, dim, device=device) * 0.02)
        for i in range(num_layers):
            setattr(self, f"EncoderBlock_{i}", EncoderBlock(dim, num_heads, expand_ratio, dtype, device))
        self.num_layers = num_layers
        self.LayerNorm_0 = LayerNorm(dim, device)

    def forward(self, inputs, is_training, pos_added: bool = False, cls_only: bool = False):
        """``pos_added``: ``inputs`` already hold the position embedding (ops.encoder_tokens).
        ``cls_only``: return only token 0 of the normalised output, [B, E] (what ViT's head reads,
        vit.py:95): the final residual add and LayerNorm (row-wise) then run on those rows only."""
        x = inputs if pos_added else inputs.float() + self.AddAbsPosEmbed_0.pos_embed
        blocks = [getattr(self, f"EncoderBlock_{i}") for i in range(self.num_layers)]
        if self.dtype == torch.bfloat16 and blocks and ops.layer_norm_ok(x):
            # Same math as vit.py:19-31,57, with every residual add fused into the LayerNorm that
            # follows it (the next block's LayerNorm_0, or the final one): one HBM pass each; every
            # Dense kernel of the encoder cast to bf16 in one launch up front.
            ops.cast_weights(encoder_weight_groups(blocks))
            try:
                # (x, h): the residual gradient is added inside the LayerNorm backward kernel
                x, h = ops.layer_norm_pass(x, blocks[0].LayerNorm_0.scale, blocks[0].LayerNorm_0.bias)
                for i, blk in enumerate(blocks):
                    a = blk.SelfAttentionBlock_0(h, is_training=is_training)
                    x, h = ops.add_layer_norm(x, a, blk.LayerNorm_1.scale, blk.LayerNorm_1.bias)
                    f = blk.FFBlock_0(h, self.dtype)
                    if i + 1 < len(blocks):
                        nxt = blocks[i + 1].LayerNorm_0
                        x, h = ops.add_layer_norm(x, f, nxt.scale, nxt.bias)
                    elif cls_only:
                        h = ops.cls_add_layer_norm(x, f, self.LayerNorm_0.scale, self.LayerNorm_0.bias)
                    else:
                        x, h = ops.add_layer_norm(x, f, self.LayerNorm_0.scale, self.LayerNorm_0.bias)
            finally:
                ops.clear_weight_cache()
            return h
        for blk in blocks:
            x = blk(x, is_training)
        y = self.LayerNorm_0(x, self.dtype)
        return y[:, 0] if cls_only else y


def patch_tokens(pe: nn.Module, inputs: torch.Tensor, patch_shape: Tuple[int, int], dtype: torch.dtype,
                 layout: str = "NHWC") -> torch.Tensor:
    """``PatchEmbedBlock_0`` (patch_embed.py:15-26) of ``inputs`` in the model call layout
    "NHWC" [B, H, W, C] or the train-step feed "HWCN" [H, W, C, B] (train.py:80): in bf16 one
    fused patch-gather GEMM (``ops.patch_embed``); otherwise (fp32 compute, shapes the kernel
    does not take) the einops rearrange and a Dense."""
    w = pe.Dense_0.kernel
    if dtype == torch.bfloat16 and ops.patch_embed_ok(inputs, w, patch_shape, layout):
        return ops.patch_embed(inputs, w, pe.Dense_0.bias, patch_shape, layout)
    if layout == "HWCN":
        inputs = inputs.permute(3, 0, 1, 2)                        # 'H W C N -> N H W C'
    b, H, W, c = inputs.shape
    ph, pw = patch_shape
    x = inputs.to(dtype).reshape(b, H // ph, ph, W // pw, pw, c).permute(0, 1, 3, 2, 4, 5)
    x = x.reshape(b, (H // ph) * (W // pw), ph * pw * c)          # 'b (h ph) (w pw) c -> b (h w) (ph pw c)'
    return pe.Dense_0(x, dtype)


class ViT(nn.Module):
    """vit.py:61-99.  ``forward(inputs [B, H, W, 3], is_training)`` -> logits [B, classes]."""

    def __init__(self, num_classes: int, num_layers: int, num_heads: int, embed_dim: int,
                 patch_shape: Tuple[int, int], img_size: int = 224, expand_ratio: float = 4,
                 dtype: torch.dtype = torch.float32, device=None):
        super().__init__()
        assert embed_dim % num_heads == 0
        self.patch_shape, self.dtype, self.embed_dim = tuple(patch_shape), dtype, embed_dim
        ph, pw = self.patch_shape
        self.PatchEmbedBlock_0 = nn.Module()
        self.PatchEmbedBlock_0.Dense_0 = Dense(ph * pw * 3, embed_dim, use_bias=False, device=device)
        self.cls = nn.Parameter(torch.zeros(1, 1, embed_dim, device=device))
        n = (img_size // ph) * (img_size // pw) + 1
        self.Encoder_0 = Encoder(n, embed_dim, num_layers, num_heads, expand_ratio, dtype, device)
        self.Dense_0 = Dense(embed_dim, num_classes, zero_init=True, device=device)

    def cast_groups(self):
        """Every Dense kernel the bf16 forward reads as a bf16 copy (the encoder's column-block
        groups, the patch embedding, the head): the optimizer may keep these copies
        (FusedAdamW ``cast_groups``).  None when the model computes in fp32."""
        if self.dtype != torch.bfloat16:
            return None
        blocks = [getattr(self.Encoder_0, f"EncoderBlock_{i}") for i in range(self.Encoder_0.num_layers)]
        return (encoder_weight_groups(blocks) + [[self.PatchEmbedBlock_0.Dense_0.kernel]] +
                [[self.Dense_0.kernel]])

    def forward(self, inputs: torch.Tensor, is_training: bool, layout: str = "NHWC") -> torch.Tensor:
        """``layout`` "HWCN": ``inputs`` is the train-step feed [H, W, C, B] (train.py:80)."""
        x = patch_tokens(self.PatchEmbedBlock_0, inputs, self.patch_shape, self.dtype, layout)
        b = x.shape[0]
        pos = self.Encoder_0.AddAbsPosEmbed_0.pos_embed
        if self.dtype == torch.bfloat16 and ops.encoder_tokens_ok(x, self.cls, pos):
            # concat(cls, tokens) + pos_embed into the fp32 residual stream in one pass
            x = self.Encoder_0(ops.encoder_tokens(x, self.cls, pos), is_training, pos_added=True, cls_only=True)
        else:
            x = torch.cat([self.cls.expand(b, 1, self.embed_dim), x.float()], dim=1)   # fp32 (promotion)
            x = self.Encoder_0(x, is_training, cls_only=True)
        return self.Dense_0(x, self.dtype)   # the class token (vit.py:95-98)


# name -> (layers, heads, embed_dim, patch); create_model.py:10-37 plus the DeiT entries (survey D10)
MODEL_CONFIGS = {
    "vit_b_patch32": (12, 12, 768, 32),
    "vit_b_patch16": (12, 12, 768, 16),
    "vit_l_patch32": (24, 16, 1024, 32),
    "vit_l_patch16": (24, 16, 1024, 16),
    "deit_ti_patch16": (12, 3, 192, 16),
    "deit_s_patch16": (12, 6, 384, 16),
}


def create_model(model_name: str, num_classes: int = 1000, dtype: torch.dtype = torch.float32,
                 img_size: int = 224, device=None) -> ViT:
    """``create_model`` (models/create_model.py:6-215) for the ViT/DeiT family."""
    if model_name not in MODEL_CONFIGS:
        raise ValueError(f"unknown model {model_name!r}; ViT/DeiT family: {sorted(MODEL_CONFIGS)}")
    L, Hh, C, p = MODEL_CONFIGS[model_name]
    return ViT(num_classes=num_classes, num_layers=L, num_heads=Hh, embed_dim=C, patch_shape=(p, p),
               img_size=img_size, dtype=dtype, device=device)


def vit_flops_per_image(model_name: str, img_size: int = 224, num_classes: int = 1000) -> float:
    """Forward FLOPs per image (2 per MAC): patch GEMM + per layer 4 projections, QK^T, AV and
    the MLP + head.  Training = 3x."""
    L, Hh, C, p = MODEL_CONFIGS[model_name]
    n = (img_size // p) ** 2 + 1
    per_layer = 2 * n * C * 3 * C + 2 * n * n * C * 2 + 2 * n * C * C + 2 * n * C * 4 * C * 2
    return float(2 * (n - 1) * p * p * 3 * C + L * per_layer + 2 * C * num_classes)
