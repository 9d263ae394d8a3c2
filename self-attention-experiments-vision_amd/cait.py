"""CaiT -- the talking-heads / class-attention caller of the attention hot path
(BASELINE configs[4]: CaiT-S24, talking-heads self-attention + class-attention layers + LayerScale).

Mirrors models/cait.py:10-186 (ClassSelfAttentionBlock, EncoderBlock, Encoder, CAEncoderBlock,
CaiT), models/layers/normalizations/layerscale.py:5-23 (LayerScaleBlock) and
models/layers/regularization/stochastic_depth.py:6-28 (StochasticDepthBlock), with Flax-style
submodule names so the parameter tree matches (``Encoder_0/EncoderBlock_i/LayerScaleBlock_0/
layerscale``, ``CAEncoderBlock_i/ClassSelfAttentionBlock_0/queries/kernel``, ``cls``, ...).

Numerics: fp32 params, ``dtype`` compute, fp32 residual stream.  Survey D7: the reference does
not pass ``dtype`` to the self-attention trunk (cait.py:147-154), so its trunk runs in fp32 even
for a bf16 model; this build runs the trunk in the model's ``dtype`` (the bf16 config of
BASELINE) -- ``trunk_dtype=torch.float32`` restores the reference behaviour.
Hot path: every self-attention layer runs the fused talking-heads kernels
(``ops.talking_heads_attention``), every class-attention layer the fused core with Nq = 1
(CLS query), every FF block ``ops.ff_block`` (GELU fused into the GEMM epilogues).
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn as nn

from . import ops
from .layers.attention import ClassSelfAttentionBlock, SelfAttentionBlock
from .vit import Dense, FFBlock, LayerNorm, encoder_weight_groups, patch_tokens

__all__ = ["CaiT", "create_cait", "CAIT_CONFIGS", "cait_flops_per_image", "LayerScaleBlock",
           "StochasticDepthBlock"]


class LayerScaleBlock(nn.Module):
    """layerscale.py:13-23: ``inputs * layerscale`` (param [C] filled with eps, cast to dtype)."""

    def __init__(self, dim: int, eps: float, device=None):
        super().__init__()
        self.layerscale = nn.Parameter(torch.full((dim,), float(eps), device=device))

    def forward(self, x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
        return x.to(dtype) * self.layerscale.to(dtype)


class StochasticDepthBlock(nn.Module):
    """stochastic_depth.py:6-28: per-sample drop of the residual branch while training, scaled by
    1 / keep_prob.  Identity at rate 0 or in evaluation.  (The reference's train.py passes no
    'stochastic_depth' rng, so it cannot train with rate > 0; the mask here comes from torch's
    device generator, replayable inside a HIP graph.)"""

    def __init__(self, drop_rate: float):
        super().__init__()
        self.drop_rate = float(drop_rate)

    def forward(self, x: torch.Tensor, is_training: bool) -> torch.Tensor:
        if not is_training or self.drop_rate == 0.0:
            return x
        keep = 1.0 - self.drop_rate
        shape = (x.shape[0],) + (1,) * (x.ndim - 1)
        mask = torch.floor(keep + torch.rand(shape, device=x.device, dtype=torch.float32))
        return x / keep * mask.to(x.dtype)


def scaled_branch(x: torch.Tensor, ls: LayerScaleBlock, sd: StochasticDepthBlock, dtype: torch.dtype,
                  is_training: bool) -> torch.Tensor:
    """``StochasticDepth(LayerScale(x))`` as ONE elementwise pass: x * (layerscale[c] * mask[b] /
    keep), the [B, 1, C] factor built first (same math as the two blocks applied in turn,
    layerscale.py:21-23 then stochastic_depth.py:19-28, up to the bf16 rounding of the factor)."""
    f = ls.layerscale.to(dtype)
    rs = sample_scale(x.shape[0], sd, is_training, x.device)
    if rs is not None:
        f = f[None, None, :] * rs[:, None, None].to(dtype)
    return x.to(dtype) * f


# the factors of every stochastic-depth block of one training forward, drawn together
# (CaiT.forward): one uniform draw and two elementwise passes instead of four launches per block
_SD_DRAW = None


class _SDDraw:
    def __init__(self, rows: torch.Tensor, index):
        self.rows, self.index = rows, index


def draw_stochastic_depth(sds, keep: torch.Tensor, batch: int, device) -> "_SDDraw":
    """rows[i] = floor(keep_i + U[0,1)) / keep_i for every block i of ``sds`` (keep [n, 1] on the
    device): the same per-sample factor as sample_scale, for all blocks in one draw."""
    u = torch.rand((len(sds), batch), device=device, dtype=torch.float32)
    return _SDDraw(torch.floor(keep + u) / keep, {id(sd): i for i, sd in enumerate(sds)})


def sample_scale(batch: int, sd: StochasticDepthBlock, is_training: bool, device):
    """Per-sample stochastic-depth factor floor(keep + U[0,1)) / keep (stochastic_depth.py:19-28),
    or None when the block is the identity; from the forward's joint draw when there is one."""
    if not is_training or sd.drop_rate == 0.0:
        return None
    d = _SD_DRAW
    if d is not None and id(sd) in d.index and d.rows.shape[1] == batch:
        return d.rows[d.index[id(sd)]]
    keep = 1.0 - sd.drop_rate
    return torch.floor(keep + torch.rand((batch,), device=device, dtype=torch.float32)) / keep


class EncoderBlock(nn.Module):
    """cait.py:18-60: LN -> talking-heads SelfAttention -> LayerScale -> StochDepth -> + ;
    LN -> FF -> LayerScale -> StochDepth -> +."""

    def __init__(self, dim, num_heads, stoch_depth_rate, layerscale_eps, expand_ratio, dtype, device=None):
        super().__init__()
        self.dtype = dtype
        self.LayerNorm_0 = LayerNorm(dim, device)
        self.SelfAttentionBlock_0 = SelfAttentionBlock(num_heads=num_heads, talking_heads=True, dtype=dtype,
                                                       in_ch=dim, device=device)
        self.LayerScaleBlock_0 = LayerScaleBlock(dim, layerscale_eps, device)
        self.StochasticDepthBlock_0 = StochasticDepthBlock(stoch_depth_rate)
        self.LayerNorm_1 = LayerNorm(dim, device)
        self.FFBlock_0 = FFBlock(dim, expand_ratio, device)
        self.LayerScaleBlock_1 = LayerScaleBlock(dim, layerscale_eps, device)
        self.StochasticDepthBlock_1 = StochasticDepthBlock(stoch_depth_rate)

    def _ln(self, ln, x):
        if self.dtype == torch.bfloat16 and ops.layer_norm_ok(x):
            return ops.layer_norm(x, ln.scale, ln.bias)
        return ln(x, self.dtype)

    def forward(self, inputs: torch.Tensor, is_training: bool) -> torch.Tensor:
        x = self.SelfAttentionBlock_0(self._ln(self.LayerNorm_0, inputs), is_training=is_training)
        x = scaled_branch(x, self.LayerScaleBlock_0, self.StochasticDepthBlock_0, self.dtype, is_training)
        x = x + inputs                                         # fp32 residual stream
        y = self.FFBlock_0(self._ln(self.LayerNorm_1, x), self.dtype)
        y = scaled_branch(y, self.LayerScaleBlock_1, self.StochasticDepthBlock_1, self.dtype, is_training)
        return x + y


class Encoder(nn.Module):
    """cait.py:63-91 (AddAbsPosEmbed_0 + EncoderBlock_i; no final norm)."""

    def __init__(self, num_tokens, dim, num_layers, num_heads, stoch_depth_rate, layerscale_eps, expand_ratio,
                 dtype, device=None):
        super().__init__()
        self.AddAbsPosEmbed_0 = nn.Module()
        self.AddAbsPosEmbed_0.pos_embed = nn.Parameter(torch.randn(1, num_tokens, dim, device=device) * 0.02)
        self.num_layers = num_layers
        for i in range(num_layers):
            setattr(self, f"EncoderBlock_{i}", EncoderBlock(dim, num_heads, stoch_depth_rate, layerscale_eps,
                                                            expand_ratio, dtype, device))

    def forward(self, inputs: torch.Tensor, is_training: bool) -> torch.Tensor:
        x = inputs.float() + self.AddAbsPosEmbed_0.pos_embed
        blocks = [getattr(self, f"EncoderBlock_{i}") for i in range(self.num_layers)]
        if blocks and blocks[0].dtype == torch.bfloat16 and ops.layer_norm_ok(x):
            # cait.py:30-60 per block, every residual add fused with the LayerNorm that follows it
            # (this block's LayerNorm_1, the next block's LayerNorm_0): one HBM pass each
            ops.cast_weights(encoder_weight_groups(blocks))   # every Dense kernel, one launch
            try:
                return self._fused(x, blocks, is_training)
            finally:
                ops.clear_weight_cache()
        for blk in blocks:
            x = blk(x, is_training)
        return x

    @staticmethod
    def _fused(x, blocks, is_training):
        h = ops.layer_norm(x, blocks[0].LayerNorm_0.scale, blocks[0].LayerNorm_0.bias)
        for i, blk in enumerate(blocks):
            # LayerScale x stochastic depth folded into the residual add + LayerNorm kernel
            a = blk.SelfAttentionBlock_0(h, is_training=is_training)
            rs = sample_scale(x.shape[0], blk.StochasticDepthBlock_0, is_training, x.device)
            x, h = ops.add_layer_norm_scaled(x, a, blk.LayerNorm_1.scale, blk.LayerNorm_1.bias,
                                             blk.LayerScaleBlock_0.layerscale, rs)
            f = blk.FFBlock_0(h, blk.dtype)
            if i + 1 < len(blocks):
                nxt = blocks[i + 1].LayerNorm_0
                rs = sample_scale(x.shape[0], blk.StochasticDepthBlock_1, is_training, x.device)
                x, h = ops.add_layer_norm_scaled(x, f, nxt.scale, nxt.bias, blk.LayerScaleBlock_1.layerscale, rs)
            else:
                x = x + scaled_branch(f, blk.LayerScaleBlock_1, blk.StochasticDepthBlock_1, blk.dtype, is_training)
        return x


class CAEncoderBlock(nn.Module):
    """cait.py:94-129: class attention of the CLS token over [cls, patches]."""

    def __init__(self, dim, num_heads, stoch_depth_rate, layerscale_eps, expand_ratio, dtype, device=None):
        super().__init__()
        self.dtype = dtype
        self.LayerNorm_0 = LayerNorm(dim, device)
        self.ClassSelfAttentionBlock_0 = ClassSelfAttentionBlock(num_heads=num_heads, dtype=dtype, in_ch=dim,
                                                                 device=device)
        self.LayerScaleBlock_0 = LayerScaleBlock(dim, layerscale_eps, device)
        self.StochasticDepthBlock_0 = StochasticDepthBlock(stoch_depth_rate)
        self.LayerNorm_1 = LayerNorm(dim, device)
        self.FFBlock_0 = FFBlock(dim, expand_ratio, device)
        self.LayerScaleBlock_1 = LayerScaleBlock(dim, layerscale_eps, device)
        self.StochasticDepthBlock_1 = StochasticDepthBlock(stoch_depth_rate)

    def _ln(self, ln, x):
        if self.dtype == torch.bfloat16 and ops.layer_norm_ok(x):
            return ops.layer_norm(x, ln.scale, ln.bias)
        return ln(x, self.dtype)

    def forward(self, inputs: torch.Tensor, cls_token: torch.Tensor, is_training: bool) -> torch.Tensor:
        x = torch.cat([cls_token, inputs], dim=1)
        x = self.ClassSelfAttentionBlock_0(self._ln(self.LayerNorm_0, x.contiguous()), is_training=is_training)
        x = scaled_branch(x, self.LayerScaleBlock_0, self.StochasticDepthBlock_0, self.dtype, is_training)
        cls_token = cls_token + x
        y = self.FFBlock_0(self._ln(self.LayerNorm_1, cls_token.contiguous()), self.dtype)
        y = scaled_branch(y, self.LayerScaleBlock_1, self.StochasticDepthBlock_1, self.dtype, is_training)
        return cls_token + y


class CaiT(nn.Module):
    """cait.py:132-186.  ``forward(inputs [B, H, W, 3], is_training)`` -> logits [B, classes]."""

    def __init__(self, num_classes: int, num_layers: int, num_layers_token_only: int, num_heads: int,
                 embed_dim: int, patch_shape: Tuple[int, int], stoch_depth_rate: float, layerscale_eps: float,
                 img_size: int = 224, expand_ratio: float = 4, dtype: torch.dtype = torch.float32,
                 trunk_dtype: torch.dtype = None, device=None):
        super().__init__()
        self.patch_shape, self.dtype, self.embed_dim = tuple(patch_shape), dtype, embed_dim
        ph, pw = self.patch_shape
        self.PatchEmbedBlock_0 = nn.Module()
        self.PatchEmbedBlock_0.Dense_0 = Dense(ph * pw * 3, embed_dim, use_bias=False, device=device)
        n = (img_size // ph) * (img_size // pw)   # no CLS in the trunk (cait.py:143-154)
        self.Encoder_0 = Encoder(n, embed_dim, num_layers, num_heads, stoch_depth_rate, layerscale_eps,
                                 expand_ratio, trunk_dtype or dtype, device)
        self.cls = nn.Parameter(torch.zeros(1, 1, embed_dim, device=device))
        self.num_layers_token_only = num_layers_token_only
        for i in range(num_layers_token_only):
            setattr(self, f"CAEncoderBlock_{i}", CAEncoderBlock(embed_dim, num_heads, stoch_depth_rate,
                                                                layerscale_eps, expand_ratio, dtype, device))
        self.LayerNorm_0 = LayerNorm(embed_dim, device)
        self.Dense_0 = Dense(embed_dim, num_classes, zero_init=True, device=device)

    def cast_groups(self):
        """The Dense kernels whose bf16 copies the optimizer may keep (FusedAdamW ``cast_groups``):
        the trunk's column-block groups (when the trunk computes in bf16), the patch embedding and
        the head and the class-attention blocks' projections / FF (when the model does)."""
        groups = []
        blocks = [getattr(self.Encoder_0, f"EncoderBlock_{i}") for i in range(self.Encoder_0.num_layers)]
        if blocks and blocks[0].dtype == torch.bfloat16:
            groups += encoder_weight_groups(blocks)
        if self.dtype == torch.bfloat16:
            groups += [[self.PatchEmbedBlock_0.Dense_0.kernel], [self.Dense_0.kernel]]
            for i in range(self.num_layers_token_only):
                ca = getattr(self, f"CAEncoderBlock_{i}")
                groups += ca.ClassSelfAttentionBlock_0.cross_weight_groups()
                groups += [[ca.FFBlock_0.Dense_0.kernel], [ca.FFBlock_0.Dense_1.kernel]]
        return groups or None

    def _sd_blocks(self, device):
        """The stochastic-depth blocks with a non-zero rate and their keep probabilities [n, 1] on
        the device (built once: inside a graph capture no host-to-device copy may run)."""
        c = getattr(self, "_sd_cache", None)
        if c is None or c[1].device != device:
            sds = [m for m in self.modules() if isinstance(m, StochasticDepthBlock) and m.drop_rate > 0.0]
            keep = torch.tensor([[1.0 - m.drop_rate] for m in sds], dtype=torch.float32, device=device)
            c = self._sd_cache = (sds, keep)
        return c

    def forward(self, inputs: torch.Tensor, is_training: bool, layout: str = "NHWC") -> torch.Tensor:
        """``layout`` "HWCN": ``inputs`` is the train-step feed [H, W, C, B] (train.py:80)."""
        global _SD_DRAW
        x = patch_tokens(self.PatchEmbedBlock_0, inputs, self.patch_shape, self.dtype, layout)
        b = x.shape[0]
        sds, keep = self._sd_blocks(x.device)
        prev = _SD_DRAW
        if is_training and sds:   # every block's per-sample factor in one draw
            _SD_DRAW = draw_stochastic_depth(sds, keep, b, x.device)
        try:
            x = self.Encoder_0(x, is_training)
            cls_token = self.cls.expand(b, 1, self.embed_dim).float()
            for i in range(self.num_layers_token_only):
                cls_token = getattr(self, f"CAEncoderBlock_{i}")(x, cls_token, is_training)
        finally:
            _SD_DRAW = prev
        # LayerNorm over [cls, x] then take the CLS row: LN is per token, so normalising the CLS row
        # alone is the same value (cait.py:179-183) without the 197-token pass
        cls_n = self.LayerNorm_0(cls_token[:, 0], self.dtype)
        return self.Dense_0(cls_n, self.dtype)


# name -> (num_layers, token-only layers, heads, embed_dim, stoch_depth_rate, layerscale_eps);
# create_model.py:70-150 (patch 16)
CAIT_CONFIGS = {
    "cait_xxs_24": (24, 2, 4, 192, 0.05, 1e-5),
    "cait_xxs_36": (36, 2, 4, 192, 0.1, 1e-6),
    "cait_xs_24": (24, 2, 6, 288, 0.05, 1e-5),
    "cait_xs_36": (36, 2, 6, 288, 0.1, 1e-6),
    "cait_s_24": (24, 2, 8, 384, 0.1, 1e-6),
    "cait_s_36": (36, 2, 8, 384, 0.2, 1e-6),
    "cait_s_48": (48, 2, 8, 384, 0.3, 1e-6),
}


def create_cait(model_name: str, num_classes: int = 1000, dtype: torch.dtype = torch.float32,
                img_size: int = 224, stoch_depth: bool = True, device=None) -> CaiT:
    """``create_model`` (models/create_model.py) for the CaiT family.  ``stoch_depth=False`` sets
    the drop rate to 0 (deterministic steps, e.g. for parity tests)."""
    if model_name not in CAIT_CONFIGS:
        raise ValueError(f"unknown model {model_name!r}; CaiT family: {sorted(CAIT_CONFIGS)}")
    L, Lt, Hh, C, sd, eps = CAIT_CONFIGS[model_name]
    return CaiT(num_classes=num_classes, num_layers=L, num_layers_token_only=Lt, num_heads=Hh, embed_dim=C,
                patch_shape=(16, 16), stoch_depth_rate=sd if stoch_depth else 0.0, layerscale_eps=eps,
                img_size=img_size, dtype=dtype, device=device)


def cait_flops_per_image(model_name: str, img_size: int = 224, num_classes: int = 1000) -> float:
    """Forward FLOPs per image (2 per MAC): patch GEMM; per SA layer the QKV / output projections,
    QK^T, AV, the two H x H talking-heads mixes and the MLP; per CA layer the same with one query;
    head.  Training = 3x."""
    L, Lt, Hh, C, _, _ = CAIT_CONFIGS[model_name]
    n = (img_size // 16) ** 2
    sa = 2 * n * C * 3 * C + 2 * n * n * C * 2 + 2 * 2 * Hh * Hh * n * n + 2 * n * C * C + 2 * n * C * 4 * C * 2
    nk = n + 1
    ca = 2 * C * C + 2 * nk * C * 2 * C + 2 * nk * C * 2 + 2 * C * C + 2 * C * 4 * C * 2
    return float(2 * n * 16 * 16 * 3 * C + L * sa + Lt * ca + 2 * C * num_classes)
