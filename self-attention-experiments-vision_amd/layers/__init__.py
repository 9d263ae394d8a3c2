"""Drop-in layers mirroring ``models/layers`` of the reference (attention hot path only)."""
from .attention import (AttentionBlock, ClassSelfAttentionBlock, DenseGeneral, LCSelfAttentionBlock,
                        SelfAttentionBlock, TalkingHeadsBlock, flax_params, load_flax_params)
from .botnet import BoTMHSA, RelativeLogits
from .position_embed import RotaryPositionalEmbedding

__all__ = ["AttentionBlock", "SelfAttentionBlock", "TalkingHeadsBlock", "ClassSelfAttentionBlock",
           "LCSelfAttentionBlock", "DenseGeneral", "RelativeLogits", "BoTMHSA",
           "RotaryPositionalEmbedding", "flax_params", "load_flax_params"]
