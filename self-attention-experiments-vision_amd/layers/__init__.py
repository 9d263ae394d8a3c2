"""Drop-in layers mirroring ``models/layers`` of the reference (attention hot path only)."""
from .attention import (AttentionBlock, ClassSelfAttentionBlock, DenseGeneral, LCSelfAttentionBlock,
                        SelfAttentionBlock, TalkingHeadsBlock, flax_params, load_flax_params)
from .botnet import BoTMHSA, RelativeLogits
from .cvt import ConvProjectionBlock, CvTAttentionBlock, CvTSelfAttentionBlock
from .position_embed import RotaryPositionalEmbedding

__all__ = ["AttentionBlock", "SelfAttentionBlock", "TalkingHeadsBlock", "ClassSelfAttentionBlock",
           "LCSelfAttentionBlock", "DenseGeneral", "RelativeLogits", "BoTMHSA",
           "RotaryPositionalEmbedding", "ConvProjectionBlock", "CvTAttentionBlock", "CvTSelfAttentionBlock",
           "flax_params", "load_flax_params"]
