"""sae_vision_amd -- MI355X-native (gfx950) multi-head self-attention hot path of
cfoster0/self-attention-experiments-vision.

Import as ``import sae_vision_amd`` (the ``sae_vision_amd.py`` shim at the repository root maps
this hyphenated directory to that name).  Kernels live in ``libsae_attn.so`` (C ABI:
``include/sae_attn.h``); ``ops`` holds the autograd operators, ``layers`` the drop-in
modules with the reference's Flax names and signatures, ``vit`` / ``train`` the ViT/DeiT
caller and the data-parallel training step used for the img/s benchmark.
"""
from . import _lib
from ._lib import SaeError, load as load_library

__version__ = "0.1.0"
__all__ = ["SaeError", "load_library", "_lib"]
