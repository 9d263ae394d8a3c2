"""ctypes binding of the C ABI in ``include/sae_attn.h`` (``libsae_attn.so``).

This is the same binding a maintainer would add on the reference side:
plain pointers, sizes and the HIP stream handle cross the boundary, nothing else.  The
library is built in-tree by ``build.py`` / ``__graft_entry__.build()``; if it is missing
the import fails loudly -- there is no CPU or eager fallback on the product path.
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

import torch  # noqa: F401  (loads torch's libamdhip64.so.7 first so the library binds to the same HIP runtime)

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# SAE_ATTN_LIB points the tools at the development build (build.py --dev); default: release
LIB_PATH = os.environ.get("SAE_ATTN_LIB") or os.path.join(_PKG_DIR, "libsae_attn.so")

SAE_OK, SAE_EINVAL, SAE_EUNSUPPORTED, SAE_EHIP = 0, -1, -2, -3
SAE_DTYPE_F32, SAE_DTYPE_BF16 = 0, 1
SAE_FLAG_RELPOS = 1
SAE_TH_MAX_HEADS = 16
SAE_TH_MAX_HEAD_DIM = 64
ABI_VERSION = 1

_i32, _i64, _f32, _vp, _sz = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t
_S3 = _i64 * 3


SAE_LAYOUT_NHWC, SAE_LAYOUT_HWCN = 0, 1


class SaePatchDesc(ctypes.Structure):
    """Mirror of ``sae_patch_desc`` (include/sae_attn.h)."""
    _fields_ = [("batch", _i32), ("height", _i32), ("width", _i32), ("channels", _i32),
                ("patch_h", _i32), ("patch_w", _i32), ("embed", _i32), ("layout", _i32), ("dtype", _i32)]


class SaeAttnDesc(ctypes.Structure):
    """Mirror of ``sae_attn_desc`` (include/sae_attn.h)."""
    _fields_ = [
        ("batch", _i32), ("heads", _i32), ("seq_q", _i32), ("seq_k", _i32), ("head_dim", _i32),
        ("dtype", _i32), ("flags", _i32), ("scale", _f32),
        ("q_stride", _S3), ("k_stride", _S3), ("v_stride", _S3), ("o_stride", _S3),
        ("do_stride", _S3), ("dq_stride", _S3), ("dk_stride", _S3), ("dv_stride", _S3),
        ("rel_h", _i32), ("rel_w", _i32),
    ]


# (name, restype, argtypes) for every entry point declared in include/sae_attn.h
_PROTOS = [
    ("sae_attn_desc_init", None, [ctypes.POINTER(SaeAttnDesc), _i32, _i32, _i32, _i32, _i32, _i32, _f32]),
    ("sae_attn_fwd", _i32, [_vp, ctypes.POINTER(SaeAttnDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("sae_attn_bwd_workspace_bytes", _sz, [ctypes.POINTER(SaeAttnDesc)]),
    ("sae_attn_bwd", _i32, [_vp, ctypes.POINTER(SaeAttnDesc)] + [_vp] * 14),
    ("sae_relpos_bias_fwd", _i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _S3, _vp, _vp, _vp, _vp]),
    ("sae_relpos_bias_bwd_workspace_bytes", _sz, [_i32, _i32, _i32, _i32]),
    ("sae_relpos_bias_bwd", _i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _S3, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _S3, _vp, _vp, _vp]),
    ("sae_rotary", _i32, [_vp, _i32, _i32, _i32, _i32, _i32, _vp, _S3, _vp, _S3, _vp, _vp, _i32]),
    ("sae_th_attn_fwd", _i32, [_vp, ctypes.POINTER(SaeAttnDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("sae_th_attn_bwd_workspace_bytes", _sz, [ctypes.POINTER(SaeAttnDesc)]),
    ("sae_th_attn_bwd", _i32, [_vp, ctypes.POINTER(SaeAttnDesc)] + [_vp] * 13),
    ("sae_attn_fwd_rotary", _i32, [_vp, ctypes.POINTER(SaeAttnDesc)] + [_vp] * 7),
    ("sae_attn_bwd_rotary", _i32, [_vp, ctypes.POINTER(SaeAttnDesc)] + [_vp] * 12),
    ("sae_th_attn_fwd_rotary", _i32, [_vp, ctypes.POINTER(SaeAttnDesc)] + [_vp] * 9),
    ("sae_th_attn_bwd_rotary", _i32, [_vp, ctypes.POINTER(SaeAttnDesc)] + [_vp] * 15),
    ("sae_gemm_dw_workspace_bytes", _sz, [_i32, _i32, _i32]),
    ("sae_gemm_dw", _i32, [_vp, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _i64, _vp, _i32, _vp]),
    ("sae_gemm_dw_blocked", _i32, [_vp, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _vp, _i32, _vp]),
    ("sae_gemm_f32_workspace_bytes", _sz, [_i32, _i32, _i32]),
    ("sae_gemm_f32", _i32, [_vp, _i32, _i32, _i32, _vp, _i64, _i64, _vp, _i64, _i64, _vp, _vp, _i64, _vp, _i32, _vp]),
    ("sae_gemm_nt", _i32, [_vp, _i32, _i32, _i32, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _i32, _vp, _i64, _vp]),
    ("sae_gemm_nt_route", _i32, [_i32, _i32, _i32, _i32]),
    ("sae_patch_embed_fwd", _i32, [_vp, ctypes.POINTER(SaePatchDesc), _vp, _vp, _vp, _vp]),
    ("sae_patch_embed_bwd_workspace_bytes", _sz, [ctypes.POINTER(SaePatchDesc)]),
    ("sae_patch_embed_bwd", _i32, [_vp, ctypes.POINTER(SaePatchDesc), _vp, _vp, _vp, _vp, _i32, _vp]),
    ("sae_patch_gather", _i32, [_vp, ctypes.POINTER(SaePatchDesc), _vp, _vp]),
    ("sae_weight_cast", _i32, [_vp, _i32, _i32, _vp, _vp, _vp]),
    ("sae_weight_cast_multi", _i32, [_vp, _i32, _vp]),
    ("sae_layernorm_fwd", _i32, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32]),
    ("sae_layernorm_bwd_workspace_bytes", _sz, [_i32, _i32]),
    ("sae_layernorm_bwd", _i32, [_vp, _i32, _i32] + [_vp] * 11),
    ("sae_layernorm_fwd_scaled", _i32, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _vp,
                                        _i32]),
    ("sae_layernorm_bwd_scaled", _i32, [_vp, _i32, _i32] + [_vp] * 14 + [_i32, _vp]),
    ("sae_adamw_plan", _i32, [_i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    ("sae_adamw_step", _i32, [_vp, _i64, _vp, _vp, _f32, _f32, _f32, _f32, _f32]),
    ("sae_adamw_cast_plan", _i32, [_i32] + [_vp] * 11 + [_vp, _i64, _vp]),
    ("sae_adamw_step_cast", _i32, [_vp, _i64, _vp, _i64, _vp, _vp, _f32, _f32, _f32, _f32, _f32]),
    ("sae_tokens_fwd", _i32, [_vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    ("sae_tokens_bwd", _i32, [_vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    ("sae_smoothed_ce_fwd", _i32, [_vp, _i32, _i32, _vp, _i64, _i32, _vp, _f32, _vp, _vp, _vp]),
    ("sae_smoothed_ce_bwd", _i32, [_vp, _i32, _i32, _vp, _i64, _i32, _vp, _f32, _vp, _vp, _vp, _i64]),
    ("sae_occupy_cus", _i32, [_vp, _i32, _i32, _i32, _f32]),
    ("sae_flag_bump", _i32, [_vp, _vp, _i32]),
    ("sae_stream_wait_flag", _i32, [_vp, _vp, ctypes.c_uint32]),
    ("sae_last_error", ctypes.c_char_p, []),
    ("sae_abi_version", _i32, []),
    ("sae_build_info", ctypes.c_char_p, []),
]
EXPORTED_SYMBOLS = [p[0] for p in _PROTOS]

_lib = None


class WeightCastItem(ctypes.Structure):
    """Mirror of ``sae_weight_cast_item`` (include/sae_attn.h)."""
    _fields_ = [("w", ctypes.c_void_p), ("w16", ctypes.c_void_p), ("wt16", ctypes.c_void_p),
                ("K", ctypes.c_int32), ("N", ctypes.c_int32), ("ld16", ctypes.c_int32), ("ldT", ctypes.c_int32),
                ("col0", ctypes.c_int32)]


class AdamwChunk(ctypes.Structure):
    """Mirror of ``sae_adamw_chunk`` (include/sae_attn.h)."""
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("n", ctypes.c_int32), ("vec", ctypes.c_int32)]


class AdamwCastTile(ctypes.Structure):
    """Mirror of ``sae_adamw_cast_tile`` (include/sae_attn.h)."""
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("m", ctypes.c_void_p), ("v", ctypes.c_void_p),
                ("w16", ctypes.c_void_p), ("wt16", ctypes.c_void_p)] + \
        [(f, ctypes.c_int32) for f in ("K", "N", "ld16", "ldT", "col0", "k0", "n0", "pad")]


SAE_ADAMW_CHUNK = 2048


class SaeError(RuntimeError):
    """A non-zero status from the C ABI (message from ``sae_last_error``)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"sae_attn error {code}: {msg}")
        self.code = code


def load(path: str = LIB_PATH):
    """Load (once) and return the ctypes library.  Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"HIP library {path} not found: build it with `python build.py` (or "
            "__graft_entry__.build()); sae_vision_amd has no CPU fallback")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, res, args in _PROTOS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.sae_abi_version() != ABI_VERSION:
        raise ImportError(f"{path}: ABI version {lib.sae_abi_version()} != {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc: int):
    if rc != SAE_OK:
        raise SaeError(rc, load().sae_last_error().decode())


def s3(strides: Sequence[int]):
    return _S3(*[int(x) for x in strides])
