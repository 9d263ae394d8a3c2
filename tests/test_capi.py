"""CPU tests of the C ABI boundary: the in-tree library loads, exports every function
include/sae_attn.h declares, agrees on the descriptor layout, and rejects bad descriptors
before touching the GPU (validation runs on the host)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sae_attn.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sae_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import sae_vision_amd
    lib = sae_vision_amd.load_library()
    names = header_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    nm = subprocess.run(["nm", "-D", "--defined-only", sae_vision_amd._lib.LIB_PATH], capture_output=True,
                        text=True).stdout
    exported = set(re.findall(r" T (sae_\w+)", nm))
    assert set(names) <= exported, set(names) - exported
    assert set(sae_vision_amd._lib.EXPORTED_SYMBOLS) == set(names)


def test_library_is_gfx950():
    """The embedded HIP fat binary carries a gfx950 code object (and no other target)."""
    import sae_vision_amd
    blob = open(sae_vision_amd._lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_abi_version_and_desc_layout():
    import sae_vision_amd
    from sae_vision_amd import _lib as L
    lib = sae_vision_amd.load_library()
    assert lib.sae_abi_version() == L.ABI_VERSION
    # sizeof(sae_attn_desc): 8 x int32 + 24 x int64 + 2 x int32 (natural alignment)
    assert ctypes.sizeof(L.SaeAttnDesc) == 8 * 4 + 24 * 8 + 2 * 4
    d = L.SaeAttnDesc()
    lib.sae_attn_desc_init(ctypes.byref(d), 2, 6, 197, 197, 64, L.SAE_DTYPE_BF16, 0.125)
    assert list(d.q_stride) == [197 * 6 * 64, 6 * 64, 64]
    assert list(d.dv_stride) == [197 * 6 * 64, 6 * 64, 64]
    assert d.scale == pytest.approx(0.125)


@pytest.mark.parametrize("field,value,msg", [
    ("head_dim", 256, "head_dim 256"),
    ("dtype", 7, "dtype 7"),
    ("seq_k", 0, ">= 1"),
    ("flags", 8, "unknown flags"),
])
def test_validation_errors(field, value, msg):
    import sae_vision_amd
    from sae_vision_amd import _lib as L
    lib = sae_vision_amd.load_library()
    d = L.SaeAttnDesc()
    lib.sae_attn_desc_init(ctypes.byref(d), 1, 1, 4, 4, 64, L.SAE_DTYPE_F32, 1.0)
    setattr(d, field, value)
    dummy = ctypes.c_void_p(16)
    rc = lib.sae_attn_fwd(None, ctypes.byref(d), dummy, dummy, dummy, None, None, dummy, None)
    assert rc in (L.SAE_EINVAL, L.SAE_EUNSUPPORTED)
    assert msg in lib.sae_last_error().decode()


def test_relpos_grid_validation():
    import sae_vision_amd
    from sae_vision_amd import _lib as L
    lib = sae_vision_amd.load_library()
    d = L.SaeAttnDesc()
    lib.sae_attn_desc_init(ctypes.byref(d), 1, 1, 49, 49, 64, L.SAE_DTYPE_F32, 1.0)
    d.flags, d.rel_h, d.rel_w = L.SAE_FLAG_RELPOS, 7, 6
    dummy = ctypes.c_void_p(16)
    rc = lib.sae_attn_fwd(None, ctypes.byref(d), dummy, dummy, dummy, dummy, dummy, dummy, None)
    assert rc == L.SAE_EINVAL and "does not match seq_k" in lib.sae_last_error().decode()


def test_talking_heads_envelope():
    import sae_vision_amd
    from sae_vision_amd import _lib as L
    lib = sae_vision_amd.load_library()
    d = L.SaeAttnDesc()
    dummy = ctypes.c_void_p(16)
    # bf16 (aligned) takes up to SAE_TH_MAX_HEADS = 16 heads (cait_m_*), the fp32 path up to 8
    lib.sae_attn_desc_init(ctypes.byref(d), 1, 17, 8, 8, 48, L.SAE_DTYPE_BF16, 1.0)
    rc = lib.sae_th_attn_fwd(None, ctypes.byref(d), dummy, dummy, dummy, dummy, dummy, dummy, dummy)
    assert rc == L.SAE_EUNSUPPORTED and "heads <= 16" in lib.sae_last_error().decode()
    lib.sae_attn_desc_init(ctypes.byref(d), 1, 12, 8, 8, 64, L.SAE_DTYPE_F32, 1.0)
    rc = lib.sae_th_attn_fwd(None, ctypes.byref(d), dummy, dummy, dummy, dummy, dummy, dummy, dummy)
    assert rc == L.SAE_EUNSUPPORTED and "12 heads > 8" in lib.sae_last_error().decode()


def test_product_path_refuses_cpu_tensors():
    """No CPU fallback: the ops raise instead of computing on the host."""
    import torch
    import sae_vision_amd.ops as ops
    q = torch.zeros(1, 4, 1, 64)
    with pytest.raises(RuntimeError, match="GPU only"):
        ops.attention(q, q, q)


def test_missing_library_fails_loudly(tmp_path):
    from sae_vision_amd import _lib as L
    old = L._lib
    try:
        L._lib = None
        with pytest.raises(ImportError, match="no CPU fallback"):
            L.load(str(tmp_path / "nope.so"))
    finally:
        L._lib = old


def test_patch_embed_validation():
    """sae_patch_desc layout and the host-side shape checks of the patch-embedding entry points."""
    import sae_vision_amd
    from sae_vision_amd import _lib as L
    lib = sae_vision_amd.load_library()
    assert ctypes.sizeof(L.SaePatchDesc) == 9 * 4
    dummy = ctypes.c_void_p(16)
    cases = [
        (L.SaePatchDesc(12, 32, 32, 3, 16, 16, 384, L.SAE_LAYOUT_HWCN, L.SAE_DTYPE_BF16), "batch % 8"),
        (L.SaePatchDesc(8, 40, 32, 3, 16, 16, 384, L.SAE_LAYOUT_NHWC, L.SAE_DTYPE_BF16), "whole number"),
        (L.SaePatchDesc(8, 30, 30, 3, 10, 10, 384, L.SAE_LAYOUT_NHWC, L.SAE_DTYPE_BF16), "% 64"),
        (L.SaePatchDesc(8, 32, 32, 3, 16, 16, 384, 5, L.SAE_DTYPE_BF16), "layout 5"),
    ]
    for d, msg in cases:
        rc = lib.sae_patch_embed_fwd(None, ctypes.byref(d), dummy, dummy, None, dummy)
        assert rc != L.SAE_OK and msg in lib.sae_last_error().decode(), (msg, lib.sae_last_error())
        assert lib.sae_patch_embed_bwd_workspace_bytes(ctypes.byref(d)) == 0
    ok = L.SaePatchDesc(128, 224, 224, 3, 16, 16, 384, L.SAE_LAYOUT_HWCN, L.SAE_DTYPE_F32)
    assert lib.sae_patch_embed_bwd_workspace_bytes(ctypes.byref(ok)) > 0


def test_adamw_cast_plan_tiles_and_refusals():
    """sae_adamw_cast_plan (host only, no GPU): 64 x 64 tiles per Dense kernel with the column
    offset / leading dimensions carried into each tile, the capacity check, and SAE_EUNSUPPORTED
    for shapes or buffers the vector tile path does not take."""
    import sae_vision_amd._lib as L
    lib = L.load()
    base = 1 << 20   # fake 16-byte-aligned device addresses: the planner only does arithmetic

    def plan(K, N, col0=0, ld16=None, off=0, cap=64):
        arr = lambda t, *v: (t * len(v))(*v)
        P, G, M, V = (arr(ctypes.c_void_p, base + 0x1000 * i + off) for i in range(4))
        W16, WT = arr(ctypes.c_void_p, base + 0x100000), arr(ctypes.c_void_p, base + 0x200000)
        tiles = (L.AdamwCastTile * cap)()
        n = ctypes.c_int64(0)
        rc = lib.sae_adamw_cast_plan(1, P, G, M, V, arr(ctypes.c_int32, K), arr(ctypes.c_int32, N), W16,
                                     arr(ctypes.c_int32, ld16 if ld16 is not None else col0 + N), WT,
                                     arr(ctypes.c_int32, K), arr(ctypes.c_int32, col0), tiles, cap, ctypes.byref(n))
        return rc, n.value, tiles

    rc, n, t = plan(68, 100, col0=36, ld16=136)
    assert rc == L.SAE_OK and n == 4
    assert sorted((x.k0, x.n0) for x in t[:4]) == [(0, 0), (0, 64), (64, 0), (64, 64)]
    assert all(x.K == 68 and x.N == 100 and x.col0 == 36 and x.ld16 == 136 and x.ldT == 68 for x in t[:4])
    rc, n, _ = plan(384, 1152, cap=10)            # 6 x 18 tiles > capacity: counted, refused
    assert rc == L.SAE_EINVAL and n == 108
    assert plan(66, 100)[0] == L.SAE_EUNSUPPORTED            # K not a multiple of 4
    assert plan(68, 100, col0=2, ld16=104)[0] == L.SAE_EUNSUPPORTED   # column offset
    assert plan(68, 100, off=8)[0] == L.SAE_EUNSUPPORTED     # fp32 buffers not 16-byte aligned
    assert plan(68, 100, col0=8, ld16=100)[0] == L.SAE_EINVAL          # ld16 < col0 + N
