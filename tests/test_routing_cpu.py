"""Projection routing (CPU: the routing predicates only, no device needed).

Every forward and input-gradient GEMM of every attention encoder width in the reference's model
registry (models/create_model.py:6-215 -- ViT-B/L, CaiT XXS..M, CeiT, CvT, TNT inner / outer;
plus DeiT-Ti/S of SURVEY D10) must run on this repo's ``sae_gemm_nt``: ``ops.use_gemm_nt`` sends
it there, and ``sae_gemm_nt_route`` (the C ABI's kernel choice, include/sae_attn.h) must name a
HIP kernel for it.  The projections are attention.py:29-37,60-63 and the FF block ff.py:8-34.
The rocprofv3 step profiles confirm on the GPU that no library GEMM runs (profiles/)."""
import pytest

import sae_vision_amd.ops as ops
from sae_vision_amd import _lib as L

NONE, TILE128, KTAIL, GEMM8, GEMM8X = 0, 1, 2, 3, 4

# (model, embed width C, FF hidden) -- create_model.py line cited per entry
WIDTHS = [
    ("vit_b (create_model.py:10-23)", 768, 3072),
    ("vit_l (create_model.py:24-37)", 1024, 4096),
    ("tnt_s outer (create_model.py:50-56)", 640, 2560),
    ("tnt_s inner (create_model.py:50-56)", 40, 160),
    ("tnt_b outer (create_model.py:57-63)", 384, 1536),
    ("tnt_b inner (create_model.py:57-63)", 24, 96),
    ("ceit_t (create_model.py:64-68)", 192, 768),
    ("ceit_s (create_model.py:69-73)", 384, 1536),
    ("ceit_b (create_model.py:74-78)", 768, 3072),
    ("cait_xxs (create_model.py:79-96)", 192, 768),
    ("cait_xs (create_model.py:97-114)", 288, 1152),
    ("cait_s (create_model.py:115-141)", 384, 1536),
    ("cait_m (create_model.py:142-168)", 768, 3072),
    ("cvt stage 1 (create_model.py:169-183)", 64, 256),
    ("cvt stage 2 (create_model.py:169-183)", 192, 768),
    ("cvt-13/21 stage 3 (create_model.py:169-178)", 368, 1472),
    ("cvt-w24 stage 3 (create_model.py:179-183)", 1024, 4096),
    ("deit_ti (SURVEY D10)", 192, 768),
    ("deit_s (SURVEY D10)", 384, 1536),
]


def _shapes(C, hidden):
    # (K, N, epilogue) of every forward / input-gradient GEMM of one encoder block
    return {
        "qkv_fwd": (C, 3 * C, 0), "qkv_dx": (3 * C, C, 0),
        "oproj_fwd": (C, C, 0), "oproj_dx": (C, C, 0),
        "ff0_fwd_gelu": (C, hidden, 1), "ff0_dx": (hidden, C, 0),
        "ff1_fwd": (hidden, C, 0), "ff1_dx_dgelu": (C, hidden, 2),
    }


@pytest.fixture(scope="module")
def lib():
    return L.load()


@pytest.mark.parametrize("name,C,hidden", WIDTHS)
def test_every_width_routes_to_hip(lib, name, C, hidden):
    for M in (128, 197 * 32, 197 * 128):   # a classifier-head-sized call and two batch sizes
        for what, (K, N, epi) in _shapes(C, hidden).items():
            assert ops.use_gemm_nt(K, N), f"{name} {what} (K={K}, N={N}) would run on the library GEMM"
            r = lib.sae_gemm_nt_route(M, N, K, epi)
            assert r != NONE, f"{name} {what} (M={M}, K={K}, N={N}) has no HIP kernel"
            assert (r == KTAIL) == (K % 64 != 0), (name, what, r)


def test_baseline_shapes_take_the_persistent_kernels(lib):
    """The DeiT-S, ViT-B@384 and CaiT-S24 training shapes keep the round-4 kernel choice."""
    M_s, M_b = 128 * 197, 32 * 577
    for what, (K, N, epi) in _shapes(384, 1536).items():
        assert lib.sae_gemm_nt_route(M_s, N, K, epi) == GEMM8, what
    expect_b = {"qkv_fwd": GEMM8, "ff0_fwd_gelu": GEMM8, "ff1_dx_dgelu": TILE128,
                "qkv_dx": GEMM8X, "oproj_fwd": GEMM8X, "oproj_dx": GEMM8X, "ff0_dx": GEMM8X, "ff1_fwd": GEMM8X}
    for what, (K, N, epi) in _shapes(768, 3072).items():
        assert lib.sae_gemm_nt_route(M_b, N, K, epi) == expect_b[what], what
    # ViT-L: the 1024 / 4096-feature outputs at K >= 768 fill 256-wide tiles
    for K, N in ((1024, 1024), (4096, 1024), (3072, 1024), (1024, 4096)):
        assert lib.sae_gemm_nt_route(M_b, N, K, 0) == GEMM8X, (K, N)
    assert lib.sae_gemm_nt_route(M_b, 3072, 1024, 0) == GEMM8   # ViT-L QKV forward
    # small M (classifier head) and shallow K stay on the 128-row kernel
    assert lib.sae_gemm_nt_route(128, 1000, 384, 0) == TILE128
    assert lib.sae_gemm_nt_route(128, 384, 1000, 0) == KTAIL
    assert lib.sae_gemm_nt_route(M_s, 576, 192, 0) == TILE128


def test_unsupported_shapes(lib):
    assert lib.sae_gemm_nt_route(1024, 1000, 12, 0) == NONE
    assert lib.sae_gemm_nt_route(1024, 10, 384, 0) == NONE
    assert lib.sae_gemm_nt_route(0, 64, 64, 0) == NONE
    assert not ops.use_gemm_nt(12, 64) and not ops.use_gemm_nt(64, 10)


def test_library_switch():
    """ops.GEMM_LIB = True (A/B runs only) hands the projections to the library GEMM."""
    old = ops.GEMM_LIB
    try:
        ops.GEMM_LIB = True
        assert not ops.use_gemm_nt(768, 2304)
    finally:
        ops.GEMM_LIB = old
    assert ops.use_gemm_nt(768, 2304)
