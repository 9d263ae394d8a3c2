"""Projection routing of the BASELINE configurations (CPU: the routing predicates only).

Every forward and input-gradient GEMM of the DeiT-S (configs[1]), ViT-B/16@384 (configs[2]) and
CaiT-S24 (configs[4]) encoders must be routed to this repo's ``sae_gemm_nt`` (ops.use_gemm_nt):
the projections of attention.py:29-37,60-63 and the FF block of ff.py:8-34.  The rocprofv3 step
profiles (profiles/r04o_step_kernels.txt) confirm on the GPU that no library GEMM runs."""
import pytest

import sae_vision_amd.ops as ops


def _shapes(C, hidden):
    # (K, N) of every forward / input-gradient GEMM of one encoder block
    return {
        "qkv_fwd": (C, 3 * C), "qkv_dx": (3 * C, C),
        "oproj_fwd": (C, C), "oproj_dx": (C, C),
        "ff0_fwd": (C, hidden), "ff0_dx": (hidden, C),
        "ff1_fwd": (hidden, C), "ff1_dx": (C, hidden),
    }


@pytest.mark.parametrize("name,C", [("deit_s", 384), ("vit_b_384", 768), ("cait_s24", 384)])
def test_every_block_gemm_routes_to_hip(name, C):
    for what, (K, N) in _shapes(C, 4 * C).items():
        assert ops.use_gemm_nt(K, N), f"{name} {what} (K={K}, N={N}) would run on the library GEMM"


def test_routing_flags_restore_the_round3_split():
    """ops.GEMM_LIB_WIDE = 1 / 2 (A/B switches) hand the ViT-B deep shapes back to the library."""
    old = ops.GEMM_LIB_WIDE
    try:
        ops.GEMM_LIB_WIDE = 1
        assert not ops.use_gemm_nt(768, 2304) and not ops.use_gemm_nt(3072, 768)
        ops.GEMM_LIB_WIDE = 2
        assert ops.use_gemm_nt(768, 2304) and not ops.use_gemm_nt(3072, 768)
    finally:
        ops.GEMM_LIB_WIDE = old
    assert ops.use_gemm_nt(3072, 768)
