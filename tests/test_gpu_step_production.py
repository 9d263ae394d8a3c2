"""Composed training-step parity at production row counts.

The other oracle-compared module / step tests run below the M >= 4096 routing threshold of the
persistent GEMMs, so there the projections take the 128-row kernel.  Here a one-block ViT at the
DeiT-S width (C 384, H 6, N 197, batch 24: M = 4,728 token rows) and at the ViT-B/16@384 width
(C 768, H 12, N 577, batch 8: M = 4,616) runs the whole bf16 training step -- patch GEMM, fused
add + LayerNorm, packed QKV GEMM, fused attention core, output projection, FF block with the GELU /
GELU' epilogues, head, smoothed CE, and every weight gradient -- with the projections on the
kernels the benchmark uses: ``gemm8`` (DeiT-S) and ``gemm8`` + ``gemm8x`` (ViT-B), weight gradients
on the LDS-DMA split-token kernel.  The routes are asserted through ``sae_gemm_nt_route`` (the C
ABI's own kernel choice) for every GEMM of the block, and the logits, loss and every parameter
gradient are compared with the bf16 program of the reference (oracle/vit_ref.py
``vit_loss_and_grads_bf16``: the bf16 rounding points of create_model(dtype=bfloat16) and the bf16
cotangents of its JAX autodiff, models/vit.py:18-99, attention.py:29-63, ff.py:8-34, train.py:77-92)
at the north_star bf16 bar of 2e-2."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import vit_ref  # noqa: E402

GEMM8, GEMM8X = 3, 4


def rel_err(a, b):
    a = a.detach().double().cpu().numpy() if hasattr(a, "detach") else np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _ff_epilogues():
    # the epilogue codes the FF block actually passes (ops.py: FF_GELU_GRAD on by default saves
    # gelu'(h) in Dense_0's forward and multiplies by it in Dense_1's input gradient)
    import sae_vision_amd.ops as ops
    if ops.FF_GELU_GRAD:
        return ops.EPI_GELU_GRAD, ops.EPI_MUL_AUX
    return ops.EPI_GELU, ops.EPI_DGELU


def _block_gemms(M, C, hidden):
    # (K, N, epilogue) of the forward / input-gradient GEMMs of one encoder block
    e_fwd, e_dx = _ff_epilogues()
    return {"qkv_fwd": (C, 3 * C, 0), "qkv_dx": (3 * C, C, 0), "oproj_fwd": (C, C, 0), "oproj_dx": (C, C, 0),
            "ff0_fwd": (C, hidden, e_fwd), "ff0_dx": (hidden, C, 0), "ff1_fwd": (hidden, C, 0),
            "ff1_dx": (C, hidden, e_dx)}


@pytest.mark.parametrize("name,B,img,C,H,expect", [
    ("deit_s_width", 24, 224, 384, 6, {k: GEMM8 for k in ("qkv_fwd", "qkv_dx", "oproj_fwd", "oproj_dx", "ff0_fwd",
                                                           "ff0_dx", "ff1_fwd", "ff1_dx")}),
    ("vit_b384_width", 8, 384, 768, 12, {"qkv_fwd": GEMM8, "ff0_fwd": GEMM8, "qkv_dx": GEMM8X, "oproj_fwd": GEMM8X,
                                         "oproj_dx": GEMM8X, "ff0_dx": GEMM8X, "ff1_fwd": GEMM8X,
                                         "ff1_dx": GEMM8}),
])
def test_train_step_production_rows_vs_oracle(dev, name, B, img, C, H, expect):
    import torch
    import sae_vision_amd.train as train
    import sae_vision_amd.vit as vit
    from sae_vision_amd import _lib as L

    N = (img // 16) ** 2 + 1
    M = B * N
    assert M >= 4096
    lib = L.load()
    for what, (K, Nf, epi) in _block_gemms(M, C, 4 * C).items():
        if what in expect:
            got = lib.sae_gemm_nt_route(M, Nf, K, epi)
            assert got == expect[what], f"{name} {what}: route {got}, expected {expect[what]}"

    torch.manual_seed(0)
    m = vit.ViT(num_classes=1000, num_layers=1, num_heads=H, embed_dim=C, patch_shape=(16, 16), img_size=img,
                dtype=torch.bfloat16, device=dev)
    with torch.no_grad():
        m.Dense_0.kernel.normal_(0, 0.05)   # the reference zero-inits the head: give the trunk a gradient
    params = {k: v.detach().double().cpu().numpy() for k, v in m.named_parameters()}
    rng = np.random.default_rng(0)
    images = rng.standard_normal((B, img, img, 3)).astype(np.float32)
    labels = rng.integers(0, 1000, size=B)
    loss_ref, logits_ref, grads_ref = vit_ref.vit_loss_and_grads_bf16(params, images, labels, 1, H, 16)
    logits = m(torch.tensor(images, device=dev), is_training=True)
    loss = train.smoothed_cross_entropy(logits, torch.tensor(labels, device=dev), 0.1)
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(logits.float(), logits_ref) <= 2e-2
    assert abs(float(loss) - loss_ref) <= 2e-2 * abs(loss_ref)
    errs = {k: rel_err(p.grad, grads_ref[k]) for k, p in m.named_parameters()}
    worst = max(errs, key=errs.get)
    print(f"{name}: max grad rel err vs the bf16 chain {errs[worst]:.3e} ({worst})")
    for k, err in errs.items():
        assert err <= 2e-2, f"{name} {k}: rel err {err:.3e}"
