"""Patch embedding (models/layers/stems/patch_embed.py:15-26) with the patch gather fused into the
GEMM operand staging, from the model-call layout NHWC and from the train-step feed HWCN
(train.py:80 'H W C N -> N H W C', input_pipeline.py:187-191).

Checker: ``oracle/vit_ref.patchify`` (+ ``hwcn_to_nhwc``) and float64 products of the same
bf16-rounded images and kernel (train.py:81 casts the images to bf16; Flax Dense casts the kernel
to the compute dtype).  Outputs are bf16: bar 2e-2 of the largest magnitude (north_star bf16);
dW accumulates in fp32: bar 1e-3.  The GEMM row order differs between the layouts but every
output element is the same dot product in the same k order, so NHWC and HWCN forwards agree bit
for bit."""
import numpy as np
import pytest
import torch

import vit_ref

pytestmark = pytest.mark.gpu

CASES = [  # (B, H, W, C, ph, pw, E)
    (8, 32, 48, 3, 16, 16, 384),     # DeiT-S stem on a small image
    (16, 224, 224, 3, 16, 16, 384),  # DeiT-S/16 at 224 px (196 patches)
    (8, 64, 64, 3, 32, 32, 768),     # patch 32 (vit_b_patch32), K = 3072
    (24, 32, 32, 3, 16, 8, 136),     # rectangular patch, K = 384, embed not a tile multiple
    (3, 48, 32, 3, 16, 16, 64),      # batch not a multiple of 8 (NHWC only)
]


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30))


def _ref(images_nhwc, w, b, patch):
    """float64 tokens and the patch matrix (bf16-rounded inputs, as the kernel sees them)."""
    x = images_nhwc.to(torch.bfloat16).double().cpu().numpy()
    wk = w.to(torch.bfloat16).double().cpu().numpy()
    A = vit_ref.patchify(x, patch)
    y = A @ wk
    if b is not None:
        y = y + b.double().cpu().numpy()
    return torch.from_numpy(y), A


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("layout", ["NHWC", "HWCN"])
@pytest.mark.parametrize("idt", [torch.bfloat16, torch.float32])
def test_patch_embed_fwd_bwd(dev, case, layout, idt):
    import sae_vision_amd.ops as ops
    B, H, W, C, ph, pw, E = case
    if layout == "HWCN" and B % 8:
        pytest.skip("HWCN takes batch % 8 == 0 (the ops fall back to the rearrange + Dense)")
    g = torch.Generator(device=dev).manual_seed(B * 7 + E)
    img = torch.randn(B, H, W, C, device=dev, generator=g)
    K = ph * pw * C
    w = torch.randn(K, E, device=dev, generator=g) / K ** 0.5
    b = torch.randn(E, device=dev, generator=g) * 0.1 if E == 136 else None
    if b is not None:
        b.requires_grad_(True)
    w.requires_grad_(True)
    feed = img.to(idt)
    if layout == "HWCN":
        feed = feed.permute(1, 2, 3, 0).contiguous()    # the feed's [H, W, C, N]
        assert np.array_equal(vit_ref.hwcn_to_nhwc(feed.float().cpu().numpy()), img.to(idt).float().cpu().numpy())
    assert ops.patch_embed_ok(feed, w, (ph, pw), layout)
    y = ops.patch_embed(feed, w, b, (ph, pw), layout)
    assert y.dtype == torch.bfloat16 and tuple(y.shape) == (B, (H // ph) * (W // pw), E)
    yref, A = _ref(img.to(idt), w.detach(), b.detach() if b is not None else None, (ph, pw))
    assert _rel(y.cpu(), yref) < 2e-2
    dy = torch.randn(y.shape, device=dev, generator=g).to(torch.bfloat16)
    y.backward(dy)
    dyn = dy.double().cpu().numpy().reshape(-1, E)
    dw_ref = torch.from_numpy(A.reshape(-1, K).T @ dyn)
    assert _rel(w.grad.cpu(), dw_ref) < 1e-3
    if b is not None:
        assert _rel(b.grad.cpu(), torch.from_numpy(dyn.sum(0))) < 1e-3


def test_patch_embed_layouts_agree_bitwise(dev):
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(5)
    img = torch.randn(16, 64, 64, 3, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(768, 384, device=dev, generator=g) / 768 ** 0.5
    y0 = ops.patch_embed(img, w, None, (16, 16), "NHWC")
    y1 = ops.patch_embed(img.permute(1, 2, 3, 0).contiguous(), w, None, (16, 16), "HWCN")
    assert torch.equal(y0, y1)


def test_patch_embed_rejects(dev):
    import sae_vision_amd.ops as ops
    from sae_vision_amd._lib import SaeError
    w = torch.zeros(768, 384, device=dev)
    img = torch.zeros(12, 32, 32, 3, device=dev)
    with pytest.raises(SaeError, match="batch % 8"):    # HWCN batch of 12
        ops.patch_embed(img.permute(1, 2, 3, 0).contiguous(), w, None, (16, 16), "HWCN")
    with pytest.raises(SaeError, match="whole number"):
        ops.patch_embed(torch.zeros(8, 40, 32, 3, device=dev), w, None, (16, 16), "NHWC")
    with pytest.raises(NotImplementedError):
        ops.patch_embed(img.requires_grad_(True), w, None, (16, 16))


@pytest.mark.parametrize("layout", ["NHWC", "HWCN"])
def test_vit_forward_layouts(dev, layout):
    """The ViT stem through the fused gather matches the rearrange + Dense stem (fp32 model path
    on the same bf16 images) and the NHWC / HWCN feeds give the same logits."""
    from sae_vision_amd.vit import ViT
    torch.manual_seed(0)
    m = ViT(num_classes=10, num_layers=2, num_heads=3, embed_dim=192, patch_shape=(16, 16), img_size=64,
            dtype=torch.bfloat16, device=dev)
    img = torch.randn(8, 64, 64, 3, device=dev).to(torch.bfloat16)
    feed = img if layout == "NHWC" else img.permute(1, 2, 3, 0).contiguous()
    with torch.no_grad():
        y = m(feed, is_training=False, layout=layout)
        y_nhwc = m(img, is_training=False)
    assert torch.equal(y, y_nhwc)


@pytest.mark.parametrize("idt", [torch.bfloat16, torch.float32])
def test_patch_gather_hwcn_exact(dev, idt):
    """sae_patch_gather writes the patch matrix of an HWCN feed bit for bit: rows n L + p, columns
    (ky Pw + kx) C + c, each image value rounded to bf16 (oracle: vit_ref.patchify of the NHWC view)."""
    import ctypes
    import sae_vision_amd.ops as ops
    from sae_vision_amd import _lib as L
    B, H, W, C, ph, pw, E = 16, 64, 48, 3, 16, 16, 384
    g = torch.Generator(device=dev).manual_seed(11)
    img = torch.randn(B, H, W, C, device=dev, generator=g).to(idt)
    feed = img.permute(1, 2, 3, 0).contiguous()
    desc = ops._patch_desc(feed, (ph, pw), E, "HWCN")
    Lp, K = (H // ph) * (W // pw), ph * pw * C
    pm = torch.empty((B * Lp, K), dtype=torch.bfloat16, device=dev)
    L.check(L.load().sae_patch_gather(ops._stream(feed), ctypes.byref(desc), ops._ptr(feed), ops._ptr(pm)))
    ref = vit_ref.patchify(img.to(torch.bfloat16).float().cpu().numpy(), (ph, pw)).reshape(B * Lp, K)
    assert np.array_equal(pm.float().cpu().numpy(), ref)


def test_patch_embed_gathered_vs_fused(dev, monkeypatch):
    """The DeiT-S stem (M = 25,088 token rows: gemm8 / gemm_dw8 on the gathered patch matrix) against
    the fused HWCN loaders: the same bf16 operands, so outputs agree to bf16 rounding and dW to
    fp32 summation order."""
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(12)
    B, H, W, C, E = 128, 224, 224, 3, 384
    feed = torch.randn(H, W, C, B, device=dev, generator=g)
    w = (torch.randn(768, E, device=dev, generator=g) / 768 ** 0.5).requires_grad_(True)
    b = (torch.randn(E, device=dev, generator=g) * 0.1).requires_grad_(True)
    dy = torch.randn(B, 196, E, device=dev, generator=g).to(torch.bfloat16)
    outs = {}
    for gathered in (True, False):
        monkeypatch.setattr(ops, "PATCH_GATHER", gathered)
        w.grad = b.grad = None
        y = ops.patch_embed(feed, w, b, (16, 16), "HWCN")
        y.backward(dy)
        outs[gathered] = (y.detach().float(), w.grad.clone(), b.grad.clone())
    (y1, dw1, db1), (y0, dw0, db0) = outs[True], outs[False]
    assert _rel(y1, y0) < 1e-2
    assert _rel(dw1, dw0) < 1e-4 and _rel(db1, db0) < 1e-4
