"""Residual add + LayerNorm kernels (sae_layernorm_fwd/bwd) and the fused ViT encoder path
against the CPU oracle (oracle/vit_ref.py restating models/vit.py:9-99).

LayerNorm statistics are fp32 in both; the output is bf16 (Flax nn.LayerNorm(dtype=bfloat16)),
so y is checked at the bf16 bar (2e-2 of max|ref|); x + delta, dx and dscale / dbias are fp32
sums of the same bf16 inputs and are checked at 1e-5."""
import numpy as np
import pytest
import torch

import vit_ref
from _util import rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,C", [(25216, 384), (1000, 768), (37, 192), (5, 1024), (3, 4), (37, 384), (11, 512), (3, 128)])
@pytest.mark.parametrize("with_delta", [False, True])
def test_add_layer_norm(dev, M, C, with_delta):
    import torch
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(M + C)
    x = (torch.randn(M, C, device=dev, generator=g) * 3 + 1).requires_grad_()
    gamma = (torch.rand(C, device=dev, generator=g) + 0.5).requires_grad_()
    beta = torch.randn(C, device=dev, generator=g).requires_grad_()
    delta = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16).requires_grad_() if with_delta else None
    dy = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
    dxo = torch.randn(M, C, device=dev, generator=g) if with_delta else None
    if with_delta:
        xo, y = ops.add_layer_norm(x, delta, gamma, beta)
        torch.autograd.backward([xo, y], [dxo, dy])
    else:
        y = ops.layer_norm(x, gamma, beta)
        y.backward(dy)
    xs = x.detach().double().cpu().numpy()
    if with_delta:
        xs = xs + delta.detach().double().cpu().numpy()
        assert rel_err(xo, xs) <= 1e-6
    s, b = gamma.detach().double().cpu().numpy(), beta.detach().double().cpu().numpy()
    yr, cache = vit_ref.layer_norm(xs, s, b)
    assert y.dtype == torch.bfloat16
    assert rel_err(y.float(), yr) <= 2e-2
    dx, ds, db = vit_ref.layer_norm_bwd(dy.double().cpu().numpy(), s, cache)
    if with_delta:
        dx = dx + dxo.double().cpu().numpy()
        assert rel_err(delta.grad.float(), dx) <= 2e-2
    assert rel_err(x.grad, dx) <= 1e-5
    assert rel_err(gamma.grad, ds) <= 1e-5
    assert rel_err(beta.grad, db) <= 1e-5


def test_layer_norm_deterministic(dev):
    import torch
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(25216, 384, device=dev, generator=g)
    gamma, beta = torch.ones(384, device=dev), torch.zeros(384, device=dev)
    dy = torch.randn(25216, 384, device=dev, generator=g).to(torch.bfloat16)
    outs = []
    for _ in range(2):
        xx, gg, bb = x.clone().requires_grad_(), gamma.clone().requires_grad_(), beta.clone().requires_grad_()
        ops.layer_norm(xx, gg, bb).backward(dy)
        outs.append((xx.grad, gg.grad, bb.grad))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_vit_train_grads_vs_oracle(dev):
    """Whole bf16 ViT training step (patch GEMM, fused add+LayerNorm, fused attention, HIP weight
    gradients, FF, head, smoothed CE) vs the fp64 numpy oracle with the same parameters."""
    import torch
    import sae_vision_amd.vit as vit
    import sae_vision_amd.train as train
    torch.manual_seed(0)
    m = vit.ViT(num_classes=10, num_layers=2, num_heads=2, embed_dim=64, patch_shape=(8, 8), img_size=32,
                dtype=torch.bfloat16, device=dev)
    with torch.no_grad():
        m.Dense_0.kernel.normal_(0, 0.1)
    params = {k: v.detach().double().cpu().numpy() for k, v in m.named_parameters()}
    rng = np.random.default_rng(0)
    images = rng.standard_normal((4, 32, 32, 3))
    labels = rng.integers(0, 10, size=4)
    # the bf16 program of the reference (bf16 rounding points of create_model(dtype=bfloat16) and
    # the bf16 cotangents of its JAX autodiff), at the stated bf16 bar of 2e-2
    loss_ref, logits_ref, grads_ref = vit_ref.vit_loss_and_grads_bf16(params, images, labels, 2, 2, 8)
    logits = m(torch.tensor(images, device=dev, dtype=torch.float32), is_training=True)
    loss = train.smoothed_cross_entropy(logits, torch.tensor(labels, device=dev), 0.1)
    loss.backward()
    errs = {k: rel_err(p.grad, grads_ref[k]) for k, p in m.named_parameters()}
    print("max grad rel err vs bf16 chain:", max(errs.values()), max(errs, key=errs.get))
    assert rel_err(logits.float(), logits_ref) <= 2e-2
    assert abs(float(loss) - loss_ref) <= 2e-2 * abs(loss_ref)
    for k, err in errs.items():
        assert err <= 2e-2, f"{k}: rel err {err:.3e}"


@pytest.mark.parametrize("rowscale", [False, True])
@pytest.mark.parametrize("B,N", [(6, 196), (3, 37)])
def test_add_layer_norm_scaled(dev, rowscale, B, N):
    """CaiT form: x + delta * bf16(layerscale) * rowscale[sample], LayerNorm, and every gradient
    against float64 autograd of the same math (layerscale.py:21-23, stochastic_depth.py:19-28)."""
    import sae_vision_amd.ops as ops
    g = torch.Generator(device=dev).manual_seed(31)
    C = 384   # (3 x 37: an odd row count -- two rows a wave at C = 384 leaves the last half-wave empty)
    x = torch.randn(B, N, C, device=dev, generator=g)
    delta = torch.randn(B, N, C, device=dev, generator=g).to(torch.bfloat16)
    gamma = torch.rand(C, device=dev, generator=g) + 0.5
    beta = torch.randn(C, device=dev, generator=g) * 0.1
    ls = torch.rand(C, device=dev, generator=g) + 0.1
    rs = torch.tensor([0.0, 1.25, 1.25, 0.0, 1.25, 1.25][:B], device=dev) if rowscale else None
    dxo = torch.randn(B, N, C, device=dev, generator=g)
    dy = torch.randn(B, N, C, device=dev, generator=g).to(torch.bfloat16)

    leaves = [t.clone().requires_grad_(True) for t in (x, gamma, beta, ls)]
    d_leaf = delta.clone().requires_grad_(True)
    xo, y = ops.add_layer_norm_scaled(leaves[0], d_leaf, leaves[1], leaves[2], leaves[3], rs)
    torch.autograd.backward([xo, y], [dxo, dy])

    r = [t.clone().double().requires_grad_(True) for t in (x, gamma, beta, ls)]
    rd = delta.clone().double().requires_grad_(True)
    f = r[3].detach().to(torch.bfloat16).double() + (r[3] - r[3].detach())   # bf16 value, identity gradient
    if rs is not None:
        f = f[None, None, :] * rs.double()[:, None, None]
    xr = r[0] + rd * f
    mu = xr.mean(-1, keepdim=True)
    var = ((xr - mu) ** 2).mean(-1, keepdim=True)
    yr = (xr - mu) / torch.sqrt(var + 1e-6) * r[1] + r[2]
    torch.autograd.backward([xr, yr], [dxo.double(), dy.double()])
    rel = lambda a, b: float((a.double() - b).abs().max() / b.abs().max().clamp_min(1e-30))
    assert rel(xo, xr) <= 1e-6
    assert rel(y, yr) <= 1e-2
    assert rel(leaves[0].grad, r[0].grad) <= 1e-5
    assert rel(d_leaf.grad, rd.grad) <= 1e-2
    for got, want, name in ((leaves[1].grad, r[1].grad, "gamma"), (leaves[2].grad, r[2].grad, "beta"),
                            (leaves[3].grad, r[3].grad, "layerscale")):
        assert rel(got, want) <= 1e-4, name
