"""The encoder input (sae_tokens_fwd / _bwd: models/vit.py:82-85 class-token concatenate +
AddAbsPosEmbed, vit.py:46 / position_embed.py:48) against the torch composition it replaces,
and the encoder's first LayerNorm returning its input (ops.layer_norm_pass) against LayerNorm +
an explicit residual branch.  Forward values and the bf16 token gradient are bit-exact (same fp32
add, same rounding); the batch sums of dcls / dpos agree to fp32 summation order."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,L,E", [(128, 196, 384), (3, 576, 768), (5, 16, 8)])
def test_encoder_tokens_matches_torch(dev, B, L, E):
    from sae_vision_amd import ops
    g = torch.Generator(device=dev).manual_seed(B + L + E)
    tok = torch.randn(B, L, E, device=dev, generator=g).to(torch.bfloat16)
    cls = torch.randn(1, 1, E, device=dev, generator=g)
    pos = torch.randn(1, L + 1, E, device=dev, generator=g)
    dx = torch.randn(B, L + 1, E, device=dev, generator=g)
    t1, c1, p1 = (t.clone().requires_grad_(True) for t in (tok, cls, pos))
    t2, c2, p2 = (t.clone().requires_grad_(True) for t in (tok, cls, pos))
    x1 = ops.encoder_tokens(t1, c1, p1)
    x2 = torch.cat([c2.expand(B, 1, E), t2.float()], dim=1) + p2
    assert torch.equal(x1, x2)
    x1.backward(dx)
    x2.backward(dx)
    assert t1.grad.dtype == torch.bfloat16 and torch.equal(t1.grad, t2.grad)
    for a, b in ((c1.grad, c2.grad), (p1.grad, p2.grad)):
        assert float((a - b).abs().max()) <= 1e-5 * float(b.abs().max()), float((a - b).abs().max())


def test_layer_norm_pass_residual_gradient(dev):
    from sae_vision_amd import ops
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(2, 197, 384, device=dev, generator=g)
    gamma = 1 + 0.1 * torch.randn(384, device=dev, generator=g)
    beta = 0.1 * torch.randn(384, device=dev, generator=g)
    w = torch.randn(2, 197, 384, device=dev, generator=g)
    dy = torch.randn(2, 197, 384, device=dev, generator=g)
    xa = x.clone().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    ra, ha = ops.layer_norm_pass(xa, gamma, beta)
    hb = ops.layer_norm(xb, gamma, beta)
    assert torch.equal(ha, hb) and torch.equal(ra, xa)
    ((ra * w).sum() + (ha.float() * dy).sum()).backward()
    ((xb * w).sum() + (hb.float() * dy).sum()).backward()
    err = float((xa.grad - xb.grad).abs().max() / xb.grad.abs().max())
    assert err <= 1e-6, err


def test_cls_add_layer_norm_matches_full(dev):
    """The final residual add + LayerNorm on the class-token rows only equals the full pass's token 0
    (bit-exact forward: the LayerNorm is row-wise); gradients agree with autograd through the full
    pass to fp32 summation order."""
    from sae_vision_amd import ops
    g = torch.Generator(device=dev).manual_seed(9)
    B, N, E = 4, 197, 384
    x = torch.randn(B, N, E, device=dev, generator=g)
    f = torch.randn(B, N, E, device=dev, generator=g).to(torch.bfloat16)
    gamma = (1 + 0.1 * torch.randn(E, device=dev, generator=g)).requires_grad_(True)
    beta = (0.1 * torch.randn(E, device=dev, generator=g)).requires_grad_(True)
    dy = torch.randn(B, E, device=dev, generator=g).to(torch.bfloat16)
    xa, fa = x.clone().requires_grad_(True), f.clone().requires_grad_(True)
    xb, fb = x.clone().requires_grad_(True), f.clone().requires_grad_(True)
    ga, ba = gamma.detach().clone().requires_grad_(True), beta.detach().clone().requires_grad_(True)
    ha = ops.cls_add_layer_norm(xa, fa, ga, ba)
    hb = ops.add_layer_norm(xb, fb, gamma, beta)[1][:, 0]
    assert ha.shape == (B, E) and torch.equal(ha, hb)
    (ha.float() * dy.float()).sum().backward()
    (hb.float() * dy.float()).sum().backward()
    for a, b in ((xa.grad, xb.grad), (fa.grad.float(), fb.grad.float()), (ga.grad, gamma.grad), (ba.grad, beta.grad)):
        assert float((a - b).abs().max()) <= 1e-6 * max(1.0, float(b.abs().max())), float((a - b).abs().max())
