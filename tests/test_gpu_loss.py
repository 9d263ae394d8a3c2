"""The training loss (sae_smoothed_ce_fwd / _bwd, train.py:77-90: optax.smooth_labels + mean
softmax cross entropy) against torch's label-smoothed cross entropy in fp32 on the same logits:
the loss within 1e-5 relative, dlogits within fp32 rounding (fp32 logits) or one bf16 rounding
(bf16 logits, whose gradient is returned in bf16)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,K", [(128, 1000), (7, 10), (300, 37), (1, 1000)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("alpha", [0.1, 0.0])
def test_smoothed_ce_matches_torch(dev, R, K, dt, alpha):
    from sae_vision_amd import ops
    g = torch.Generator(device=dev).manual_seed(R * K)
    x = (3 * torch.randn(R, K, device=dev, generator=g)).to(dt)
    y = torch.randint(0, K, (R,), device=dev, generator=g)
    xa = x.clone().requires_grad_(True)
    xr = x.float().clone().requires_grad_(True)
    loss = ops.smoothed_cross_entropy(xa, y, alpha)
    ref = F.cross_entropy(xr, y, label_smoothing=alpha)
    assert abs(float(loss) - float(ref)) <= 1e-5 * abs(float(ref)), (float(loss), float(ref))
    (1.7 * loss).backward()
    (1.7 * ref).backward()
    assert xa.grad.dtype == dt
    tol = 1e-6 if dt == torch.float32 else 2 ** -8
    err = float((xa.grad.float() - xr.grad).abs().max() / xr.grad.abs().max())
    assert err <= tol, err


def test_smoothed_ce_deterministic_and_strided(dev):
    """Same bits on every call; a row-strided logits view (the head output sliced) is read in place."""
    from sae_vision_amd import ops
    g = torch.Generator(device=dev).manual_seed(1)
    big = torch.randn(64, 1024, device=dev, generator=g).to(torch.bfloat16)
    x = big[:, :1000]
    y = torch.randint(0, 1000, (64,), device=dev, generator=g)
    a = ops.smoothed_cross_entropy(x, y)
    b = ops.smoothed_cross_entropy(x, y)
    assert torch.equal(a, b)
    ref = F.cross_entropy(x.float(), y, label_smoothing=0.1)
    assert abs(float(a) - float(ref)) <= 1e-5 * abs(float(ref))


def test_smoothed_ce_rejects_cpu():
    from sae_vision_amd import ops
    with pytest.raises(RuntimeError, match="GPU only"):
        ops.smoothed_cross_entropy(torch.randn(2, 5), torch.zeros(2, dtype=torch.int64))
