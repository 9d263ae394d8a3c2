"""CaiT caller on the GPU (models/cait.py): logits shape like the reference's cait_test.py, the
forward against the float64 oracle (oracle/cait_ref.py: the whole composition -- patch embed,
talking-heads trunk with LayerScale, class attention over [cls, x], final norm and head) for the
fp32 and the bf16 model, the bf16 model's gradients against the bf16-emulated oracle chain
(cait_ref.cait_logits_bf16), and the HIP-graph training step with stochastic depth on."""
import numpy as np
import pytest
import torch

import cait_ref

pytestmark = pytest.mark.gpu


def _small(dtype, dev, sd=0.0):
    from sae_vision_amd import cait
    torch.manual_seed(0)
    m = cait.CaiT(num_classes=10, num_layers=2, num_layers_token_only=2, num_heads=4, embed_dim=192,
                  patch_shape=(16, 16), stoch_depth_rate=sd, layerscale_eps=1e-5, img_size=64, dtype=dtype,
                  device=dev)
    with torch.no_grad():   # exercise every branch: unit LayerScale, a non-zero head
        for n, p in m.named_parameters():
            if n.endswith("layerscale"):
                p.fill_(1.0)
        m.Dense_0.kernel.normal_(0.0, 0.05)
    return m


def test_cait_logits_shape(dev):
    from sae_vision_amd import cait
    m = cait.create_cait("cait_xxs_24", 1000, torch.bfloat16, device=dev)
    x = torch.randn(2, 224, 224, 3, device=dev)
    y = m(x, is_training=False)
    assert y.shape == (2, 1000)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
def test_cait_forward_matches_oracle(dev, dtype, tol):
    m = _small(dtype, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(4, 64, 64, 3, device=dev, generator=g)
    with torch.no_grad():
        y = m(x, is_training=False).double().cpu().numpy()
    P = {n: p.detach().double().cpu().numpy() for n, p in m.named_parameters()}
    xin = x.to(dtype).double().cpu().numpy()       # the images as the model sees them
    ref = cait_ref.cait_forward(P, xin, num_layers=2, num_layers_token_only=2, patch=16)
    err = float(np.abs(y - ref).max() / np.abs(ref).max())
    print(f"cait {dtype}: max rel err {err:.2e}")
    assert err <= tol


def test_cait_bf16_grads_match_oracle(dev):
    """The bf16 model's logits and EVERY parameter gradient against the bf16-emulated oracle chain
    (oracle/cait_ref.cait_logits_bf16: float64 with the Flax modules' bf16 rounding points, autograd
    rounding each bf16 value's cotangent to bf16 = JAX autodiff of the bf16 program), at the stated
    2e-2: talking-heads trunk (fp32 mixes), LayerScale, class attention (Nq = 1), FF, LayerNorms,
    patch embedding, head."""
    import torch.nn.functional as F
    m = _small(torch.bfloat16, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(4, 64, 64, 3, device=dev, generator=g)
    lab = torch.randint(0, 10, (4,), device=dev, generator=g)
    y = m(x, is_training=True)
    F.cross_entropy(y.float(), lab).backward()
    P = {n: p.detach().double().cpu().requires_grad_(True) for n, p in m.named_parameters()}
    ref = cait_ref.cait_logits_bf16(P, x.double().cpu(), num_layers=2, num_layers_token_only=2, patch=16)
    F.cross_entropy(ref, lab.cpu()).backward()
    rel = lambda a, b: float((a.double().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-30))
    assert rel(y.float().detach(), ref.detach()) <= 2e-2
    bad = {}
    for n, p in m.named_parameters():
        e = rel(p.grad, P[n].grad)
        if not e <= 2e-2:
            bad[n] = e
    assert not bad, bad


def test_cait_graph_step_stochastic_depth(dev):
    from sae_vision_amd import train
    m = _small(torch.bfloat16, dev, sd=0.1)
    step = train.TrainStep(m, global_batch=8, device=dev, graph=True)
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn(8, 64, 64, 3, device=dev, generator=g)
    lab = torch.randint(0, 10, (8,), device=dev, generator=g)
    losses = [float(step(x, lab)) for _ in range(4)]
    assert all(l == l and abs(l) < 1e4 for l in losses), losses
    assert step._g is not None          # captured (torch's generator is graph-safe)
