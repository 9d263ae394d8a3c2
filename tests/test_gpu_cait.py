"""CaiT caller on the GPU (models/cait.py): logits shape like the reference's cait_test.py, the
forward against the float64 oracle (oracle/cait_ref.py: the whole composition -- patch embed,
talking-heads trunk with LayerScale, class attention over [cls, x], final norm and head) for the
fp32 and the bf16 model, the bf16 gradients against the fp32 model's (whose kernels are pinned to
the oracle op by op in test_gpu_variants.py), and the HIP-graph training step with stochastic
depth on."""
import copy

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


def test_cait_bf16_matches_fp32(dev):
    m32 = _small(torch.float32, dev)
    m16 = copy.deepcopy(m32)
    m16.dtype = torch.bfloat16
    for mod in m16.modules():
        if hasattr(mod, "dtype") and isinstance(getattr(mod, "dtype"), torch.dtype):
            mod.dtype = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(4, 64, 64, 3, device=dev, generator=g)
    lab = torch.randint(0, 10, (4,), device=dev, generator=g)
    outs = []
    for m in (m32, m16):
        y = m(x, is_training=True)
        loss = torch.nn.functional.cross_entropy(y.float(), lab)
        loss.backward()
        outs.append((y.float().detach(), {n: p.grad.detach().clone() for n, p in m.named_parameters()}))
    (y32, g32), (y16, g16) = outs
    rel = lambda a, b: float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
    assert rel(y16, y32) <= 3e-2
    for n in ("Dense_0.kernel", "CAEncoderBlock_1.FFBlock_0.Dense_1.kernel",
              "CAEncoderBlock_0.ClassSelfAttentionBlock_0.queries.kernel",
              "Encoder_0.EncoderBlock_1.SelfAttentionBlock_0.TalkingHeadsBlock_0.talking_heads_transform",
              "Encoder_0.EncoderBlock_0.SelfAttentionBlock_0.keys.kernel", "PatchEmbedBlock_0.Dense_0.kernel"):
        assert rel(g16[n], g32[n]) <= 6e-2, n


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
