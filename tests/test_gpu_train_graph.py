"""The HIP-graph training step (TrainStep(graph=True): forward, loss, backward and AdamW captured
once and replayed) must do what the eager step does: same losses and parameters over several
steps from the same initial state and data."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("flat", [False, True])
def test_graph_step_matches_eager(dev, flat):
    """flat=True: the multi-rank structure (flat gradient buffer, forward + backward graph, the
    all-reduce point, optimizer graph) at world 1, against the plain eager step."""
    from sae_vision_amd import train, vit
    torch.manual_seed(0)
    m_e = vit.create_model("deit_ti_patch16", 1000, torch.bfloat16, device=dev)
    m_g = copy.deepcopy(m_e)
    s_e = train.TrainStep(m_e, global_batch=8, device=dev)
    s_g = train.TrainStep(m_g, global_batch=8, device=dev, graph=True, flat_grads=flat)
    g = torch.Generator(device=dev).manual_seed(3)
    data = [(torch.randn(8, 224, 224, 3, device=dev, generator=g),
             torch.randint(0, 1000, (8,), device=dev, generator=g)) for _ in range(4)]
    # the graph step's first call warms up, restores the parameters and optimizer state, captures
    # (executing nothing) and replays once: exactly one optimizer step on data[0], as eager
    le = [float(s_e(*data[0]))]
    lg = [float(s_g(*data[0]))]
    assert s_g._g is not None and (s_g._g_opt is not None) == flat
    for x, y in data[1:]:
        le.append(float(s_e(x, y)))
        lg.append(float(s_g(x, y)))
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-3 * abs(a), (le, lg)
    for (n, pe), pg in zip(m_e.named_parameters(), m_g.parameters()):
        err = float((pe - pg).abs().max())
        assert err <= 1e-3 * max(1.0, float(pe.abs().max())), (n, err)
