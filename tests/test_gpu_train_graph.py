"""The HIP-graph training step (TrainStep(graph=True): forward, loss, backward and AdamW captured
once and replayed) must do what the eager step does: same losses and parameters over several
steps from the same initial state and data."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model,split", [("deit_ti_patch16", False), ("deit_ti_patch16", True), ("cait", False)])
def test_graph_step_matches_eager(dev, model, split):
    """The graph step (flat gradient buffer with in-place sinks, only the non-sunk gradient ranges
    zeroed between replays, one-launch FusedAdamW) against the round-1 eager step (autograd's
    per-parameter gradients, torch's AdamW); split=True: the multi-rank structure (forward +
    backward graph, the all-reduce point, optimizer graph) at world 1; CaiT: parameters whose
    gradients autograd still accumulates (class token, position embedding) beside sunk ones."""
    from sae_vision_amd import cait, train, vit
    torch.manual_seed(0)
    if model == "cait":
        m_e = cait.create_cait("cait_xxs_24", 1000, torch.bfloat16, stoch_depth=False, device=dev)
    else:
        m_e = vit.create_model(model, 1000, torch.bfloat16, device=dev)
    m_g = copy.deepcopy(m_e)
    s_e = train.TrainStep(m_e, global_batch=8, device=dev, flat_grads=False)
    s_g = train.TrainStep(m_g, global_batch=8, device=dev, graph=True, two_graphs=split)
    assert s_g.flat and isinstance(s_g.opt, train.FusedAdamW) and not s_e.flat
    g = torch.Generator(device=dev).manual_seed(3)
    data = [(torch.randn(8, 224, 224, 3, device=dev, generator=g),
             torch.randint(0, 1000, (8,), device=dev, generator=g)) for _ in range(4)]
    # the graph step's first call warms up, restores the parameters and optimizer state, captures
    # (executing nothing) and replays once: exactly one optimizer step on data[0], as eager
    le = [float(s_e(*data[0]))]
    lg = [float(s_g(*data[0]))]
    assert s_g._g is not None and (s_g._g_opt is not None) == split
    for x, y in data[1:]:
        le.append(float(s_e(x, y)))
        lg.append(float(s_g(x, y)))
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-3 * abs(a), (le, lg)
    if model != "cait":   # every ViT parameter has a sink: nothing left to zero between replays
        assert s_g._zero_ranges == []
    for (n, pe), pg in zip(m_e.named_parameters(), m_g.parameters()):
        err = float((pe - pg).abs().max())
        assert err <= 1e-3 * max(1.0, float(pe.abs().max())), (n, err)


@pytest.mark.parametrize("model", ["deit_ti_patch16", "cait"])
def test_flat_grad_sinks_bitwise(dev, model):
    """The multi-rank step's in-place gradient sinks (ops.set_grad_sinks: the backward kernels write
    every Dense / FF / LayerNorm / patch-embedding gradient straight into its view of the flat
    buffer) give the same gradient bits as autograd's own accumulation, and a parameter
    feeding two sink-writing ops in one backward is refused."""
    from sae_vision_amd import cait, ops, train, vit
    torch.manual_seed(0)
    if model == "cait":
        m_a = cait.create_cait("cait_xxs_24", 1000, torch.bfloat16, stoch_depth=False, device=dev)
    else:
        m_a = vit.create_model(model, 1000, torch.bfloat16, device=dev)
    m_b = copy.deepcopy(m_a)
    m_b.load_state_dict(m_a.state_dict())
    s_a = train.TrainStep(m_a, global_batch=8, device=dev, flat_grads=False)
    s_b = train.TrainStep(m_b, global_batch=8, device=dev, flat_grads=True)
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(8, 224, 224, 3, device=dev, generator=g)
    y = torch.randint(0, 1000, (8,), device=dev, generator=g)
    s_a._fwd_bwd(x, y)
    s_b._fwd_bwd(x, y)
    torch.cuda.synchronize()
    for (n, pa), pb in zip(m_a.named_parameters(), m_b.parameters()):
        assert pa.grad is not None and pb.grad is not None, n
        assert pb.grad.data_ptr() >= s_b._flat.data_ptr(), n            # still the flat view
        assert torch.equal(pa.grad, pb.grad), (n, float((pa.grad - pb.grad).abs().max()))
    # outside the training step's sink window a backward keeps autograd's accumulate semantics
    g1 = [p.grad.clone() for p in m_b.parameters()]
    train.smoothed_cross_entropy(m_b(x, is_training=True), y).backward()
    torch.cuda.synchronize()
    for (n, p), g in zip(m_b.named_parameters(), g1):
        assert torch.allclose(p.grad, 2 * g, rtol=1e-5, atol=1e-6), n
    # inside one window a parameter's sink can be written once: a second backward is refused
    ops.begin_backward_sinks()
    try:
        train.smoothed_cross_entropy(m_b(x, is_training=True), y).backward()
        with pytest.raises(RuntimeError, match="written twice"):
            train.smoothed_cross_entropy(m_b(x, is_training=True), y).backward()
    finally:
        ops.end_backward_sinks()
    ops.set_grad_sinks(None)


def test_fused_adamw_matches_torch(dev):
    """sae_adamw_step (one launch over every parameter, chunk table built once, device step
    counter) against torch.optim.AdamW on the same gradients for several steps: odd sizes (scalar
    tail chunks) and sizes past one chunk."""
    from sae_vision_amd import train
    g = torch.Generator(device=dev).manual_seed(11)
    shapes = [(384, 1152), (7,), (1000,), (3, 2051), (384,)]
    ref = [torch.randn(s, device=dev, generator=g) for s in shapes]
    mine = [t.clone() for t in ref]
    for t in ref + mine:
        t.requires_grad_(True)
    flat = torch.zeros(sum(t.numel() for t in mine), device=dev)
    off = 0
    for t in mine:
        t.grad = flat[off:off + t.numel()].view_as(t)
        off += t.numel()
    kw = dict(lr=3e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4)
    opt_ref = torch.optim.AdamW(ref, foreach=False, **kw)
    opt = train.FusedAdamW(mine, flat, **kw)
    for _ in range(5):
        for a, b in zip(ref, mine):
            gr = torch.randn(a.shape, device=dev, generator=g)
            a.grad = gr.clone()
            b.grad.copy_(gr)
        opt_ref.step()
        opt.step()
    assert int(opt.step_count.item()) == 5
    for a, b in zip(ref, mine):
        err = float((a.detach() - b.detach()).abs().max() / a.detach().abs().max())
        assert err <= 2e-6, err


def test_grad_sink_follows_param_grad(dev):
    """A sink is only used while it is still the parameter's .grad: after the gradient is reset
    (zero_grad(set_to_none=True)) autograd's own accumulation takes over again."""
    from sae_vision_amd import ops, vit
    torch.manual_seed(0)
    m = vit.create_model("deit_ti_patch16", 1000, torch.bfloat16, device=dev)
    params = [p for p in m.parameters()]
    flat = torch.zeros(sum(p.numel() for p in params), device=dev)
    off = 0
    for p in params:
        p.grad = flat[off:off + p.numel()].view_as(p)
        off += p.numel()
    ops.set_grad_sinks(params, [p.grad for p in params])
    for p in params:
        p.grad = None            # reset: the registered views are no longer the gradients
    ops.begin_backward_sinks()
    try:
        x = torch.randn(2, 224, 224, 3, device=dev)
        m(x, is_training=True).float().sum().backward()
    finally:
        ops.end_backward_sinks()
    assert all(p.grad is not None for p in params)
    assert float(flat.abs().max()) == 0.0   # nothing went into the stale views
    ops.set_grad_sinks(None)


@pytest.mark.parametrize("flagged", ["1", "0"])
@pytest.mark.parametrize("model", ["deit_ti_patch16", "cait"])
def test_world1_rccl_overlapped_step(dev, model, flagged):
    """The multi-rank step's collective path on one GPU (tests/world1_rccl_case.py): a one-rank
    RCCL group, the bucket all-reduces launched from inside the backward on the communication
    stream and captured with the rest of the step in ONE HIP graph; losses and parameters equal to
    the no-collective graph step's bit for bit.  Run in a child process: the RCCL communicator and
    the graphs that captured its collectives live and die there (the child tears them down in the
    right order) and its stderr is reported if it fails."""
    import subprocess
    import sys
    import os
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "world1_rccl_case.py")
    env = dict(os.environ, SAE_FLAGGED=flagged)   # the default flag-gated structure / the in-graph fork
    r = subprocess.run([sys.executable, "-u", script, model], capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0 and "WORLD1_OK" in r.stdout, \
        f"SAE_FLAGGED={flagged} rc {r.returncode}\nstdout:\n{r.stdout[-2000:]}\nstderr:\n{r.stderr[-4000:]}"


def test_fused_adamw_cast_copies(dev):
    """sae_adamw_step_cast: parameters bit-identical to sae_adamw_step's, and the bf16 copies the
    update writes (plain [K, sum N] at the column offsets and its transpose) equal to the bf16
    cast of the updated fp32 weights; partial 64 x 64 edge tiles (K 68, N 100) included, one
    parameter outside every group (the flat chunk path in the same launch)."""
    from sae_vision_amd import ops, train
    g = torch.Generator(device=dev).manual_seed(13)
    shapes = [(68, 100), (68, 36), (384, 1152), (7,), (256, 68)]
    base = [torch.randn(s, device=dev, generator=g) for s in shapes]

    def make():
        ps = [t.clone().requires_grad_(True) for t in base]
        offs, n = train.flat_layout(ps)
        flat = torch.zeros(n, device=dev)
        for p, o in zip(ps, offs):
            p.grad = flat[o:o + p.numel()].view_as(p)
        return ps, flat

    a, fa = make()
    b, fb = make()
    kw = dict(lr=3e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4)
    groups = [[b[0], b[1]], [b[2]], [b[4]]]
    opt_a = train.FusedAdamW(a, fa, **kw)
    opt_b = train.FusedAdamW(b, fb, cast_groups=groups, **kw)
    try:
        assert len(opt_b.cast_groups) == 3 and opt_b.n_tiles == 2 * 2 + 2 * 1 + 6 * 18 + 4 * 2
        for _ in range(4):
            for p, q in zip(a, b):
                gr = torch.randn(p.shape, device=dev, generator=g)
                p.grad.copy_(gr)
                q.grad.copy_(gr)
            opt_a.step()
            opt_b.step()
        torch.cuda.synchronize()
        for p, q in zip(a, b):
            assert torch.equal(p, q)
        for ws, (w16, wt16) in zip(groups, opt_b.copies):
            ref = torch.cat([w.detach() for w in ws], dim=1).to(torch.bfloat16)
            assert torch.equal(w16, ref) and torch.equal(wt16, ref.t().contiguous())
            assert ops._cast_lookup(ws)[0] is w16          # served to the forward as is
        # an in-place change outside the optimizer is noticed: the next lookup re-casts
        with torch.no_grad():
            b[2].mul_(0.5)
        w16, wt16 = ops._cast_lookup([b[2]])
        torch.cuda.synchronize()
        assert torch.equal(w16, b[2].detach().to(torch.bfloat16))
    finally:
        opt_b.close()
    assert ops._wkey([b[2]]) not in ops._PERSIST
    # a parameter named by two groups is updated once: the second group is left to the forward
    c, fc = make()
    opt_c = train.FusedAdamW(c, fc, cast_groups=[[c[2]], [c[2]], [c[0], c[0]]], **kw)
    try:
        assert [len(g) for g in opt_c.cast_groups] == [1]
    finally:
        opt_c.close()


@pytest.mark.parametrize("model,graph", [("deit_ti_patch16", False), ("deit_ti_patch16", True), ("cait", True)])
def test_train_step_persistent_casts_bitwise(dev, model, graph):
    """Training steps with the optimizer writing the bf16 Dense copies (no cast in the forward)
    give the same losses and parameters, bit for bit, as steps that cast every forward (DeiT-Ti;
    CaiT-XXS: trunk groups, class-attention cross projections, talking-heads transform sinks)."""
    from sae_vision_amd import cait, ops, train, vit
    torch.manual_seed(0)
    if model == "cait":
        m_a = cait.create_cait("cait_xxs_24", 1000, torch.bfloat16, stoch_depth=False, device=dev)
    else:
        m_a = vit.create_model(model, 1000, torch.bfloat16, device=dev)
    m_b = copy.deepcopy(m_a)
    s_a = train.TrainStep(m_a, global_batch=8, device=dev, graph=graph, persistent_casts=False)
    s_b = train.TrainStep(m_b, global_batch=8, device=dev, graph=graph)
    assert not s_a.opt.cast_groups
    assert len(s_b.opt.cast_groups) == len(m_b.cast_groups())   # every group the model names
    g = torch.Generator(device=dev).manual_seed(3)
    data = [(torch.randn(8, 224, 224, 3, device=dev, generator=g),
             torch.randint(0, 1000, (8,), device=dev, generator=g)) for _ in range(3)]
    try:
        la = [float(s_a(x, y)) for x, y in data]
        lb = [float(s_b(x, y)) for x, y in data]
        assert la == lb, (la, lb)
        for (n, pa), pb in zip(m_a.named_parameters(), m_b.parameters()):
            assert torch.equal(pa, pb), n
    finally:
        s_b.opt.close()


def test_graph_step_sees_weights_loaded_after_capture(dev):
    """a replayed step graph holds no weight cast (the optimizer writes the bf16
    copies), so weights loaded in place after the capture (load_state_dict) must re-cast the
    copies before the next replay: the step after the load equals, bit for bit, a step that casts
    every forward (persistent_casts=False) from the same loaded state."""
    from sae_vision_amd import train, vit
    torch.manual_seed(0)
    m_a = vit.create_model("deit_ti_patch16", 1000, torch.bfloat16, device=dev)
    m_b = copy.deepcopy(m_a)
    fresh = copy.deepcopy(m_a).state_dict()          # the state loaded mid-run
    s_a = train.TrainStep(m_a, global_batch=8, device=dev, graph=True, persistent_casts=False)
    s_b = train.TrainStep(m_b, global_batch=8, device=dev, graph=True)
    g = torch.Generator(device=dev).manual_seed(7)
    data = [(torch.randn(8, 224, 224, 3, device=dev, generator=g),
             torch.randint(0, 1000, (8,), device=dev, generator=g)) for _ in range(3)]
    try:
        for m, s in ((m_a, s_a), (m_b, s_b)):
            s(*data[0])                                  # capture + first replay
            s(*data[1])
            m.load_state_dict(fresh)                     # in place: same storage, versions move
        la, lb = float(s_a(*data[2])), float(s_b(*data[2]))
        assert la == lb, (la, lb)
        for (n, pa), pb in zip(m_a.named_parameters(), m_b.parameters()):
            assert torch.equal(pa, pb), n
    finally:
        s_b.close()
        s_a.close()
