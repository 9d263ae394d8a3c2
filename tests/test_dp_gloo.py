"""Multi-process data-parallel path on CPU (gloo, world size 2).

The training step (sae_vision_amd.train.TrainStep, the rebuild of the reference's
pmap(train_step) + lax.pmean(grads), train.py:94-96,230: flat gradient buffer, bucketed SUM
all-reduce of the gradients of loss / world) must give every rank the same parameters as a
single process stepping on the concatenated global batch (global-mean gradient, survey D9),
starting from rank 0's initial state whatever the other ranks initialised.
On the GPU the same bucket logic runs inside the captured step graph (the all-reduces forked onto a
communication stream).  The attention kernels themselves are replicas (GPU only); this checks the
collective / bucketing / optimizer path with a small CPU model.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sae_vision_amd import ops as _ops


class TinyNet(torch.nn.Module):
    def __init__(self, seed: int = 0):
        super().__init__()
        torch.manual_seed(seed)
        self.l1 = torch.nn.Linear(12, 16)
        self.l2 = torch.nn.Linear(16, 5)

    def forward(self, x, is_training: bool):
        return self.l2(torch.nn.functional.gelu(self.l1(x.flatten(1))))


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(8, 3, 4, generator=g), torch.randint(0, 5, (8,), generator=g)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from sae_vision_amd import train
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, y = _data()
    per = x.shape[0] // world
    # each rank initialises from its own seed: the step broadcasts rank 0's state at construction
    step = train.TrainStep(TinyNet(seed=rank), global_batch=x.shape[0], bucket_cap_mb=0.0001)
    # the flat gradient buffer: every .grad a view into it, buckets tile it from the end (the
    # order the backward completes the parameters), each at least the cap unless it is the last
    # every view 16-byte aligned (the in-place gradient kernels' vector stores; l2.bias has 5 elements)
    n = step._flat.numel()
    b = step._buckets
    assert b[0][1] == n and b[-1][0] == 0 and all(b[i][0] == b[i + 1][1] for i in range(len(b) - 1))
    assert len(b) > 1 and all(p.grad.data_ptr() >= step._flat.data_ptr() for p in step.model.parameters())
    assert all(p.grad.data_ptr() % 16 == 0 for p in step.model.parameters())
    # the buckets' all-reduces are launched from inside the backward, as each bucket completes
    assert step.collective == "overlap"
    launched = []
    orig = step._launch_bucket
    step._launch_bucket = lambda bi: (launched.append((bi, len(step._ready))), orig(bi))[1]
    for _ in range(3):
        step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
    # bucket 0 (the last parameters) goes out before the backward has finished every gradient
    assert launched[0][0] == 0 and launched[0][1] < len(list(step.model.parameters())), launched
    assert sorted(bi for bi, _ in launched[:len(b)]) == list(range(len(b)))
    flat = torch.cat([p.detach().flatten() for p in step.model.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        torch.save(torch.stack(gathered), out)
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_ddp_matches_single_process(tmp_path):
    from sae_vision_amd import train
    out = str(tmp_path / "params.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    assert torch.equal(got[0], got[1]), "ranks diverged"
    x, y = _data()
    ref = train.TrainStep(TinyNet(), global_batch=x.shape[0])
    for _ in range(3):
        ref(x, y)
    flat = torch.cat([p.detach().flatten() for p in ref.model.parameters()])
    torch.testing.assert_close(got[0], flat, rtol=1e-5, atol=1e-6)


def test_smoothed_cross_entropy_matches_optax_formula():
    from sae_vision_amd import train
    logits = torch.randn(4, 10, dtype=torch.float64)
    labels = torch.tensor([1, 3, 9, 0])
    y = torch.nn.functional.one_hot(labels, 10).double() * 0.9 + 0.1 / 10      # optax.smooth_labels
    ref = -(y * torch.log_softmax(logits, -1)).sum(-1).mean()
    torch.testing.assert_close(train.smoothed_cross_entropy(logits, labels, 0.1).double(), ref)


class _MixTH(torch.autograd.Function):
    """A CPU stand-in for the talking-heads op's gradient handling (ops._TalkingHeads): y = x T1 +
    x T2 with the transforms' gradients going through ops._th_sinks / _claim / _unsunk exactly as
    the HIP op's backward does (the sink written in place, the listener told via ops._sinking)."""

    @staticmethod
    def forward(ctx, x, t1, t2):
        from sae_vision_amd import ops
        ctx.save_for_backward(x, t1, t2)
        ctx.sinks = ops._th_sinks(t1, t2)
        return x @ t1 + x @ t2

    @staticmethod
    @_ops._sinking
    def backward(ctx, dy):
        from sae_vision_amd import ops
        x, t1, t2 = ctx.saved_tensors
        g = x.t() @ dy
        s1, s2 = ctx.sinks
        s1, s2 = ops._claim(s1), ops._claim(s2)
        if s1 is not None:
            s1.copy_(g)
        if s2 is not None:
            s2.copy_(g)
        return dy @ (t1 + t2).t(), ops._unsunk(g.clone(), s1), ops._unsunk(g.clone(), s2)


class AliasTHNet(torch.nn.Module):
    """One [H, H] parameter used as BOTH transforms (a shared talking-heads transform)."""

    def __init__(self, seed: int = 0):
        super().__init__()
        torch.manual_seed(seed)
        self.l1 = torch.nn.Linear(12, 8)
        self.t = torch.nn.Parameter(torch.randn(8, 8) * 0.3)
        self.l2 = torch.nn.Linear(8, 5)

    def forward(self, x, is_training: bool):
        return self.l2(_MixTH.apply(self.l1(x.flatten(1)), self.t, self.t))


def _alias_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from sae_vision_amd import train
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, y = _data()
    per = x.shape[0] // world
    step = train.TrainStep(AliasTHNet(seed=rank), global_batch=x.shape[0], bucket_cap_mb=0.0001)
    assert step.collective == "overlap"
    ti = [i for i, p in enumerate(step._params) if p is step.model.t][0]
    lo, hi = step._offs[ti], step._offs[ti] + step.model.t.numel()
    seen = []
    orig = step._launch_bucket

    def spy(bi):
        blo, bhi = step._buckets[bi]
        if blo <= lo and hi <= bhi:   # the bucket holding the shared transform: its gradient as launched
            seen.append(step._flat[lo:hi].clone())
        return orig(bi)
    step._launch_bucket = spy
    for _ in range(2):
        step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
        assert seen and torch.isfinite(seen[-1]).all()
    flat = torch.cat([p.detach().flatten() for p in step.model.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    if rank == 0:
        torch.save({"params": torch.stack(gathered)}, out)
    dist.destroy_process_group()


def test_aliased_transform_bucket_waits_for_accumulation(tmp_path):
    """a parameter fed to one op as both talking-heads transforms must not count as
    final when dT1's sink is written -- autograd still adds dT2.  With the fix neither is sunk and
    the post-accumulate hook releases the bucket; the 2-rank result equals the single process."""
    from sae_vision_amd import ops, train
    out = str(tmp_path / "alias.pt")
    mp.spawn(_alias_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    assert torch.equal(got["params"][0], got["params"][1]), "ranks diverged"
    x, y = _data()
    ref = train.TrainStep(AliasTHNet(), global_batch=x.shape[0])
    for _ in range(2):
        ref(x, y)
    flat = torch.cat([p.detach().flatten() for p in ref.model.parameters()])
    torch.testing.assert_close(got["params"][0], flat, rtol=1e-5, atol=1e-6)
    # the sink decision itself: one parameter as both transforms -> neither sunk
    p = torch.nn.Parameter(torch.zeros(4, 4))
    p.grad = torch.zeros(4, 4)
    ops.set_grad_sinks([p], [p.grad])
    ops.begin_backward_sinks()
    try:
        assert ops._th_sinks(p, p) == (None, None)
        q = torch.nn.Parameter(torch.zeros(4, 4))
        q.grad = torch.zeros(4, 4)
        ops.set_grad_sinks([q], [q.grad])
        s1, s2 = ops._th_sinks(p, q)
        assert s1 is not None and s2 is not None
    finally:
        ops.end_backward_sinks()
        ops.set_grad_sinks(None)


def _capture_fail_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from sae_vision_amd import train
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x, y = _data()
    per = x.shape[0] // world
    step = train.TrainStep(TinyNet(seed=rank), global_batch=x.shape[0], bucket_cap_mb=0.0001)
    # all ranks captured: the graph stays on everywhere
    step.graph = True
    step._flag_pg = dist.new_group(backend="gloo")
    step._settle_capture(True)
    both_ok = step.graph
    # rank 1's capture fails (injected): every rank must turn the graph off, not just rank 1
    step._settle_capture(rank != 1)
    after_fail = step.graph
    # ... and the eager steps that follow stay in lockstep (same collectives on both ranks)
    for _ in range(2):
        step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
    flat = torch.cat([p.detach().flatten() for p in step.model.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    flags = [None] * world
    dist.all_gather_object(flags, (both_ok, after_fail))
    if rank == 0:
        torch.save({"params": torch.stack(gathered), "flags": flags}, out)
    step.close()
    dist.destroy_process_group()


def test_capture_failure_on_one_rank_turns_graphs_off_everywhere(tmp_path):
    """a capture failure at world > 1 is an all-ranks decision (train.py
    TrainStep._settle_capture: MIN flag all-reduce over a gloo group), never a per-rank eager
    fallback beside peers that replay graphs."""
    from sae_vision_amd import train
    out = str(tmp_path / "capfail.pt")
    mp.spawn(_capture_fail_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    assert got["flags"] == [(True, False), (True, False)], got["flags"]
    assert torch.equal(got["params"][0], got["params"][1]), "ranks diverged"
    x, y = _data()
    ref = train.TrainStep(TinyNet(), global_batch=x.shape[0])
    for _ in range(2):
        ref(x, y)
    flat = torch.cat([p.detach().flatten() for p in ref.model.parameters()])
    torch.testing.assert_close(got["params"][0], flat, rtol=1e-5, atol=1e-6)


def test_init_distributed_connects_eagerly(monkeypatch):
    """init_distributed asks RCCL for peer connections at communicator
    creation (NCCL_RUNTIME_CONNECT=0) so the gradient group's first collective -- issued inside the
    step's graph capture -- does no connection setup there; a user's own setting wins."""
    from sae_vision_amd import train
    monkeypatch.delenv("NCCL_RUNTIME_CONNECT", raising=False)
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("SAE_DIST_BACKEND", "nccl")
    train.init_distributed()   # world 1, no SAE_WORLD1_RCCL: no process group is created
    assert os.environ.get("NCCL_RUNTIME_CONNECT") == "0"
    monkeypatch.setenv("NCCL_RUNTIME_CONNECT", "1")
    train.init_distributed()
    assert os.environ["NCCL_RUNTIME_CONNECT"] == "1"
    assert not dist.is_initialized()
