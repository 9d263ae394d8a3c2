"""Multi-process data-parallel path on CPU (gloo, world size 2).

The training step (sae_vision_amd.train.TrainStep, the rebuild of the reference's
pmap(train_step) + lax.pmean(grads), train.py:94-96,230: flat gradient buffer, bucketed SUM
all-reduce of the gradients of loss / world) must give every rank the same parameters as a
single process stepping on the concatenated global batch (global-mean gradient, survey D9),
starting from rank 0's initial state whatever the other ranks initialised.
The GPU step runs the same code between its two HIP graphs.  The attention kernels themselves are replicas (GPU only); this checks the
collective / bucketing / optimizer path with a small CPU model.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


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
