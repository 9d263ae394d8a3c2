"""Probe: can a world-size-1 RCCL (backend 'nccl') all-reduce be captured into a HIP graph on a
side stream (fork/join with the compute stream), and does the replay give the right values?"""
import os
import sys
import time

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1)
print("backend", dist.get_backend(), "nccl version", torch.cuda.nccl.version(), flush=True)
x = torch.randn(1 << 20, device=dev)
# eager warm-up (communicator init)
dist.all_reduce(x)
torch.cuda.synchronize()
buf = torch.zeros(8 << 20, device=dev)
src = torch.randn(8 << 20, device=dev)
comm = torch.cuda.Stream(device=dev)
g = torch.cuda.CUDAGraph()
cur = torch.cuda.current_stream()
s = torch.cuda.Stream(device=dev)
s.wait_stream(cur)
with torch.cuda.stream(s):
    buf.copy_(src); buf.mul_(2.0)
    comm.wait_stream(s); 
    with torch.cuda.stream(comm):
        dist.all_reduce(buf[: 4 << 20])
    buf[4 << 20:].add_(1.0)
    s.wait_stream(comm)
cur.wait_stream(s)
torch.cuda.synchronize()
try:
    with torch.cuda.graph(g):
        buf.copy_(src)
        buf.mul_(2.0)
        comm.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(comm):
            w = dist.all_reduce(buf[: 4 << 20], async_op=False)
        buf[4 << 20:].add_(1.0)
        torch.cuda.current_stream().wait_stream(comm)
        out = buf.sum()
    print("captured", flush=True)
except Exception as e:
    print("CAPTURE FAILED:", repr(e), flush=True)
    sys.exit(3)
src.normal_()
g.replay()
torch.cuda.synchronize()
ref = torch.cat([src[: 4 << 20] * 2, src[4 << 20:] * 2 + 1])
print("max err", float((buf - ref).abs().max()), "sum", float(out), float(ref.sum()), flush=True)
t0 = time.perf_counter()
for _ in range(20):
    g.replay()
torch.cuda.synchronize()
print("replay us", (time.perf_counter() - t0) / 20 * 1e6, flush=True)
dist.destroy_process_group()
print("OK", flush=True)
