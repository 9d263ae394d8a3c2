"""Probe: do timing events recorded during HIP-graph capture time the replayed kernels?"""
import torch
a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
s = torch.cuda.Stream()
evs = []
with torch.cuda.stream(s):
    for _ in range(3):
        a @ a
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(4):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            b = a @ a
            e1.record()
            evs.append((e0, e1))
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
print("in-graph event ms:", [round(x.elapsed_time(y), 4) for x, y in evs])
t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0.record(); g.replay(); t1.record(); torch.cuda.synchronize()
print("whole replay ms:", round(t0.elapsed_time(t1), 4), "expected ~4 x", round(2 * 4096**3 / 1e12 / 1.0, 3), "ms at 1 PF")
