"""Probe: what does a forked branch cost inside a replayed HIP graph?

The training step's graph forks each gradient bucket's all-reduce onto a communication stream
(comm.wait_stream(compute); kernel on comm; compute.wait_stream(comm) before AdamW).  Here a
chain of `n` GEMM kernels on the capture stream (about the length of a backward) gets `f` forks
of one tiny kernel each, spread along the chain, joined at the end; variants: no fork, forks
with no kernel (event edges only), forks of a kernel that spins for `us` microseconds on a few
workgroups, and all `f` forked kernels on the main stream instead (no fork).

    python tools/probe/graph_fork.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import sae_vision_amd.ops as ops
    dev = torch.device("cuda:0")
    a = torch.randn(4096, 1024, device=dev, dtype=torch.bfloat16)
    b = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
    main_s, comm = torch.cuda.Stream(), torch.cuda.Stream()
    n = 200

    evs = []

    def body(forks, mode, us):
        at = set(int((i + 1) * n / (forks + 1)) for i in range(forks)) if forks else set()
        x = a
        evs.clear()
        for i in range(n):
            x = (x @ b)[:, :1024]
            if i in at:
                if mode == "main":
                    ops.occupy_cus(main_s, 16, us, lds_bytes=0)
                elif mode == "extern":
                    # an event-record node on the (linear) graph; the branch runs outside the graph
                    e = torch.cuda.Event(external=True)
                    e.record(main_s)
                    evs.append(e)
                else:
                    comm.wait_stream(main_s)
                    if mode == "kernel":
                        with torch.cuda.stream(comm):
                            ops.occupy_cus(comm, 16, us, lds_bytes=0)
        if forks and mode not in ("main", "extern"):
            main_s.wait_stream(comm)
        return x

    def after(mode, us):
        # "extern": the forked kernels are launched eagerly on the comm stream after the replay is
        # enqueued, each behind its event; the main stream joins the comm stream at the end
        if mode == "extern" and evs:
            for e in evs:
                comm.wait_event(e)
                with torch.cuda.stream(comm):
                    ops.occupy_cus(comm, 16, us, lds_bytes=0)
            main_s.wait_stream(comm)

    results = []
    cases = [(0, "-", 0), (1, "kernel", 0), (4, "kernel", 0), (4, "kernel", 100), (0, "-", 0)]
    if os.environ.get("PROBE_FULL"):
        cases = [(0, "-", 0), (4, "edge", 0), (4, "kernel", 0), (4, "kernel", 100), (4, "main", 0),
                 (1, "kernel", 0), (8, "kernel", 0), (16, "kernel", 0), (0, "-", 0)]
    print("env:", {k: v for k, v in os.environ.items() if k.startswith("DEBUG_")}, flush=True)
    for forks, mode, us in cases:
        with torch.cuda.stream(main_s):
            for _ in range(2):
                body(forks, mode, us)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=main_s, capture_error_mode="thread_local"):
                body(forks, mode, us)
            for _ in range(3):
                g.replay()
                after(mode, us)
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ms = []
            for _ in range(10):
                t0.record()
                g.replay()
                after(mode, us)
                t1.record()
                t1.synchronize()
                ms.append(t0.elapsed_time(t1))
        ms.sort()
        results.append((forks, mode, us, ms[len(ms) // 2]))
        print(f"forks={forks:2d} {mode:6s} us={us:4d}: replay {ms[len(ms) // 2]:.3f} ms (min {ms[0]:.3f})", flush=True)
        del g
    base = results[0][3]
    for forks, mode, us, m in results[1:]:
        if forks:
            print(f"  {forks} x {mode} (us={us}): +{(m - base) * 1e3:.1f} us total, +{(m - base) * 1e3 / forks:.1f} us per fork")


if __name__ == "__main__":
    main()
