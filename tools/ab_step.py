#!/usr/bin/env python3
"""A/B of the DeiT-S/16 training step inside ONE process (cdna_hip_programming.md §5.4 rule 24):
variants interleaved over several rounds, median ms/step each, plus the host-side submission time
of a step (perf_counter around the step without a sync) to show whether the step is launch-bound.

    python tools/ab_step.py [--rounds 4] [--steps 10]
Variants: ``fused`` (HIP FF block: GELU / GELU' in the GEMM epilogues), ``lib`` (library GEMMs +
torch GELU), ``graph`` (fused, the whole step replayed as one HIP graph).
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--model", default="deit_s_patch16")
    a = ap.parse_args()
    import torch
    from sae_vision_amd import ops, train, vit
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = vit.create_model(a.model, 1000, torch.bfloat16, device=dev)
    step_e = train.TrainStep(model, global_batch=a.batch, device=dev)
    step_g = train.TrainStep(model, global_batch=a.batch, device=dev, graph=True)
    g = torch.Generator(device=dev).manual_seed(1234)
    images = torch.randn(a.batch, 224, 224, 3, device=dev, generator=g)
    labels = torch.randint(0, 1000, (a.batch,), device=dev, generator=g)
    variants = {"fused": (True, step_e), "lib": (False, step_e), "graph": (True, step_g)}
    res = {k: [] for k in variants}
    host = {k: [] for k in variants}
    for k, (v, step) in variants.items():   # warm every path
        ops.FF_FUSED = v
        for _ in range(3):
            step(images, labels)
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for k, (v, step) in variants.items():
            ops.FF_FUSED = v
            step(images, labels)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hs = 0.0
            for _ in range(a.steps):
                h0 = time.perf_counter()
                step(images, labels)
                hs += time.perf_counter() - h0
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / a.steps * 1e3)
            host[k].append(hs / a.steps * 1e3)
    for k in variants:
        print(f"{k:6s} ms/step median {statistics.median(res[k]):7.3f} min {min(res[k]):7.3f} "
              f"img/s {a.batch / statistics.median(res[k]) * 1e3:8.1f} | host submit ms/step "
              f"{statistics.median(host[k]):6.3f}", flush=True)


if __name__ == "__main__":
    main()
