#!/usr/bin/env python3
"""Same-process A/B of a dev-library knob on the graph-replayed training step
(cdna_hip_programming.md section 5.4 rule 24): one TrainStep(graph=True) per variant, each captured
with its environment knob set (the C-ABI reads dev knobs at launch, i.e. at capture), replays
interleaved over rounds; median ms/step.

    SAE_ATTN_LIB=<pkg>/libsae_attn_dev.so python tools/ab_knob.py KNOB=v1 [KNOB=v2 ...] [--model m]
    e.g. python tools/ab_knob.py SAE_NT_NO_G8=1 SAE_NT_NO_G8=0
         python tools/ab_knob.py ops.GEMM_LIB_WIDE=1 ops.GEMM_LIB_WIDE=0   (module flags of ops)
"""
import argparse
import copy
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--model", default="deit_s_patch16")
    ap.add_argument("--img-size", type=int, default=224)
    a = ap.parse_args()
    import torch
    from sae_vision_amd import cait, train, vit
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    if a.model.startswith("cait"):
        base = cait.create_cait(a.model, 1000, torch.bfloat16, device=dev)
    else:
        base = vit.create_model(a.model, 1000, torch.bfloat16, img_size=a.img_size, device=dev)
    g = torch.Generator(device=dev).manual_seed(1234)
    images = torch.randn(a.batch, a.img_size, a.img_size, 3, device=dev, generator=g)
    labels = torch.randint(0, 1000, (a.batch,), device=dev, generator=g)
    steps = {}
    from sae_vision_amd import ops
    for v in a.variants:
        k, val = v.split("=")
        if k.startswith("ops."):   # a module flag of ops (routing decisions are taken at capture)
            old = getattr(ops, k[4:])
            setattr(ops, k[4:], type(old)(int(val)) if isinstance(old, bool) else type(old)(val))
        else:
            os.environ[k] = val
        s = train.TrainStep(copy.deepcopy(base), global_batch=a.batch, device=dev, graph=True)
        s(images, labels)        # capture under this knob
        if k.startswith("ops."):
            setattr(ops, k[4:], old)
        else:
            os.environ.pop(k)
        steps[v] = s
    torch.cuda.synchronize()
    res = {v: [] for v in steps}
    for _ in range(a.rounds):
        for v, s in steps.items():
            s(images, labels)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                s(images, labels)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / a.steps * 1e3)
    for v in steps:
        print(f"{a.model} {v:24s} ms/step median {statistics.median(res[v]):7.3f} min {min(res[v]):7.3f} "
              f"img/s {a.batch / statistics.median(res[v]) * 1e3:8.1f}", flush=True)


if __name__ == "__main__":
    main()
