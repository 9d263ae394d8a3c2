#!/usr/bin/env python3
"""One weight-gradient shape (ops.gemm_dw: gemm_dw8 + the split reduction), launched `iters`
times (a target for rocprofv3 --pmc passes).

    python tools/probe/dw_one.py M I J [bias] [iters]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import sae_vision_amd.ops as ops
    M, I, J = (int(v) for v in sys.argv[1:4])
    bias = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    dev = torch.device("cuda:0")
    x = torch.randn(M, I, device=dev).to(torch.bfloat16)
    dy = torch.randn(M, J, device=dev).to(torch.bfloat16)
    dw = torch.empty(I, J, device=dev)
    db = torch.empty(J, device=dev) if bias else None
    for _ in range(iters):
        ops.gemm_dw(x, dy, dw, db)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.gemm_dw(x, dy, dw, db)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    print(f"gemm_dw M={M} I={I} J={J} bias={bias}: {us:.1f} us {2 * M * I * J / us / 1e6:.1f} TF/s")


if __name__ == "__main__":
    main()
