#!/usr/bin/env python3
"""One sae_gemm_nt shape, launched `iters` times (a target for rocprofv3 --pmc passes).

    python tools/probe/gemm_one.py M K N [epi] [iters]      epi: 0 none, 1 GELU, 2 GELU'
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import sae_vision_amd.ops as ops
    M, K, N = (int(v) for v in sys.argv[1:4])
    epi = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    dev = torch.device("cuda:0")
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    bt = torch.randn(N, K, device=dev).to(torch.bfloat16)
    bias = torch.randn(N, device=dev) if epi != ops.EPI_DGELU else None
    aux = torch.randn(M, N, device=dev).to(torch.bfloat16) if epi == ops.EPI_DGELU else None
    for _ in range(iters):
        ops.gemm_nt(a, bt, bias, epi, aux=aux)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.gemm_nt(a, bt, bias, epi, aux=aux)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    print(f"gemm_nt M={M} K={K} N={N} epi={epi}: {us:.1f} us {2 * M * N * K / us / 1e6:.1f} TF/s")


if __name__ == "__main__":
    main()
