#!/usr/bin/env python3
"""Probe library GEMM (torch.matmul -> hipBLASLt) throughput at the DeiT-S / ViT-B training shapes.

    python tools/gemm_probe.py
"""
import torch


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    dev = torch.device("cuda:0")
    M = 128 * 197
    shapes = [  # (name, M, K, N)
        ("qkv_fwd", M, 384, 1152), ("oproj_fwd", M, 384, 384), ("ff1_fwd", M, 384, 1536), ("ff2_fwd", M, 1536, 384),
        ("square8k", 8192, 8192, 8192), ("square4k", 4096, 4096, 4096),
        ("b384_ff1", 32 * 577, 768, 3072), ("b384_ff2", 32 * 577, 3072, 768),
    ]
    for name, m, k, n in shapes:
        a = torch.randn(m, k, device=dev).to(torch.bfloat16)
        b = torch.randn(k, n, device=dev).to(torch.bfloat16)
        ms = bench(lambda: a @ b)
        # weight gradient orientation: a^T @ dy  ([k, m] x [m, n])
        dy = torch.randn(m, n, device=dev).to(torch.bfloat16)
        ms_w = bench(lambda: a.t() @ dy)
        ms_x = bench(lambda: dy @ b.t())
        f = 2.0 * m * n * k
        print(f"{name:10s} M={m:6d} K={k:5d} N={n:5d}  fwd {ms*1e3:8.1f} us {f/ms/1e9:7.1f} TF | "
              f"dW {ms_w*1e3:8.1f} us {f/ms_w/1e9:7.1f} TF | dX {ms_x*1e3:8.1f} us {f/ms_x/1e9:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
