#!/usr/bin/env python3
"""Projection GEMM throughput at the DeiT-S / ViT-B training shapes: the library GEMM
(torch.matmul -> hipBLASLt) for y = x W, dX = dY W^T, dW = X^T dY, next to this repo's
split-token weight-gradient kernel (sae_gemm_dw, fp32 out + fused bias sum).

    python tools/gemm_probe.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


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
    import sae_vision_amd.ops as ops
    dev = torch.device("cuda:0")
    M = 128 * 197
    shapes = [  # (name, M, K, N)
        ("qkv", M, 384, 1152), ("oproj", M, 384, 384), ("ff1", M, 384, 1536), ("ff2", M, 1536, 384),
        ("qkv_dx", M, 1152, 384),
        ("b384_qkv", 32 * 577, 768, 2304), ("b384_ff1", 32 * 577, 768, 3072), ("b384_ff2", 32 * 577, 3072, 768),
    ]
    for name, m, k, n in shapes:
        a = torch.randn(m, k, device=dev).to(torch.bfloat16)
        b = torch.randn(k, n, device=dev).to(torch.bfloat16)
        dy = torch.randn(m, n, device=dev).to(torch.bfloat16)
        dw = torch.empty(k, n, device=dev)
        db = torch.empty(n, device=dev)
        ms = bench(lambda: a @ b)
        ms_x = bench(lambda: dy @ b.t())
        ms_w = bench(lambda: a.t() @ dy)
        ms_h = bench(lambda: ops.gemm_dw(a, dy, dw, db))
        bt = b.t().contiguous()
        ms_nt = bench(lambda: ops.gemm_nt(a, bt))
        ms_ntx = bench(lambda: ops.gemm_nt(dy, b))
        f = 2.0 * m * n * k
        print(f"{name:9s} sae_gemm_nt fwd {ms_nt*1e3:7.1f} us {f/ms_nt/1e9:7.1f} TF | dX {ms_ntx*1e3:7.1f} us "
              f"{f/ms_ntx/1e9:7.1f} TF", flush=True)
        if n == 4 * k:   # FF Dense_0: GEMM + GELU (library + torch elementwise) vs the fused epilogue
            bias = torch.zeros(n, device=dev)
            hh = torch.randn(m, n, device=dev).to(torch.bfloat16)
            ms_lg = bench(lambda: torch.nn.functional.gelu(torch.addmm(bias.to(torch.bfloat16), a, b), approximate="tanh"))
            ms_ng = bench(lambda: ops.gemm_nt(a, bt, bias, ops.EPI_GELU))
            dyk = torch.randn(m, k, device=dev).to(torch.bfloat16)
            bk = torch.randn(n, k, device=dev).to(torch.bfloat16)   # Dense_1 kernel [hid, out]
            ms_ld = bench(lambda: torch.ops.aten.gelu_backward(dyk @ bk.t(), hh, approximate="tanh"))
            ms_nd = bench(lambda: ops.gemm_nt(dyk, bk, None, ops.EPI_DGELU, aux=hh))
            print(f"{name:9s} Dense_0+GELU lib {ms_lg*1e3:7.1f} us fused {ms_ng*1e3:7.1f} us | "
                  f"Dense_1 dX+GELU' lib {ms_ld*1e3:7.1f} us fused {ms_nd*1e3:7.1f} us", flush=True)
        print(f"{name:9s} M={m:6d} K={k:5d} N={n:5d} | fwd {ms*1e3:7.1f} us {f/ms/1e9:7.1f} TF | dX {ms_x*1e3:7.1f} us "
              f"{f/ms_x/1e9:7.1f} TF | dW lib {ms_w*1e3:7.1f} us {f/ms_w/1e9:7.1f} TF | dW+db hip {ms_h*1e3:7.1f} us "
              f"{f/ms_h/1e9:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
