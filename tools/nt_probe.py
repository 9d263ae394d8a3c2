#!/usr/bin/env python3
"""sae_gemm_nt tile-height A/B at the projection / FF shapes, beside the library GEMM.

    SAE_ATTN_LIB=<pkg>/libsae_attn_dev.so python tools/nt_probe.py

Needs the dev library (SAE_NT_VARIANT: 1 = 128-token tiles, 2 = 256-token tiles, 3 / 4 = LDS-DMA
staging with 3 / 4 stage buffers, 0 = the release policy; NT_VARIANTS picks them, the first is the
bit-equality reference; NT_PROBE_SHAPES filters shapes).  Per shape: y = x W (fwd, bt = W^T), dX = dY W^T, and for the FF shapes the GELU
and GELU' epilogues; each variant's output is checked bit-equal to the 128-token tile's.
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
    Mb = int(os.environ.get("NT_PROBE_B384", "64")) * 577
    Ms = 128 * 197
    shapes = [  # (name, M, K, N, gelu)
        ("s_qkv", Ms, 384, 1152, False), ("s_oproj", Ms, 384, 384, False), ("s_ff1", Ms, 384, 1536, True),
        ("s_qkv_dx", Ms, 1152, 384, False), ("s_ff1_dx", Ms, 1536, 384, False),
        ("b_qkv", Mb, 768, 2304, False), ("b_ff1", Mb, 768, 3072, True),
        ("b_ff2", Mb, 3072, 768, False), ("b_qkv_dx", Mb, 2304, 768, False),
    ]
    only = os.environ.get("NT_PROBE_SHAPES")
    if only:
        shapes = [x for x in shapes if x[0] in only.split(",")]
    variants = os.environ.get("NT_VARIANTS", "1,2,0").split(",")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, m, k, n, gelu in shapes:
        a = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(k, n, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        wt = w.t().contiguous()
        dy = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16)
        f = 2.0 * m * n * k
        row = [f"{name:9s} M={m:6d} K={k:5d} N={n:5d}"]
        lib_f = bench(lambda: a @ w)
        lib_x = bench(lambda: dy @ w.t())
        row.append(f"lib fwd {f/lib_f/1e9:6.0f} dX {f/lib_x/1e9:6.0f} TF")
        outs = {}
        for var in variants:
            os.environ["SAE_NT_VARIANT"] = var
            t_f = bench(lambda: ops.gemm_nt(a, wt))
            t_x = bench(lambda: ops.gemm_nt(dy, w))
            o = (ops.gemm_nt(a, wt), ops.gemm_nt(dy, w))
            s = f"v{var} fwd {f/t_f/1e9:6.0f} dX {f/t_x/1e9:6.0f}"
            if gelu:
                bias = torch.zeros(n, device=dev)
                t_g = bench(lambda: ops.gemm_nt(a, wt, bias, ops.EPI_GELU))
                hh = torch.randn(m, n, device=dev, generator=torch.Generator(device=dev).manual_seed(1)).to(torch.bfloat16)
                t_d = bench(lambda: ops.gemm_nt(a, wt, None, ops.EPI_DGELU, aux=hh))
                o = o + (ops.gemm_nt(a, wt, bias, ops.EPI_GELU)[0], ops.gemm_nt(a, wt, None, ops.EPI_DGELU, aux=hh))
                s += f" gelu {f/t_g/1e9:6.0f} dgelu {f/t_d/1e9:6.0f}"
            outs[var] = o
            eq = all(torch.equal(x, y) for x, y in zip(o, outs[variants[0]]))
            row.append(s + ("" if eq else " MISMATCH"))
        os.environ["SAE_NT_VARIANT"] = "0"
        print(" | ".join(row), flush=True)


if __name__ == "__main__":
    main()
