#!/usr/bin/env python3
"""Per-shape A/B of sae_gemm_nt dev-knob variants at the DeiT-S / ViT-B step shapes.

    SAE_ATTN_LIB=<pkg>/libsae_attn_dev.so python tools/g8_shape_ab.py KNOB=v1,v2,... [--iters 20]

Each (shape, knob value) is timed as a HIP graph of 10 back-to-back calls (HIP events around the
replay, median of `iters` replays), values interleaved per shape so box drift hits all equally.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

M = 128 * 197
SHAPES = [  # (name, M, K, N, epilogue)
    ("qkv", M, 384, 1152, 0), ("oproj", M, 384, 384, 0), ("ff0_gelu", M, 384, 1536, 3), ("ff1", M, 1536, 384, 0),
    ("qkv_dx", M, 1152, 384, 0), ("ff0_dx", M, 1536, 384, 0), ("ff1_dx_mul", M, 384, 1536, 4),
    ("b384_qkv", 32 * 577, 768, 2304, 0),
]


def main():
    import sae_vision_amd.ops as ops
    knob, vals = sys.argv[1].split("=")
    vals = vals.split(",")
    iters = int(sys.argv[sys.argv.index("--iters") + 1]) if "--iters" in sys.argv else 20
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    s = torch.cuda.Stream(device=dev)
    for name, m, k, n, epi in SHAPES:
        a = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        bt = (torch.randn(n, k, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        bias = torch.randn(n, device=dev, generator=g) if epi != 4 else None
        aux = torch.randn(m, n, device=dev, generator=g).to(torch.bfloat16) if epi == 4 else None
        flop = 2.0 * m * n * k
        res = {}
        for rep in range(2):
            for v in vals:
                os.environ[knob] = v
                with torch.cuda.stream(s):
                    for _ in range(2):
                        ops.gemm_nt(a, bt, bias, epi, aux=aux)
                    torch.cuda.synchronize()
                    gr = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gr, stream=s):
                        for _ in range(10):
                            ops.gemm_nt(a, bt, bias, epi, aux=aux)
                    ts = []
                    for _ in range(iters):
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(s)
                        gr.replay()
                        e1.record(s)
                        e1.synchronize()
                        ts.append(e0.elapsed_time(e1) * 100.0)   # us per call
                ts.sort()
                res.setdefault(v, []).append(ts[len(ts) // 2])
                del gr
        line = "  ".join(f"{knob}={v}: {min(res[v]):7.1f} us {flop / min(res[v]) / 1e6:6.0f} TF" for v in vals)
        print(f"{name:12s} M={m:6d} K={k:5d} N={n:5d} | {line}", flush=True)


if __name__ == "__main__":
    main()
