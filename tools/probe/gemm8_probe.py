#!/usr/bin/env python3
"""gemm8.h variants (tools/probe/libgemm8_probe.so) against the release sae_gemm_nt and the library
GEMM at the projection / FF shapes: correctness vs an fp32 product, TF/s (events around 20 launches).

    python tools/probe/gemm8_probe.py [variants=0,1,2,...] [shapes=s_qkv,...]
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
LIB = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgemm8_probe.so"))
LIB.g8_run.restype = ctypes.c_int
LIB.g8_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                       ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p,
                       ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
# variant % 10: tile / stage depth / ring; variant >= 10: persistent grid of 256 workgroups
NAMES = {0: "256x256 bk32 ns3", 1: "256x192 bk32 ns3", 2: "256x192 bk32 ns4", 3: "256x192 bk64 ns2",
         4: "256x128 bk32 ns4", 5: "256x128 bk64 ns2"}
# 40-45: gemm8x ping-pong (43 = 256 x 256 BAL, 45 = 224 x 256 BAL); 50 / 51 / 53: persistent 224 x 256 bk32 ns3,
# 192 x 192 bk64 ns2, 224 x 192 bk64 ns2 (tile heights that fill 256 CUs at M = 25,216 / 18,464)


def bench(fn, iters=40):
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


def run(var, a, bt, c, epi=0, bias=None, aux=None, c2=None):
    st = torch.cuda.current_stream().cuda_stream
    M, K = a.shape
    N = bt.shape[0]
    rc = LIB.g8_run(var, st, M, N, K, a.data_ptr(), a.stride(0), bt.data_ptr(), bt.stride(0),
                    bias.data_ptr() if bias is not None else None, c.data_ptr(), c.stride(0), epi,
                    aux.data_ptr() if aux is not None else None, aux.stride(0) if aux is not None else 0,
                    c2.data_ptr() if c2 is not None else None)
    if rc:
        raise RuntimeError(f"g8_run rc {rc}")


def main():
    import sae_vision_amd.ops as ops
    args = dict(x.split("=") for x in sys.argv[1:])
    variants = [int(v) for v in args.get("variants", "0,1,2,3,4,5,10,11,12,13,14,15").split(",")]
    dev = torch.device("cuda:0")
    Ms, Mb = 128 * 197, 32 * 577
    shapes = [  # name, M, K, N, epi
        ("s_qkv", Ms, 384, 1152, 0), ("s_oproj", Ms, 384, 384, 0), ("s_ff1", Ms, 384, 1536, 1),
        ("s_ff2", Ms, 1536, 384, 0), ("s_ff1dx", Ms, 384, 1536, 2), ("s_qkvdx", Ms, 1152, 384, 0),
        ("b_qkv", Mb, 768, 2304, 0), ("b_ff1", Mb, 768, 3072, 1), ("b_ff2", Mb, 3072, 768, 0),
        ("b_qkvdx", Mb, 2304, 768, 0), ("b_oproj", Mb, 768, 768, 0), ("b_ff1dx", Mb, 768, 3072, 2),
        ("big", 4096, 4096, 4096, 0),
    ]
    if "shapes" in args:
        shapes = [s for s in shapes if s[0] in args["shapes"].split(",")]
    g = torch.Generator(device=dev).manual_seed(0)
    for name, M, K, N, epi in shapes:
        a = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        bt = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(torch.bfloat16)
        bias = torch.randn(N, device=dev, generator=g) * 0.1 if epi != 2 else None
        aux = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16) if epi == 2 else None
        ref = a.float() @ bt.float().t()
        if bias is not None:
            ref = ref + bias
        f = 2.0 * M * N * K
        row = [f"{name:8s} M={M:6d} K={K:5d} N={N:5d} epi={epi}"]
        c_rel = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if epi == 0:
            t = bench(lambda: ops.gemm_nt(a, bt, bias))
            t_lib = bench(lambda: torch.addmm(bias.to(torch.bfloat16), a, bt.t()))
            row.append(f"rel {f / t / 1e9:5.0f} lib {f / t_lib / 1e9:5.0f}")
        elif epi == 1:
            t = bench(lambda: ops.gemm_nt(a, bt, bias, ops.EPI_GELU))
            row.append(f"rel {f / t / 1e9:5.0f}")
        else:
            t = bench(lambda: ops.gemm_nt(a, bt, None, ops.EPI_DGELU, aux=aux))
            row.append(f"rel {f / t / 1e9:5.0f}")
        for v in variants:
            c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            c2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if epi == 1 else None
            try:
                run(v, a, bt, c, epi, bias, aux, c2)
            except RuntimeError as e:
                row.append(f"v{v} ERR {e}")
                continue
            torch.cuda.synchronize()
            h = (c2 if epi == 1 else c).float()
            if epi == 2:
                # c = bf16(bf16(acc) * gelu'(aux))
                want = ops.gemm_nt(a, bt, None, ops.EPI_DGELU, aux=aux).float()
                err = float((c.float() - want).abs().max() / want.abs().max())
            else:
                err = float((h - ref).abs().max() / ref.abs().max())
                if epi == 1:
                    g1 = ops.gemm_nt(a, bt, bias, ops.EPI_GELU)[0].float()
                    err = max(err, float((c.float() - g1).abs().max() / g1.abs().max()))
            tv = bench(lambda: run(v, a, bt, c, epi, bias, aux, c2))
            row.append(f"v{v} {f / tv / 1e9:5.0f}{' BAD %.1e' % err if err > 2e-2 else ''}")
        print(" | ".join(row), flush=True)


if __name__ == "__main__":
    main()
