#!/usr/bin/env python3
"""sae_gemm_f32 beside the library fp32 GEMM at the fp32 projection shapes (forward, input
gradient, weight gradient + db), CUDA-event timed, TF/s against the 157.3 TF f32 MFMA peak."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sae_vision_amd.ops as ops  # noqa: E402

SHAPES = [  # (name, tokens, in, out)
    ("s_qkv", 25216, 384, 1152),
    ("s_oproj", 25216, 384, 384),
    ("s_ff1", 25216, 384, 1536),
    ("s_ff2", 25216, 1536, 384),
    ("b_oproj", 18464, 768, 768),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    dev = torch.device("cuda", 0)
    for name, T, I, J in SHAPES:
        x = torch.randn(T, I, device=dev)
        w = torch.randn(I, J, device=dev) / I ** 0.5
        b = torch.randn(J, device=dev)
        dy = torch.randn(T, J, device=dev)
        db = torch.empty(J, device=dev)
        f = 2.0 * T * I * J
        row = [f"{name:8s} T={T:6d} I={I:5d} J={J:5d} |"]
        for lab, ours, lib in (
                ("fwd", lambda: ops.gemm_f32(x, w, b), lambda: torch.addmm(b, x, w)),
                ("dx", lambda: ops.gemm_f32(dy, w.t()), lambda: dy @ w.t()),
                ("dw", lambda: ops.gemm_f32(x.t(), dy, colsum=db), lambda: (x.t() @ dy, dy.sum(0)))):
            t0, t1 = timeit(ours), timeit(lib)
            row.append(f"{lab} {t0 * 1e6:7.1f} us {f / t0 / 1e12:6.1f} TF (lib {f / t1 / 1e12:6.1f}) |")
        print(" ".join(row), flush=True)


if __name__ == "__main__":
    main()
