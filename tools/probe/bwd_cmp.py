#!/usr/bin/env python3
"""Backward variants of the dev library against float64 autograd (max |g - ref| / max |ref| for dq,
dk, dv), key ranges > 256 (the two-pass / bwd5 path).  SAE_ATTN_LIB=<pkg>/libsae_attn_dev.so."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import sae_vision_amd.ops as ops
    variants = sys.argv[1].split(",") if len(sys.argv) > 1 else [""]
    dev = torch.device("cuda:0")
    shapes = [(2, 577, 577, 12, 64), (1, 300, 300, 2, 64), (1, 257, 257, 3, 64), (2, 577, 577, 4, 48),
              (1, 1000, 700, 2, 64), (1, 400, 320, 2, 64)]
    for B, Nq, Nk, H, D in shapes:
        g = torch.Generator(device=dev).manual_seed(Nq * 7 + Nk)
        q, k, v, do = (torch.randn(B, n, H, D, device=dev, generator=g).to(torch.bfloat16) for n in (Nq, Nk, Nk, Nq))
        sc = 1.0 / math.sqrt(D)
        qd, kd, vd = (t.double().requires_grad_(True) for t in (q, k, v))
        s = torch.einsum("bqhd,bkhd->bhqk", qd, kd) * sc
        o = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), vd)
        o.backward(do.double())
        os.environ["SAE_FWD_VARIANT"] = ""
        of, lse = ops._fwd(q, k, v, sc)
        line = f"B{B} Nq{Nq} Nk{Nk} H{H} D{D}:"
        outs = {}
        for var in variants:
            os.environ["SAE_BWD_VARIANT"] = var
            dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
            ops._bwd(q, k, v, of, lse, do, dq, dk, dv, sc)
            torch.cuda.synchronize()
            errs = [float((x.double() - r.grad).abs().max() / r.grad.abs().max()) for x, r in ((dq, qd), (dk, kd), (dv, vd))]
            outs[var] = (dq, dk, dv)
            line += f"  [{var or 'def'}] " + " ".join(f"{e:.1e}" for e in errs)
        ref = outs[variants[0]]
        same = {var: all(torch.equal(a_, b_) for a_, b_ in zip(outs[var], ref)) for var in variants[1:]}
        print(line, "| bit-equal to first:", same, flush=True)


if __name__ == "__main__":
    main()
