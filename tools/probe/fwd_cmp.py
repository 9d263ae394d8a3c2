#!/usr/bin/env python3
"""Forward variants of the dev library against a float64 reference (max |o - ref| / max |ref|, lse
max abs error), several shapes incl. ragged ones.  SAE_ATTN_LIB=<pkg>/libsae_attn_dev.so."""
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
    shapes = [(2, 577, 577, 12, 64), (4, 197, 197, 6, 64), (3, 196, 196, 8, 48), (2, 65, 65, 2, 64),
              (2, 33, 33, 2, 64), (2, 17, 17, 3, 64), (1, 300, 128, 2, 64), (1, 64, 64, 1, 64), (1, 128, 129, 1, 64)]
    for B, Nq, Nk, H, D in shapes:
        g = torch.Generator(device=dev).manual_seed(Nq + Nk)
        q, k, v = (torch.randn(B, n, H, D, device=dev, generator=g).to(torch.bfloat16) for n in (Nq, Nk, Nk))
        sc = 1.0 / math.sqrt(D)
        s = torch.einsum("bqhd,bkhd->bhqk", q.double(), k.double()) * sc
        ref = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), v.double())
        lref = torch.logsumexp(s, -1)
        line = f"B{B} Nq{Nq} Nk{Nk} H{H} D{D}:"
        for var in variants:
            os.environ["SAE_FWD_VARIANT"] = var
            o, lse = ops._fwd(q, k, v, sc)
            torch.cuda.synchronize()
            e = float((o.double() - ref).abs().max() / ref.abs().max())
            el = float((lse.double().view(B, H, Nq) - lref).abs().max())
            line += f"  [{var or 'def'}] o {e:.2e} lse {el:.2e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
