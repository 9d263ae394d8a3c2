#!/usr/bin/env python3
"""Bitwise comparison of attention backward schedule variants on the development library.

    SAE_ATTN_LIB=<pkg>/libsae_attn_dev.so python tools/variant_check.py --shapes vitb384 --bwd-variants 4,5,6

Every variant must produce the same dq / dk / dv bits as the default dispatch (variant 0): the
variants re-order instructions, not arithmetic.
"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="vitb384")
    ap.add_argument("--bwd-variants", default="4")
    ap.add_argument("--fwd-variants", default="")
    args = ap.parse_args()
    import torch
    import sae_vision_amd.ops as ops
    from attn_bench import SHAPES

    dev = torch.device("cuda:0")
    bad = 0
    for shape in args.shapes.split(","):
        B, Nq, Nk, H, D = SHAPES[shape]
        g = torch.Generator(device=dev).manual_seed(1)
        q, k, v, do = (torch.randn(B, n, H, D, device=dev, generator=g).to(torch.bfloat16) for n in (Nq, Nk, Nk, Nq))
        sc = 1.0 / math.sqrt(D)

        def run(fv, bv):
            os.environ["SAE_FWD_VARIANT"], os.environ["SAE_BWD_VARIANT"] = fv, bv
            o, lse = ops._fwd(q, k, v, sc)
            dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
            ops._bwd(q, k, v, o, lse, do, dq, dk, dv, sc)
            torch.cuda.synchronize()
            return o, lse, dq, dk, dv

        ref = run("", "")
        for fv in (args.fwd_variants.split(",") if args.fwd_variants else [""]):
            for bv in (args.bwd_variants.split(",") if args.bwd_variants else [""]):
                got = run(fv, bv)
                for name, x, y in zip(("o", "lse", "dq", "dk", "dv"), ref, got):
                    same = torch.equal(x, y)
                    err = float((x.double() - y.double()).abs().max())
                    print(f"{shape} f{fv or 0} b{bv or 0} {name}: {'bitwise equal' if same else 'DIFFERS'} (max abs {err:.3g})",
                          flush=True)
                    bad += 0 if same else 1
    print("VARIANT_CHECK", "OK" if bad == 0 else f"{bad} DIFFER")


if __name__ == "__main__":
    main()
