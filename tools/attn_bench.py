#!/usr/bin/env python3
"""Microbenchmark of the fused attention kernels (fwd, bwd) at the BASELINE shapes.

    python tools/attn_bench.py [--iters 50] [--shapes deit_s,vitb384,...] [--dtype bf16]

Times each C-ABI call inside HIP graphs of 10 back-to-back launches (HIP events around the
replay, median over iterations, per-launch time = replay time / 10) and
prints TFLOP/s and GB/s with the algorithmic counts of SURVEY §8d.
"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {  # name: (B, Nq, Nk, H, D)
    "deit_s": (128, 197, 197, 6, 64),
    "deit_s_b256": (256, 197, 197, 6, 64),
    "vitb384": (64, 577, 577, 12, 64),
    "cait_s24": (256, 196, 196, 8, 48),
    "cait_ca": (256, 1, 197, 8, 48),
    "bot14": (256, 196, 196, 4, 128),
    "bot7": (256, 49, 49, 4, 128),
    "cvt1": (64, 3136, 784, 1, 64),
    "cait_m24": (128, 196, 196, 16, 48),
    # the per-workgroup work of a key-split single-pass backward at the ViT-B/16@384 headline
    # (same query x key products as vitb384): 3 key ranges of 192 or 2.25 of 256
    "vb_k192": (192, 577, 192, 12, 64),
    "vb_k256": (144, 577, 256, 12, 64),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", default="deit_s,vitb384,cait_s24,cait_ca,bot14,bot7")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--json", default=None)
    ap.add_argument("--th", action="store_true", help="talking-heads attention (orthogonal T1, T2)")
    ap.add_argument("--rope", action="store_true", help="fused rotary (base 10000) on q / k (--th)")
    ap.add_argument("--rel", action="store_true",
                    help="BoTNet relative logits (square Hs = Ws = sqrt(Nk) grid, N(0, 1/D) bias tables)")
    ap.add_argument("--fwd-variants", default="", help="comma list of SAE_FWD_VARIANT values to A/B (dev build: SAE_ATTN_LIB=<pkg>/libsae_attn_dev.so)")
    ap.add_argument("--bwd-variants", default="", help="comma list of SAE_BWD_VARIANT values to A/B")
    ap.add_argument("--knob", default="", help="NAME=v1,v2,...: any dev-library knob to A/B (dev build)")
    args = ap.parse_args()
    import torch
    import sae_vision_amd.ops as ops

    dev = torch.device("cuda:0")
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    elt = 2 if args.dtype == "bf16" else 4
    results = {}
    fv = args.fwd_variants.split(",") if args.fwd_variants else [os.environ.get("SAE_FWD_VARIANT", "")]
    bv = args.bwd_variants.split(",") if args.bwd_variants else [os.environ.get("SAE_BWD_VARIANT", "")]
    kname, kvals = (args.knob.split("=") + [""])[:2] if args.knob else ("", "")
    kv = kvals.split(",") if kname else [""]
    runs = [(n, f, b, x) for n in args.shapes.split(",") for f in fv for b in bv for x in kv]
    for shape, fvar, bvar, kval in runs:
        os.environ["SAE_FWD_VARIANT"], os.environ["SAE_BWD_VARIANT"] = fvar, bvar
        if kname:
            os.environ[kname] = kval
        name = shape + ("+rel" if args.rel else "") + ("+rope" if args.rope else "") + (f"@f{fvar}" if len(fv) > 1 else "") + (f"@b{bvar}" if len(bv) > 1 else "")
        name += f"@{kname}={kval}" if len(kv) > 1 else ""
        B, Nq, Nk, H, D = SHAPES[shape]
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B, Nq, H, D, device=dev, generator=g).to(dt)
        k = torch.randn(B, Nk, H, D, device=dev, generator=g).to(dt)
        v = torch.randn(B, Nk, H, D, device=dev, generator=g).to(dt)
        do = torch.randn(B, Nq, H, D, device=dev, generator=g).to(dt)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        sc = 1.0 / math.sqrt(D)
        if args.th:
            th1, th2 = (torch.linalg.qr(torch.randn(H, H, device=dev, generator=g))[0].contiguous() for _ in range(2))
            rp = 10000.0 if args.rope else None
            o, lse, _, _ = ops._th_fwd(q, k, v, th1, th2, sc, rope=rp)
            fwd_call = lambda: ops._th_fwd(q, k, v, th1, th2, sc, rope=rp)
            bwd_call = lambda: ops._th_bwd(q, k, v, th1, th2, lse, do, dq, dk, dv, sc, rope=rp)
        elif args.rel:
            hs = int(round(math.sqrt(Nk)))
            assert hs * hs == Nk and Nq == Nk, "--rel: square key grid"
            bh = torch.randn(B, H, Nq, hs, device=dev, generator=g) / math.sqrt(D)
            bw = torch.randn(B, H, Nq, hs, device=dev, generator=g) / math.sqrt(D)
            grid = (hs, hs)
            o, lse = ops._fwd(q, k, v, sc, bh, bw, grid)
            fwd_call = lambda: ops._fwd(q, k, v, sc, bh, bw, grid)
            bwd_call = lambda: ops._bwd(q, k, v, o, lse, do, dq, dk, dv, sc, bh, bw, grid)
        else:
            o, lse = ops._fwd(q, k, v, sc)
            fwd_call = lambda: ops._fwd(q, k, v, sc)
            bwd_call = lambda: ops._bwd(q, k, v, o, lse, do, dq, dk, dv, sc)
        bwd_call()
        torch.cuda.synchronize()
        # HIP graphs of `reps` back-to-back launches: no host launch gaps inside the timed region
        reps = 10
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                fwd_call()
                bwd_call()
        torch.cuda.current_stream().wait_stream(s)
        gf, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(gf):
            for _ in range(reps):
                fwd_call()
        with torch.cuda.graph(gb):
            for _ in range(reps):
                bwd_call()
        tf, tb = [], []
        for _ in range(args.iters):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            gf.replay()
            e[1].record()
            gb.replay()
            e[2].record()
            torch.cuda.synchronize()
            tf.append(e[0].elapsed_time(e[1]) / reps)
            tb.append(e[1].elapsed_time(e[2]) / reps)
        tf.sort()
        tb.sort()
        mf, mb = tf[len(tf) // 2] / 1e3, tb[len(tb) // 2] / 1e3
        ff, fb = 4.0 * B * H * Nq * Nk * D, 8.0 * B * H * Nq * Nk * D
        if args.th:   # + the two H x H head mixes: 2 x 2 H^2 Nq Nk fwd, 2 x 4 H^2 Nq Nk bwd
            ff += 4.0 * B * H * H * Nq * Nk
            fb += 8.0 * B * H * H * Nq * Nk
        bf = elt * B * H * D * (2 * Nq + 2 * Nk) + 4 * B * H * Nq
        bb = elt * B * H * D * (4 * Nq + 4 * Nk) + 8 * B * H * Nq
        r = {"fwd_us": round(mf * 1e6, 1), "bwd_us": round(mb * 1e6, 1),
             "fwd_tflops": round(ff / mf / 1e12, 1), "bwd_tflops": round(fb / mb / 1e12, 1),
             "fwdbwd_tflops": round((ff + fb) / (mf + mb) / 1e12, 1),
             "fwd_gbs": round(bf / mf / 1e9), "bwd_gbs": round(bb / mb / 1e9)}
        results[name] = r
        print(f"{name:16s} B={B:4d} Nq={Nq:5d} Nk={Nk:5d} H={H:3d} D={D:4d} | fwd {r['fwd_us']:8.1f} us "
              f"{r['fwd_tflops']:7.1f} TF {r['fwd_gbs']:6d} GB/s | bwd {r['bwd_us']:8.1f} us {r['bwd_tflops']:7.1f} TF "
              f"{r['bwd_gbs']:6d} GB/s | fwd+bwd {r['fwdbwd_tflops']:7.1f} TF", flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
