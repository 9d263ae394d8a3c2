#!/usr/bin/env python3
"""Per-workgroup timeline of the attention kernels (diagnostic build knob SAE_DBG & 64).

    python tools/wg_timeline.py --shape vitb384 --which fwd|bwd [--variant N]

Each workgroup's thread 0 stamps s_memrealtime (100 MHz) at kernel entry (0), after the
prologue barrier (1), after the tile loop (2) and after the epilogue (3), plus HW_ID / XCC_ID.
Prints the kernel span, workgroup lifetime percentiles, the prologue / loop / epilogue shares
and how many workgroups were resident per CU on average.  Only SHARES are meaningful (the
stamps themselves perturb timing).
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
    ap.add_argument("--shape", default="vitb384")
    ap.add_argument("--which", default="fwd")
    ap.add_argument("--dbg", type=int, default=0)
    args = ap.parse_args()
    import numpy as np
    import torch
    import sae_vision_amd.ops as ops
    from attn_bench import SHAPES

    B, Nq, Nk, H, D = SHAPES[args.shape]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    q, k, v, do = (torch.randn(B, n, H, D, device=dev, generator=g).to(torch.bfloat16) for n in (Nq, Nk, Nk, Nq))
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    sc = 1.0 / math.sqrt(D)
    o, lse = ops._fwd(q, k, v, sc)
    for _ in range(3):
        ops._fwd(q, k, v, sc)
        ops._bwd(q, k, v, o, lse, do, dq, dk, dv, sc)
    buf = torch.zeros(1 << 20, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    os.environ["SAE_DBG"] = str(64 | args.dbg)
    os.environ["SAE_DBG_BUF"] = "%x" % buf.data_ptr()
    if args.which == "fwd":
        ops._fwd(q, k, v, sc)
    else:
        ops._bwd(q, k, v, o, lse, do, dq, dk, dv, sc)
    torch.cuda.synchronize()
    del os.environ["SAE_DBG"], os.environ["SAE_DBG_BUF"]
    a = buf.cpu().numpy().reshape(-1, 8)
    n = int((a[:, 0] != 0).sum())
    a = a[:n].astype(np.float64)
    t0 = a[:, 0].min()
    ts = (a[:, :4] - t0) / 100.0   # microseconds
    span = ts[:, 3].max()
    life = ts[:, 3] - ts[:, 0]
    pro = ts[:, 1] - ts[:, 0]
    loop = ts[:, 2] - ts[:, 1]
    epi = ts[:, 3] - ts[:, 2]
    hw = a[:, 6].astype(np.int64)
    cu = ((a[:, 7].astype(np.int64) & 0xF) << 8) | ((hw >> 8) & 0xF) | (((hw >> 13) & 0x7) << 4)
    ncu = len(set(cu.tolist()))
    resident = life.sum() / (span * ncu)
    pct = lambda x: " ".join(f"{np.percentile(x, p):7.2f}" for p in (5, 50, 95))
    print(f"{args.which} {args.shape}: {n} workgroups on {ncu} CU ids, span {span:.1f} us, "
          f"mean resident workgroups per CU {resident:.2f}")
    print(f"  lifetime us p5/p50/p95 {pct(life)}")
    print(f"  prologue us           {pct(pro)}   share {pro.sum() / life.sum():.3f}")
    print(f"  loop us               {pct(loop)}   share {loop.sum() / life.sum():.3f}")
    print(f"  epilogue us           {pct(epi)}   share {epi.sum() / life.sum():.3f}")
    starts = np.sort(ts[:, 0])
    print(f"  start times p0/p25/p50/p75/p100 " + " ".join(f"{np.percentile(starts, p):7.1f}" for p in (0, 25, 50, 75, 100)))


if __name__ == "__main__":
    main()
