#!/usr/bin/env python3
"""Where a kernel's cycles go: in-kernel s_memtime stamps of the attention kernels.

    SAE_ATTN_LIB=<pkg>/libsae_attn_stamp.so python tools/stamps.py --shapes deit_s,vitb384

Needs the diagnostic build (``python build.py --stamps``): lane 0 of every wave stores the shader
clock at fixed points (slot 0 = entry, 1 = prologue done, 2.. = after each tile's barrier, 30 =
loop done, 31 = exit; bwd3: 1 / 2 = the two prologue barriers, 3.. = the query tiles).  The
dQ pass of the two-pass backward records at block offset 4096.  Prints, per kernel launch, the
phase medians of wave 0 in cycles and the dispatch profile (how many blocks start per round).
"""
import argparse
import ctypes
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

SLOTS, WAVES, RECS = 32, 16, 1 << 22


def read(lib):
    buf = np.zeros(RECS, dtype=np.uint64)
    rc = lib.sae_dev_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes), 0)
    assert rc == 0
    return buf.reshape(-1, WAVES, SLOTS)


def clear(lib):
    assert lib.sae_dev_stamps(None, ctypes.c_size_t(0), 1) == 0


def report(name, st, blocks, boff=0, nwaves=4):
    s = st[boff:boff + blocks].astype(np.int64)
    w0 = s[:, 0, :]
    ok = w0[:, 0] > 0
    w0 = w0[ok]
    if len(w0) == 0:
        print(f"{name}: no stamps")
        return
    t0 = w0[:, 0].min()
    start = w0[:, 0] - t0
    end = w0[:, 31] - t0
    dur = w0[:, 31] - w0[:, 0]
    rt = (w0[:, 29] - w0[:, 28]).astype(np.float64)
    clk = np.median(dur / np.maximum(rt, 1) * 100.0)   # MHz
    print(f"== {name}: {len(w0)} blocks, in-kernel clock {clk:.0f} MHz")
    print(f"   block life median {np.median(dur):.0f} cyc (p10 {np.percentile(dur, 10):.0f}, p90 {np.percentile(dur, 90):.0f})")
    # phases
    used = [k for k in list(range(1, 28)) + [30] if (w0[:, k] > 0).mean() > 0.5]
    prev = 0
    out = []
    for k in used:
        m = w0[:, k] > 0
        d = w0[m, k] - w0[m, prev if (w0[m, prev] > 0).all() else 0]
        out.append(f"{prev}->{k}:{np.median(d):.0f}")
        prev = k
    d = w0[:, 31] - w0[:, prev]
    out.append(f"{prev}->31:{np.median(d):.0f}")
    print("   phases (median cyc): " + " ".join(out))
    # (s_memtime is not synchronised across XCDs: start offsets are only meaningful within one XCD)
    # wave skew inside a block: end of the loop (slot 30) across waves
    sk = []
    for wv in range(1, nwaves):
        a = s[ok, wv, 30]
        m = a > 0
        if m.any():
            sk.append(np.median(np.abs(a[m] - s[ok][m, 0, 30])))
    if sk:
        print(f"   wave skew at loop end (median |w - w0| cyc): {' '.join(f'{x:.0f}' for x in sk)}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="deit_s,vitb384")
    args = ap.parse_args()
    import torch
    import sae_vision_amd.ops as ops
    import sae_vision_amd._lib as L
    from attn_bench import SHAPES

    lib = L.load()
    lib.sae_dev_stamps.restype = ctypes.c_int32
    lib.sae_dev_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32]
    dev = torch.device("cuda:0")
    for shape in args.shapes.split(","):
        B, Nq, Nk, H, D = SHAPES[shape]
        g = torch.Generator(device=dev).manual_seed(0)
        dt = torch.bfloat16
        q, k, v, do = (torch.randn(B, n, H, D, device=dev, generator=g).to(dt) for n in (Nq, Nk, Nk, Nq))
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        sc = 1.0 / math.sqrt(D)
        for _ in range(20):
            o, lse = ops._fwd(q, k, v, sc)
            ops._bwd(q, k, v, o, lse, do, dq, dk, dv, sc)
        torch.cuda.synchronize()
        clear(lib)
        torch.cuda.synchronize()
        o, lse = ops._fwd(q, k, v, sc)
        torch.cuda.synchronize()
        st = read(lib)
        nqb = (Nq + 127) // 128
        report(f"{shape} fwd2", st, nqb * B * H)
        clear(lib)
        torch.cuda.synchronize()
        ops._bwd(q, k, v, o, lse, do, dq, dk, dv, sc)
        torch.cuda.synchronize()
        st = read(lib)
        if Nk <= 256:
            report(f"{shape} bwd3", st, B * H, nwaves=8)
        else:
            report(f"{shape} bwd2 dq", st, nqb * B * H, boff=4096)
            report(f"{shape} bwd2 dkdv", st, ((Nk + 127) // 128) * B * H)


if __name__ == "__main__":
    main()
