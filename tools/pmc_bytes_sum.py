#!/usr/bin/env python3
"""Summarise tools/pmc_bytes.sh output: per kernel, average per dispatch, the gfx950 request-size
read bytes (32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B) beside the FETCH_SIZE-style figure
(64 B per TCC_EA0_RDREQ, the guide's x2 correction applied = 128 B per request), plus L2 hit rate.

    python tools/pmc_bytes_sum.py <outdir> [kernel-substring ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(outdir):
    per = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [values per dispatch]
    for f in sorted(glob.glob(os.path.join(outdir, "pass*", "**", "*counter_collection.csv"), recursive=True)):
        acc = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in acc.items():
            per[names[d]][c].append(v)
    return per


def main(outdir, subs):
    per = load(outdir)
    print(f"{'kernel':60s} {'n':>4s} {'RDREQ':>10s} {'32B':>9s} {'64B':>9s} {'128B':>9s} "
          f"{'exact_MB':>9s} {'x2_MB':>8s} {'ratio':>6s} {'L2hit':>6s} {'wr_MB':>7s}")
    for k, c in sorted(per.items(), key=lambda kv: -sum(kv[1].get("TCC_EA0_RDREQ_sum", [0]))):
        if subs and not any(s in k for s in subs):
            continue
        avg = {n: sum(v) / len(v) for n, v in c.items()}
        rd = avg.get("TCC_EA0_RDREQ_sum", 0)
        b32, b64, b128 = (avg.get(f"TCC_EA0_RDREQ_{s}B_sum", 0) for s in (32, 64, 128))
        exact = 32 * b32 + 64 * b64 + 128 * b128
        x2 = 128 * rd
        hit, miss = avg.get("TCC_HIT_sum", 0), avg.get("TCC_MISS_sum", 0)
        wr = 64 * avg.get("TCC_EA0_WRREQ_64B_sum", 0) + 32 * (avg.get("TCC_EA0_WRREQ_sum", 0) - avg.get("TCC_EA0_WRREQ_64B_sum", 0))
        name = k.split("(")[0].replace("void ", "")[:60]
        print(f"{name:60s} {len(c.get('TCC_EA0_RDREQ_sum', [])):4d} {rd:10.0f} {b32:9.0f} {b64:9.0f} {b128:9.0f} "
              f"{exact / 1e6:9.2f} {x2 / 1e6:8.2f} {exact / max(x2, 1):6.2f} {hit / max(hit + miss, 1):6.2f} {wr / 1e6:7.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
