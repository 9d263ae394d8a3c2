#!/usr/bin/env python3
"""Per-step kernel breakdown of a graph-replayed training step from a rocprofv3 run (the rocpd
SQLite database or the --output-format csv kernel trace): the kernels between the last two
optimizer launches (adamw_cast), grouped by name.

    python tools/prof_step.py <rocprof output dir> [top]
"""
import collections
import csv
import glob
import os
import sqlite3
import sys


def load(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if dbs:
        con = sqlite3.connect(dbs[0])
        return [(n, s, e) for n, s, e in con.execute("select name, start, end from kernels order by start")]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    return [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]


def main(d, top=18):
    tr = load(d)
    idx = [i for i, (n, _, _) in enumerate(tr) if "adamw_cast" in n]
    a, b = idx[-2], idx[-1]
    seg = tr[a + 1:b + 1]
    by = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e in seg:
        k = n.split("(")[0][:90]
        by[k][0] += 1
        by[k][1] += (e - s) / 1e3
    busy = sum(v[1] for v in by.values())
    wall = (tr[b][2] - tr[a][2]) / 1e3
    print(f"# {d}: one step = {len(seg)} kernels, {busy:.0f} us of kernel time, {wall:.0f} us wall")
    for k, (c, t) in sorted(by.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{t:9.1f} us {100 * t / busy:5.1f}% {c:4d} x {t / c:7.1f} us  {k}")
    lib = [k for k in by if k.startswith("Cijk") or "gemm" in k.lower() and "sae::" not in k]
    print("# library GEMM kernels in the step:", lib if lib else "none")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 18)
