#!/usr/bin/env python3
"""One training step's kernels in launch order from a rocprofv3 ``*_kernel_trace.csv``.

    python tools/step_timeline.py <kernel_trace.csv> [kernels_per_step] [--gaps]

The trace of ``bench.py --profile`` holds warm-up and timed steps back to back; the last
``kernels_per_step`` dispatches (default: the distance between the last two AdamW launches) are one
step.  Prints each dispatch (short name, grid, duration, gap since the previous end) and a summary by
(kernel, grid) -- the shapes that share a kernel name (e.g. the gemm8 launches) come apart by grid.
"""
import csv
import re
import sys
from collections import OrderedDict


def short(name):
    name = re.sub(r"\(.*$", "", name)
    name = name.replace("void ", "").replace("sae::", "")
    return name[:70]


def main(path, per_step=None, gaps=False):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if per_step is None:
        idx = [i for i, r in enumerate(rows) if "adamw_cast" in r["Kernel_Name"]]
        per_step = idx[-1] - idx[-2]
        rows = rows[idx[-2] + 1: idx[-1] + 1]
    else:
        rows = rows[-per_step:]
    t0 = int(rows[0]["Start_Timestamp"])
    t1 = int(rows[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
    print(f"# {path}: one step = {len(rows)} dispatches, wall {(t1 - t0) / 1e3:.1f} us, "
          f"kernel time {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us")
    groups = OrderedDict()
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = (int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]))
        key = (short(r["Kernel_Name"]), grid)
        g = groups.setdefault(key, [])
        g.append((e - s) / 1e3)
        if gaps:
            gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
            print(f"{key[0]:70s} grid {str(grid):14s} {(e - s) / 1e3:8.1f} us  gap {gap:6.1f}")
        prev_end = e
    print(f"\n{'kernel':70s} {'grid':14s} {'n':>3s} {'mean_us':>8s} {'total_us':>9s} {'pct':>6s}")
    for (k, grid), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k:70s} {str(grid):14s} {len(v):3d} {sum(v) / len(v):8.1f} {sum(v):9.1f} {100 * sum(v) / (busy / 1e3):6.1f}")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0], int(args[1]) if len(args) > 1 else None, "--gaps" in sys.argv)
