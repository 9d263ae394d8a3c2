#!/usr/bin/env python3
"""Per-kernel average of rocprofv3 PMC counters from tools/pmc.sh output directories.

usage: python tools/pmc_summary.py <outdir> [kernel-substring ...]
Derived: MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 256 CU * 4 SIMD)... reported raw;
HBM bytes = FETCH_SIZE*1024*2 (gfx950 FETCH_SIZE reads half of a wide coalesced stream,
MI355X_MICROARCH.md §HBM) + WRITE_SIZE*1024.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(out, pats):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(out, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if pats and not any(p in name for p in pats):
                continue
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for name, cs in acc.items():
        avg = {k: sum(v) / len(v) for k, v in cs.items()}
        res[name] = avg
        short = name.split("(")[0][:90]
        print(f"== {short}")
        for k in sorted(avg):
            print(f"   {k:28s} {avg[k]:16.1f}")
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            print(f"   {'hbm_bytes (corrected)':28s} {avg['FETCH_SIZE'] * 1024 * 2 + avg['WRITE_SIZE'] * 1024:16.1f}")
        if "SQ_WAVE_CYCLES" in avg:
            wc = avg["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if k in avg:
                    print(f"   {k + '/WAVE_CYCLES':28s} {avg[k] / wc:16.3f}")
    return res


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
