#!/usr/bin/env python3
"""Summarise a rocprofv3 ``*_kernel_stats.csv`` (--kernel-trace --stats) into a short table.

usage: python tools/prof_summary.py <kernel_stats.csv> [top_n]
"""
import csv
import sys


def main(path, top=30):
    rows = list(csv.DictReader(open(path)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {path}\n# total kernel time {total / 1e6:.3f} ms over {sum(int(r['Calls']) for r in rows)} launches")
    print(f"{'kernel':100s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{r['Name'][:100]:100s} {r['Calls']:>6s} {float(r['AverageNs']) / 1e3:9.2f} "
              f"{float(r['MinNs']) / 1e3:9.2f} {float(r['MaxNs']) / 1e3:9.2f} {float(r['Percentage']):6.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
