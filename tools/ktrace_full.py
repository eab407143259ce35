#!/usr/bin/env python3
"""Per-kernel launch durations of a rocprofv3 kernel_trace.csv, restricted to the launches of the
full-size merges (each kernel's launches with its largest grid): the figures bench.py's HIP-event
timings describe, without the smaller PCIe-sample / census merges of the same command.

usage: tools/ktrace_full.py <run_kernel_trace.csv> [name filter]"""
import csv
import sys
from collections import defaultdict


def main():
    flt = sys.argv[2] if len(sys.argv) > 2 else "::k_"
    by = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        n = r["Kernel_Name"]
        if flt not in n:
            continue
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        short = n.replace("(anonymous namespace)::", "").replace("void ", "", 1)
        by[short.split("(")[0]].append((g, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows = []
    for n, v in by.items():
        gmax = max(g for g, _ in v)
        full = [d for g, d in v if g == gmax]
        rows.append((sum(full), n, len(full), len(v), sum(full) / len(full), min(full), max(full)))
    print(f"{'kernel':70s} {'full':>5} {'all':>5} {'avg us':>10} {'min':>10} {'max':>10}")
    for tot, n, nf, na, avg, mn, mx in sorted(rows, reverse=True):
        print(f"{n[-70:]:70s} {nf:5d} {na:5d} {avg:10.1f} {mn:10.1f} {mx:10.1f}")


if __name__ == "__main__":
    main()
