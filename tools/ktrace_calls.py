#!/usr/bin/env python3
"""Per-call timeline of a streaming merge (cfg5: one crdt_merge per delta) from a rocprofv3 kernel trace:
the launches between two consecutive anchor kernels (default: the largest-grid k_apply launches) form one
call; prints, as medians over the calls, each kernel's duration, the device-busy time, the call's span
(anchor start to next anchor start) and the idle time inside it.  With a HIP API trace beside it
(rocprofv3 --hip-trace), also the median count and time of each host API per call.

usage: tools/ktrace_calls.py <run_kernel_trace.csv> [anchor substring] [run_hip_api_trace.csv]
STOP_AT=<substring>[|<substring>...]: a call ends at its last kernel before the first launch matching it (span = busy + gaps)."""
import csv
import os
import statistics
import sys
from collections import defaultdict


def main():
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_apply"
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        n = r["Kernel_Name"].replace("void ", "", 1).replace("(anonymous namespace)::", "").split("(")[0]
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, g))
    rows.sort()
    anc = [x for x in rows if anchor in x[2]]
    gmax = max(x[3] for x in anc)
    starts = [x[0] for x in anc if x[3] == gmax]
    per = defaultdict(list)
    busy, span, idle, nk = [], [], [], []
    stop = os.environ.get("STOP_AT")                     # e.g. k_put_rows: the bench's table reset ends a call
    for a, b in zip(starts, starts[1:]):
        ks = [x for x in rows if a <= x[0] < b]
        if stop:
            cut = [x[0] for x in ks if any(t in x[2] for t in stop.split("|"))]
            if cut:
                ks = [x for x in ks if x[0] < cut[0]]
            b = max(x[1] for x in ks)
        dur = defaultdict(float)
        for s, e, n, _ in ks:
            dur[n] += (e - s) / 1e3
        for n, d in dur.items():
            per[n].append(d)
        bsy = sum((e - s) for s, e, _, _ in ks) / 1e3
        busy.append(bsy)
        span.append((b - a) / 1e3)
        idle.append((b - a) / 1e3 - bsy)
        nk.append(len(ks))
    calls = len(span)
    print(f"{calls} calls (anchor {anchor}, grid {gmax}): median span {statistics.median(span):.1f} us, "
          f"device busy {statistics.median(busy):.1f} us, idle {statistics.median(idle):.1f} us, "
          f"{statistics.median(nk):.0f} launches per call")
    for n, v in sorted(per.items(), key=lambda kv: -statistics.median(kv[1])):
        print(f"  {n[-60:]:60s} {len(v):4d} calls  median {statistics.median(v):8.1f} us")
    if len(sys.argv) > 3:
        api = []
        for r in csv.DictReader(open(sys.argv[3])):
            api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
        cnt, tm = defaultdict(list), defaultdict(list)
        for a, b in zip(starts, starts[1:]):
            c, t = defaultdict(int), defaultdict(float)
            for s, e, f in api:
                if a <= s < b:
                    c[f] += 1
                    t[f] += (e - s) / 1e3
            for f in c:
                cnt[f].append(c[f])
                tm[f].append(t[f])
        print("host API per call (median count, median time):")
        for f in sorted(cnt, key=lambda f: -statistics.median(tm[f])):
            if len(cnt[f]) * 2 < calls:
                continue
            print(f"  {f:40s} {statistics.median(cnt[f]):5.0f}  {statistics.median(tm[f]):8.1f} us")


if __name__ == "__main__":
    main()
