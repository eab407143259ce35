#!/usr/bin/env python3
"""HBM traffic per merge step from two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE) of one
bench.py command, written as the JSON bench.py reads for roofline.traffic.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE tallies each 128-B memory-side
read at 64 B, so it is doubled (round 1 calibrated it on a known 8 GiB stream); WRITE_SIZE is
taken as reported.  Only this library's kernels are summed (the workload generator's torch
kernels and the per-step table reset, k_put_rows, are not part of a merge step).

usage: tools/pmc_step.py <fetch dir> <write dir> <merges in the run> <out.json> <command args json>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    per = defaultdict(float)
    calls = defaultdict(int)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if row.get("Counter_Name") != counter or "::k_" not in name or "k_put_rows" in name:
                continue
            short = name.split("::", 1)[1].split("(")[0]
            per[short] += float(row["Counter_Value"])
            calls[short] += 1
    return per, calls


def main():
    fdir, wdir, merges, out, cmd = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5]
    fetch, calls = load(fdir, "FETCH_SIZE")
    write, _ = load(wdir, "WRITE_SIZE")
    kernels = sorted(set(fetch) | set(write), key=lambda k: -(2 * fetch.get(k, 0) + write.get(k, 0)))
    rows = {k: {"read_bytes_per_step": int(2 * fetch.get(k, 0) * 1024 / merges),
                "write_bytes_per_step": int(write.get(k, 0) * 1024 / merges),
                "dispatches_per_step": calls.get(k, 0) / merges} for k in kernels}
    rd = sum(r["read_bytes_per_step"] for r in rows.values())
    wr = sum(r["write_bytes_per_step"] for r in rows.values())
    res = {"hbm_bytes_per_step": rd + wr, "read_bytes_per_step": rd, "write_bytes_per_step": wr,
           "merges_in_run": merges, "correction": "FETCH_SIZE x 2 (gfx950: 128-B reads tallied at 64 B), "
           "WRITE_SIZE as reported; FETCH/WRITE_SIZE in KB", "kernels": rows}
    res.update(json.loads(cmd))
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("hbm_bytes_per_step", "read_bytes_per_step", "write_bytes_per_step")}))
    for k, r in rows.items():
        print(f"  {k:34s} read {r['read_bytes_per_step'] / 1e9:7.2f} GB  write {r['write_bytes_per_step'] / 1e9:7.2f} GB")


if __name__ == "__main__":
    main()
