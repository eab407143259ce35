"""Summarise rocprofv3 PMC / kernel-trace CSVs of tools/gpu_profile.sh per kernel."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_r1"


def short(name):
    for k in ("k_apply", "k_scan", "k_clock", "k_verify", "k_resolve", "k_put_rows", "k_gather<32, 4, false>",
              "k_gather<16, 4, false>", "k_stream", "k_fill"):
        if k.split("<")[0] in name and (("<" not in k) or k.replace(" ", "") in name.replace(" ", "")):
            return k
    return None


out = defaultdict(dict)
for f in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")) + \
        glob.glob(os.path.join(d, "ub_fetch", "*counter_collection.csv")):
    acc = defaultdict(lambda: defaultdict(list))
    for row in csv.DictReader(open(f)):
        k = short(row.get("Kernel_Name", ""))
        if k:
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in acc.items():
        for c, vals in cs.items():
            out[k][c] = {"per_dispatch_mean": sum(vals) / len(vals), "dispatches": len(vals)}
trace = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))
if trace:
    for row in csv.DictReader(open(trace[0])):
        k = short(row["Name"])
        if k:
            out[k]["duration_ns_avg"] = float(row["AverageNs"])
            out[k]["calls"] = int(row["Calls"])
print(json.dumps(out, indent=1))
