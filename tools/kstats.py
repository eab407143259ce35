#!/usr/bin/env python3
"""Print the crdt kernels of a rocprofv3 kernel_stats.csv: calls, average and total time."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "k_" in n:
        print(f"{n[:60]:60s} {r['Calls']:>6} {float(r['AverageNs']) / 1000:10.1f} us  "
              f"total {float(r['TotalDurationNs']) / 1e6:8.2f} ms")
