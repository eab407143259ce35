"""HBM bytes per dispatch of each library kernel from two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE).

gfx950 correction (MI355X_MICROARCH.md, HBM section; tools/pmc_step.py): FETCH_SIZE counts each 128-B memory-side
read at 64 B, so it is doubled; WRITE_SIZE as reported.  Both are in KiB.
usage: tools/pmc_kernels.py <fetch dir> <write dir>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d, counter):
    tot, calls = defaultdict(float), defaultdict(int)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if row.get("Counter_Name") != counter or "::k_" not in name:
                continue
            short = name.split("::", 1)[1].split("(")[0]
            tot[short] += float(row["Counter_Value"])
            calls[short] += 1
    return tot, calls


def main():
    fetch, fc = load(sys.argv[1], "FETCH_SIZE")
    write, wc = load(sys.argv[2], "WRITE_SIZE")
    print(f"{'kernel':64s} {'calls':>5s} {'read MB':>10s} {'written MB':>11s}   (per dispatch; FETCH_SIZE x 2)")
    for k in sorted(set(fetch) | set(write), key=lambda k: -(2 * fetch.get(k, 0) / max(fc.get(k, 1), 1))):
        r = 2 * fetch.get(k, 0) * 1024 / max(fc.get(k, 1), 1) / 1e6
        w = write.get(k, 0) * 1024 / max(wc.get(k, 1), 1) / 1e6
        print(f"{k[:64]:64s} {fc.get(k, 0):5d} {r:10.1f} {w:11.1f}")


if __name__ == "__main__":
    main()
