#!/bin/bash
# WRITE_SIZE per kernel of the default bench workload under a library switch setting:
# tools/gpu_pmc_write_ab.sh "VAR=value" (one --pmc pass of its own run)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$(echo "$1" | tr '=,' '__')
env "$1" true || exit 2
export "$1"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$tag -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-census --no-pcie > gpurun_out/pmcw_$tag.log 2>&1
rc=$?; echo "[write $tag] exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmcw_$tag.log; exit $rc; }
python3 - "$tag" <<'PY'
import csv, glob, sys
from collections import defaultdict
tag = sys.argv[1]
per = defaultdict(float)
for f in glob.glob(f"gpurun_out/pmcw_{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r.get("Kernel_Name", "")
        if r.get("Counter_Name") == "WRITE_SIZE" and "::k_part" in n:
            per[n.split("::", 1)[1].split("(")[0]] += float(r["Counter_Value"])
for k, v in sorted(per.items(), key=lambda x: -x[1]):
    print(f"{tag} {k}: {v * 1024 / 3 / 1e9:.2f} GB written per step")
PY
