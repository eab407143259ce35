#!/bin/bash
# SQ counters of the partition scatters and the resolve on the default bench workload (one --pmc
# pass per group, each its own run under its own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_scatter
mkdir -p $OUT
BENCH="bench.py --steps 1 --warmup 0 --no-cpu --no-census --no-pcie"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_part_scatter|k_resolve_packed" --output-format csv -d $OUT/p$i -o run -- python3 $BENCH > $OUT/p$i.log 2>&1
  rc=$?; echo "[pmc $i] exit $rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 - <<'PY'
import csv, glob
from collections import defaultdict
vals = defaultdict(lambda: defaultdict(float))
for f in glob.glob("gpurun_out/pmc_scatter/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "").split("::", 1)[-1].split("(")[0]
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in vals.items():
    print(k)
    for c in sorted(d):
        print(f"  {c:26s} {d[c]:.4g}")
PY
