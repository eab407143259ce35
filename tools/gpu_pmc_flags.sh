#!/bin/bash
# SQ counters of the flagged form's kernels beside the order-free ones (tools/prof_flags.py with MIX=1:
# steps alternate flags / no flags), one --pmc pass.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=${OUT:-pmc_flags_sq}
rm -rf gpurun_out/$OUT
CTRS=${CTRS:-SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU}
MIX=1 STEPS=4 timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/$OUT -o run -- python3 tools/prof_flags.py > gpurun_out/$OUT.log 2>&1
rc=$?; echo "[pmc] exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/$OUT.log; exit $rc; }
OUT=$OUT python3 - <<'PY'
import csv, glob, collections, os
f = glob.glob(f"gpurun_out/{os.environ['OUT']}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    if not k.startswith("k_"): continue
    k = k.split("(")[0]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, c in acc.items():
    if c.get("SQ_WAVE_CYCLES", 0) < 1e8: continue
    w = c["SQ_WAVE_CYCLES"]
    print(f"{k[:60]:60s} " + "  ".join(
        f"{n[3:]} {v / w:.3f}" if n.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY")) else f"{n[3:]} {v:.4g}"
        for n, v in sorted(c.items())))
PY
