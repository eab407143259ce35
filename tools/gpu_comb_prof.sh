#!/bin/bash
# Kernel trace of the combine probe at one rank's share of N = 8 (tools/combine_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_comb
N=${N:-8} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_comb -o run -- python3 tools/combine_probe.py > gpurun_out/prof_comb.log 2>&1
rc=$?; echo "[prof] exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_comb.log; exit $rc; }
grep -E "mean|distinct" gpurun_out/prof_comb.log
f=$(find gpurun_out/prof_comb -name "*kernel_stats.csv" | head -1); python3 tools/kstats.py "$f" > gpurun_out/prof_comb_top.txt; head -30 gpurun_out/prof_comb_top.txt
