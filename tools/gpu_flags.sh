#!/bin/bash
# Flagged-form check and profile: the flag diagnostic (correctness under form switches), then the 1B
# fan-in with flags under a rocprofv3 kernel trace.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/diag_flags.py > gpurun_out/diag_flags.log 2>&1 || { tail -20 gpurun_out/diag_flags.log; exit 1; }
grep -c "mismatches=0 " gpurun_out/diag_flags.log
rm -rf gpurun_out/prof_flags
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_flags -o run -- python3 tools/prof_flags.py > gpurun_out/prof_flags.log 2>&1 || { tail -20 gpurun_out/prof_flags.log; exit 1; }
f=$(find gpurun_out/prof_flags -name "*kernel_stats.csv" | head -1); python3 tools/kstats.py "$f" > gpurun_out/prof_flags_top.txt
grep step gpurun_out/prof_flags.log; head -12 gpurun_out/prof_flags_top.txt
