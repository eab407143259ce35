#!/bin/bash
# In-process A/B of a flagged-form switch on the 1B fan-in with flags (AB="VAR=a,b", STEPS), then the
# flag diagnostic (correctness under form switches).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prof_flags.py > gpurun_out/flags_ab.log 2>&1 || { tail -20 gpurun_out/flags_ab.log; exit 1; }
grep "A/B" gpurun_out/flags_ab.log
timeout -k 10 240 python -u tools/diag_flags.py > gpurun_out/diag_flags.log 2>&1 || { tail -20 gpurun_out/diag_flags.log; exit 1; }
grep -c "mismatches=0 " gpurun_out/diag_flags.log
