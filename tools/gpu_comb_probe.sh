#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for n in ${NS:-2 8}; do
  N=$n timeout -k 10 300 python -u tools/combine_probe.py > gpurun_out/comb_probe_$n.log 2>&1
  rc=$?; echo "[N=$n] exit $rc"; grep -E "mean|distinct" gpurun_out/comb_probe_$n.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/comb_probe_$n.log; exit $rc; }
done
