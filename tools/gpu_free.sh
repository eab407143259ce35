#!/bin/bash
# Sorted-path parity in both count modes, then cfg3 / sorted fan-in with and without exact counts.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sorted" \
  > gpurun_out/pytest_sorted.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_sorted.log; [ $rc -eq 0 ] || exit $rc
for mode in free exact free exact; do
  extra=""; [ $mode = exact ] && extra="--exact-counts"
  timeout -k 10 300 python -u bench.py --config cfg3 --steps 5 --warmup 2 --no-pcie $extra > gpurun_out/cfg3_$mode.json 2> gpurun_out/cfg3_$mode.log
  rc=$?; [ $rc -eq 0 ] || { echo "[cfg3 $mode] exit $rc"; tail -5 gpurun_out/cfg3_$mode.log; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/cfg3_$mode.json')); print('$mode', d['ms_per_step'], d['config']['step_ms_all'], d['parity']['equal'], d['roofline']['frac'])"
done
