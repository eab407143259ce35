#!/bin/bash
# Sorted-path parity (every sorted test), then cfg3 with full-size parity, then the A/B against a reference build.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sorted" \
  > gpurun_out/pytest_sorted.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_sorted.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config cfg3 --steps 5 --warmup 2 --no-census --no-pcie > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.log
rc=$?; echo "[cfg3] exit $rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/bench_cfg3.json')); print(d['ms_per_step'], d['config']['step_ms_all'], d['parity'])"
bash tools/gpu_ab.sh "--config cfg3 --steps 6 --warmup 2" "$@"
