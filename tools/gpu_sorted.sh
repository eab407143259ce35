#!/bin/bash
# Sorted-path session: parity tests for both paths, then benches + a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "sorted" \
  > gpurun_out/pytest_sorted.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_sorted.log; echo "[pytest sorted] exit $rc"; [ $rc -eq 0 ] || exit $rc
for spec in "$@"; do
  name=$(echo "$spec" | cut -d: -f1); cmd=$(echo "$spec" | cut -d: -f2-)
  timeout -k 10 400 python -u bench.py $cmd > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.log
  rc=$?; echo "[bench $name] exit $rc"; cat gpurun_out/bench_$name.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_sorted -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-census --path sorted > gpurun_out/trace_sorted.log 2>&1
rc=$?; echo "[trace] exit $rc"; exit $rc
