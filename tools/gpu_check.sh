#!/bin/bash
# GPU parity suite, then the streaming (cfg5) and default fan-in benches; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/t_gpu.log; [ $rc -eq 0 ] || exit $rc
for spec in "$@"; do
  name=$(echo "$spec" | cut -d: -f1); args=$(echo "$spec" | cut -d: -f2-)
  timeout -k 10 400 python -u bench.py $args > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.log
  rc=$?; echo "[bench $name] exit $rc"; cat gpurun_out/bench_$name.json; [ $rc -eq 0 ] || exit $rc
done
