#!/bin/bash
# Round 2: GPU parity suite (incl. the library's collective merge), then a short default bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KARGS=(); [ -n "${KEXPR:-}" ] && KARGS=(-k "$KEXPR")
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests "${KARGS[@]}" > gpurun_out/t_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/t_gpu.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|error" gpurun_out/t_gpu.log | head -20; exit $rc; }
for spec in "$@"; do
  name=$(echo "$spec" | cut -d: -f1); args=$(echo "$spec" | cut -d: -f2-)
  timeout -k 10 500 python -u bench.py $args > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.log
  rc=$?; echo "[bench $name] exit $rc"; cat gpurun_out/bench_$name.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$name.log; exit $rc; }
done
