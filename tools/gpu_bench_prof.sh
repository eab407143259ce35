#!/bin/bash
# Default bench + rocprofv3 kernel-trace of the same command (short run).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log
rc=$?; echo "[bench] exit $rc"; cat gpurun_out/bench_default.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-census "$@" > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "[rocprof] exit $rc"; [ $rc -eq 0 ] || exit $rc
find gpurun_out/prof -name "*stats*" | head
