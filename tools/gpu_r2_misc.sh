#!/bin/bash
# Round 2: new API / ABI parity tests, the carry-fold reproduction, the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_api.py > gpurun_out/t_api.log 2>&1
rc=$?; tail -3 gpurun_out/t_api.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|FAILED" gpurun_out/t_api.log | head -20; exit $rc; }
timeout -k 10 120 tools/repro_carry_fold > gpurun_out/repro_carry_fold.txt 2>&1
echo "[repro] exit $?"; cat gpurun_out/repro_carry_fold.txt
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log
rc=$?; echo "[bench] exit $rc"; cat gpurun_out/bench_default.json; [ $rc -eq 0 ] || tail -20 gpurun_out/bench_default.log
