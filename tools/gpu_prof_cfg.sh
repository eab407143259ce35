#!/bin/bash
# GPU parity suite, then a rocprofv3 kernel-trace summary of one bench config.
# usage: tools/gpu_prof_cfg.sh <name> <bench args...>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
name=$1; shift
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/t_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py "$@" --no-cpu > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.log
rc=$?; echo "[bench $name] exit $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -o run -- python3 bench.py "$@" --steps 2 --warmup 1 --no-cpu --no-census > gpurun_out/prof_$name.log 2>&1
rc=$?; echo "[prof $name] exit $rc"; exit $rc
