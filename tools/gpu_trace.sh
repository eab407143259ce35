#!/bin/bash
# rocprofv3 kernel trace of one bench configuration: gpurun_out/trace_<name>/
# usage: tools/gpu_trace.sh <name> <bench args...>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
name=$1; shift
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$name -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-census "$@" > gpurun_out/trace_$name.log 2>&1
rc=$?; echo "[trace $name] exit $rc"; tail -3 gpurun_out/trace_$name.log
exit $rc
