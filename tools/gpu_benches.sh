#!/bin/bash
# Several bench.py configurations back to back; stops at the first crash/timeout.
# usage: tools/gpu_benches.sh "<name>:<bench args>" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for spec in "$@"; do
  name=$(echo "$spec" | cut -d: -f1); cmd=$(echo "$spec" | cut -d: -f2-)
  timeout -k 10 400 python -u bench.py $cmd > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.log
  rc=$?; echo "[bench $name] exit $rc"; cat gpurun_out/bench_$name.json
  [ $rc -eq 0 ] || exit $rc
done
