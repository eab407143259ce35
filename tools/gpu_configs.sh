#!/bin/bash
# The non-default BASELINE configs (cfg2 / cfg3 / cfg5) through bench.py, plus a rocprofv3
# kernel-trace summary of cfg5 (streaming deltas: one crdt_merge per 10M-record delta).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in cfg2 cfg3 cfg5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.log
  rc=$?; echo "[$c] exit $rc"; cat gpurun_out/bench_$c.json; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg5 -o run -- python3 bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu --no-census > gpurun_out/prof_cfg5.log 2>&1
rc=$?; echo "[prof cfg5] exit $rc"; exit $rc
