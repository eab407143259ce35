#!/bin/bash
# Round 2: the other BASELINE configs (parity cases, not bench lines) on the current tree.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for spec in "cfg2:--config cfg2 --steps 10 --warmup 2 --no-census" "cfg3:--config cfg3 --steps 5 --warmup 2" "cfg5:--config cfg5 --steps 3 --warmup 1" "gather:--path gather --row-bytes 32 --steps 3 --warmup 1 --no-cpu --no-pcie" "fanin:--steps 5 --warmup 2 --no-cpu --no-pcie --no-census"; do
  name=$(echo "$spec" | cut -d: -f1); args=$(echo "$spec" | cut -d: -f2-)
  timeout -k 10 500 python -u bench.py $args > gpurun_out/r02_bench_$name.json 2> gpurun_out/r02_bench_$name.log
  rc=$?; echo "[$name] exit $rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r02_bench_$name.log; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r02_bench_$name.json')); p=d.get('parity') or {}
print('$name', d['value'], d['ms_per_step'], d['config'].get('merge_path'), 'parity', p.get('equal'))"
done
