#!/bin/bash
# Round 3: the other BASELINE configs and the exact-count fan-in on the current tree, then a kernel
# trace of cfg3.  Every GPU step has its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "cfg2:--config cfg2 --steps 10 --warmup 2 --no-census" "cfg3:--config cfg3 --steps 5 --warmup 2" "cfg5:--config cfg5 --steps 3 --warmup 1" "exact_counts:--exact-counts --no-cpu --no-pcie"; do
  name=$(echo "$spec" | cut -d: -f1); args=$(echo "$spec" | cut -d: -f2-)
  timeout -k 10 500 python -u bench.py $args > gpurun_out/r03_bench_$name.json 2> gpurun_out/r03_bench_$name.log
  rc=$?; echo "[$name] exit $rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r03_bench_$name.log; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03_bench_$name.json')); p=d.get('parity') or {}
w=d.get('with_win_flags') or {}
print('$name', d['value'], d['ms_per_step'], d['config'].get('merge_path'), 'parity', p.get('equal'), 'flags', w.get('ms_per_step'), w.get('merge_path'), w.get('flags_equal_gather'))"
done
rm -rf gpurun_out/r03_prof_cfg3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof_cfg3 -o run -- python3 bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu --no-census --no-pcie > gpurun_out/r03_prof_cfg3.log 2>&1
rc=$?; echo "[prof cfg3] exit $rc"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/r03_prof_cfg3 -name "*kernel_trace.csv" | head -1); python3 tools/ktrace_full.py "$f" > gpurun_out/r03_prof_cfg3_full.txt; head -24 gpurun_out/r03_prof_cfg3_full.txt
