#!/bin/bash
# Closing lines of cfg2 and cfg5 on the final tree (default bench options for each config: CPU baseline and parity on).
set -o pipefail
mkdir -p gpurun_out
for c in cfg2 cfg5; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/r05z_bench_$c.json 2> gpurun_out/r05z_bench_$c.log || { tail -20 gpurun_out/r05z_bench_$c.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r05z_bench_$c.json')); print('$c', d['ms_per_step'], d['value'], d['roofline']['frac'], (d.get('parity') or {}).get('equal'), d['cpu_baseline']['value'])"
done
