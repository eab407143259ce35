#!/bin/bash
# Round-5 closing measurements on the final tree: the default bench line, cfg3, and the N = 8 loopback probe.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r05c}
timeout -k 10 420 python -u bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_default.json')); print('default', d['ms_per_step'], d['roofline']['frac'], d['with_win_flags']['ms_per_step'], (d.get('parity') or {}).get('equal'))"
timeout -k 10 300 python -u bench.py --config cfg3 --steps 10 --warmup 2 > gpurun_out/${TAG}_bench_cfg3.json 2> gpurun_out/${TAG}_bench_cfg3.log || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_cfg3.json')); print('cfg3', d['ms_per_step'], d['roofline']['frac'], (d.get('parity') or {}).get('equal'))"
N=8 STEPS=2 MODES=route_l1,route_l1_head timeout -k 10 400 python -u tools/route_probe.py > gpurun_out/${TAG}_probe_n8.log 2>&1 || exit $?
grep -E "mean|rows" gpurun_out/${TAG}_probe_n8.log
