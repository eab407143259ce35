#!/bin/bash
# K2 records-per-thread sweep (CRDT_APPLY_ITEMS) over the bench configs; one JSON line each.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in fanin cfg3 cfg5; do
  for it in ${ITEMS:-0 1 2 4}; do
    CRDT_APPLY_ITEMS=$it timeout -k 10 300 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu --no-census \
      > gpurun_out/tune_${cfg}_$it.json 2> gpurun_out/tune_${cfg}_$it.log
    rc=$?; [ $rc -eq 0 ] || { echo "[$cfg items=$it] exit $rc"; tail -5 gpurun_out/tune_${cfg}_$it.log; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/tune_${cfg}_$it.json')); print('$cfg items=$it', round(d['value']/1e9,2), 'G rec/s', d['ms_per_step'], 'ms', 'K2', d['roofline']['avg_launch_us'], 'us', d['breakdown_ms'])"
  done
done
