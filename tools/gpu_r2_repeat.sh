#!/bin/bash
# The default bench command run N times in separate processes on one box (process-to-process
# spread: each process gets its own physical placement of the table and partition buffers).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in $(seq 1 ${1:-3}); do
  timeout -k 10 400 python -u bench.py --no-cpu --no-pcie > gpurun_out/r02_repeat_$i.json 2> gpurun_out/r02_repeat_$i.log
  rc=$?; echo "[run $i] exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r02_repeat_$i.log; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r02_repeat_$i.json')); p=d['roofline']['dominant_kernel']['phases_ms_per_step']
print('run $i', d['ms_per_step'], round(d['value']/1e9, 2), 'G/s', p, 'parity', (d.get('parity') or {}).get('equal'))"
done
