#!/bin/bash
# A/B of library builds on one bench command: tools/gpu_ab.sh "<bench args>" lib1 lib2 ...
# (each lib under crdt_amd/, loaded through CRDT_LIB_PATH); stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
args="$1"; shift
for lib in "$@"; do
  CRDT_LIB_PATH=$PWD/crdt_amd/$lib timeout -k 10 300 python -u bench.py $args --no-cpu --no-census \
    > gpurun_out/ab_$lib.json 2> gpurun_out/ab_$lib.log
  rc=$?; echo "[$lib] exit $rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$lib.json')); print('$lib', d['ms_per_step'], d['config'].get('step_ms_all'))"
done
