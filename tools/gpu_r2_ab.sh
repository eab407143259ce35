#!/bin/bash
# Round 2: targeted GPU tests (KEXPR), then an in-process A/B of a library switch on the default
# bench workload: tools/gpu_r2_ab.sh "VAR=a,b" [steps]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${KEXPR:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests -k "$KEXPR" > gpurun_out/t_ab.log 2>&1
  rc=$?; tail -3 gpurun_out/t_ab.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error" gpurun_out/t_ab.log | head; exit $rc; }
fi
timeout -k 10 600 python -u bench.py --steps ${2:-16} --warmup 2 --no-cpu --no-census --no-pcie --ab "$1" \
  > gpurun_out/ab.json 2> gpurun_out/ab.log
rc=$?; grep "A/B" gpurun_out/ab.log; python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print(d['ms_per_step'], d['roofline']['dominant_kernel']['phases_ms_per_step'])"; exit $rc
