#!/bin/bash
# Perf probe: a parity subset (pytest -k "$KEXPR", default: sorted), then one bench line per
# "name:ENV=... args" spec, then (PROF=1) a rocprofv3 kernel trace of the last spec.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${KEXPR:-sorted}" != "none" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "${KEXPR:-sorted}" > gpurun_out/t_probe.log 2>&1
  rc=$?; tail -3 gpurun_out/t_probe.log; [ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/t_probe.log | head; exit $rc; }
fi
last=""
for spec in "$@"; do
  name=$(echo "$spec" | cut -d: -f1); rest=$(echo "$spec" | cut -d: -f2-)
  envs=$(echo "$rest" | cut -d'|' -f1); args=$(echo "$rest" | cut -d'|' -f2-)
  env $envs timeout -k 10 400 python -u bench.py $args > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.log
  rc=$?; echo "[bench $name] exit $rc"; python3 -c "
import json,sys; d=json.load(open('gpurun_out/bench_$name.json')); print('$name', d['ms_per_step'], d['config']['merge_path'], d['roofline'].get('frac'), d['breakdown_ms'])" || true
  [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$name.log; exit $rc; }
  last="$envs|$args"
  if [ "${PROF:-0}" = "all" ]; then   # a kernel trace of every spec, each in its own directory
    timeout -k 10 400 env $envs rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -o run -- python3 bench.py $args --steps 2 --warmup 1 --no-cpu --no-census --no-pcie > gpurun_out/prof_$name.log 2>&1
    rc=$?; echo "[prof $name] exit $rc"; [ $rc -eq 0 ] || exit $rc
    f=$(find gpurun_out/prof_$name -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 tools/kstats.py "$f" | head -${PROF_TOP:-12}
  fi
done
if [ "${PROF:-0}" = "1" ] && [ -n "$last" ]; then
  envs=$(echo "$last" | cut -d'|' -f1); args=$(echo "$last" | cut -d'|' -f2-)
  for e in $envs; do export "$e"; done
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_probe -o run -- python3 bench.py $args --steps 2 --warmup 1 --no-cpu --no-census --no-pcie > gpurun_out/prof_probe.log 2>&1
  rc=$?; echo "[prof] exit $rc"; f=$(find gpurun_out/prof_probe -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && python3 tools/kstats.py "$f"
fi
