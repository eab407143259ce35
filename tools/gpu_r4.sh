#!/bin/bash
# Round-4 GPU steps.  STAGE selects; every GPU step has its own time limit; stops at the first failure.
#   flags : the flagged / ordered GPU tests, then the 1B flagged merge timing (tools/prof_flags.py)
#   tests : the whole -m gpu suite (TESTS="-k expr" narrows it)
#   shard : the multi-rank GPU tests (gloo ranks on one GPU, RCCL single rank)
#   probe : one rank's local work at config 4's shares (tools/route_probe.py, PROBE_N="8 2")
#   cfg3  : cfg3 with the sparse-bucket resolve on / off (in-process A/B), then its per-kernel PMC traffic
#   fprof : kernel trace of the 1B flagged merge (tools/prof_flags.py)
#   bench : the default bench line + its PMC traffic + a kernel trace (profiles evidence)
#   suite : the whole -m gpu suite, then smoke()
#   spread: the short bench in REPS processes, clocks / power per step
#   misc  : wide-frame fan-in with flags, anchored-form PMC, flagged-form SQ counters
#   cfgpath: cfg5 and cfg2 on each store path (gather K2 vs sorted)
#   cfg5prof: cfg5's per-call kernel / HIP API timeline (tools/ktrace_calls.py)
#   place : the level-1 scatter per allocation of the partition buffers (tools/place_probe.py)
#   ab    : in-process A/B of the 1B flagged merge (AB="VAR=a,b")
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r4}
case "${STAGE:-flags}" in
  flags)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests \
      -k "(flagged or sorted or exact or ordered) and not rank" > gpurun_out/${TAG}_pytest_flags.log 2>&1
    rc=$?; tail -3 gpurun_out/${TAG}_pytest_flags.log; [ $rc -eq 0 ] || exit $rc
    STEPS=${STEPS:-6} timeout -k 10 300 python -u tools/prof_flags.py > gpurun_out/${TAG}_flags_time.log 2>&1
    rc=$?; tail -8 gpurun_out/${TAG}_flags_time.log; exit $rc ;;
  tests)
    timeout -k 10 1100 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests ${TESTS:-} \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1
    rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; exit $rc ;;
  shard)
    timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu tests \
      -k "${TESTS:-rank or route or combine or shard or mismatch or rccl}" > gpurun_out/${TAG}_pytest_shard.log 2>&1
    rc=$?; tail -3 gpurun_out/${TAG}_pytest_shard.log; exit $rc ;;
  probe)
    for n in ${PROBE_N:-8 2}; do
      N=$n STEPS=${STEPS:-3} timeout -k 10 400 python -u tools/route_probe.py > gpurun_out/${TAG}_probe_n$n.log 2>&1
      rc=$?; grep -E "mean|rows|home" gpurun_out/${TAG}_probe_n$n.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_probe_n$n.log; exit $rc; }
    done ;;
  cfg3)
    timeout -k 10 500 python -u bench.py --config cfg3 --steps ${STEPS:-8} --warmup 2 --no-cpu --no-pcie \
      --ab ${AB:-CRDT_SPARSE_T=0,1024} > gpurun_out/${TAG}_cfg3_ab.json 2> gpurun_out/${TAG}_cfg3_ab.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_cfg3_ab.log; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_cfg3_ab.log; exit $rc; }
    [ -n "${NO_PMC:-}" ] && exit 0
    ARGS="--config cfg3 --steps 1 --warmup 0 --no-cpu --no-census --no-pcie" MERGES=1 PMC_OUT=${TAG}_pmc_cfg3.json \
      bash tools/gpu_pmc_bench.sh ;;
  fprof)
    rm -rf gpurun_out/${TAG}_prof_flags
    STEPS=${STEPS:-3} timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_flags -o run \
      -- python3 tools/prof_flags.py > gpurun_out/${TAG}_prof_flags.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_prof_flags.log; exit $rc; }
    f=$(find gpurun_out/${TAG}_prof_flags -name "*kernel_trace.csv" | head -1)
    python3 tools/ktrace_full.py "$f" > gpurun_out/${TAG}_prof_flags_full.txt; grep step gpurun_out/${TAG}_prof_flags.log
    head -24 gpurun_out/${TAG}_prof_flags_full.txt ;;
  bench)
    # the default bench line, its PMC traffic (two --pmc passes) and a kernel trace of the same command
    timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.log
    rc=$?; cat gpurun_out/${TAG}_bench_default.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench_default.log; exit $rc; }
    PMC_OUT=${TAG}_pmc_bench.json bash tools/gpu_pmc_bench.sh || exit $?
    rm -rf gpurun_out/${TAG}_prof_bench
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_bench -o run \
      -- python3 bench.py --no-cpu > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.log
    rc=$?; echo "[prof] exit $rc"; [ $rc -eq 0 ] || exit $rc
    t=$(find gpurun_out/${TAG}_prof_bench -name "*kernel_trace.csv" | head -1)
    python3 tools/ktrace_full.py "$t" > gpurun_out/${TAG}_prof_bench_full.txt; head -16 gpurun_out/${TAG}_prof_bench_full.txt ;;
  suite)
    timeout -k 10 1000 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1
    rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
    rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; exit $rc ;;
  spread)
    # process-to-process spread: the same short bench in REPS processes, each line with its per-step clocks
    for i in $(seq 1 ${REPS:-3}); do
      [ -n "${CONTIG_ALT:-}" ] && export CRDT_ALLOC_CONTIG=$(( i % 2 ))
      [ -n "${SHUFFLE_ALT:-}" ] && export CRDT_ALLOC_SHUFFLE=$(( i % 2 ))
      [ -n "${PLACE_ALT:-}" ] && export CRDT_PLACE_TRIES=$(( i % 2 ? 3 : 1 ))
      timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu --no-census --no-pcie \
        > gpurun_out/${TAG}_spread_$i.json 2> gpurun_out/${TAG}_spread_$i.log
      rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_spread_$i.log; exit $rc; }
      python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_spread_$i.json')); g=d.get('gpu_clocks') or {}
print('run $i contig=${CRDT_ALLOC_CONTIG:-0} shuffle=${CRDT_ALLOC_SHUFFLE:-0} place=${CRDT_PLACE_TRIES:-3}', d.get('placement'), d['ms_per_step'], 'part1', d['roofline']['dominant_kernel']['phases_ms_per_step']['part1'], 'copy', g.get('copy_GBs'), [(s.get('step_ms'), s.get('part1_ms'), s.get('sclk_mhz'), s.get('power_w')) for s in g.get('per_step', [])])"
    done ;;
  misc)
    # the wide clock frame with win flags; the anchored form's PMC traffic (item 3);
    # SQ counters of the flagged form's kernels (item 2)
    timeout -k 10 600 python -u bench.py --millis-span 67108864 --steps 3 --warmup 1 --no-pcie --no-cpu-copy16 \
      --cpu-seconds 5 > gpurun_out/${TAG}_bench_wide26.json 2> gpurun_out/${TAG}_bench_wide26.log
    rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench_wide26.log; exit $rc; }
    python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench_wide26.json')); w=d['with_win_flags']
print('wide26', d['ms_per_step'], d['roofline']['dominant_kernel']['plan'].get('key16'), 'flags', w['ms_per_step'], w['merge_path'], w['flagged_form'], w.get('flags_equal_gather'), 'parity', (d['parity'] or {}).get('equal'))"
    CRDT_SORTED_FORM=262144 PMC_OUT=${TAG}_pmc_anchored.json bash tools/gpu_pmc_bench.sh || exit $?
    OUT=${TAG}_pmc_flags_sq bash tools/gpu_pmc_flags.sh ;;
  cfgpath)
    # single-changeset configs on each store path: cfg2 (10M + 10M) and cfg5 (100 streaming 10M deltas)
    for cfg in ${CFGS:-cfg5 cfg2}; do
      for path in gather sorted; do
        timeout -k 10 400 python -u bench.py --config $cfg --path $path --steps 3 --warmup 1 --no-cpu --no-pcie \
          > gpurun_out/${TAG}_${cfg}_$path.json 2> gpurun_out/${TAG}_${cfg}_$path.log
        rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_${cfg}_$path.log; exit $rc; }
        python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_${cfg}_$path.json'))
print('$cfg $path', d['ms_per_step'], d['config'].get('merge_path'), 'frac', d['roofline']['frac'], 'parity', (d.get('parity') or {}).get('equal'))"
      done
    done ;;
  cfg5prof)
    # cfg5's per-call timeline: kernel + HIP API trace of one step (100 merge calls)
    rm -rf gpurun_out/${TAG}_prof_cfg5
    timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/${TAG}_prof_cfg5 -o run \
      -- python3 bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu --no-pcie --no-census \
      > gpurun_out/${TAG}_prof_cfg5.json 2> gpurun_out/${TAG}_prof_cfg5.log
    rc=$?; echo "[prof] exit $rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_prof_cfg5.log; exit $rc; }
    k=$(find gpurun_out/${TAG}_prof_cfg5 -name "*kernel_trace.csv" | head -1)
    h=$(find gpurun_out/${TAG}_prof_cfg5 -name "*hip_api_trace.csv" | head -1)
    python3 tools/ktrace_calls.py "$k" k_apply "$h" > gpurun_out/${TAG}_cfg5_calls.txt; cat gpurun_out/${TAG}_cfg5_calls.txt ;;
  place)
    # the level-1 scatter per allocation of the partition buffers, in one process (tools/place_probe.py)
    A=${A:-5} STEPS=${STEPS:-3} timeout -k 10 500 python -u tools/place_probe.py > gpurun_out/${TAG}_place.log 2>&1
    rc=$?; grep allocation gpurun_out/${TAG}_place.log; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_place.log; exit $rc; } ;;
  ab)
    STEPS=${STEPS:-9} timeout -k 10 400 python -u tools/prof_flags.py > gpurun_out/${TAG}_flags_ab.log 2>&1
    rc=$?; grep -E "A/B|step" gpurun_out/${TAG}_flags_ab.log | tail -12; exit $rc ;;
esac
