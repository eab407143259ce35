#!/bin/bash
# Round-5 GPU stages (run under gpurun from the repo root).  STAGE=check: sorted-path parity subset, then
# an in-process A/B of the persistent partition scatters (CRDT_SORTED_FORM bit 2097152 = one tile per
# workgroup) on the 1B fan-in.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r5}
case "${STAGE:-check}" in
  libab) ;;
  check)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
      -k "sorted_golden or packed_kinds or odd_level1 or form_switches or flagged_equals or routed_fanin or eight_rank_route_l1 or place_tuner or split_hot" \
      > gpurun_out/${TAG}_check.log 2>&1 || { tail -30 gpurun_out/${TAG}_check.log; exit 1; }
    tail -3 gpurun_out/${TAG}_check.log
    timeout -k 10 420 python -u bench.py --steps 8 --warmup 2 --ab CRDT_SORTED_FORM=0,2097152 --no-cpu --no-census \
      --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_persist.json 2> gpurun_out/${TAG}_ab_persist.log
    rc=$?; grep "A/B\|placement" gpurun_out/${TAG}_ab_persist.log; exit $rc ;;
  cfg5pmc)
    # cfg5 (100 streaming 10M-record merges on K2): k_apply's HBM bytes per launch (FETCH_SIZE, WRITE_SIZE in
    # separate passes), then records per thread of K2 in one process (CRDT_APPLY_ITEMS A/B)
    ARGS="--config cfg5 --path gather --steps 1 --warmup 0 --no-cpu --no-census --no-pcie --flag-steps 0" MERGES=1 \
      PMC_PATH=gather PMC_OUT=${TAG}_pmc_cfg5.json bash tools/gpu_pmc_bench.sh || exit $?
    timeout -k 10 420 python -u bench.py --config cfg5 --path gather --steps 3 --warmup 1 --no-cpu --no-census \
      --no-pcie --flag-steps 0 --ab CRDT_APPLY_ITEMS=0,1,2,4,8 > gpurun_out/${TAG}_cfg5_items.json \
      2> gpurun_out/${TAG}_cfg5_items.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_cfg5_items.log; exit $rc ;;
  cfg3trace)
    # cfg3's per-merge timeline: device-busy time vs the merge's span (launch gaps), anchor = the clock scan
    rm -rf gpurun_out/${TAG}_prof_cfg3
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_cfg3 -o run \
      -- python3 bench.py --config cfg3 --steps 5 --warmup 2 --no-cpu --no-pcie --no-census --flag-steps 0 \
      > gpurun_out/${TAG}_prof_cfg3.json 2> gpurun_out/${TAG}_prof_cfg3.log
    rc=$?; echo "[prof] exit $rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_prof_cfg3.log; exit $rc; }
    k=$(find gpurun_out/${TAG}_prof_cfg3 -name "*kernel_trace.csv" | head -1)
    STOP_AT="fill|Fill|k_put_rows" python3 tools/ktrace_calls.py "$k" k_scan > gpurun_out/${TAG}_cfg3_calls.txt; cat gpurun_out/${TAG}_cfg3_calls.txt
    python3 tools/ktrace_full.py "$k" > gpurun_out/${TAG}_cfg3_full.txt ;;
  final)
    # the round's default bench line, its kernel trace (--stats) and its PMC traffic, then the scatters' SQ counters
    timeout -k 10 420 python -u bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.log
    rc=$?; tail -3 gpurun_out/${TAG}_bench_default.log; [ $rc -eq 0 ] || exit $rc
    rm -rf gpurun_out/${TAG}_prof_bench
    timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_bench -o run \
      -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-pcie --no-census > gpurun_out/${TAG}_prof_bench.json \
      2> gpurun_out/${TAG}_prof_bench.log
    rc=$?; echo "[prof] exit $rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_prof_bench.log; exit $rc; }
    k=$(find gpurun_out/${TAG}_prof_bench -name "*kernel_trace.csv" | head -1)
    python3 tools/ktrace_full.py "$k" > gpurun_out/${TAG}_prof_bench_full.txt; head -12 gpurun_out/${TAG}_prof_bench_full.txt
    PMC_OUT=${TAG}_pmc_bench.json bash tools/gpu_pmc_bench.sh || exit $?
    bash tools/gpu_pmc_scatter.sh > gpurun_out/${TAG}_pmc_scatter_sq.txt 2>&1; rc=$?; tail -40 gpurun_out/${TAG}_pmc_scatter_sq.txt; exit $rc ;;
  ab)
    timeout -k 10 420 python -u bench.py --steps ${STEPS:-8} --warmup 2 --ab "$AB" --no-cpu --no-census --no-pcie \
      --flag-steps 0 ${ARGS:-} > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.log
    rc=$?; grep "A/B\|placement" gpurun_out/${TAG}_ab.log; exit $rc ;;
esac
# STAGE=libab: the default bench in alternating processes on the in-tree library and on LIB_B (same box)
if [ "${STAGE}" = "libab" ]; then
  for i in 1 2; do
    for lib in new "${LIB_B}"; do
      if [ "$lib" = new ]; then unset CRDT_LIB_PATH; else export CRDT_LIB_PATH=$lib; fi
      timeout -k 10 300 python -u bench.py --steps ${STEPS:-6} --warmup 2 --no-cpu --no-census --no-pcie --flag-steps 0 ${ARGS:-} \
        > gpurun_out/${TAG}_libab_${i}_$(basename $lib).json 2> gpurun_out/${TAG}_libab_${i}_$(basename $lib).log || exit $?
      python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_libab_${i}_$(basename $lib).json')); ph=d['roofline']['dominant_kernel']['phases_ms_per_step']; print('$lib', d['ms_per_step'], ph, (d.get('placement') or {}).get('level1_ms'), 'flags', (d.get('with_win_flags') or {}).get('ms_per_step'))"
    done
  done
fi
