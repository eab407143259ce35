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
      timeout -k 10 300 python -u bench.py --steps ${STEPS:-6} --warmup 2 --no-cpu --no-census --no-pcie --flag-steps 0 \
        > gpurun_out/${TAG}_libab_${i}_$(basename $lib).json 2> gpurun_out/${TAG}_libab_${i}_$(basename $lib).log || exit $?
      python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_libab_${i}_$(basename $lib).json')); ph=d['roofline']['dominant_kernel']['phases_ms_per_step']; print('$lib', d['ms_per_step'], ph, d.get('placement',{}).get('level1_ms'))"
    done
  done
fi
