#!/bin/bash
# PMC passes on the sorted path's kernels (one counter group per run, each under its own timeout).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sorted
mkdir -p $OUT
BENCH="bench.py --steps 1 --warmup 0 --no-cpu --no-census --path sorted --records 250000000 --replicas 256 $*"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex "k_part|k_resolve_b" --output-format csv -d $OUT/p$i -o run -- python3 $BENCH > $OUT/p$i.log 2>&1
  rc=$?; echo "[pmc $i] exit $rc"; [ $rc -eq 0 ] || exit $rc
done
