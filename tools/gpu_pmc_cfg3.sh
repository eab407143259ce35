#!/bin/bash
# HBM traffic of the sorted path's kernels on cfg3 (order-free form, the bench default):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes, each under its own timeout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_cfg3
mkdir -p $OUT
BENCH="bench.py --config cfg3 --steps 1 --warmup 0 --no-cpu --no-census --no-pcie"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex "k_part|k_resolve|k_scan" --output-format csv -d $OUT/p$i -o run -- python3 $BENCH > $OUT/p$i.log 2>&1
  rc=$?; echo "[pmc $i] exit $rc"; [ $rc -eq 0 ] || exit $rc
done
