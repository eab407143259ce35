#!/bin/bash
# rocprofv3 evidence for bench.py: kernel-trace stats, then one PMC pass per counter group.
# Each pass runs under its own hard timeout; a crash/timeout ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_r1
mkdir -p $OUT
BENCH="bench.py --steps 2 --warmup 1 --no-cpu --no-census $*"
stop_on() { case "$1" in 0) ;; 124|137|134|139) echo "[$2] exit $1 -> stop"; exit $1 ;; *) echo "[$2] exit $1" ;; esac; }
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1; stop_on $? list
grep -o -E "\b(FETCH_SIZE|WRITE_SIZE|TCC_EA0_RDREQ(_32B)?(_sum)?|TCC_EA0_WRREQ(_64B)?(_sum)?|TCC_HIT(_sum)?|TCC_MISS(_sum)?)\b" $OUT/counters.txt | sort -u > $OUT/counters_found.txt
cat $OUT/counters_found.txt | tr '\n' ' '; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1
stop_on $? trace
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  name=$(echo $grp | tr ' ' '+')
  timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$name -o run -- python3 $BENCH > $OUT/pmc_$name.log 2>&1
  stop_on $? "pmc $grp"
done
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/ub_fetch -o run -- ./tools/ubench_gather > $OUT/ub_fetch.log 2>&1
stop_on $? "ubench pmc"
find $OUT -name "*.csv" | head -30
