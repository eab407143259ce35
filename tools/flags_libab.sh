#!/bin/bash
# The flagged merge (with_win_flags, the census on) in alternating processes on the in-tree library and LIB_B.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r5fl}
for i in 1 2; do
  for lib in new "${LIB_B}"; do
    if [ "$lib" = new ]; then unset CRDT_LIB_PATH; else export CRDT_LIB_PATH=$lib; fi
    out=gpurun_out/${TAG}_${i}_$(basename $lib)
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-pcie --flag-steps ${FSTEPS:-4} > $out.json 2> $out.log || exit $?
    python3 -c "import json; d=json.load(open('$out.json')); w=d['with_win_flags']; print('$lib', d['ms_per_step'], 'flags', w['ms_per_step'], w.get('flags_equal_gather'))"
  done
done
