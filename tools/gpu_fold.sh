#!/bin/bash
# The split buckets' part folds over a compact part list (k_fold_items): parity subset, then the fan-in
# (order-free and flagged) and cfg3 in alternating processes against LIB_B (the library before).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r5fold}
LIB_B=${LIB_B:-tools/ab/libcrdt_prev.so}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${KSEL:-split or combine_hot or routed_fanin or eight_rank_route_l1 or equals_gather_fanin or hot_keys}" > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for i in 1 2; do
  for lib in new "${LIB_B}"; do
    if [ "$lib" = new ]; then unset CRDT_LIB_PATH; else export CRDT_LIB_PATH=$lib; fi
    out=gpurun_out/${TAG}_${i}_$(basename $lib)
    timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-pcie --flag-steps 4 > $out.json 2> $out.log || exit $?
    python3 -c "import json; d=json.load(open('$out.json')); w=d['with_win_flags']; print('$lib', d['ms_per_step'], 'flags', w['ms_per_step'], w.get('flags_equal_gather'), (d.get('parity') or {}).get('equal'))"
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 10 --warmup 2 --no-cpu --no-pcie > $out.cfg3.json 2> $out.cfg3.log || exit $?
    python3 -c "import json; d=json.load(open('$out.cfg3.json')); print('$lib cfg3', d['ms_per_step'], (d.get('parity') or {}).get('equal'))"
  done
done
