#!/bin/bash
# route_l1's head fold (round 5): its parity tests, then the loopback probe at N = 8
# (one rank's local work and the bytes it sends, route_l1 vs route_l1 with the head fold).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r5h}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_failures.py -x -v --timeout 300 \
    --timeout-method thread -k "${K:-routed_fanin_equals or loopback_route_ways or eight_rank_route_l1 or route_tune or head}" \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
for n in ${NS:-8}; do
  N=$n STEPS=${STEPS:-2} MODES=${MODES:-route_l1,route_l1_head} timeout -k 10 600 python -u tools/route_probe.py \
    > gpurun_out/${TAG}_probe_n$n.log 2>&1 || { tail -30 gpurun_out/${TAG}_probe_n$n.log; exit 1; }
  echo "N=$n"; grep -E "mean|rows" gpurun_out/${TAG}_probe_n$n.log
done
