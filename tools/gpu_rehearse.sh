#!/bin/bash
# The driver's N = 8 commands rehearsed as 8 gloo ranks on ONE GPU (round 5): the fan-in (config 4) and the
# streaming config 5, each at full size, per-rank logs under gpurun_out/${TAG}_{fanin,cfg5}_logs.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r5r}
for cfg in ${CFGS:-fanin cfg5}; do
  extra="--no-presharded"; [ $cfg = cfg5 ] && extra=""
  CRDT_BENCH_BACKEND=gloo timeout -k 10 ${LIMIT:-480} python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29537 --log-dir gpurun_out/${TAG}_${cfg}_logs --redirects 3 \
    bench.py --config $cfg --gpus 8 --steps ${STEPS:-2} --warmup 1 $extra --no-cpu-copy16 --cpu-seconds 5 \
    > gpurun_out/${TAG}_${cfg}.out 2>&1
  rc=$?; echo "$cfg torchrun rc=$rc"
  f=$(find gpurun_out/${TAG}_${cfg}_logs -path "*/0/stdout.log" | head -1)
  python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{\"metric\"'):
        d=json.loads(l); p=d.get('parity') or {}
        print('$cfg', d['ms_per_step'], 'ms', 'parity', p.get('equal'), p.get('digest_blocks'), 'tune', (d.get('route_tune') or {}).get('best'))"
  [ $rc -eq 0 ] || exit $rc
done
