#!/bin/bash
# The driver's fan-in bench at N ranks (gloo, all on ONE GPU), full size: NS="2 4".
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r5rn}
for n in ${NS:-2 4}; do
  CRDT_BENCH_BACKEND=gloo timeout -k 10 ${LIMIT:-500} python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2954$n --log-dir gpurun_out/${TAG}_n${n}_logs --redirects 3 \
    bench.py --gpus $n --steps 2 --warmup 1 --no-presharded --no-cpu-copy16 --cpu-seconds 5 > gpurun_out/${TAG}_n$n.out 2>&1
  rc=$?; echo "N=$n torchrun rc=$rc"
  f=$(find gpurun_out/${TAG}_n${n}_logs -path "*/0/stdout.log" | head -1)
  python3 -c "
import json
for l in open('$f'):
    if l.startswith('{\"metric\"'):
        d=json.loads(l); p=d.get('parity') or {}
        print('N=$n', d['ms_per_step'], 'ms parity', p.get('equal'), p.get('digest_blocks'), 'tune', d.get('route_tune'), 'exchange', d.get('exchange'))"
  [ $rc -eq 0 ] || exit $rc
done
