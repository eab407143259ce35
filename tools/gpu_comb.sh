#!/bin/bash
# Map-side combine checks: the small combine tests, then the N = 2 bench path over gloo (one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests -k "${TESTS:-combine}" > gpurun_out/comb_tests.log 2>&1
echo "[tests] exit $?"; tail -3 gpurun_out/comb_tests.log
CRDT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29563 bench.py --gpus 2 --steps 2 --warmup 1 --records 4000000 --replicas 16 ${BENCH_ARGS:-} > gpurun_out/comb_bench2.json 2> gpurun_out/comb_bench2.log
echo "[bench2] exit $?"
python3 -c "
import json; d=json.load(open('gpurun_out/comb_bench2.json')); print(d['ms_per_step'], json.dumps(d.get('parity')), d['roofline']['dominant_kernel'].get('plan'))" || tail -30 gpurun_out/comb_bench2.log
