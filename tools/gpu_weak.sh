#!/bin/bash
# Rehearsal of the weak-scaling (parts) protocol: N ranks on the one GPU of a gpurun box, gloo
# collectives (RCCL needs a GPU per rank). Checks the protocol end to end, not the scaling.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
N=${1:-2}; REC=${2:-250000000}; shift 2 2>/dev/null; EXTRA="$*"
CRDT_BENCH_BACKEND=gloo timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N --steps 3 --warmup 1 --records $REC \
  --no-cpu $EXTRA > gpurun_out/bench_weak$N.json 2> gpurun_out/bench_weak$N.log
rc=$?
echo "[weak$N] exit $rc"; cat gpurun_out/bench_weak$N.json; tail -5 gpurun_out/bench_weak$N.log
exit $rc
