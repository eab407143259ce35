#!/bin/bash
# Round evidence: default bench (with CPU baselines + census), rocprofv3 kernel-trace stats of
# the same command, host-ingest end to end, 2-rank gloo rehearsal of the multi-GPU bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on() { case "$1" in 0) ;; *) echo "[$2] exit $1 -> stop"; exit $1 ;; esac; }
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log
stop_on $? bench; cat gpurun_out/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-census > gpurun_out/prof_default.log 2>&1
stop_on $? rocprof
timeout -k 10 300 python -u tools/ingest_bench.py --records 1000000 --gpu > gpurun_out/ingest.json 2> gpurun_out/ingest.log
stop_on $? ingest; cat gpurun_out/ingest.json
CRDT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --records 250000000 > gpurun_out/bench_weak2.json 2> gpurun_out/bench_weak2.log
stop_on $? weak2; cat gpurun_out/bench_weak2.json
