#!/bin/bash
# Round-3 GPU steps.  STAGE selects what runs; every GPU step has its own time limit and the
# script stops at the first failure.
#   tests  : the -m gpu tests named by TESTS (pytest -k expression; default: all)
#   bench  : the default bench line (BENCH_ARGS appended), output gpurun_out/r03_${TAG}.json
#   ab     : bench.py --ab $AB (in-process A/B of a library switch)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
for stage in ${STAGE:-tests}; do
  case "$stage" in
    tests)
      timeout -k 10 ${TLIM:-900} python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests \
        ${TESTS:+-k "$TESTS"} > gpurun_out/r03_pytest_${TAG}.log 2>&1
      rc=$?; tail -5 gpurun_out/r03_pytest_${TAG}.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1
      rc=$?; tail -2 gpurun_out/r03_smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 ${TLIM:-600} python -u bench.py ${BENCH_ARGS:-} > gpurun_out/r03_${TAG}.json 2> gpurun_out/r03_${TAG}.log
      rc=$?; cat gpurun_out/r03_${TAG}.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r03_${TAG}.log; exit $rc; } ;;
    ab)
      timeout -k 10 ${TLIM:-600} python -u bench.py --no-cpu --no-census --no-pcie --steps ${ABSTEPS:-8} --warmup 2 \
        --ab "$AB" ${BENCH_ARGS:-} > gpurun_out/r03_ab_${TAG}.json 2> gpurun_out/r03_ab_${TAG}.log
      rc=$?; grep "A/B" gpurun_out/r03_ab_${TAG}.log; [ $rc -eq 0 ] || { tail -20 gpurun_out/r03_ab_${TAG}.log; exit $rc; } ;;
    route8)   # config 4's N = 8 path rehearsed with 8 ranks on one GPU over the gloo crdt_comm_ops table
      CRDT_BENCH_BACKEND=gloo timeout -k 10 ${TLIM:-600} python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node ${NR:-8} --master-addr 127.0.0.1 --master-port ${PORT:-29517} bench.py --gpus ${NR:-8} \
        --records ${RECS:-16000000} --steps 2 --warmup 1 --cpu-seconds 3 ${BENCH_ARGS:-} \
        > gpurun_out/r03_bench_route${NR:-8}_gloo.json 2> gpurun_out/r03_bench_route${NR:-8}_gloo.log
      rc=$?; cat gpurun_out/r03_bench_route${NR:-8}_gloo.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/r03_bench_route${NR:-8}_gloo.log; exit $rc; } ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
