#!/bin/bash
# Round-6 GPU stages (run under gpurun from the repo root).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r6}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
case "${STAGE:-comm}" in
  comm)
    # the collective deadline: stalled / lost peers over gloo (2 and 8 ranks), RCCL's abort on one rank, the
    # injected failures (point 6 new), the single-rank RCCL parity tests
    timeout -k 10 900 $PYT tests/test_gpu_failures.py > gpurun_out/${TAG}_pytest_failures.log 2>&1 \
      || { tail -40 gpurun_out/${TAG}_pytest_failures.log; exit 1; }
    tail -3 gpurun_out/${TAG}_pytest_failures.log
    timeout -k 10 300 $PYT tests/test_gpu_parity.py -k "rccl" > gpurun_out/${TAG}_pytest_rccl.log 2>&1 \
      || { tail -40 gpurun_out/${TAG}_pytest_rccl.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_rccl.log ;;
  full)
    timeout -k 10 1100 $PYT tests -m gpu > gpurun_out/${TAG}_pytest_full.log 2>&1 \
      || { tail -40 gpurun_out/${TAG}_pytest_full.log; exit 1; }
    tail -3 gpurun_out/${TAG}_pytest_full.log ;;
  bench)
    timeout -k 10 420 python -u bench.py ${ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log
    rc=$?; tail -4 gpurun_out/${TAG}_bench.log; exit $rc ;;
  *) echo "unknown STAGE"; exit 2 ;;
esac
