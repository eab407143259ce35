#!/bin/bash
# One GPU session: parity tests, smoke, short benches. Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok_or_stop() {  # $1 = exit code, $2 = step name; tests may fail (1) but a crash/timeout ends the session
  case "$1" in
    0|1|2|5) echo "[$2] exit $1" ;;
    *) echo "[$2] exit $1 -> stopping"; exit "$1" ;;
  esac
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
ok_or_stop $? pytest
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
ok_or_stop $? smoke
cat gpurun_out/smoke.log
for spec in "${@}"; do
  name=$(echo "$spec" | cut -d: -f1); cmd=$(echo "$spec" | cut -d: -f2-)
  timeout -k 10 400 python -u bench.py $cmd > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.log
  ok_or_stop $? "bench $name"
  cat gpurun_out/bench_$name.json
done
