#!/bin/bash
# Round-3 evidence.  STAGE=a: the GPU parity suite and smoke.  STAGE=b: the PMC traffic of the default
# bench workload (two --pmc passes), the default bench line (reading that PMC summary), and a
# rocprofv3 kernel trace of the same command.  Every GPU step has its own time limit; the script
# stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${STAGE:-a}" = "a" ]; then
  timeout -k 10 1000 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/r03_pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/r03_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke.log 2>&1
  rc=$?; tail -2 gpurun_out/r03_smoke.log; [ $rc -eq 0 ] || exit $rc
else
  bash tools/gpu_pmc_bench.sh || exit $?
  cp gpurun_out/r03_pmc_bench.json profiles/r03_pmc_bench.json
  timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.log
  rc=$?; cat gpurun_out/r03_bench_default.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r03_bench_default.log; exit $rc; }
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof_bench -o run -- python3 bench.py --no-cpu > gpurun_out/r03_prof_bench.json 2> gpurun_out/r03_prof_bench.log
  rc=$?; echo "[prof] exit $rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/r03_prof_bench -name "*kernel_stats.csv" | head -1); python3 tools/kstats.py "$f" > gpurun_out/r03_prof_bench_top.txt
  t=$(find gpurun_out/r03_prof_bench -name "*kernel_trace.csv" | head -1); python3 tools/ktrace_full.py "$t" > gpurun_out/r03_prof_bench_full.txt; head -14 gpurun_out/r03_prof_bench_full.txt
  python3 -c "import json; d=json.load(open('gpurun_out/r03_prof_bench.json')); print('profiled run:', d['ms_per_step'], json.dumps(d['roofline']['dominant_kernel']))"
fi
