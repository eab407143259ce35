#!/bin/bash
# The default bench line under a rocprofv3 kernel trace: the JSON line and the per-kernel durations come from
# ONE command, so bench.py's HIP-event average for the dominant kernel and the trace's can be compared directly.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05d}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 -u bench.py "$@" > gpurun_out/${TAG}_bench_prof.json 2> gpurun_out/${TAG}_bench_prof.log || { tail -20 gpurun_out/${TAG}_bench_prof.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_prof.json')); k=d['roofline']['dominant_kernel']; print(d['ms_per_step'], d['roofline']['frac'], k['avg_launch_us'], k['frac'], (d.get('parity') or {}).get('equal'))"
kt=$(find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" | head -1)
python3 tools/ktrace_full.py "$kt" > gpurun_out/${TAG}_prof_bench_full.txt && head -12 gpurun_out/${TAG}_prof_bench_full.txt
ks=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1)
cp "$ks" gpurun_out/${TAG}_prof_bench_kernel_stats.csv
rm -f "$kt"
