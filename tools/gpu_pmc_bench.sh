#!/bin/bash
# HBM traffic of the default bench's merge step: two rocprofv3 --pmc passes (FETCH_SIZE, then
# WRITE_SIZE: they cannot share a pass on gfx950), each its own run, then tools/pmc_step.py.
# ARGS = the bench workload (the default one); the run merges warmup + steps times.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${ARGS:-"--steps 2 --warmup 1 --no-cpu --no-census --no-pcie"}
MERGES=${MERGES:-3}                 # merges the command runs (warmup + steps)
export CRDT_PLACE_TRIES=1           # (no placement-trial merges: the bytes of a step do not depend on them)
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py $ARGS > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "[fetch] exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_fetch.log; exit $rc; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py $ARGS > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "[write] exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_write.log; exit $rc; }
CMD=$(python3 -c "
import json, sys; sys.argv=['bench.py']+'$ARGS'.split(); sys.path.insert(0,'.')
import bench; a=bench.parse(); print(json.dumps({'command_args': bench.pmc_args(a), 'merge_path': '${PMC_PATH:-sorted}', 'command': 'python bench.py $ARGS'}))")
python3 tools/pmc_step.py gpurun_out/pmc_fetch gpurun_out/pmc_write $MERGES gpurun_out/${PMC_OUT:-r03_pmc_bench.json} "$CMD"
