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
  perf1)
    # sorted / flagged parity subset (the new flag-pass staging, XCD order, the two-stream resolve), then in-process
    # A/Bs: the order-free step (overlap on / off), the flagged merge (new forms vs the old ones), cfg3
    timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "sorted or flagged" > gpurun_out/${TAG}_pytest_sorted.log 2>&1 \
      || { tail -40 gpurun_out/${TAG}_pytest_sorted.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_sorted.log
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --ab CRDT_SORTED_FORM=0,8388608 --no-cpu --no-census \
      --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_overlap.json 2> gpurun_out/${TAG}_ab_overlap.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_overlap.log; [ $rc -eq 0 ] || exit $rc
    STEPS=16 AB=CRDT_SORTED_FORM=0,8388608,6291456,14680064 timeout -k 10 300 python -u tools/prof_flags.py \
      > gpurun_out/${TAG}_ab_flags.log 2>&1
    rc=$?; grep "A/B\|DIFFER" gpurun_out/${TAG}_ab_flags.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 12 --warmup 2 --ab CRDT_SORTED_FORM=0,8388608 --no-cpu \
      --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_cfg3.json 2> gpurun_out/${TAG}_ab_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_cfg3.log; exit $rc ;;
  flags)
    # the flag passes' forms in one process (0: XCD order + 4-byte staging + 8-record gather; 2097152: plain order;
    # 4194304: byte staging; 6291456: both old), under the kernel trace for the passes' own times
    timeout -k 10 300 $PYT tests/test_gpu_parity.py -k "flagged" > gpurun_out/${TAG}_pytest_flagged.log 2>&1 \
      || { tail -40 gpurun_out/${TAG}_pytest_flagged.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_flagged.log
    export TMPDIR=/tmp
    rm -rf gpurun_out/${TAG}_prof_flags
    STEPS=20 AB=CRDT_SORTED_FORM=0,2097152,4194304,6291456 timeout -k 10 400 rocprofv3 --kernel-trace --stats \
      --output-format csv -d gpurun_out/${TAG}_prof_flags -o run -- python3 tools/prof_flags.py \
      > gpurun_out/${TAG}_ab_flags.log 2>&1
    rc=$?; grep "A/B\|DIFFER" gpurun_out/${TAG}_ab_flags.log; [ $rc -eq 0 ] || exit $rc
    k=$(find gpurun_out/${TAG}_prof_flags -name "*kernel_stats.csv" | head -1)
    grep -i "flags_back\|pflags\|scatter1\|scatter2_seg" "$k" | cut -c1-400 ;;
  compact)
    # the compact form: sorted parity subset (compact cases included), then in-process A/Bs on the fan-in and cfg3
    timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "sorted or compact or flagged_equals" \
      > gpurun_out/${TAG}_pytest_sorted.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_sorted.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_sorted.log
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --ab CRDT_SORTED_FORM=0,1048576 --no-cpu --no-census \
      --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_compact.json 2> gpurun_out/${TAG}_ab_compact.log
    rc=$?; grep "A/B\|placement" gpurun_out/${TAG}_ab_compact.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 12 --warmup 2 --ab CRDT_SORTED_FORM=0,1048576 --no-cpu \
      --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_compact_cfg3.json 2> gpurun_out/${TAG}_ab_compact_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_compact_cfg3.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 420 python -u bench.py --steps 5 --warmup 2 > gpurun_out/${TAG}_bench_default.json \
      2> gpurun_out/${TAG}_bench_default.log
    rc=$?; tail -2 gpurun_out/${TAG}_bench_default.log; exit $rc ;;
  perf2)
    # the flagged form's compact variant (parity subset, then the flagged merge with compact on / off in one process);
    # the routed fan-in tests (head owner work beside the pieces) and the N = 8 loopback probe
    timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "flagged or compact or loopback or routed_fanin or eight_rank_route_l1" \
      > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest.log
    STEPS=12 AB=CRDT_SORTED_FORM=0,1048576 timeout -k 10 300 python -u tools/prof_flags.py > gpurun_out/${TAG}_ab_flags.log 2>&1
    rc=$?; grep "A/B\|DIFFER\|step 0" gpurun_out/${TAG}_ab_flags.log; [ $rc -eq 0 ] || exit $rc
    N=8 STEPS=3 MODES=route_l1,route_l1_head timeout -k 10 600 python -u tools/route_probe.py \
      > gpurun_out/${TAG}_route_probe_n8.txt 2>&1
    rc=$?; tail -25 gpurun_out/${TAG}_route_probe_n8.txt; exit $rc ;;
  ceiling)
    # the streaming ceilings the floors are priced at: the micro-benchmark (grid-stride and
    # block-contiguous copies, the runtime's D2D copy, smaller buffers, the level-1 scatter's own shape), then the
    # default bench line on the same box (its torch copy figure, gpu_clocks.copy_GBs)
    timeout -k 10 300 ./tools/ubench_stream 8 > gpurun_out/${TAG}_ubench_stream.txt 2>&1
    rc=$?; tail -12 gpurun_out/${TAG}_ubench_stream.txt; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 420 python -u bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.log
    rc=$?; tail -2 gpurun_out/${TAG}_bench_default.log; exit $rc ;;
  profiles)
    # the closing tree's evidence for the default command: the bench line under the kernel trace (bench.py's HIP-event
    # average for the dominant kernel beside the trace's), then its HBM bytes (two --pmc passes) into PMC_OUT, which
    # bench.py's roofline.traffic reads
    TAG=$TAG bash tools/gpu_prof_same.sh || exit 1
    PMC_OUT=${PMC_OUT:-r06_pmc_bench.json} bash tools/gpu_pmc_bench.sh ;;
  cfg3)
    # cfg3 on the compact form: the level-1 tile and the sparse-bucket threshold re-tuned in one process each, then a
    # kernel trace of five merges (per-kernel times against the floors)
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 12 --warmup 2 --ab CRDT_L1_TILE=0,28672 --no-cpu \
      --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_cfg3_l1tile.json 2> gpurun_out/${TAG}_cfg3_l1tile.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_cfg3_l1tile.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 12 --warmup 2 --ab CRDT_SPARSE_T=2048,1024,4096 --no-cpu \
      --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_cfg3_sparse.json 2> gpurun_out/${TAG}_cfg3_sparse.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_cfg3_sparse.log; [ $rc -eq 0 ] || exit $rc
    export TMPDIR=/tmp
    rm -rf gpurun_out/${TAG}_prof_cfg3
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_cfg3 -o run \
      -- python3 bench.py --config cfg3 --steps 5 --warmup 2 --no-cpu --no-pcie --no-census --flag-steps 0 \
      > gpurun_out/${TAG}_prof_cfg3.json 2> gpurun_out/${TAG}_prof_cfg3.log
    rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_prof_cfg3.log; exit $rc; }
    k=$(find gpurun_out/${TAG}_prof_cfg3 -name "*kernel_trace.csv" | head -1)
    python3 tools/ktrace_full.py "$k" > gpurun_out/${TAG}_cfg3_full.txt; head -16 gpurun_out/${TAG}_cfg3_full.txt
    rm -f "$k" ;;
  scanjx)
    # the clock scan's step-major grid (CRDT_SORTED_FORM bit 16777216): parity subset, then in-process A/Bs on cfg3
    # (four steps per changeset: the workgroup rounds' tail) and the 1B fan-in
    timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "scan_step_major or packed_form_switches or fused_small" \
      > gpurun_out/${TAG}_pytest_scanjx.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_scanjx.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_scanjx.log
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 16 --warmup 2 --ab CRDT_SORTED_FORM=0,16777216 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_scanjx_cfg3.json 2> gpurun_out/${TAG}_ab_scanjx_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_scanjx_cfg3.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --ab CRDT_SORTED_FORM=0,16777216 --no-cpu --no-census \
      --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_scanjx.json 2> gpurun_out/${TAG}_ab_scanjx.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_scanjx.log; exit $rc ;;
  cfg3b)
    # the scan grid's default (auto: step-major on cfg3) against forced changeset-major, parity subset first; then the
    # flag passes' SQ counters (stage flagsq)
    timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "scan_step_major or packed_form_switches or fused_small" \
      > gpurun_out/${TAG}_pytest_scanjx.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_scanjx.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_scanjx.log
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 16 --warmup 2 --ab CRDT_SORTED_FORM=0,33554432 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_scanjx_cfg3.json 2> gpurun_out/${TAG}_ab_scanjx_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_scanjx_cfg3.log; [ $rc -eq 0 ] || exit $rc
    STAGE=flagsq TAG=$TAG bash tools/gpu_r6.sh ;;
  sparsek)
    # the sparse buckets in their own kernel (k_resolve_sparse; CRDT_SORTED_FORM bit 67108864 = inside k_resolve_packed):
    # parity subset, in-process A/B on cfg3 and the fan-in, then cfg3's kernel trace
    timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "sparse or packed_form_switches or sorted_compact or scan_step_major" \
      > gpurun_out/${TAG}_pytest_sparsek.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_sparsek.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_sparsek.log
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 16 --warmup 2 --ab CRDT_SORTED_FORM=0,67108864 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_sparsek_cfg3.json 2> gpurun_out/${TAG}_ab_sparsek_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_sparsek_cfg3.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --ab CRDT_SORTED_FORM=0,67108864 --no-cpu --no-census \
      --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_sparsek.json 2> gpurun_out/${TAG}_ab_sparsek.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_sparsek.log; [ $rc -eq 0 ] || exit $rc
    export TMPDIR=/tmp
    rm -rf gpurun_out/${TAG}_prof_cfg3
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_cfg3 -o run \
      -- python3 bench.py --config cfg3 --steps 5 --warmup 2 --no-cpu --no-pcie --no-census --flag-steps 0 \
      > gpurun_out/${TAG}_prof_cfg3.json 2> gpurun_out/${TAG}_prof_cfg3.log
    rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_prof_cfg3.log; exit $rc; }
    k=$(find gpurun_out/${TAG}_prof_cfg3 -name "*kernel_trace.csv" | head -1)
    python3 tools/ktrace_full.py "$k" > gpurun_out/${TAG}_cfg3_full.txt; head -24 gpurun_out/${TAG}_cfg3_full.txt
    rm -f "$k" ;;
  fbpre)
    # the flag passes with the tile's positions loaded first (CRDT_SORTED_FORM bit 134217728): every flagged test with
    # the bit set, then the flagged merge A/B (old / new) in one process under the kernel trace
    CRDT_SORTED_FORM=134217728 timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "flagged" \
      > gpurun_out/${TAG}_pytest_fbpre.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_fbpre.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_fbpre.log
    export TMPDIR=/tmp
    rm -rf gpurun_out/${TAG}_prof_fbpre
    STEPS=12 AB=CRDT_SORTED_FORM=0,134217728 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/${TAG}_prof_fbpre -o run -- python3 tools/prof_flags.py > gpurun_out/${TAG}_ab_fbpre.log 2>&1
    rc=$?; grep "A/B\|DIFFER" gpurun_out/${TAG}_ab_fbpre.log; [ $rc -eq 0 ] || exit $rc
    k=$(find gpurun_out/${TAG}_prof_fbpre -name "*kernel_stats.csv" | head -1)
    grep -i "flags_back\|pflags" "$k" | cut -c1-300
    find gpurun_out/${TAG}_prof_fbpre -name "*kernel_trace.csv" -delete ;;
  lists)
    # round-6 closing forms: the flag passes with positions first (default; 134217728 = round 5's, 536870912 = level 2
    # in 512-thread workgroups), the packed resolve's per-kernel item lists (default; 268435456 = every item slot);
    # sorted / flagged / sparse parity, then A/Bs on the flagged merge (kernel trace), cfg3 and the fan-in
    timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "flagged or sorted or sparse or compact or scan_step or fused" \
      > gpurun_out/${TAG}_pytest_lists.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_lists.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_lists.log
    export TMPDIR=/tmp
    rm -rf gpurun_out/${TAG}_prof_fb
    STEPS=12 AB=CRDT_SORTED_FORM=0,134217728,536870912 timeout -k 10 400 rocprofv3 --kernel-trace --stats \
      --output-format csv -d gpurun_out/${TAG}_prof_fb -o run -- python3 tools/prof_flags.py > gpurun_out/${TAG}_ab_fb.log 2>&1
    rc=$?; grep "A/B\|DIFFER" gpurun_out/${TAG}_ab_fb.log; [ $rc -eq 0 ] || exit $rc
    k=$(find gpurun_out/${TAG}_prof_fb -name "*kernel_stats.csv" | head -1)
    grep -i "flags_back" "$k" | cut -c1-250
    find gpurun_out/${TAG}_prof_fb -name "*kernel_trace.csv" -delete
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 16 --warmup 2 --ab CRDT_SORTED_FORM=0,268435456 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_lists_cfg3.json 2> gpurun_out/${TAG}_ab_lists_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_lists_cfg3.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --ab CRDT_SORTED_FORM=0,268435456 --no-cpu --no-census \
      --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_lists.json 2> gpurun_out/${TAG}_ab_lists.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_lists.log; [ $rc -eq 0 ] || exit $rc
    rm -rf gpurun_out/${TAG}_prof_cfg3
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_cfg3 -o run \
      -- python3 bench.py --config cfg3 --steps 5 --warmup 2 --no-cpu --no-pcie --no-census --flag-steps 0 \
      > gpurun_out/${TAG}_prof_cfg3.json 2> gpurun_out/${TAG}_prof_cfg3.log
    rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_prof_cfg3.log; exit $rc; }
    k=$(find gpurun_out/${TAG}_prof_cfg3 -name "*kernel_trace.csv" | head -1)
    python3 tools/ktrace_full.py "$k" > gpurun_out/${TAG}_cfg3_full.txt; head -26 gpurun_out/${TAG}_cfg3_full.txt
    rm -f "$k" ;;
  lists2)
    # the ordered (flagged) resolve on item lists (default; 268435456 = every slot) and the level-1 flag pass staging
    # 28 bytes per batch (1073741824): flagged parity, then the flagged merge A/B under the kernel trace
    timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "flagged or sorted_sparse or packed_form" \
      > gpurun_out/${TAG}_pytest_lists2.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_lists2.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_lists2.log
    export TMPDIR=/tmp
    rm -rf gpurun_out/${TAG}_prof_fb
    STEPS=12 AB=CRDT_SORTED_FORM=0,268435456,1073741824 timeout -k 10 400 rocprofv3 --kernel-trace --stats \
      --output-format csv -d gpurun_out/${TAG}_prof_fb -o run -- python3 tools/prof_flags.py > gpurun_out/${TAG}_ab_fb.log 2>&1
    rc=$?; grep "A/B\|DIFFER" gpurun_out/${TAG}_ab_fb.log; [ $rc -eq 0 ] || exit $rc
    find gpurun_out/${TAG}_prof_fb -name "*kernel_trace.csv" -delete ;;
  scanw5)
    # the fused-histogram scan at 5 waves per SIMD (bit 1073741824): parity subset, A/B on the fan-in and cfg3; then
    # cfg3's HBM bytes per kernel (FETCH_SIZE / WRITE_SIZE passes, tools/gpu_pmc_cfg3.sh)
    timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "packed_form_switches or scan_step_major or sorted_compact" \
      > gpurun_out/${TAG}_pytest_scanw5.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_scanw5.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_scanw5.log
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --ab CRDT_SORTED_FORM=0,1073741824 --no-cpu --no-census \
      --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_scanw5.json 2> gpurun_out/${TAG}_ab_scanw5.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_scanw5.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 16 --warmup 2 --ab CRDT_SORTED_FORM=0,1073741824 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_scanw5_cfg3.json 2> gpurun_out/${TAG}_ab_scanw5_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_scanw5_cfg3.log; [ $rc -eq 0 ] || exit $rc
    bash tools/gpu_pmc_cfg3.sh || exit 1
    python3 tools/pmc_kernels.py gpurun_out/pmc_cfg3/p1 gpurun_out/pmc_cfg3/p2 > gpurun_out/${TAG}_pmc_cfg3.txt 2>&1
    rc=$?; cat gpurun_out/${TAG}_pmc_cfg3.txt; rm -rf gpurun_out/pmc_cfg3; exit $rc ;;
  posT)
    # the flagged level 1's tile-strided positions from registers (default; 2147483648 = LDS-staged at the input
    # index): flagged parity, then the flagged merge A/B under the kernel trace
    timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "flagged" \
      > gpurun_out/${TAG}_pytest_posT.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_posT.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_posT.log
    export TMPDIR=/tmp
    rm -rf gpurun_out/${TAG}_prof_posT
    STEPS=12 AB=CRDT_SORTED_FORM=0,2147483648 timeout -k 10 400 rocprofv3 --kernel-trace --stats \
      --output-format csv -d gpurun_out/${TAG}_prof_posT -o run -- python3 tools/prof_flags.py > gpurun_out/${TAG}_ab_posT.log 2>&1
    rc=$?; grep "A/B\|DIFFER" gpurun_out/${TAG}_ab_posT.log; [ $rc -eq 0 ] || exit $rc
    find gpurun_out/${TAG}_prof_posT -name "*kernel_trace.csv" -delete
    k=$(find gpurun_out/${TAG}_prof_posT -name "*kernel_stats.csv" | head -1)
    grep -i "flags_back\|scatter1" "$k" | cut -c1-200 ;;
  sparset)
    # the sparse threshold re-tuned on the closing tree's cfg3 (k_resolve_sparse), then the default bench line
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 18 --warmup 2 --ab CRDT_SPARSE_T=2048,4096,8192 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_sparset_cfg3.json 2> gpurun_out/${TAG}_ab_sparset_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_sparset_cfg3.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 420 python -u bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.log
    rc=$?; tail -2 gpurun_out/${TAG}_bench_default.log; exit $rc ;;
  hist4)
    # the level-2 histogram with four tiles per workgroup (default; 1073741824 = one): parity subset, A/B on the fan-in,
    # cfg3 and the flagged merge
    timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "packed_form_switches or sorted or compact or flagged_equals" \
      > gpurun_out/${TAG}_pytest_hist4.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_hist4.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_hist4.log
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --ab CRDT_SORTED_FORM=0,1073741824 --no-cpu --no-census \
      --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_hist4.json 2> gpurun_out/${TAG}_ab_hist4.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_hist4.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 16 --warmup 2 --ab CRDT_SORTED_FORM=0,1073741824 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_hist4_cfg3.json 2> gpurun_out/${TAG}_ab_hist4_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_hist4_cfg3.log; [ $rc -eq 0 ] || exit $rc
    export TMPDIR=/tmp
    rm -rf gpurun_out/${TAG}_prof_h4
    STEPS=12 AB=CRDT_SORTED_FORM=0,1073741824 timeout -k 10 400 rocprofv3 --kernel-trace --stats \
      --output-format csv -d gpurun_out/${TAG}_prof_h4 -o run -- python3 tools/prof_flags.py > gpurun_out/${TAG}_ab_h4flags.log 2>&1
    rc=$?; grep "A/B\|DIFFER" gpurun_out/${TAG}_ab_h4flags.log; [ $rc -eq 0 ] || exit $rc
    find gpurun_out/${TAG}_prof_h4 -name "*kernel_trace.csv" -delete
    k=$(find gpurun_out/${TAG}_prof_h4 -name "*kernel_stats.csv" | head -1)
    grep -i "hist16w" "$k" | cut -c1-160 ;;
  spside)
    # the sparse buckets on the side stream (1073741824) against the default: parity subset, cfg3 A/B
    timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "sparse or packed_form_switches" \
      > gpurun_out/${TAG}_pytest_spside.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_spside.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_spside.log
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 20 --warmup 2 --ab CRDT_SORTED_FORM=0,1073741824 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_spside_cfg3.json 2> gpurun_out/${TAG}_ab_spside_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_spside_cfg3.log; exit $rc ;;
  closing)
    # the closing tree's evidence: the default command under the kernel trace + its PMC bytes (r06_pmc_bench.json),
    # the cfg3 line with full-table parity, then the driver's N = 8 command as 8 gloo ranks on this GPU
    STAGE=profiles TAG=$TAG bash tools/gpu_r6.sh || exit 1
    timeout -k 10 420 python -u bench.py --config cfg3 > gpurun_out/${TAG}_bench_cfg3.json 2> gpurun_out/${TAG}_bench_cfg3.log
    rc=$?; tail -2 gpurun_out/${TAG}_bench_cfg3.log; [ $rc -eq 0 ] || exit $rc
    NS=8 TAG=${TAG}n8 LIMIT=600 bash tools/gpu_rehearse_n.sh ;;
  libab)
    # the tree's library against build_ab/libcrdt_prev.so (CRDT_LIB_PATH), alternating processes: the fan-in, cfg3
    # and the flagged merge; parity subset on the tree's library first
    timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "sorted or compact or flagged" \
      > gpurun_out/${TAG}_pytest_libab.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_libab.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_libab.log
    for i in 1 2; do
      for lib in tree prev; do
        L=""; [ $lib = prev ] && L=$PWD/build_ab/libcrdt_prev.so
        CRDT_LIB_PATH=$L timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu --no-census --no-pcie \
          --flag-steps 0 > gpurun_out/${TAG}_${lib}_$i.json 2> gpurun_out/${TAG}_${lib}_$i.log || exit 1
        CRDT_LIB_PATH=$L timeout -k 10 300 python -u bench.py --config cfg3 --steps 12 --warmup 2 --no-cpu --no-census \
          --no-pcie --flag-steps 0 > gpurun_out/${TAG}_${lib}_cfg3_$i.json 2> gpurun_out/${TAG}_${lib}_cfg3_$i.log || exit 1
        CRDT_LIB_PATH=$L STEPS=6 timeout -k 10 300 python -u tools/prof_flags.py > gpurun_out/${TAG}_${lib}_flags_$i.log 2>&1 || exit 1
        python3 -c "
import json
a=json.load(open('gpurun_out/${TAG}_${lib}_$i.json')); b=json.load(open('gpurun_out/${TAG}_${lib}_cfg3_$i.json'))
f=[l for l in open('gpurun_out/${TAG}_${lib}_flags_$i.log') if l.startswith('A/B') or 'mean' in l]
print('$lib $i fanin', a['ms_per_step'], a['roofline']['dominant_kernel']['phases_ms_per_step'], 'cfg3', b['ms_per_step'], f[-1].strip() if f else '')"
      done
    done ;;
  scanacc)
    # the sorted path's scan publishing its frame once per workgroup (k_scan_hv; 1073741824 = per tile, round 5):
    # parity subset, A/B on the fan-in (phases), cfg3 and the flagged merge
    timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "packed_form_switches or sorted or compact or flagged" \
      > gpurun_out/${TAG}_pytest_scanacc.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_scanacc.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_scanacc.log
    timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --ab CRDT_SORTED_FORM=0,1073741824,4096 --no-cpu --no-census \
      --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_scanacc.json 2> gpurun_out/${TAG}_ab_scanacc.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_scanacc.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 18 --warmup 2 --ab CRDT_SORTED_FORM=0,1073741824,4096 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_scanacc_cfg3.json 2> gpurun_out/${TAG}_ab_scanacc_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_scanacc_cfg3.log; [ $rc -eq 0 ] || exit $rc
    STEPS=12 AB=CRDT_SORTED_FORM=0,1073741824,4096 timeout -k 10 300 python -u tools/prof_flags.py \
      > gpurun_out/${TAG}_ab_scanacc_flags.log 2>&1
    rc=$?; grep "A/B\|DIFFER" gpurun_out/${TAG}_ab_scanacc_flags.log; exit $rc ;;
  scanpf)
    # the sorted path's scan with the next tile in flight (k_scan_pf, default; 4096 = k_scan): parity subset, A/B on
    # the fan-in, cfg3 and the flagged merge
    timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "packed_form_switches or sorted or compact or flagged or scan_step" \
      > gpurun_out/${TAG}_pytest_scanpf.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_scanpf.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_scanpf.log
    timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --ab CRDT_SORTED_FORM=0,4096 --no-cpu --no-census \
      --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_scanpf.json 2> gpurun_out/${TAG}_ab_scanpf.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_scanpf.log; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 16 --warmup 2 --ab CRDT_SORTED_FORM=0,4096 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_scanpf_cfg3.json 2> gpurun_out/${TAG}_ab_scanpf_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_scanpf_cfg3.log; [ $rc -eq 0 ] || exit $rc
    STEPS=12 AB=CRDT_SORTED_FORM=0,4096 timeout -k 10 300 python -u tools/prof_flags.py > gpurun_out/${TAG}_ab_scanpf_flags.log 2>&1
    rc=$?; grep "A/B\|DIFFER" gpurun_out/${TAG}_ab_scanpf_flags.log; exit $rc ;;
  cfgs)
    # the other single-GPU configs on the closing tree, each with its parity: cfg2 (one 10M changeset), cfg5 (100
    # streaming 10M-record deltas)
    for cfg in cfg2 cfg5; do
      timeout -k 10 420 python -u bench.py --config $cfg > gpurun_out/${TAG}_bench_$cfg.json 2> gpurun_out/${TAG}_bench_$cfg.log
      rc=$?; tail -1 gpurun_out/${TAG}_bench_$cfg.log; [ $rc -eq 0 ] || exit $rc
      python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_$cfg.json')); print('$cfg', d['ms_per_step'], d['value'], d['roofline']['frac'], (d.get('parity') or {}).get('equal'))"
    done ;;
  cfg5jx)
    # cfg5 with the scan's step-major grid (the default: its 10M-record deltas are ~2.4K workgroups) against forced off
    timeout -k 10 420 python -u bench.py --config cfg5 --steps 8 --warmup 2 --ab CRDT_SORTED_FORM=0,33554432 --no-cpu --no-census --no-pcie \
      > gpurun_out/${TAG}_ab_cfg5jx.json 2> gpurun_out/${TAG}_ab_cfg5jx.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_cfg5jx.log; exit $rc ;;
  fb1024)
    # the level-1 flag pass in 1024-thread workgroups (bit 2) against 512: flagged parity, then the flagged merge A/B
    # under the kernel trace
    timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "flagged" \
      > gpurun_out/${TAG}_pytest_fb1024.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_fb1024.log; exit 1; }
    tail -2 gpurun_out/${TAG}_pytest_fb1024.log
    export TMPDIR=/tmp
    rm -rf gpurun_out/${TAG}_prof_fb
    STEPS=12 AB=CRDT_SORTED_FORM=0,2 timeout -k 10 400 rocprofv3 --kernel-trace --stats \
      --output-format csv -d gpurun_out/${TAG}_prof_fb -o run -- python3 tools/prof_flags.py > gpurun_out/${TAG}_ab_fb1024.log 2>&1
    rc=$?; grep "A/B\|DIFFER" gpurun_out/${TAG}_ab_fb1024.log; [ $rc -eq 0 ] || exit $rc
    find gpurun_out/${TAG}_prof_fb -name "*kernel_trace.csv" -delete
    k=$(find gpurun_out/${TAG}_prof_fb -name "*kernel_stats.csv" | head -1)
    grep -i "flags_back" "$k" | cut -c1-200 ;;
  sweep)
    timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "random_sweep" > gpurun_out/${TAG}_pytest_sweep.log 2>&1 \
      || { tail -60 gpurun_out/${TAG}_pytest_sweep.log; exit 1; }
    tail -3 gpurun_out/${TAG}_pytest_sweep.log ;;
  sparset2)
    timeout -k 10 300 python -u bench.py --config cfg3 --steps 18 --warmup 2 --ab CRDT_SPARSE_T=2048,1024,1536 \
      --no-cpu --no-census --no-pcie --flag-steps 0 > gpurun_out/${TAG}_ab_sparset2_cfg3.json 2> gpurun_out/${TAG}_ab_sparset2_cfg3.log
    rc=$?; grep "A/B" gpurun_out/${TAG}_ab_sparset2_cfg3.log; exit $rc ;;
  flagsq)
    # SQ counters of the flag passes on the closing tree: the wait / issue breakdown (each counter
    # checked against rocprofv3 -L first), then the LDS / VALU pass of tools/gpu_pmc_flags.sh
    export TMPDIR=/tmp
    timeout -k 10 120 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || exit 1
    C2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
    for c in $C2; do grep -qw "$c" gpurun_out/${TAG}_counters.txt || { echo "no counter $c"; exit 1; }; done
    OUT=${TAG}_pmc_flags_sq bash tools/gpu_pmc_flags.sh > gpurun_out/${TAG}_pmc_flags_sq.txt 2>&1
    rc=$?; cat gpurun_out/${TAG}_pmc_flags_sq.txt | cut -c1-400; [ $rc -eq 0 ] || exit $rc
    CTRS="$C2" OUT=${TAG}_pmc_flags_sq2 bash tools/gpu_pmc_flags.sh > gpurun_out/${TAG}_pmc_flags_sq2.txt 2>&1
    rc=$?; cat gpurun_out/${TAG}_pmc_flags_sq2.txt | cut -c1-400; exit $rc ;;
  full)
    timeout -k 10 1100 $PYT tests -m gpu > gpurun_out/${TAG}_pytest_full.log 2>&1 \
      || { tail -40 gpurun_out/${TAG}_pytest_full.log; exit 1; }
    tail -3 gpurun_out/${TAG}_pytest_full.log ;;
  bench)
    timeout -k 10 420 python -u bench.py ${ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log
    rc=$?; tail -4 gpurun_out/${TAG}_bench.log; exit $rc ;;
  *) echo "unknown STAGE"; exit 2 ;;
esac
