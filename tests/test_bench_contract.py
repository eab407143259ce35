"""bench.py's output contract on a small fan-in: one JSON line with the driver's keys, the
roofline and cpu_baseline objects, and full-table parity against the OpenMP oracle.

Runs bench.py as a child process (one extra GPU process) at 1/250 of the default size so it
finishes in seconds; the default-size line is in profiles/r01_bench_default.json."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _run_bench(*extra):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
           "--records", "4000000", "--replicas", "16", "--keys", str(1 << 22), "--local", str(1 << 21),
           "--cpu-seconds", "0.5", "--no-pcie", *extra]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["gather", "sorted"])
def test_bench_line_contract(gpu_device, path):
    d = _run_bench("--path", path)
    for k in KEYS:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "strong" and d["data"] == "synthetic"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["records"] == 4000000 and d["config"]["merge_path"] == path
    rf, job = d["roofline"], d["job"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    # the contract fraction: SURVEY 8(d)'s B_alg over distinct keys / step time
    b_alg = 20 * d["config"]["records"] + 12 * job["U_touch"] + 24 * job["U_win"]
    assert job["B_alg_bytes"] == b_alg
    assert abs(rf["frac"] - b_alg / (d["ms_per_step"] / 1e3) / 8e12) < 2e-3
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0
    assert d["parity"]["equal"] is True and d["parity"]["fields_differing"] == 0
    pl = d["placement"]                                        # the level-1 placement tuner (sorted path only)
    assert (pl["kept"] is not None and len(pl["level1_ms"]) == pl["candidates"]) if path == "sorted" \
        else pl is None or pl["kept"] is None


@pytest.mark.gpu
def test_bench_two_ranks_routed(gpu_device):
    """The N > 1 bench path (config 4: the same records in total, replica j on rank j % N, routed
    to key % N inside the library's collective merge) with 2 ranks on one GPU over the gloo
    communicator: the driver's N = 2..8 runs take the same code with RCCL, one GPU per rank."""
    env = dict(os.environ, CRDT_BENCH_BACKEND="gloo", CRDT_ROUTE_TUNE="1")   # (64 changesets: the tuner runs)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29561", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--records", "4000000", "--replicas", "64"]
    # (default key space: torch.distributed.run's own parser takes `--local` for `--local-addr`)
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]                  # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["parallelism"] == "keyshard2-routed" and d["config"]["records"] == 4000000
    assert d["value"] == pytest.approx(4000000 / (d["ms_per_step"] / 1e3), rel=1e-3)
    assert d["presharded"]["value"] > 0
    assert d["job"]["U_touch"] > 0 and d["job"]["U_win"] > 0
    ab = d["route_ab"]                                          # one timed step per way of routing
    assert ab["combine"]["combined"] and not ab["route"]["route_l1"] and not ab["route"]["combined"]
    assert all(ab[m]["ms"] > 0 for m in ("route_l1", "combine", "route"))
    tune = d["route_tune"]                                      # the way every timed step took, measured
    ways = ("route_l1", "combine", "route_l1_4", "route_l1_1", "route_l1_head")
    assert tune["best"] in ways and all(tune[f"{w}_ms"] > 0 for w in ways)
    assert ab["default_plan"]["combined"] == (tune["best"] == "combine")
