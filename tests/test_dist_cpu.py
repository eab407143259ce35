"""Sharded replica protocol on CPU: gloo, world size 2 and 3.

Each rank owns keys ``key % G`` (slot ``key // G``); tests/_phase_model.py restates
crdt_amd/csrc/comm_path.inc::merge_sharded in numpy and issues its collectives through
``crdt_amd.dist.GlooComm`` — the communicator the GPU tests hand the library.  Three
input layouts, each against the single-table sequential C oracle (every row, every win
flag, canonical, exception fields, counts):

* routed: changeset j arrives whole on rank j % G (north star config 4);
* parts: every changeset is split over the ranks without regard to ownership, its
  iteration order rank-major;
* presharded: every rank holds exactly the records it owns (no record exchange).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from crdt_amd.dist import GlooComm, home_part, route_by_owner
from tests._cases import ABSENT_MOD, CASE_SPECS, make_case, oracle_run
from tests._phase_model import ShardModel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def layout(case, world, rank, kind):
    """(the case in the iteration order the layout implies, this rank's rows, its offsets)."""
    key, offs = case["key"], case["offsets"].astype(np.int64)
    R = len(offs) - 1
    if kind == "routed":
        sel, part_offs = home_part(offs, world, rank)
        return case, sel, part_offs
    # parts / presharded: part of record x of changeset j on rank owner(x); changeset order rank-major
    if kind == "parts":
        owner = (np.arange(len(key)) * 7 + 3) % world
    else:
        owner = key.astype(np.int64) % world
    order = []
    for j in range(R):
        seg = np.arange(offs[j], offs[j + 1])
        for r in range(world):
            order.extend(seg[owner[seg] == r])
    order = np.array(order, dtype=np.int64)
    g = dict(case)
    for f in ("key", "lt", "rank", "val"):
        g[f] = case[f][order]
    if case["millis"] is not None:
        g["millis"] = case["millis"][order]
    own = owner[order]
    cs = np.repeat(np.arange(R), np.diff(offs))
    sel = np.nonzero(own == rank)[0]
    counts = np.bincount(cs[sel], minlength=R)
    return g, sel, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)


def _worker(rank, world, port, case_kw, kind, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case, sel, part_offs = layout(make_case(**case_kw), world, rank, kind)
        cap = -(-case["n_ids"] // world)
        t = ShardModel(cap, case["local_rank"], case["c0"], world, rank)
        loc = case["local"]
        ids = np.arange(case["n_local"])
        mine = (ids % world == rank) & (loc["mod"] != ABSENT_MOD)
        t.put_rows(ids[mine] // world, loc["lt"][mine], loc["rank"][mine], loc["val"][mine], loc["mod"][mine])
        key = case["key"][sel]
        if kind == "presharded":
            key = key // world
        millis = None if case["millis"] is None else case["millis"][sel]
        flags = np.zeros(len(sel), np.uint8)
        res = t.merge(key, case["lt"][sel], case["rank"][sel], case["val"][sel], part_offs, case["wall"],
                      GlooComm(dist), millis=millis, win_flags=flags, presharded=kind == "presharded")
        q.put((rank, res, t.lt, t.rank, t.val, t.mod, sel, flags))
    finally:
        dist.destroy_process_group()


def run_sharded(kw, world, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kw, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda o: o[0])


def check(kw, world, kind):
    case, _, _ = layout(make_case(**kw), world, 0, kind)
    orows, ores, oflags = oracle_run(case)
    flags = np.zeros(len(case["key"]), np.uint8)
    for rank, res, lt, rk, val, mod, sel, fl in run_sharded(kw, world, kind):
        for f in ("status", "n_stored", "exc_changeset", "exc_index", "canonical_lt", "drift_ms", "counter",
                  "n_present", "n_won"):
            assert res[f] == ores[f], (kind, rank, f, res[f], ores[f])
        flags[sel] = fl
        keys = np.arange(case["n_ids"])
        mine = keys % world == rank
        slots = keys[mine] // world
        for f, a in (("lt", lt), ("rank", rk), ("val", val), ("mod", mod)):
            assert np.array_equal(a[slots], orows[f][mine]), (kind, f)
    assert np.array_equal(flags, oflags)


@pytest.mark.parametrize("name", ["r4_ties", "dup_node", "drift", "drift_late", "send_overflow", "send_drift",
                                  "explicit_millis", "neg_mod", "dup_and_drift", "empty_changesets"])
def test_routed_two_ranks(name):
    check(dict(CASE_SPECS)[name], 2, "routed")


@pytest.mark.parametrize("name", ["r4_ties", "dup_node", "drift", "drift_late", "explicit_millis",
                                  "dup_and_drift"])
def test_parts_two_ranks(name):
    check(dict(CASE_SPECS)[name], 2, "parts")


@pytest.mark.parametrize("name", ["r4_ties", "drift", "send_overflow", "r8_tombstones"])
def test_presharded_two_ranks(name):
    check(dict(CASE_SPECS)[name], 2, "presharded")


@pytest.mark.parametrize("kind", ["routed", "parts"])
def test_three_ranks(kind):
    check(dict(seed=333, R=7, per_cs=120, dup_frac=0.003, force=[(4, 17, "drift")]), 3, kind)


def test_route_by_owner_is_stable():
    key = np.array([5, 2, 7, 4, 9, 6], np.uint32)
    routes = route_by_owner(key, np.array([0, 3, 6], np.uint64), 2)
    assert routes[0][0].tolist() == [1, 3, 5] and routes[0][1].tolist() == [0, 1, 3]
    assert routes[1][0].tolist() == [0, 2, 4] and routes[1][1].tolist() == [0, 2, 3]


def test_home_part_layout():
    sel, offs = home_part(np.array([0, 3, 5, 9], np.uint64), 2, 0)
    assert sel.tolist() == [0, 1, 2, 5, 6, 7, 8] and offs.tolist() == [0, 3, 3, 7]
    sel, offs = home_part(np.array([0, 3, 5, 9], np.uint64), 2, 1)
    assert sel.tolist() == [3, 4] and offs.tolist() == [0, 0, 2, 2]


# ---- a host transport bounds its own operations (crdt_set_comm_timeout) ------------------
def _timeout_worker(rank, world, port, q, what):
    import datetime
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    comm = GlooComm(dist, timeout=1.0)
    dist.barrier()
    if rank == world - 1:                       # the stalled (or lost) peer
        if what == "exit":
            os._exit(17)
        time.sleep(5.0)
    words = np.zeros(4, np.int64)
    t0 = time.monotonic()
    try:
        {"reduce": lambda: comm.all_reduce(words, 1),
         "gather": lambda: comm.all_gather(words, np.zeros(4 * world, np.int64)),
         "exit": lambda: comm.all_reduce(words, 1),
         "a2a": lambda: comm.all_to_all_v([np.zeros(8 * world, np.uint8)], [np.zeros(8 * world, np.uint8)], [1],
                                          [0 if d == rank else 8 for d in range(world)], [8 * d for d in range(world)],
                                          [0 if d == rank else 8 for d in range(world)], [8 * d for d in range(world)])}[what]()
        err = None
    except Exception as e:  # noqa: BLE001 -- the timeout surfaces as the transport's error
        err = type(e).__name__
    q.put((rank, err, time.monotonic() - t0))
    q.close()
    q.join_thread()
    os._exit(0)


@pytest.mark.parametrize("what,world", [("reduce", 2), ("gather", 3), ("a2a", 2), ("exit", 3)])
def test_gloo_comm_timeout_bounds_each_operation(what, world):
    """GlooComm(timeout=1 s): an operation whose peer stalls (or exited) raises on the waiting ranks within
    the bound — the error the library turns into CRDT_E_COMM — instead of blocking until the peer returns."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timeout_worker, args=(r, world, port, q, what)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=120) for _ in range(world - 1)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=30)
    for rank, err, el in outs:
        if rank == world - 1:
            continue
        assert err is not None, (rank, el)
        assert el < 4.0, (rank, el)             # the stalled peer slept 5 s: the bound ended the wait


def test_bench_watchdog_reports_and_exits():
    """bench.py's per-rank watchdog: a call that overruns its bound prints the rank's phase and exits 4."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import time, bench; w = bench.Watchdog(3); w.arm(10, 'early'); w.disarm(); "
            "w.arm(0.6, 'merge step (merging)'); time.sleep(10); print('not reached')")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=60)
    assert r.returncode == 4, (r.returncode, r.stderr[-500:])
    assert "rank 3: WATCHDOG: merge step (merging) overran" in r.stderr, r.stderr[-500:]
    assert "not reached" not in r.stdout
