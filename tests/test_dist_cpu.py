"""Multi-rank protocol of crdt_amd/dist.py on CPU: gloo, world_size 2 (and 3).

Each rank owns keys ``key % G`` and is home to changesets ``j % G``; the phase
algebra runs in tests/_phase_model.py (a numpy restatement of the device
kernels).  The sharded result must equal the single-table sequential C oracle:
every row, every win flag, the canonical, the exception fields."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from crdt_amd.dist import route_by_owner, sharded_merge, torch_reducers
from tests._cases import ABSENT_MOD, CASE_SPECS, make_case, oracle_run
from tests._phase_model import PhaseModel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _split(case, world, rank):
    key, offs = case["key"], case["offsets"]
    R = len(offs) - 1
    routes = route_by_owner(key, offs, world)
    idx, own_offs = routes[rank]
    millis = case["millis"]
    owned = ((key[idx] // world).astype(np.uint32), case["lt"][idx], case["rank"][idx], case["val"][idx],
             own_offs, None)
    # home: full changesets j % world == rank, empty otherwise (same R everywhere)
    counts = np.diff(offs.astype(np.int64))
    sel = np.concatenate([np.arange(offs[j], offs[j + 1]) for j in range(R) if j % world == rank] or
                         [np.zeros(0, np.int64)]).astype(np.int64)
    hc = np.where(np.arange(R) % world == rank, counts, 0)
    home_offs = np.concatenate([[0], np.cumsum(hc)]).astype(np.uint64)
    home = (None, case["lt"][sel], case["rank"][sel], None, home_offs,
            None if millis is None else millis[sel])
    return owned, home, idx


def _worker(rank, world, port, case_kw, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        case = make_case(**case_kw)
        cap = -(-case["n_ids"] // world)
        t = PhaseModel(cap, case["local_rank"], case["c0"])
        loc = case["local"]
        ids = np.arange(case["n_local"])
        mine = (ids % world == rank) & (loc["mod"] != ABSENT_MOD)
        t.put_rows(ids[mine] // world, loc["lt"][mine], loc["rank"][mine], loc["val"][mine], loc["mod"][mine])
        owned, home, idx = _split(case, world, rank)
        R = len(case["offsets"]) - 1
        d_max = torch.zeros(max(R, 1), dtype=torch.int64)
        d_ev = torch.zeros(4, dtype=torch.int64)
        flags = np.zeros(len(idx), np.uint8)
        red_max, red_min = torch_reducers(dist)
        res = sharded_merge(t, home, owned, case["wall"], d_max, d_ev, red_max, red_min, win_flags=flags)
        q.put((rank, res, t.lt, t.rank, t.val, t.mod, idx, flags))
    finally:
        dist.destroy_process_group()


def run_sharded(case_kw, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case_kw, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda o: o[0])


@pytest.mark.parametrize("name", ["r4_ties", "dup_node", "drift", "send_overflow", "send_drift",
                                  "explicit_millis", "neg_mod", "dup_and_drift"])
def test_two_rank_sharded_equals_single_table(name):
    kw = dict(CASE_SPECS)[name]
    case = make_case(**kw)
    orows, ores, oflags = oracle_run(case)
    world = 2
    outs = run_sharded(kw, world)
    n_present = n_won = 0
    flags = np.zeros(len(case["key"]), np.uint8)
    for rank, res, lt, rk, val, mod, idx, fl in outs:
        for f in ("status", "n_stored", "exc_changeset", "exc_index", "canonical_lt", "drift_ms", "counter"):
            assert res[f] == ores[f], (name, rank, f, res[f], ores[f])
        n_present += res["n_present"]
        n_won += res["n_won"]
        flags[idx] = fl
        keys = np.arange(case["n_ids"])
        mine = keys % world == rank
        slots = keys[mine] // world
        assert np.array_equal(lt[slots], orows["lt"][mine])
        assert np.array_equal(mod[slots], orows["mod"][mine])
        assert np.array_equal(rk[slots], orows["rank"][mine])
        assert np.array_equal(val[slots], orows["val"][mine])
    assert (n_present, n_won) == (ores["n_present"], ores["n_won"])
    assert np.array_equal(flags, oflags)


def test_three_ranks():
    kw = dict(seed=333, R=7, per_cs=120, dup_frac=0.003, force=[(4, 17, "drift")])
    case = make_case(**kw)
    _, ores, _ = oracle_run(case)
    for rank, res, *_ in run_sharded(kw, 3):
        assert res["status"] == ores["status"] and res["canonical_lt"] == ores["canonical_lt"]
        assert res["n_stored"] == ores["n_stored"] and res["exc_index"] == ores["exc_index"]


def test_route_by_owner_is_stable():
    key = np.array([5, 2, 7, 4, 9, 6], np.uint32)
    routes = route_by_owner(key, np.array([0, 3, 6], np.uint64), 2)
    assert routes[0][0].tolist() == [1, 3, 5] and routes[0][1].tolist() == [0, 1, 3]
    assert routes[1][0].tolist() == [0, 2, 4] and routes[1][1].tolist() == [0, 2, 3]


# ---------------------------------------------------------------- "parts" protocol
def _parts_case(kw, world):
    """One global case; changeset j's iteration order is rank-major (rank r's owned records first
    for r = 0, then 1, ...).  Returns the reordered global case and each rank's part."""
    case = make_case(**kw)
    key, offs = case["key"], case["offsets"].astype(np.int64)
    order = []
    for j in range(len(offs) - 1):
        seg = np.arange(offs[j], offs[j + 1])
        for r in range(world):
            order.extend(seg[key[seg] % world == r])
    order = np.array(order, dtype=np.int64)
    g = dict(case)
    for f in ("key", "lt", "rank", "val"):
        g[f] = case[f][order]
    if case["millis"] is not None:
        g["millis"] = case["millis"][order]
    return g


def _parts_worker(rank, world, port, case_kw, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from crdt_amd.dist import sharded_merge_parts, torch_all_gather
        case = _parts_case(case_kw, world)
        cap = -(-case["n_ids"] // world)
        t = PhaseModel(cap, case["local_rank"], case["c0"])
        loc = case["local"]
        ids = np.arange(case["n_local"])
        mine = (ids % world == rank) & (loc["mod"] != ABSENT_MOD)
        t.put_rows(ids[mine] // world, loc["lt"][mine], loc["rank"][mine], loc["val"][mine], loc["mod"][mine])
        routes = route_by_owner(case["key"], case["offsets"], world)
        idx, offs_r = routes[rank]
        millis = None if case["millis"] is None else case["millis"][idx]
        part = ((case["key"][idx] // world).astype(np.uint32), case["lt"][idx], case["rank"][idx],
                case["val"][idx], offs_r, millis)
        counts = np.stack([np.diff(routes[r][1].astype(np.int64)) for r in range(world)])
        ibase = counts[:rank].sum(axis=0) if rank else np.zeros(counts.shape[1], np.int64)
        R = len(case["offsets"]) - 1
        d_max = torch.zeros(max(R, 1), dtype=torch.int64)
        d_ev = torch.zeros(4, dtype=torch.int64)
        flags = np.zeros(len(idx), np.uint8)
        red_max, red_min = torch_reducers(dist)
        res = sharded_merge_parts(t, part, case["wall"], ibase, d_max, d_ev, torch_all_gather(dist), red_max,
                                  red_min, rank, win_flags=flags)
        q.put((rank, res, t.lt, t.rank, t.val, t.mod, idx, flags))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["r4_ties", "dup_node", "drift", "drift_late", "send_overflow",
                                  "explicit_millis", "dup_and_drift"])
def test_parts_protocol_equals_single_table(name):
    kw = dict(CASE_SPECS)[name]
    world = 2
    case = _parts_case(kw, world)
    orows, ores, oflags = oracle_run(case)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_parts_worker, args=(r, world, port, kw, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=120) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    flags = np.zeros(len(case["key"]), np.uint8)
    tot = [0, 0]
    for rank, res, lt, rk, val, mod, idx, fl in outs:
        for f in ("status", "n_stored", "exc_changeset", "exc_index", "canonical_lt", "drift_ms", "counter"):
            assert res[f] == ores[f], (name, rank, f, res[f], ores[f])
        tot[0] += res["n_present"]
        tot[1] += res["n_won"]
        flags[idx] = fl
        keys = np.arange(case["n_ids"])
        mine = keys % world == rank
        slots = keys[mine] // world
        for f, a in (("lt", lt), ("rank", rk), ("val", val), ("mod", mod)):
            assert np.array_equal(a[slots], orows[f][mine]), f
    assert tot == [ores["n_present"], ores["n_won"]]
    assert np.array_equal(flags, oflags)


# ---------------------------------------------------------------- routed protocol (all-to-all)
def _home_batch(case, world, rank):
    """Changesets j % world == rank in full (keys included), the others empty."""
    offs = case["offsets"]
    R = len(offs) - 1
    sel = np.concatenate([np.arange(offs[j], offs[j + 1]) for j in range(R) if j % world == rank] or
                         [np.zeros(0, np.int64)]).astype(np.int64)
    hc = np.where(np.arange(R) % world == rank, np.diff(offs.astype(np.int64)), 0)
    home_offs = np.concatenate([[0], np.cumsum(hc)]).astype(np.uint64)
    millis = case["millis"]
    return (case["key"][sel], case["lt"][sel], case["rank"][sel], case["val"][sel], home_offs,
            None if millis is None else millis[sel]), sel


def _routed_worker(rank, world, port, case_kw, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from crdt_amd.dist import sharded_merge_routed, torch_all_gather, torch_all_to_all, torch_alloc
        case = make_case(**case_kw)
        cap = -(-case["n_ids"] // world)
        t = PhaseModel(cap, case["local_rank"], case["c0"])
        loc = case["local"]
        ids = np.arange(case["n_local"])
        mine = (ids % world == rank) & (loc["mod"] != ABSENT_MOD)
        t.put_rows(ids[mine] // world, loc["lt"][mine], loc["rank"][mine], loc["val"][mine], loc["mod"][mine])
        home, sel = _home_batch(case, world, rank)
        R = len(case["offsets"]) - 1
        d_max = torch.zeros(max(R, 1), dtype=torch.int64)
        d_ev = torch.zeros(4, dtype=torch.int64)
        flags = torch.zeros(len(sel), dtype=torch.uint8)
        red_max, red_min = torch_reducers(dist)
        res = sharded_merge_routed(t, home, case["wall"], d_max, d_ev, red_max, red_min, torch_all_gather(dist),
                                   torch_all_to_all(dist), rank, world, torch_alloc("cpu"), win_flags=flags)
        q.put((rank, res, t.lt, t.rank, t.val, t.mod, sel, flags.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,world", [("r4_ties", 2), ("dup_node", 2), ("drift_late", 2), ("send_overflow", 2),
                                        ("r8_tombstones", 3), ("explicit_millis", 2), ("empty_changesets", 2)])
def test_routed_protocol_equals_single_table(name, world):
    kw = dict(CASE_SPECS)[name]
    case = make_case(**kw)
    orows, ores, oflags = oracle_run(case)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_routed_worker, args=(r, world, port, kw, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=120) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    flags = np.zeros(len(case["key"]), np.uint8)
    tot = [0, 0]
    for rank, res, lt, rk, val, mod, sel, fl in outs:
        for f in ("status", "n_stored", "exc_changeset", "exc_index", "canonical_lt", "drift_ms", "counter"):
            assert res[f] == ores[f], (name, rank, f, res[f], ores[f])
        tot[0] += res["n_present"]
        tot[1] += res["n_won"]
        flags[sel] = fl
        keys = np.arange(case["n_ids"])
        mine = keys % world == rank
        slots = keys[mine] // world
        for f, a in (("lt", lt), ("rank", rk), ("val", val), ("mod", mod)):
            assert np.array_equal(a[slots], orows[f][mine]), f
    assert tot == [ores["n_present"], ores["n_won"]]
    assert np.array_equal(flags, oflags)


def test_route_plan_layout():
    from crdt_amd.dist import route_plan
    # 2 ranks, 3 changesets: rank 0 holds j = 0, 2; rank 1 holds j = 1
    ca = np.zeros((2, 3, 2), np.int64)
    ca[0, 0] = [3, 2]
    ca[0, 2] = [1, 4]
    ca[1, 1] = [5, 0]
    sb, ss, rs, b, e = route_plan(ca, 0)
    assert ss.tolist() == [4, 6] and rs.tolist() == [4, 5]
    assert sb[:, 0].tolist() == [0, 3, 3] and sb[:, 1].tolist() == [4, 6, 6]
    assert b.tolist() == [0, 4, 3] and e.tolist() == [3, 9, 4]
