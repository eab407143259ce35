"""GPU parity on the BASELINE.json workload generators (crdt_amd/workload.py).

* fan-in and cfg3 (heavy (millis, counter) ties decided by node rank), cfg2 — at reduced sizes,
  bit-exact against the C restatement (every row, every win flag, the result fields);
* cfg5 streaming (one merge call per delta, advancing wall, 10% tombstones, drift / duplicate-node
  injection): reduced size bit-exact per call against the C restatement; full size (100M keys,
  100 x 10M) through size-independent properties — the stop point, the exception fields, the
  canonical (A7 of SURVEY §8(a)) and a 50K-key sample of rows replayed delta by delta.
"""
import numpy as np
import pytest

from tests._cases import ABSENT_MOD

pytestmark = pytest.mark.gpu

FIELDS = ("status", "n_stored", "exc_changeset", "exc_index", "canonical_lt", "drift_ms", "counter",
          "n_present", "n_won")


def _np(t, dt):
    return t.cpu().numpy().astype(dt)


def wl_case(wl):
    """A generated (single-rank) workload as a numpy case for the oracle."""
    loc, own = wl["local"], wl["owned"]
    n_local = int(wl["n_local_rows"])
    slot = _np(loc["slot"], np.int64)
    assert np.array_equal(slot, np.arange(n_local))
    cap = int(wl["capacity"])
    return {
        "key": _np(own["key"], np.uint32), "lt": _np(own["lt"], np.int64), "rank": _np(own["rank"], np.uint32),
        "val": _np(own["val"], np.uint32), "offsets": np.asarray(wl["owned_offsets"], np.uint64),
        "millis": None, "wall": int(wl["wall"]), "c0": int(wl["c0"]), "local_rank": 0, "n_ids": cap,
        "n_local": n_local,
        "local": {"lt": _np(loc["lt"], np.int64), "rank": _np(loc["rank"], np.uint32),
                  "val": _np(loc["val"], np.uint32), "mod": _np(loc["mod"], np.int64)},
    }


def _device_table(wl):
    from crdt_amd import DeviceTable
    t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
    loc = wl["local"]
    t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
    t.canonical = wl["c0"]
    return t


def _oracle_table(case):
    from oracle.oracle_c import OracleTable
    t = OracleTable(case["n_ids"], 0, case["c0"])
    loc = case["local"]
    keep = loc["mod"] != ABSENT_MOD
    ids = np.arange(case["n_local"], dtype=np.uint32)[keep]
    t.put_rows(ids, loc["lt"][keep], loc["rank"][keep], loc["val"][keep], loc["mod"][keep])
    return t


def _check_batch(wl):
    import torch
    case = wl_case(wl)
    t = _device_table(wl)
    own = wl["owned"]
    flags = torch.zeros(max(int(case["offsets"][-1]), 1), dtype=torch.uint8, device="cuda")
    res, _ = t.merge(own["key"], own["lt"], own["rank"], own["val"], wl["owned_offsets"], wl["wall"],
                     win_flags=flags)
    lt, rank, val, mod = t.read_rows(np.arange(case["n_ids"], dtype=np.uint32))
    t.close()
    o = _oracle_table(case)
    ores, oflags = o.merge(case["key"], case["lt"], case["rank"], case["val"], case["offsets"], case["wall"])
    ores = ores.as_dict()
    rows = o.rows
    for f, a in (("lt", lt), ("rank", rank), ("val", val), ("mod", mod)):
        assert np.array_equal(a, rows[f]), f
    assert np.array_equal(flags[:len(oflags)].cpu().numpy(), oflags)
    for k in FIELDS:
        assert res[k] == ores[k], (k, res[k], ores[k])
    return res


def test_fanin_reduced_vs_oracle(gpu_device):
    from crdt_amd.workload import gen_fanin
    res = _check_batch(gen_fanin(total=4_000_000, R=64, K=1 << 22, n_local=1 << 21, device="cuda"))
    assert res["status"] == 0 and res["n_won"] > 0


def test_cfg3_reduced_ties_vs_oracle(gpu_device):
    from crdt_amd.workload import gen_cfg3
    wl = gen_cfg3(device="cuda", total=2_000_000, K=2_000_000, R=256)
    lt = wl["owned"]["lt"]
    assert int(torch_unique_count(lt)) <= 32            # 8 millis x 4 counters: ties everywhere
    res = _check_batch(wl)
    assert res["status"] == 0 and 0 < res["n_won"] < res["n_present"]


def torch_unique_count(t):
    import torch
    return torch.unique(t).numel()


def test_cfg2_reduced_vs_oracle(gpu_device):
    from crdt_amd.workload import gen_cfg2
    res = _check_batch(gen_cfg2(device="cuda", n_local=1_000_000, n_remote=1_000_000))
    assert res["n_present"] > 0 and res["n_stored"] == 1


# ------------------------------------------------------------------------------- cfg5
def _run_calls(t, wl, flags=None):
    """One merge call per delta, stopping at the first exception (as the caller's loop would)."""
    own, offs, out = wl["owned"], wl["owned_offsets"], []
    for d in range(wl["R"]):
        b, e = int(offs[d]), int(offs[d + 1])
        fl = False if flags is None else flags[b:e]
        r, _ = t.merge(own["key"][b:e], own["lt"][b:e], own["rank"][b:e], own["val"][b:e],
                       np.array([0, e - b], np.uint64), int(wl["walls"][d]), win_flags=fl)
        out.append(r)
        if r["status"]:
            break
    return out


@pytest.mark.parametrize("inject", [None, "drift", "dup"])
def test_cfg5_reduced_streaming_vs_oracle(gpu_device, inject):
    import torch
    from crdt_amd.workload import gen_cfg5
    wl = gen_cfg5(device="cuda", K=1_000_000, n_delta=100_000, deltas=60, inject=inject, inject_at=(37, 49_999))
    case = wl_case(wl)
    t = _device_table(wl)
    flags = torch.zeros(int(wl["total"]), dtype=torch.uint8, device="cuda")
    got = _run_calls(t, wl, flags)
    lt, rank, val, mod = t.read_rows(np.arange(case["n_ids"], dtype=np.uint32))
    t.close()
    o = _oracle_table(case)
    offs = case["offsets"]
    oflags = np.zeros(int(offs[-1]), np.uint8)
    for d, r in enumerate(got):
        b, e = int(offs[d]), int(offs[d + 1])
        ores, of = o.merge(case["key"][b:e], case["lt"][b:e], case["rank"][b:e], case["val"][b:e],
                           np.array([0, e - b], np.uint64), int(wl["walls"][d]))
        oflags[b:e] = of
        ores = ores.as_dict()
        for k in FIELDS:
            assert r[k] == ores[k], (d, k, r[k], ores[k])
    rows = o.rows
    for f, a in (("lt", lt), ("rank", rank), ("val", val), ("mod", mod)):
        assert np.array_equal(a, rows[f]), f
    assert np.array_equal(flags.cpu().numpy(), oflags)
    assert (val == 0xFFFFFFFF).any()                      # tombstones were stored
    if inject is None:
        assert len(got) == 60 and all(r["status"] == 0 for r in got)
    else:
        assert len(got) == 38
        last = got[-1]
        assert last["status"] == (1 if inject == "drift" else 2)
        assert last["exc_index"] == 49_999 and last["n_stored"] == 0
        if inject == "drift":
            assert last["drift_ms"] == 60_001


@pytest.mark.parametrize("inject", ["drift", "dup"])
def test_cfg5_full_scale_injection(gpu_device, inject):
    """100M-key table, 10M-record deltas: the stop point and the A7 partial state at full size."""
    import torch
    from crdt_amd.workload import gen_cfg5
    wl = gen_cfg5(device="cuda", inject=inject)
    K, n = wl["K"], wl["n_per_replica"]
    t = _device_table(wl)
    got = _run_calls(t, wl)
    assert len(got) == 38
    last = got[-1]
    assert last["status"] == (1 if inject == "drift" else 2)
    assert (last["exc_changeset"], last["exc_index"], last["n_stored"]) == (0, 4_999_999, 0)
    if inject == "drift":
        assert last["drift_ms"] == 60_001
    # canonical: C_j = send(max(C_{j-1}, M_j)) over the 37 clean deltas, then the running max of
    # delta 37's records before the failing one (hlc.dart:80-97, crdt.dart:77-94)
    lt = wl["owned"]["lt"]
    c = wl["c0"]
    rj = []
    for d in range(37):
        r = max(c, int(lt[d * n:(d + 1) * n].max().item()))
        rj.append(r)
        c = max(r + 1, int(wl["walls"][d]) << 16)
        assert got[d]["canonical_lt"] == c and got[d]["status"] == 0
    expect = max(c, int(lt[37 * n:37 * n + 4_999_999].max().item()))
    assert last["canonical_lt"] == expect == t.canonical
    # 50K sampled keys replayed delta by delta (keys are an affine bijection per delta)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    keys = torch.randint(0, K, (50_000,), device="cuda", generator=g)
    loc = wl["local"]
    row_lt, row_rank = loc["lt"][keys].clone(), loc["rank"][keys].to(torch.int64)
    row_val, row_mod = loc["val"][keys].to(torch.int64), loc["mod"][keys].clone()
    own = wl["owned"]
    for d in range(37):
        a, b = wl["affine"][d]
        pos = ((keys - b) % K * pow(a, -1, K)) % K
        here = pos < n
        x = d * n + torch.where(here, pos, torch.zeros_like(pos))
        l, r = own["lt"][x], own["rank"][x].to(torch.int64)
        win = here & ((l > row_lt) | ((l == row_lt) & (r > row_rank)))
        row_lt = torch.where(win, l, row_lt)
        row_rank = torch.where(win, r, row_rank)
        row_val = torch.where(win, own["val"][x].to(torch.int64), row_val)
        row_mod = torch.where(win, torch.full_like(row_mod, rj[d]), row_mod)
    glt, grank, gval, gmod = t.read_rows(keys.cpu().numpy().astype(np.uint32))
    t.close()
    assert np.array_equal(glt, row_lt.cpu().numpy())
    assert np.array_equal(grank, row_rank.cpu().numpy().astype(np.uint32))
    assert np.array_equal(gval, (row_val.cpu().numpy() & 0xFFFFFFFF).astype(np.uint32))
    want = row_mod.cpu().numpy()
    bad = np.flatnonzero(gmod != want)
    stamps = {v: d for d, v in enumerate(rj)}
    assert len(bad) == 0, (len(bad), [(int(keys[i]), int(gmod[i]), int(want[i]), stamps.get(int(gmod[i])),
                                       stamps.get(int(want[i]))) for i in bad[:8]])


def _cfg5_shard_worker(rank, world, port, q, kw):
    """One rank of configs[4] on N GPUs at reduced size: its parts of every delta, one collective
    routed crdt_merge per delta (gloo communicator, all ranks on cuda:0)."""
    import os

    import torch.distributed as dist

    from crdt_amd import DeviceTable
    from crdt_amd.dist import GlooComm
    from crdt_amd.workload import gen_cfg5
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = gen_cfg5(device="cuda", rank=rank, world=world, **kw)
        t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
        t.set_row_bytes(32)
        loc, home, offs = wl["local"], wl["home"], wl["home_offsets"]
        t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
        t.canonical = wl["c0"]
        t.comm_init_ops(world, rank, GlooComm(dist))
        results, mid = [], None
        for d in range(wl["R"]):
            b, e = int(offs[d]), int(offs[d + 1])
            res, _ = t.merge(home["key"][b:e], home["lt"][b:e], home["rank"][b:e], home["val"][b:e],
                             np.array([0, e - b], np.uint64), int(wl["walls"][d]), win_flags=False)
            results.append(res)
            if d == 9:
                mid = t.read_rows(np.arange(wl["capacity"], dtype=np.uint32))
            if res["status"] != 0:
                break
        q.put((rank, results, mid, t.read_rows(np.arange(wl["capacity"], dtype=np.uint32))))
        t.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("inject", [None, "drift"])
def test_cfg5_two_rank_streaming_vs_oracle(gpu_device, inject):
    """configs[4] ('8 x MI355X streaming') rehearsed with 2 ranks on one GPU over gloo at reduced size
    (400K keys, 40 deltas x 100K records, 10 % tombstones): every delta split into 2 contiguous parts,
    one collective routed merge per delta, a drift injected at (37, 49,999) (on rank 0's part: the
    exception index is the position in the whole delta).  Every call's status, stop point, exception
    fields and canonical on both ranks, and both shards' rows after delta 9 and at the end, against
    the C oracle merging the whole deltas in order (crdt.dart:77-94)."""
    import torch.multiprocessing as mp

    from crdt_amd.workload import gen_cfg5
    from oracle.oracle_c import OracleTable
    from tests.test_dist_cpu import _free_port
    kw = dict(K=400_000, n_delta=100_000, deltas=40, inject=inject, inject_at=(37, 49_999))
    wl = gen_cfg5(device="cuda", **kw)
    own = {k: _np(v, np.int64) for k, v in wl["owned"].items()}
    loc = wl["local"]
    o = OracleTable(wl["capacity"], 0, wl["c0"])
    o.put_rows(_np(loc["slot"], np.uint32), _np(loc["lt"], np.int64), _np(loc["rank"], np.uint32),
               _np(loc["val"], np.uint32), _np(loc["mod"], np.int64))
    offs = wl["owned_offsets"]
    expect, mid_rows = [], None
    for d in range(wl["R"]):
        b, e = int(offs[d]), int(offs[d + 1])
        r, _ = o.merge(own["key"][b:e].astype(np.uint32), own["lt"][b:e], own["rank"][b:e].astype(np.uint32),
                       own["val"][b:e].astype(np.uint32), np.array([0, e - b], np.uint64), int(wl["walls"][d]),
                       want_flags=False)
        expect.append(r.as_dict())
        if d == 9:
            mid_rows = o.rows.copy()
        if r.status != 0:
            break
    del wl
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cfg5_shard_worker, args=(r, world, port, q, kw)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, results, mid, final in outs:
        assert len(results) == len(expect), (rank, len(results), len(expect))
        for d, (got, want) in enumerate(zip(results, expect)):
            for f in FIELDS:
                assert got[f] == want[f], (rank, d, f, got[f], want[f])
        for rows, ref in ((mid, mid_rows), (final, o.rows)):
            sh = ref[rank::world]
            for f, a in zip(("lt", "rank", "val", "mod"), rows):
                assert np.array_equal(a[:len(sh)], sh[f]), (rank, f)
    assert (expect[-1]["status"] != 0) == (inject is not None)
    if inject:
        # one call per delta: the drift stops call 37 at its record 49,999 (changeset 0 of that call)
        assert (len(expect), expect[-1]["exc_changeset"], expect[-1]["exc_index"]) == (38, 0, 49_999)
