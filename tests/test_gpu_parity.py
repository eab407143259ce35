"""GPU parity: the HIP merge path (through the C-ABI) against the golden vectors
and the C restatement, bit for bit — rows, win flags, canonical, exceptions."""
import numpy as np
import pytest

from tests._cases import ABSENT_MOD, CASE_SPECS, NULL, WALL, make_case, oracle_run
from tests.test_golden_cpu import check_rows, golden_case

pytestmark = pytest.mark.gpu

RESULT_FIELDS = ("status", "n_stored", "exc_changeset", "exc_index", "canonical_lt", "drift_ms", "counter",
                 "n_present", "n_won")


def device_run(case, device_cols=False, capacity=None, path=None, flags=True, counts=True, rank_bound=0):
    """path: None (auto) | 'gather' | 'sorted' (crdt_set_merge_path); flags=False asks for no
    per-record win flags (the sorted path's precondition), returned flags are then None;
    counts=False: crdt_set_counts(0) (the sorted path's order-free form); rank_bound:
    crdt_set_rank_bound."""
    from crdt_amd import DeviceTable
    t = DeviceTable(0, local_rank=case["local_rank"], capacity=capacity or case["n_ids"])
    if path:
        t.set_merge_path(path)
    if not counts:
        t.set_counts(False)
    if rank_bound:
        t.set_rank_bound(rank_bound)
    loc = case["local"]
    keep = loc["mod"] != ABSENT_MOD
    ids = np.arange(case["n_local"], dtype=np.uint32)[keep]
    if len(ids):
        t.put_rows(ids, loc["lt"][keep], loc["rank"][keep], loc["val"][keep], loc["mod"][keep])
    t.canonical = case["c0"]
    cols = [case["key"], case["lt"], case["rank"], case["val"]]
    millis = case["millis"]
    if device_cols:
        import torch
        cols = [torch.from_numpy(c.astype(c.dtype)).cuda() for c in cols]
        millis = None if millis is None else torch.from_numpy(millis).cuda()
    res, fl = t.merge(*cols, case["offsets"], case["wall"], millis=millis, win_flags=flags)
    if device_cols and fl is not None:
        fl = fl.cpu().numpy()
    lt, rank, val, mod = t.read_rows(np.arange(case["n_ids"], dtype=np.uint32))
    assert t.canonical == res["canonical_lt"]
    res["path"] = t.last_path()
    res["plan"] = t.last_plan()
    t.close()
    return (lt, rank, val, mod), res, fl


@pytest.mark.parametrize("name", [n for n, _ in CASE_SPECS])
def test_golden_vectors(gpu_device, name):
    case, exp, expected = golden_case(name)
    rows, res, flags = device_run(case)
    check_rows(*rows, exp)
    assert np.array_equal(flags, exp["flags"])
    for k, v in expected.items():
        assert res[k] == v, (name, k, res[k], v)


def compare_with_oracle(case, **kw):
    rows, res, flags = device_run(case, **kw)
    orows, ores, oflags = oracle_run(case)
    for f, a in zip(("lt", "rank", "val", "mod"), rows):
        assert np.array_equal(a, orows[f]), f
    if flags is not None:
        assert np.array_equal(flags, oflags)
    for k in RESULT_FIELDS:
        if kw.get("counts", True) is False and res["path"] == "sorted" and k in ("n_present", "n_won"):
            assert res[k] == (1 << 64) - 1, (k, res[k])
            continue
        assert res[k] == ores[k], (k, res[k], ores[k])
    return res


@pytest.mark.parametrize("seed", range(12))
def test_random_small(gpu_device, seed):
    rng = np.random.default_rng(1000 + seed)
    kw = dict(seed=2000 + seed, R=int(rng.integers(1, 12)), per_cs=int(rng.integers(0, 500)),
              n_local=int(rng.integers(1, 600)), n_new=int(rng.integers(0, 400)),
              millis_span=int(rng.integers(1, 100)), counter_span=int(rng.integers(1, 8)),
              n_ranks=int(rng.integers(2, 40)), tomb_frac=float(rng.random() * 0.5),
              neg_mod_frac=float(rng.random() * 0.1), dup_frac=float(rng.random() * 0.01),
              drift_frac=float(rng.random() * 0.005))
    kw["local_rank"] = int(rng.integers(0, kw["n_ranks"]))
    compare_with_oracle(make_case(**kw))


def _fused_cases():
    yield make_case(seed=3100, R=7, per_cs=3000, n_local=5000, n_new=2000, millis_span=40, counter_span=3,
                    n_ranks=9, dup_frac=0.002, drift_frac=0.002, local_rank=2)
    yield make_case(seed=3101, R=2, per_cs=200_000, n_local=300_000, n_new=100_000,
                    force=[(1, 150_001, "drift")], millis_span=1 << 12)
    yield make_case(seed=3102, R=40, per_cs=500, n_local=8000, n_new=4000, millis_span=5, counter_span=2,
                    n_ranks=41, force=[(33, 17, "dup")], local_rank=0)
    yield make_case(seed=3103, R=1, per_cs=300_000, n_local=200_000, n_new=200_000, millis_span=1 << 14)


@pytest.mark.parametrize("k", range(4))
def test_fused_small_merge_equals_unfused(gpu_device, monkeypatch, k):
    """crdt_merge's fused form (tile max inside k_clock<true>, resolve by the last k_verify<true>
    workgroup) against the separate kernels (CRDT_NO_FUSE) and the oracle."""
    case = list(_fused_cases())[k]
    fused = device_run(case)
    monkeypatch.setenv("CRDT_NO_FUSE", "1")
    plain = device_run(case)
    for a, b in zip(fused[0], plain[0]):
        assert np.array_equal(a, b)
    assert np.array_equal(fused[2], plain[2])
    for f in RESULT_FIELDS:
        assert fused[1][f] == plain[1][f], f
    monkeypatch.delenv("CRDT_NO_FUSE")
    compare_with_oracle(case)


@pytest.mark.parametrize("window", [1, 777, 3000, 1 << 20])
def test_host_batch_key_val_windows(gpu_device, monkeypatch, window):
    """Host batches: key / val are staged window by window on the copy stream under K2
    (CRDT_KV_WINDOW records per window; changesets split into pieces at window ends), with
    win flags, a late duplicate-node exception and the sorted path, against the oracle."""
    monkeypatch.setenv("CRDT_KV_WINDOW", str(window))
    case = make_case(seed=3200, R=7, per_cs=3000, n_local=12_000, n_new=6000, millis_span=30, counter_span=3,
                     n_ranks=9, local_rank=2)
    compare_with_oracle(case)
    compare_with_oracle(make_case(seed=3201, R=6, per_cs=2500, n_local=9000, n_new=4000, millis_span=20,
                                  n_ranks=7, force=[(4, 1234, "dup")], local_rank=1))
    compare_with_oracle(case, path="sorted", flags=False)


def test_device_resident_columns(gpu_device):
    """Zero-copy path: torch CUDA tensors go straight to the kernels."""
    compare_with_oracle(make_case(seed=77, R=5, per_cs=3000, n_local=6000, n_new=3000), device_cols=True)


def test_large_single_changeset(gpu_device):
    """One changeset of 1M records: many scan tiles, many apply blocks."""
    from tests._cases import WALL
    res = compare_with_oracle(make_case(seed=78, R=1, per_cs=1_000_000, n_local=1_200_000, n_new=800_000,
                                        millis_span=1 << 16, base=WALL - 70_000))
    assert res["status"] == 0 and res["n_won"] > 0


def test_many_changesets(gpu_device):
    compare_with_oracle(make_case(seed=79, R=300, per_cs=2000, n_local=40_000, n_new=20_000, millis_span=8,
                                  counter_span=4, n_ranks=301))


def test_exception_in_late_tile(gpu_device):
    """A raising record deep inside a big changeset: candidate tile far from the start."""
    case = make_case(seed=80, R=2, per_cs=200_000, n_local=300_000, n_new=100_000,
                     force=[(1, 150_001, "drift")], millis_span=1 << 12)
    res = compare_with_oracle(case)
    assert res["status"] == 1 and res["exc_changeset"] == 1 and res["exc_index"] == 150_001


def test_false_candidates_do_not_raise(gpu_device):
    """Flagged records above C0 that are NOT prefix maxima must not raise."""
    rng = np.random.default_rng(5)
    case = make_case(seed=81, R=1, per_cs=50_000, n_local=60_000, n_new=0, c0=0, millis_span=1000)
    # first record is the global max (foreign); later dups exceed C0 but not the running max
    case["lt"][0] = int(case["lt"].max()) + 10
    dups = rng.choice(np.arange(1, 50_000), 500, replace=False)
    case["rank"][dups] = case["local_rank"]
    res = compare_with_oracle(case)
    assert res["status"] == 0


def test_put_stamped_and_views(gpu_device):
    from crdt_amd import DeviceTable
    from oracle.oracle_c import OracleTable
    from tests._cases import WALL
    t = DeviceTable(0, local_rank=2, capacity=100)
    o = OracleTable(100, 2, 0)
    key = np.array([5, 9, 3], np.uint32)
    val = np.array([1, NULL, 7], np.uint32)
    r1 = t.put_stamped(key, val, WALL)
    r2 = o.put_stamped(key, val, WALL)
    assert r1["canonical_lt"] == r2.canonical_lt == WALL << 16
    r1 = t.put_stamped(key[:1], val[:1], WALL)                 # same wall: counter + 1
    r2 = o.put_stamped(key[:1], val[:1], WALL)
    assert r1["canonical_lt"] == r2.canonical_lt == (WALL << 16) + 1
    lt, rank, v, mod = t.read_rows(np.arange(100, dtype=np.uint32))
    assert np.array_equal(lt, o.rows["lt"]) and np.array_equal(mod, o.rows["mod"])
    assert t.refresh_canonical(100) == o.refresh(100)
    assert np.array_equal(t.modified_since(100, (WALL << 16) + 1), o.modified_since(100, (WALL << 16) + 1))
    assert np.array_equal(t.modified_since(100, 0), np.array([3, 5, 9], np.uint32))
    t.remap_ranks(100, [0, 1, 4, 5, 6])
    assert t.read_rows(np.array([5], np.uint32))[1][0] == 4
    t.clear_rows(0, 100)
    assert np.all(t.read_rows(np.arange(100, dtype=np.uint32))[3] < 0)
    assert t.refresh_canonical(100) == 0


def test_key_out_of_range_is_reported_not_faulting(gpu_device):
    from crdt_amd import CrdtNativeError, DeviceTable
    t = DeviceTable(0, local_rank=0, capacity=64)
    with pytest.raises(CrdtNativeError):
        t.merge(np.array([1, 10_000], np.uint32), np.array([5, 6], np.int64), np.array([1, 1], np.uint32),
                np.array([0, 0], np.uint32), np.array([0, 2], np.uint64), 1 << 40)


@pytest.mark.parametrize("path", ["gather", "sorted"])
def test_row_bytes_32_and_relayout(gpu_device, path):
    """crdt_set_row_bytes: 32-B rows give the oracle's rows on both paths, and switching the row
    size of a populated table (24 -> 32 -> 24) keeps every row."""
    from crdt_amd import DeviceTable
    case = make_case(seed=61, R=80, per_cs=1200, n_local=3000, n_new=1500, millis_span=4, counter_span=2,
                     n_ranks=7, tomb_frac=0.1)
    t = DeviceTable(0, local_rank=case["local_rank"], capacity=case["n_ids"])
    t.set_row_bytes(32)
    t.set_merge_path(path)
    if path == "sorted":
        t.set_counts(False)
    loc = case["local"]
    keep = loc["mod"] != ABSENT_MOD
    ids = np.arange(case["n_local"], dtype=np.uint32)[keep]
    t.put_rows(ids, loc["lt"][keep], loc["rank"][keep], loc["val"][keep], loc["mod"][keep])
    t.canonical = case["c0"]
    t.merge(case["key"], case["lt"], case["rank"], case["val"], case["offsets"], case["wall"],
            millis=case["millis"], win_flags=False)
    orows, _, _ = oracle_run(case)
    all_ids = np.arange(case["n_ids"], dtype=np.uint32)
    for f, a in zip(("lt", "rank", "val", "mod"), t.read_rows(all_ids)):
        assert np.array_equal(a, orows[f]), f
    t.set_row_bytes(24)
    for f, a in zip(("lt", "rank", "val", "mod"), t.read_rows(all_ids)):
        assert np.array_equal(a, orows[f]), f
    t.set_row_bytes(32)
    for f, a in zip(("lt", "rank", "val", "mod"), t.read_rows(all_ids)):
        assert np.array_equal(a, orows[f]), f
    t.close()


def test_reserve_preserves_rows(gpu_device):
    from crdt_amd import DeviceTable
    t = DeviceTable(0, local_rank=0, capacity=16)
    t.put_rows(np.array([3], np.uint32), np.array([42], np.int64), np.array([1], np.uint32),
               np.array([7], np.uint32), np.array([43], np.int64))
    t.reserve(100_000)
    lt, rank, val, mod = t.read_rows(np.array([3, 99_999], np.uint32))
    assert (lt[0], rank[0], val[0], mod[0]) == (42, 1, 7, 43) and mod[1] < 0


def _init_pg(dist, rank, world, backend):
    import torch
    if backend == "nccl":                      # the bench's process group at N > 1
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)


def _make_injected(kw):
    """make_case(**kw) with an optional record that raises at (41, 123,456): kw["inject"] = "drift"
    (millis past wall + 60 s) or "dup" (the local node id, above every clock the call reaches)."""
    kw = dict(kw)
    inject = kw.pop("inject", None)
    case = make_case(**kw)
    if inject:
        x = int(case["offsets"][41]) + 123_456
        case["lt"] = case["lt"].copy()
        case["rank"] = case["rank"].copy()
        if inject == "drift":
            case["lt"][x] = (case["wall"] + 60_001) << 16
        else:
            case["lt"][x] = max(int(case["lt"].max()), case["c0"]) + 1000
            case["rank"][x] = case["local_rank"]
    return case


def _shard_gpu_worker(rank, world, port, case_kw, kind, q, backend="gloo", path="gather", counts=True,
                      again=False):
    """One rank of a sharded replica on cuda:0: the library's collective crdt_merge
    (comm_path.inc) over RCCL (backend nccl) or the host-staged gloo communicator."""
    import os

    import torch
    import torch.distributed as dist

    from crdt_amd import DeviceTable
    from crdt_amd.dist import GlooComm, attach_rccl
    from tests.test_dist_cpu import layout
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    _init_pg(dist, rank, world, backend)
    try:
        case, sel, part_offs = layout(_make_injected(case_kw), world, rank, kind)
        cap = -(-case["n_ids"] // world)
        t = DeviceTable(0, local_rank=case["local_rank"], capacity=cap)
        want_flags = path in ("gather", "sorted+flags")       # sorted+flags: the receivers' flagged form
        t.set_merge_path("sorted" if path == "sorted+flags" else path)
        t.set_counts(counts)
        loc = case["local"]
        ids = np.arange(case["n_local"])
        mine = (ids % world == rank) & (loc["mod"] != ABSENT_MOD)

        def reset():
            t.clear_rows(0, cap)
            if mine.any():
                t.put_rows((ids[mine] // world).astype(np.uint32), loc["lt"][mine], loc["rank"][mine],
                           loc["val"][mine], loc["mod"][mine])
            t.canonical = case["c0"]
        reset()
        if backend == "nccl":
            attach_rccl(t, dist)
        else:
            t.comm_init_ops(world, rank, GlooComm(dist))
        assert t.comm_info() == (world, rank)
        t.set_presharded(kind == "presharded")
        key = case["key"][sel]
        if kind == "presharded":
            key = key // world
        dev = lambda a: None if a is None else torch.from_numpy(  # noqa: E731
            np.ascontiguousarray(a.view(np.int32) if a.dtype == np.uint32 else a)).cuda()
        millis = None if case["millis"] is None else dev(case["millis"][sel])
        flags = torch.zeros(max(len(sel), 1), dtype=torch.uint8, device="cuda") if want_flags else False
        cols = (dev(key.astype(np.uint32)), dev(case["lt"][sel]), dev(case["rank"][sel]), dev(case["val"][sel]))
        res, _ = t.merge(*cols, part_offs, case["wall"], millis=millis, win_flags=flags)
        if again:                 # the same call again on this ctx (receive columns sized by the first)
            reset()
            res, _ = t.merge(*cols, part_offs, case["wall"], millis=millis, win_flags=flags)
        res["path"] = t.last_path()
        res["plan"] = t.last_plan()
        lt, rk, val, mod = t.read_rows(np.arange(cap, dtype=np.uint32))
        fl = flags[:len(sel)].cpu().numpy() if want_flags else None
        q.put((rank, res, lt, rk, val, mod, sel, fl))
        t.close()
    finally:
        dist.destroy_process_group()


def run_shard_gpu(kw, world, kind, backend="gloo", path="gather", counts=True, again=False):
    import torch.multiprocessing as mp

    from tests.test_dist_cpu import _free_port, layout
    case, _, _ = layout(_make_injected(kw), world, 0, kind)
    orows, ores, oflags = oracle_run(case)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_gpu_worker, args=(r, world, port, kw, kind, q, backend, path, counts, again))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    flags = np.zeros(len(case["key"]), np.uint8)
    for rank, res, lt, rk, val, mod, sel, fl in outs:
        for f in RESULT_FIELDS:
            if f in ("n_present", "n_won") and not counts and res["path"] == "sorted":
                assert res[f] == (1 << 64) - 1
                continue
            assert res[f] == ores[f], (kind, rank, f, res[f], ores[f])
        if fl is not None:
            flags[sel] = fl
        keys = np.arange(case["n_ids"])
        mine = keys % world == rank
        slots = keys[mine] // world
        for f, a in (("lt", lt), ("rank", rk), ("val", val), ("mod", mod)):
            assert np.array_equal(a[slots], orows[f][mine]), (kind, f)
    if path in ("gather", "sorted+flags"):
        assert np.array_equal(flags, oflags)
    return outs


def _mismatch_worker(rank, world, port, q, what):
    """Two ranks whose collective-shape settings differ (win flags on one rank only, or counts): both
    calls must fail with CRDT_E_INVALID before any exchange is posted (no hang, no corruption)."""
    import os

    import torch
    import torch.distributed as dist

    from crdt_amd import DeviceTable
    from crdt_amd.device import CrdtNativeError
    from crdt_amd.dist import GlooComm
    from tests.test_dist_cpu import layout
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    _init_pg(dist, rank, world, "gloo")
    try:
        case, sel, part_offs = layout(make_case(**dict(CASE_SPECS)["r8_tombstones"]), world, rank, "routed")
        cap = -(-case["n_ids"] // world)
        t = DeviceTable(0, local_rank=case["local_rank"], capacity=cap)
        t.comm_init_ops(world, rank, GlooComm(dist))
        if what == "counts":
            t.set_counts(rank == 0)
        flags = what == "flags" and rank == 1
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a.view(np.int32) if a.dtype == np.uint32 else a)).cuda()  # noqa: E731
        cols = (dev(case["key"][sel].astype(np.uint32)), dev(case["lt"][sel]), dev(case["rank"][sel]),
                dev(case["val"][sel]))
        c0 = t.canonical
        before = t.read_rows(np.arange(cap, dtype=np.uint32))
        try:
            t.merge(*cols, part_offs, case["wall"], win_flags=flags)
            st = 0
        except CrdtNativeError as e:
            st = e.status
        after = t.read_rows(np.arange(cap, dtype=np.uint32))
        q.put((rank, st, t.canonical == c0, all(np.array_equal(a, b) for a, b in zip(before, after))))
        t.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("what", ["flags", "counts"])
def test_two_rank_settings_mismatch_fails_fast(gpu_device, what):
    """ADVICE r3 (comm_path.inc): the ranks' collective-shape words are all-gathered with the part maxima;
    when they differ every rank returns CRDT_E_INVALID (nothing routed, canonical unchanged)."""
    import torch.multiprocessing as mp

    from tests.test_dist_cpu import _free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mismatch_worker, args=(r, 2, port, q, what)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, st, c_same, rows_same in outs:
        assert st == -1, (rank, st)
        assert c_same and rows_same, rank


@pytest.mark.parametrize("kind", ["routed", "parts", "presharded"])
@pytest.mark.parametrize("name", ["r8_tombstones", "dup_node", "drift_late", "send_overflow", "explicit_millis"])
def test_two_rank_sharded_on_device(gpu_device, name, kind):
    """The library's collective crdt_merge, 2 ranks on one GPU over the gloo communicator:
    every row of both shards, win flags, canonical, exception fields, counts vs the oracle."""
    run_shard_gpu(dict(CASE_SPECS)[name], 2, kind)


@pytest.mark.parametrize("counts", [True, False])
def test_two_rank_routed_sorted_path(gpu_device, counts):
    """Routed records resolved by the sorted path: changeset j is one segment per source rank
    (tile map with segment ends and changesets); 300 tie-heavy changesets, 3 ranks."""
    kw = dict(seed=79, R=300, per_cs=2000, n_local=40_000, n_new=20_000, millis_span=8, counter_span=4,
              n_ranks=301)
    outs = run_shard_gpu(kw, 3, "parts", path="sorted", counts=counts)
    assert all(o[1]["path"] == "sorted" for o in outs)


@pytest.mark.parametrize("kind", ["routed", "parts"])
@pytest.mark.parametrize("path", ["gather", "sorted"])
@pytest.mark.parametrize("name", ["r8_tombstones", "drift_late", "explicit_millis"])
def test_two_rank_own_chunk_in_place(gpu_device, monkeypatch, name, kind, path):
    """The second collective merge on each ctx scatters the rank's own chunk straight into the
    receive columns (sized by the first call; CRDT_PLAN_OWN_IN_PLACE): every shard row, canonical and
    exception fields vs the oracle, gather and sorted receivers (win flags keep the copy).  The
    map-side combine is off here (CRDT_COMBINE=0): it routes folded keys, not records."""
    monkeypatch.setenv("CRDT_COMBINE", "0")
    outs = run_shard_gpu(dict(CASE_SPECS)[name], 2, kind, path=path, counts=path == "gather", again=True)
    for rank, res, *_ in outs:
        assert res["plan"]["own_in_place"] == (path != "gather"), (rank, res["plan"])
        assert not res["plan"]["combined"]


@pytest.mark.parametrize("kind", ["routed", "parts"])
@pytest.mark.parametrize("name", ["r4_ties", "drift_late", "send_overflow", "explicit_millis"])
def test_two_rank_packed_wire_gather_receiver(gpu_device, monkeypatch, name, kind):
    """Order-free merge without win flags: the global frame fits, so records cross as 16-B packed
    {slot, key, val}; these batches are small, so each owner applies them on the gather path and
    unpacks (lt, rank) first (k_unpack_routed).  (The map-side combine off: with it on, owners
    always resolve on the sorted path — test_two_rank_combine.)"""
    monkeypatch.setenv("CRDT_COMBINE", "0")
    run_shard_gpu(dict(CASE_SPECS)[name], 2, kind, path="auto", counts=False)


@pytest.mark.parametrize("kind", ["routed", "parts", "presharded"])
@pytest.mark.parametrize("name", ["r4_ties", "r8_tombstones", "drift_late", "dup_node", "explicit_millis"])
def test_two_rank_flagged_receivers(gpu_device, name, kind):
    """Win flags on a sharded ctx: the owners resolve their records on the sorted path's flagged form
    (unpacked wire, the global frame; a changeset is one segment per source), the flags travel back
    to the senders — every flag, shard row, canonical, exception field and exact count vs the oracle."""
    outs = run_shard_gpu(dict(CASE_SPECS)[name], 2, kind, path="sorted+flags", counts=True, again=True)
    for rank, res, *_ in outs:
        if res["path"] == "sorted":
            assert res["plan"]["flagged"] and not res["plan"]["wire_packed"], (rank, res["plan"])


def test_three_rank_flagged_receivers_fanin(gpu_device):
    """A 300-changeset tie-heavy fan-in over 3 ranks with win flags on the receivers' flagged form."""
    kw = dict(seed=79, R=300, per_cs=2000, n_local=40_000, n_new=20_000, millis_span=8, counter_span=4,
              n_ranks=301)
    outs = run_shard_gpu(kw, 3, "routed", path="sorted+flags", counts=True)
    assert all(o[1]["plan"]["flagged"] for o in outs), [o[1]["plan"] for o in outs]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kind", ["routed", "parts"])
@pytest.mark.parametrize("name", ["r4_ties", "r8_tombstones", "drift_late", "dup_node", "send_overflow",
                                  "explicit_millis"])
def test_two_rank_combine(gpu_device, monkeypatch, name, kind, world):
    """The map-side combine (order-free, frame fits; CRDT_COMBINE=2 forces it below 64 changesets):
    each rank folds its home records into one packed maximum per key (apply_sorted's emit mode),
    routes those, and the owners resolve them on the sorted path — every shard row, canonical and
    exception fields vs the oracle."""
    monkeypatch.setenv("CRDT_COMBINE", "2")
    outs = run_shard_gpu(dict(CASE_SPECS)[name], world, kind, path="auto", counts=False)
    for rank, res, *_ in outs:
        if res["status"] == 0 or res["plan"]["combined"]:
            assert res["plan"]["combined"] == res["plan"]["wire_packed"], (rank, res["plan"])


def test_two_rank_combine_hot_and_windows(gpu_device):
    """Combine (auto: 120 changesets) with split (hot) buckets on the home fold and on the owners:
    240K records over 4096 keys, ties and tombstones, 2 ranks."""
    kw = dict(seed=85, R=120, per_cs=2000, n_local=3000, n_new=1000, millis_span=4, counter_span=3,
              n_ranks=9, tomb_frac=0.2, neg_mod_frac=0.05)
    outs = run_shard_gpu(kw, 2, "routed", path="auto", counts=False)
    assert all(o[1]["plan"]["combined"] for o in outs), [o[1]["plan"] for o in outs]


@pytest.mark.parametrize("kind", ["routed", "parts", "presharded"])
@pytest.mark.parametrize("name", ["r8_tombstones", "drift_late"])
def test_rccl_single_rank(gpu_device, name, kind):
    """The same call over RCCL (crdt_comm_init_rccl, one rank): the device-side all-gather /
    all-reduce and the grouped exchange path the bench takes at N > 1."""
    run_shard_gpu(dict(CASE_SPECS)[name], 1, kind, backend="nccl")


def test_rccl_single_rank_sorted(gpu_device):
    kw = dict(seed=80, R=200, per_cs=3000, n_local=30_000, n_new=30_000, millis_span=8, counter_span=4,
              n_ranks=201, tomb_frac=0.1)
    outs = run_shard_gpu(kw, 1, "routed", backend="nccl", path="sorted", counts=False)
    assert outs[0][1]["path"] == "sorted"


def _fanin_shard_worker(rank, world, port, q, K, total, R, calls=1):
    """Routed fan-in (gen_fanin's home layout) on one rank, `calls` times from the same table; returns this
    shard's rows after each call (with the call's result, path and plan) and the ctx's routing tuner."""
    import os

    import torch
    import torch.distributed as dist

    from crdt_amd import DeviceTable
    from crdt_amd.dist import GlooComm
    from crdt_amd.workload import gen_fanin
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = gen_fanin(total=total, R=R, K=K, n_local=K // 2, s=0.8, device="cuda", rank=rank, world=world,
                       route=True)
        t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
        t.set_counts(False)
        t.set_merge_path("sorted")
        loc, home = wl["local"], wl["home"]
        t.comm_init_ops(world, rank, GlooComm(dist))
        got = []
        for _ in range(calls):
            t.clear_rows(0, wl["capacity"])
            t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
            t.canonical = wl["c0"]
            res, _ = t.merge(home["key"], home["lt"], home["rank"], home["val"], wl["home_offsets"], wl["wall"],
                             win_flags=False)
            got.append((res, t.last_path(), t.read_rows(np.arange(wl["capacity"], dtype=np.uint32)), t.last_plan()))
        if calls == 1:
            q.put((rank,) + got[0])
        else:
            q.put((rank, got, t.route_tune()))
        t.close()
        torch.cuda.empty_cache()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("combine,route_l1,split", [("1", "1", "1"), ("0", "1", "1"), ("0", "1", "0"), ("0", "1", "4"),
                                                    ("0", "1", "3"), ("0", "0", "1"), ("0", "2", "1"), ("0", "2", "0"),
                                                    ("0", "2", "4"), ("0", "3", "1")])
def test_two_rank_routed_fanin_equals_one_gpu(gpu_device, monkeypatch, combine, route_l1, split):
    """Full-table parity at a fan-in shape: 2 ranks (replica j whole on rank j % 2, records
    routed to key % 2) give exactly the rows and canonical of the C oracle's unsharded merge — with the
    map-side combine (each rank folds its home records per key before the exchange), with the routed
    level-1 partition (home records partitioned straight into the owners' level-1 buckets, owners from
    level 2 on; route_l1 = 2: with every owner's leading level-1 digits folded at the sender, one packed
    maximum per key, sent after the pieces; 3: every digit folded), and with plain record routing."""
    monkeypatch.setenv("CRDT_COMBINE", combine)
    monkeypatch.setenv("CRDT_ROUTE_L1", route_l1)
    monkeypatch.setenv("CRDT_RL1_SPLIT", split)             # route_l1 in two pipelined pieces / in one
    monkeypatch.setenv("CRDT_ROUTE_TUNE", "0")               # the fixed rule (the tuner: the test below)
    import torch.multiprocessing as mp

    from tests.test_dist_cpu import _free_port
    K, total, R = 1 << 22, 4_000_000, 128
    ref, rows = _fanin_reference(K, total, R)                  # the C oracle, unsharded
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fanin_shard_worker, args=(r, 2, port, q, K, total, R)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(2)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, res, path, shard, plan in outs:
        assert path == "sorted"
        assert plan["combined"] == (combine == "1"), plan
        assert plan["route_l1"] == (combine == "0" and route_l1 != "0"), plan
        assert plan["rl1_head"] == (plan["route_l1"] and route_l1 in ("2", "3")), plan
        if plan["route_l1"]:                                   # pieces cut at changeset boundaries
            assert plan["rl1_pieces"] == {"0": 1, "1": 2}.get(split, int(split)), plan
        for f in ("status", "n_stored", "canonical_lt", "exc_changeset"):
            assert res[f] == ref[f], (rank, f)
        for a, b in zip(shard, rows):
            assert np.array_equal(a, b[rank::2]), rank


@pytest.mark.parametrize("tries,R", [("3", 128), ("4", 128), ("1", 128), ("3", 2048)])
def test_place_tuner_candidates_same_rows(gpu_device, monkeypatch, tries, R):
    """The level-1 placement tuner (crdt_reserve_scratch with CRDT_PLACE_TRIES candidate buffers): the
    first sorted merges run their level-1 scatter on each candidate in turn and the fastest is kept;
    every call — on every candidate and after the choice — leaves exactly the C oracle's rows.
    (2048 changesets: more than the packed key's changeset window, so a call partitions in several
    windows, every one on the candidate under trial.)"""
    from crdt_amd import DeviceTable
    from crdt_amd.workload import gen_fanin
    monkeypatch.setenv("CRDT_PLACE_TRIES", tries)
    K, total = 1 << 22, 4_000_000
    ref, rows = _fanin_reference(K, total, R)
    wl = gen_fanin(total=total, R=R, K=K, n_local=K // 2, s=0.8, device="cuda")
    loc, own = wl["local"], wl["owned"]
    t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
    t.reserve_scratch(total)
    t.set_merge_path("sorted")
    t.set_counts(False)
    n = int(tries)
    assert t.place_info()["candidates"] == n and t.place_info()["kept"] == (None if n > 1 else 0)
    for i in range(2 * n + 2):                                # (the warm-up merge, then two per candidate)
        t.clear_rows(0, wl["capacity"])
        t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
        t.canonical = wl["c0"]
        res, _ = t.merge(own["key"], own["lt"], own["rank"], own["val"], wl["owned_offsets"], wl["wall"],
                         win_flags=False)
        info = t.place_info()
        assert info["kept"] == (0 if n == 1 else None if i < 2 * n else info["kept"]), (i, info)
        assert info["merges_used"] == (0 if n == 1 else min(i + 1, 2 * n + 1)), (i, info)
        for f in ("status", "n_stored", "canonical_lt", "exc_changeset"):
            assert res[f] == ref[f], (i, f)
        for a, b in zip(t.read_rows(np.arange(K, dtype=np.uint32)), rows):
            assert np.array_equal(a, b), i
    info = t.place_info()
    if n > 1:
        assert info["kept"] in range(n) and all(m > 0 for m in info["level1_ms"]), info
        assert info["level1_ms"][info["kept"]] == min(info["level1_ms"]), info
    t.close()


@pytest.mark.parametrize("G", [4, 8])
def test_loopback_route_ways_same_rows(gpu_device, monkeypatch, G):
    """The device-memory collective path — the one RCCL takes: no host synchronisation inside the
    collectives, so the partition, the exchanges and the owners' work overlap on their three streams as
    they do on the node — on one GPU through a loopback communicator (tests/_loopback.py: rank 0 of G ranks
    that all hold its data; the peers' parts come back as device copies).  route_l1 in 1, 2, 3 and 4
    pipelined pieces (and in 2 and 1 with the head fold), record routing and the map-side fold apply the same
    records and must leave the same rows, and every row's lt / rank / value is checked against the rule restated
    on the host (_loopback_winners).  (Under the loopback, keys of different owners share rank 0's slots, so
    two records of one changeset may carry equal packed keys at one slot and the order-free fold may keep either
    value: those tie slots, predicted exactly from the records, are the only ones whose value is not pinned.)"""
    from crdt_amd import DeviceTable
    from crdt_amd.workload import gen_fanin
    from tests._loopback import LoopbackComm
    monkeypatch.setenv("CRDT_ENV_DYNAMIC", "1")
    wl = gen_fanin(total=2_000_000 * G, R=128, K=1 << 24, n_local=1 << 23, s=0.8, device="cuda", rank=0, world=G,
                   route=True)
    home, loc, cap = wl["home"], wl["local"], wl["capacity"]
    t = DeviceTable(0, local_rank=0, capacity=cap)
    t.set_counts(False)
    comm = LoopbackComm(G)
    t.comm_init_ops(G, 0, comm)
    ways = {"1": ("0", "1", "0", 1), "2": ("0", "1", "1", 2), "3": ("0", "1", "3", 3), "4": ("0", "1", "4", 4),
            "route": ("0", "0", "1", 0), "fold": ("2", "1", "1", 0), "head": ("0", "2", "1", 2),
            "head1": ("0", "2", "0", 1), "headall": ("0", "3", "1", 2)}
    rows = {}
    for name, (comb, rl1, split, pieces) in ways.items():
        monkeypatch.setenv("CRDT_COMBINE", comb)
        monkeypatch.setenv("CRDT_ROUTE_L1", rl1)
        monkeypatch.setenv("CRDT_RL1_SPLIT", split)
        for _ in range(2):                                    # (the second call reuses every buffer)
            t.clear_rows(0, cap)
            t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
            t.canonical = wl["c0"]
            res, _ = t.merge(home["key"], home["lt"], home["rank"], home["val"], wl["home_offsets"], wl["wall"],
                             win_flags=False)
            assert res["status"] == 0 and comm.error is None, (name, res, comm.error)
            # crdt_timing.sent_bytes: what the library handed the communicator for its peers
            assert t.timing()["sent_bytes"] == comm.exchange_bytes() > 0, name
            plan = t.last_plan()
            assert plan["route_l1"] == (pieces > 0) and plan["rl1_pieces"] == pieces, (name, plan)
            assert plan["combined"] == (name == "fold"), (name, plan)
            assert plan["rl1_head"] == name.startswith("head"), (name, plan)
            rows.setdefault(name, []).append(t.read_rows(np.arange(cap, dtype=np.uint32)))
    comm.exchange_ms()
    t.close()
    want_lt, want_rank, want_val, present, tie = _loopback_winners(wl, G, cap)
    ref = rows["1"][0]
    assert np.array_equal(ref[3] != ABSENT_MOD, present)
    assert np.array_equal(ref[0][present], want_lt[present]) and np.array_equal(ref[1][present], want_rank[present])
    keep = present & ~tie
    for name, runs in rows.items():
        for got in runs:                                      # (each way twice: the second reuses every buffer)
            for f in (0, 1, 3):
                assert np.array_equal(ref[f], got[f]), (name, f)
            # the value handle: the restated winner's everywhere but the loopback's tie slots
            assert np.array_equal(got[2][keep], want_val[keep]), name


def _loopback_winners(wl, G, cap):
    """What the loopback leaves, restated on the host (crdt.dart:83-84 per slot, the order-free fold's
    rule): rank 0 applies every record of its home changesets, each at slot key // G (its own and, as the
    peers' parts, those it routes to them), so a slot's winner is the maximum (lt, rank) over the local row
    and the slot's records — a record only when it beats the row (equal keeps the row), the earliest
    changeset among equal records.  Returns (lt, rank, val) per slot, the slots holding a row, and the tie
    slots, where two records of ONE changeset (different owners) carry the winning (lt, rank) and either value
    may stand."""
    home, loc = wl["home"], wl["local"]
    h = lambda a: a.cpu().numpy()                                 # noqa: E731
    slot = h(home["key"]).astype(np.int64) // G
    lt = h(home["lt"]).astype(np.int64)
    rk = h(home["rank"]).astype(np.int64)
    val = h(home["val"]).view(np.uint32)
    offs = np.asarray(wl["home_offsets"], dtype=np.int64)
    j = np.repeat(np.arange(len(offs) - 1), np.diff(offs))
    o = np.lexsort((-j, rk, lt, slot))                             # per slot: the last is the winner
    slot, lt, rk, val, j = slot[o], lt[o], rk[o], val[o], j[o]
    last = np.flatnonzero(np.r_[slot[1:] != slot[:-1], True])
    dup = np.zeros(len(slot), bool)                                # the previous record has the same key + changeset
    dup[1:] = (slot[1:] == slot[:-1]) & (lt[1:] == lt[:-1]) & (rk[1:] == rk[:-1]) & (j[1:] == j[:-1])
    w_lt = np.full(cap, np.iinfo(np.int64).min, np.int64)
    w_rk = np.zeros(cap, np.int64)
    w_val = np.zeros(cap, np.uint32)
    present = np.zeros(cap, bool)
    ls = h(loc["slot"]).astype(np.int64)
    w_lt[ls], w_rk[ls], w_val[ls], present[ls] = h(loc["lt"]), h(loc["rank"]), h(loc["val"]).view(np.uint32), True
    s = slot[last]
    beats = ~present[s] | (lt[last] > w_lt[s]) | ((lt[last] == w_lt[s]) & (rk[last] > w_rk[s]))
    ws = s[beats]
    w_lt[ws], w_rk[ws], w_val[ws], present[ws] = lt[last][beats], rk[last][beats], val[last][beats], True
    tie = np.zeros(cap, bool)
    tie[ws] = dup[last][beats]
    return w_lt, w_rk.astype(np.uint32), w_val, present, tie


def _fanin_reference(K, total, R):
    """The C oracle (oracle/merge_oracle.c, the KAT-pinned restatement) merging gen_fanin's whole job
    unsharded: (result fields, all rows as (lt, rank, val, mod))."""
    from crdt_amd.workload import gen_fanin
    from oracle.oracle_c import OracleTable
    wl = gen_fanin(total=total, R=R, K=K, n_local=K // 2, s=0.8, device="cuda")
    loc, own = wl["local"], wl["owned"]
    t = OracleTable(K, 0, wl["c0"])
    t.put_rows(*(loc[f].cpu().numpy() for f in ("slot", "lt", "rank", "val", "mod")))
    res, _ = t.merge(*(own[f].cpu().numpy() for f in ("key", "lt", "rank", "val")), wl["owned_offsets"],
                     wl["wall"], want_flags=False)
    rows = tuple(np.array(t.rows[f]) for f in ("lt", "rank", "val", "mod"))
    return res.as_dict(), rows


def test_two_rank_route_tune(gpu_device, monkeypatch):
    """The routing tuner (comm_path.inc RouteTune, the auto settings): the first calls take route_l1 in two
    pieces twice, the map-side combine twice, route_l1 in four pieces, in one and in two with the head fold twice
    each, every later call the way
    whose timed call was fastest (max over the ranks, the same way on both ranks); every call leaves
    exactly the C oracle's rows of the unsharded merge."""
    for k in ("CRDT_COMBINE", "CRDT_ROUTE_L1", "CRDT_ROUTE_TUNE", "CRDT_RL1_SPLIT"):
        monkeypatch.delenv(k, raising=False)
    import torch.multiprocessing as mp

    from tests.test_dist_cpu import _free_port
    K, total, R = 1 << 22, 4_000_000, 128
    ref, rows = _fanin_reference(K, total, R)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fanin_shard_worker, args=(r, 2, port, q, K, total, R, 12)) for r in range(2)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(2)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tunes = [o[2] for o in outs]
    assert tunes[0] == tunes[1], tunes                        # one decision, from the max over ranks
    tune = tunes[0]
    ways = ("route_l1", "combine", "route_l1_4", "route_l1_1", "route_l1_head")
    assert tune["best"] in ways and all(tune[f"{w}_ms"] > 0 for w in ways), tune
    assert tune["best"] == min(ways, key=lambda w: tune[f"{w}_ms"]), tune
    for rank, got, _ in outs:
        for i, (res, path, shard, plan) in enumerate(got):
            assert path == "sorted" and plan["route_tuned"], (rank, i, plan)
            way = tune["best"] if i >= 10 else ways[i // 2]
            assert plan["combined"] == (way == "combine") and plan["route_l1"] == (way != "combine"), (rank, i, plan)
            assert plan["rl1_head"] == (way == "route_l1_head"), (rank, i, plan)
            if way != "combine":
                assert plan["rl1_pieces"] == {"route_l1_4": 4, "route_l1_1": 1}.get(way, 2), (rank, i, plan)
            for f in ("status", "n_stored", "canonical_lt", "exc_changeset"):
                assert res[f] == ref[f], (rank, i, f)
            for a, b in zip(shard, rows):
                assert np.array_equal(a, b[rank::2]), (rank, i)


@pytest.mark.parametrize("name", ["drift_late", "dup_node", "r8_tombstones"])
def test_eight_rank_routed_small(gpu_device, name):
    """G = 8 (route_bits(8), the 8-way count exchange, grouped all-to-all over 7 peers): the small
    golden cases routed over 8 ranks on one GPU through the gloo communicator, sorted receivers in
    the order-free form — rows of all 8 shards, canonical and exception fields vs the oracle."""
    outs = run_shard_gpu(dict(CASE_SPECS)[name], 8, "routed", path="sorted", counts=False)
    assert all(o[1]["path"] in ("sorted", "gather") for o in outs)


@pytest.mark.parametrize("combine", ["1", "0"])
@pytest.mark.parametrize("inject", [None, "drift", "dup"])
def test_eight_rank_routed_packed_sorted(gpu_device, monkeypatch, inject, combine):
    """The rehearsal of config 4's 8-GPU plan: 8 ranks on one GPU over the gloo communicator,
    16M records in 64 changesets (replica j whole on rank j % 8, records routed to key % 8).  The
    global frame fits, so records cross as 16-B packed wire records and every owner resolves them
    on the sorted path; a drift or a duplicate-node record raises at (41, 123,456).  Every row of all
    8 shards, the canonical clock, status and exception fields against the C oracle.  combine = 1:
    each rank folds its home records to one packed maximum per key first (the map-side combine)."""
    monkeypatch.setenv("CRDT_COMBINE", combine)            # (64 changesets: auto combines)
    kw = dict(seed=808, R=64, per_cs=250_000, n_local=1_500_000, n_new=600_000, millis_span=1 << 12,
              counter_span=16, n_ranks=65, tomb_frac=0.1, inject=inject)
    outs = run_shard_gpu(kw, 8, "routed", path="sorted", counts=False, again=True)
    for rank, res, *_ in outs:
        assert res["path"] == "sorted" and res["plan"]["wire_packed"], (rank, res["plan"])
        assert res["plan"]["combined"] == (combine == "1"), (rank, res["plan"])
        if combine == "0":
            assert res["plan"]["own_in_place"], (rank, res["plan"])    # the second call on each ctx
        assert res["status"] == {None: 0, "drift": 1, "dup": 2}[inject], res
        if inject:
            assert (res["exc_changeset"], res["exc_index"]) == (41, 123_456), res


@pytest.mark.parametrize("inject,head", [(None, "1"), ("drift", "1"), ("dup", "1"), ("dup", "2"), ("drift", "3")])
def test_eight_rank_route_l1(gpu_device, monkeypatch, inject, head):
    """The routed level-1 partition at G = 8 (comm_path.inc, route_l1): shards of > 2^20 slots (two
    digits per owner), 16M records in 64 changesets, every rank partitioning its home records straight
    into the 8 owners' level-1 buckets (14-B records over the exchange, own part in place), the owners
    from level 2 on; a drift or duplicate-node record at (41, 123,456).  Every row of all 8 shards,
    canonical, status and exception fields vs the C oracle, on two calls per ctx (buffers reused).
    head = 2: every owner's leading level-1 digits folded at the sender (CRDT_ROUTE_L1=2); 3: every digit."""
    monkeypatch.setenv("CRDT_ROUTE_L1", head)
    kw = dict(seed=818, R=64, per_cs=250_000, n_local=6_000_000, n_new=3_000_000, millis_span=1 << 12,
              counter_span=16, n_ranks=65, tomb_frac=0.1, inject=inject)
    outs = run_shard_gpu(kw, 8, "routed", path="sorted", counts=False, again=True)
    for rank, res, *_ in outs:
        assert res["path"] == "sorted" and res["plan"]["route_l1"], (rank, res["plan"])
        assert not res["plan"]["combined"], (rank, res["plan"])
        assert res["plan"]["rl1_head"] == (head != "1"), (rank, res["plan"])
        assert res["status"] == {None: 0, "drift": 1, "dup": 2}[inject], res
        if inject:
            assert (res["exc_changeset"], res["exc_index"]) == (41, 123_456), res


# ------------------------------------------------------------------ sorted path
# The key-partitioned path (sorted_path.inc) against the same oracle: rows, canonical,
# status, exception fields and the per-record counts n_present / n_won.
def _sorted_expected(case):
    """The sorted path runs iff its preconditions hold (no flags, C0 >= 0)."""
    return "sorted" if case["c0"] >= 0 else "gather"


@pytest.mark.parametrize("name", [n for n, _ in CASE_SPECS])
@pytest.mark.parametrize("counts", [True, False])
def test_sorted_golden_vectors(gpu_device, name, counts):
    case, exp, expected = golden_case(name)
    rows, res, flags = device_run(case, path="sorted", flags=False, counts=counts)
    check_rows(*rows, exp)
    assert flags is None
    for k, v in expected.items():
        if not counts and res["path"] == "sorted" and k in ("n_present", "n_won"):
            continue
        assert res[k] == v, (name, k, res[k], v)
    assert res["path"] == _sorted_expected(case)


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("counts", [True, False])
def test_sorted_random_small(gpu_device, seed, counts):
    rng = np.random.default_rng(1000 + seed)
    kw = dict(seed=2000 + seed, R=int(rng.integers(1, 12)), per_cs=int(rng.integers(0, 500)),
              n_local=int(rng.integers(1, 600)), n_new=int(rng.integers(0, 400)),
              millis_span=int(rng.integers(1, 100)), counter_span=int(rng.integers(1, 8)),
              n_ranks=int(rng.integers(2, 40)), tomb_frac=float(rng.random() * 0.5),
              neg_mod_frac=float(rng.random() * 0.1), dup_frac=float(rng.random() * 0.01),
              drift_frac=float(rng.random() * 0.005))
    kw["local_rank"] = int(rng.integers(0, kw["n_ranks"]))
    case = make_case(**kw)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=counts)
    assert res["path"] == _sorted_expected(case)


@pytest.mark.parametrize("capacity", [None, (1 << 20) + 7, 1 << 24])
@pytest.mark.parametrize("counts", [True, False])
def test_sorted_ties_many_changesets(gpu_device, capacity, counts):
    """300 tie-heavy changesets (same key in many of them, equal (lt, rank) across them):
    one-level buckets (capacity <= 2^20) and two-level (capacity > 2^20)."""
    case = make_case(seed=79, R=300, per_cs=2000, n_local=40_000, n_new=20_000, millis_span=8,
                     counter_span=4, n_ranks=301)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=counts, capacity=capacity)
    assert res["path"] == "sorted" and res["n_won"] > 0


@pytest.mark.parametrize("counts", [True, False])
def test_sorted_hot_keys_in_one_chunk(gpu_device, counts):
    """Few keys, many changesets: every 2048-record chunk holds dozens of records per key,
    so the in-chunk same-key lists are long (ordering inside a chunk)."""
    case = make_case(seed=83, R=400, per_cs=60, n_local=50, n_new=30, millis_span=3, counter_span=2,
                     n_ranks=7)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=counts)
    assert res["path"] == "sorted"


@pytest.mark.parametrize("counts", [True, False])
def test_sorted_split_hot_bucket(gpu_device, counts):
    """All keys in one 4096-key bucket, 240K records: the bucket is resolved as 4 parts
    (part folds, carries, per-part counts) — ties and tombstones across the part cuts."""
    case = make_case(seed=85, R=120, per_cs=2000, n_local=3000, n_new=1000, millis_span=4, counter_span=3,
                     n_ranks=9, tomb_frac=0.2, neg_mod_frac=0.05)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=counts)
    assert res["path"] == "sorted" and res["n_won"] > 0


def _spread_case(case, buckets, n_ids):
    """Remap a case's key ids i -> buckets[i // 4096] * 4096 + i % 4096 on an n_ids table."""
    from tests._cases import ABSENT_MOD
    bk = np.asarray(buckets, np.int64)
    remap = lambda k: (bk[k.astype(np.int64) // 4096] * 4096 + k.astype(np.int64) % 4096)  # noqa: E731
    loc = case["local"]
    ids = remap(np.arange(case["n_local"]))
    local = {"lt": np.zeros(n_ids, np.int64), "rank": np.zeros(n_ids, np.uint32),
             "val": np.zeros(n_ids, np.uint32), "mod": np.full(n_ids, ABSENT_MOD, np.int64)}
    for f in local:
        local[f][ids] = loc[f]
    out = dict(case, n_ids=n_ids, n_local=n_ids, local=local)
    out["key"] = remap(case["key"]).astype(np.uint32)
    return out


@pytest.mark.parametrize("counts", [True, False])
def test_sorted_split_buckets_across_blocks(gpu_device, counts):
    """Split (hot) buckets at bucket ids on both sides of the 1024-bucket blocks of the item
    prefix and hot list (k_bucket_items), two-level capacity 2^24: ~80K records in each of
    six buckets (two parts each), ties and tombstones."""
    buckets = [3, 1023, 1024, 2047, 2048, 4095]
    base = make_case(seed=86, R=40, per_cs=12_000, n_local=18_000, n_new=6 * 4096 - 18_000, millis_span=4,
                     counter_span=3, n_ranks=9, tomb_frac=0.2, neg_mod_frac=0.05)
    case = _spread_case(base, buckets, 1 << 24)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=counts)
    assert res["path"] == "sorted" and res["n_won"] > 0


@pytest.mark.parametrize("counts", [True, False])
def test_sorted_windows_and_late_exception(gpu_device, counts):
    """More changesets than one 4096-changeset window; a drift record in changeset 4500
    stops the batch there (later windows and changesets untouched)."""
    case = make_case(seed=84, R=5000, per_cs=20, n_local=3000, n_new=2000, millis_span=20,
                     force=[(4500, 7, "drift")])
    res = compare_with_oracle(case, path="sorted", flags=False, counts=counts)
    assert res["status"] == 1 and res["exc_changeset"] == 4500 and res["path"] == "sorted"


@pytest.mark.parametrize("counts", [True, False])
def test_sorted_large_single_changeset(gpu_device, counts):
    from tests._cases import WALL
    case = make_case(seed=78, R=1, per_cs=1_000_000, n_local=1_200_000, n_new=800_000,
                     millis_span=1 << 16, base=WALL - 70_000)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=counts)
    assert res["status"] == 0 and res["path"] == "sorted"


def _frame_edge_case(seed):
    """Local rows placed around the frame of the records (sorted_path.inc, packed resolve): lt
    just below / at / just above the records' lt range, ranks below / inside / above theirs,
    equal (lt, rank) with a record — every clamp of pack_local against the list form's rules."""
    case = make_case(seed=seed, R=40, per_cs=2000, n_local=3000, n_new=1000, millis_span=4, counter_span=2,
                     n_ranks=9, local_rank=0, tomb_frac=0.2)
    rng = np.random.default_rng(seed)
    lo, hi = int(case["lt"].min()), int(case["lt"].max())
    rlo, rhi = int(case["rank"].min()), int(case["rank"].max())
    loc = case["local"]
    n = case["n_local"]
    lt_choices = np.array([lo - 1, lo, (lo + hi) // 2, hi, hi + 1], np.int64)
    loc["lt"] = lt_choices[rng.integers(0, 5, n)]
    rk_choices = np.array([max(rlo - 1, 0), rlo, (rlo + rhi) // 2, rhi, rhi + 1, 200], np.uint32)
    loc["rank"] = rk_choices[rng.integers(0, 6, n)]
    # a tenth of the local rows copy a record of their key exactly (equal (lt, rank): local keeps)
    first = {}
    for x, k in enumerate(case["key"].tolist()):
        first.setdefault(k, x)
    for k in rng.choice(n, n // 10, replace=False):
        if int(k) in first:
            loc["lt"][k] = case["lt"][first[int(k)]]
            loc["rank"][k] = case["rank"][first[int(k)]]
    loc["mod"] = np.where(loc["mod"] >= 0, loc["lt"], loc["mod"])
    vis = loc["mod"] >= 0
    case["c0"] = int(loc["lt"][vis].max())
    return case


@pytest.mark.parametrize("packed", ["1", "0"])
@pytest.mark.parametrize("seed", [91, 92])
def test_sorted_packed_frame_edges(gpu_device, monkeypatch, seed, packed):
    """Order-free sorted path, packed resolve (CRDT_PACKED=1) and its list form (0), on local rows
    at every edge of the records' frame; one- and two-level capacities."""
    monkeypatch.setenv("CRDT_PACKED", packed)
    case = _frame_edge_case(seed)
    for cap in (None, (1 << 20) + 3):
        res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=cap)
        assert res["path"] == "sorted"


@pytest.mark.parametrize("slack", [0, 1, 700])
@pytest.mark.parametrize("seed", [91, 92])
def test_sorted_rank_bound_frame(gpu_device, seed, slack):
    """crdt_set_rank_bound: the packed frame's rank part comes from the bound (the scan reads lt
    only) — tight and loose bounds, local rows with ranks above it, same rows as the oracle."""
    case = _frame_edge_case(seed)
    bound = int(case["rank"].max()) + 1 + slack
    for cap in (None, (1 << 20) + 3):
        res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=cap, rank_bound=bound)
        assert res["path"] == "sorted"


def _late_drift_case(seed):
    """A ClockDrift in a late changeset: stop < R, the changesets from it on are not applied."""
    case = make_case(seed=seed, R=48, per_cs=3000, n_local=4000, n_new=2000, millis_span=4, counter_span=3,
                     n_ranks=7, tomb_frac=0.1)
    x = int(case["offsets"][37]) + 5
    case["lt"][x] = (case["wall"] + 60_001) << 16
    return case


@pytest.mark.parametrize("kind", ["edges", "late_drift", "hot"])
@pytest.mark.parametrize("cap", [None, (1 << 20) + 3])
def test_sorted_hist_in_scan(gpu_device, monkeypatch, kind, cap):
    """The level-1 histogram counted by the scan (device columns, rank bound, order-free form):
    same rows / result as the oracle and as the separate histogram pass (CRDT_HIST_FUSE=0),
    including a stop < R (rows of the unapplied changesets' tiles cleared) and one / two levels."""
    if kind == "edges":
        case = _frame_edge_case(95)
    elif kind == "late_drift":
        case = _late_drift_case(96)
    else:
        case = make_case(seed=97, R=120, per_cs=2000, n_local=3000, n_new=1000, millis_span=4, counter_span=3,
                         n_ranks=9, tomb_frac=0.2)
    bound = int(case["rank"].max()) + 1
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=cap, rank_bound=bound,
                              device_cols=True)
    assert res["path"] == "sorted" and res["plan"]["hist_in_scan"], res["plan"]
    assert res["plan"]["two_level"] == (cap is not None)
    assert res["plan"]["key8"] == (cap is not None), res["plan"]      # these frames leave 4 bits free
    if kind == "late_drift":
        assert res["status"] != 0 and res["n_stored"] < len(case["offsets"]) - 1
    monkeypatch.setenv("CRDT_HIST_FUSE", "0")
    res0 = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=cap, rank_bound=bound,
                               device_cols=True)
    assert not res0["plan"]["hist_in_scan"]


@pytest.mark.parametrize("counts", [False, True])
def test_rank_bound_violation_stores_nothing(gpu_device, counts):
    """A batch rank at or above the promised bound: the packed sorted forms (order-free, and the
    ordered one exact counts take) refuse the call with CRDT_E_INVALID before writing a row
    (canonical unchanged); with the promise withdrawn the batch merges exactly."""
    from crdt_amd import CrdtNativeError, DeviceTable
    case = make_case(seed=94, R=20, per_cs=1000, n_local=2000, n_new=500, millis_span=4, counter_span=2,
                     n_ranks=9, tomb_frac=0.1)
    bound = int(case["rank"].max())               # the highest rank breaks the promise
    t = DeviceTable(0, local_rank=case["local_rank"], capacity=case["n_ids"])
    t.set_merge_path("sorted")
    t.set_counts(counts)
    t.set_rank_bound(bound)
    loc = case["local"]
    keep = loc["mod"] != ABSENT_MOD
    ids = np.arange(case["n_local"], dtype=np.uint32)[keep]
    t.put_rows(ids, loc["lt"][keep], loc["rank"][keep], loc["val"][keep], loc["mod"][keep])
    t.canonical = case["c0"]
    before = t.read_rows(np.arange(case["n_ids"], dtype=np.uint32))
    with pytest.raises(CrdtNativeError, match="invalid"):
        t.merge(case["key"], case["lt"], case["rank"], case["val"], case["offsets"], case["wall"],
                millis=case["millis"], win_flags=False)
    assert t.last_path() == "sorted"
    after = t.read_rows(np.arange(case["n_ids"], dtype=np.uint32))
    for a, b in zip(before, after):
        assert np.array_equal(a, b)
    assert t.canonical == case["c0"]
    t.set_rank_bound(0)                           # promise withdrawn: the same batch merges exactly
    res, _ = t.merge(case["key"], case["lt"], case["rank"], case["val"], case["offsets"], case["wall"],
                     millis=case["millis"], win_flags=False)
    orows, ores, _ = oracle_run(case)
    for f, a in zip(("lt", "rank", "val", "mod"), t.read_rows(np.arange(case["n_ids"], dtype=np.uint32))):
        assert np.array_equal(a, orows[f]), f
    assert res["canonical_lt"] == ores["canonical_lt"]
    t.close()


@pytest.mark.parametrize("form_off", ["64", "128", "256", "448", "512", "1024", "8192", "32768", "65536",
                                      "8388608", "16777216", "33554432", "67108864", "268435456"])
def test_sorted_packed_form_switches(gpu_device, monkeypatch, form_off):
    """CRDT_SORTED_FORM: each refinement of the packed form switched off (changed-rows-only
    resolve writes, 16-B final records, 16-B level-1 records, forward-only tile fill, the
    level-2 histogram with 2-B loads into shared bins, the level-1 scatter's / the scan's narrow
    loads, 32K-record level-2 tiles) gives the same rows."""
    monkeypatch.setenv("CRDT_SORTED_FORM", form_off)
    case = _frame_edge_case(99)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=(1 << 20) + 3,
                              rank_bound=int(case["rank"].max()) + 1, device_cols=True)
    assert res["plan"]["packed"] and res["plan"]["two_level"]
    assert res["plan"]["key8"] == (form_off in ("64", "256", "512", "1024", "8192", "32768", "65536", "8388608",
                                                 "16777216", "33554432", "67108864", "268435456")), \
        res["plan"]


@pytest.mark.parametrize("grid", ["16777216", "33554432"])
@pytest.mark.parametrize("k", range(4))
@pytest.mark.parametrize("path", ["gather", "sorted"])
def test_scan_step_major_grid(gpu_device, monkeypatch, k, path, grid):
    """CRDT_SORTED_FORM bits 16777216 / 33554432: the clock scan's step-major grid (changeset in blockIdx.x,
    step in blockIdx.y) forced on / off (by default it runs on batches of at most 8192 scan workgroups) —
    the same tile maxima, raising tiles and fused level-1 histogram, so the same rows and exception fields
    as the oracle, on multi-step changesets with a forced drift / duplicate-node record."""
    monkeypatch.setenv("CRDT_SORTED_FORM", grid)
    case = list(_fused_cases())[k]
    kw = dict(path=path)
    if path == "sorted":
        kw.update(flags=False, counts=False, rank_bound=int(case["rank"].max()) + 1, device_cols=True)
    compare_with_oracle(case, **kw)


@pytest.mark.parametrize("form", ["0", "1048576", "67108864"])
@pytest.mark.parametrize("sparse_t", ["0", "1024", "1000000000"])
@pytest.mark.parametrize("seed", [99, 5])
def test_sorted_sparse_bucket_resolve(gpu_device, monkeypatch, sparse_t, seed, form):
    """CRDT_SPARSE_T: buckets of fewer records than it fold their records from "absent" and read only
    the touched keys' rows afterwards (0: every bucket loads its rows first; 10^9: every bucket below
    the high-water mark is sparse) — the same rows, canonical and exception fields as the oracle, on
    frame edges (rows below / at / above the frame, ranks outside it, exact ties) and on a case where a
    part of the table lies above the high-water mark.  Each in k_resolve_sparse's own workgroups (the
    default; 1048576: on the 13-B records of the plain lt field) and inside k_resolve_packed (67108864)."""
    monkeypatch.setenv("CRDT_SPARSE_T", sparse_t)
    monkeypatch.setenv("CRDT_SORTED_FORM", form)
    case = _frame_edge_case(seed) if seed == 99 else _cold_bucket_case(seed)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False,
                              capacity=(1 << 20) + 3 if seed == 99 else case["n_ids"],
                              rank_bound=int(case["rank"].max()) + 1, device_cols=True)
    assert res["plan"]["packed"] and res["plan"]["two_level"]


@pytest.mark.parametrize("form", ["0", "1048576", "128"])
def test_sorted_sparse_kernel_many_rounds(gpu_device, monkeypatch, form):
    """k_resolve_sparse over buckets of 32768 records (CRDT_SPARSE_T = 10^9: every unsplit bucket is
    sparse): 16 rounds of 2048 records each, the second phase re-reading them; ties across changesets
    (few millis, small counters), tombstones and invisible rows — the oracle's rows and fields, on the
    compact, 13-B (1048576) and 16-B (128) record forms."""
    monkeypatch.setenv("CRDT_SPARSE_T", "1000000000")
    monkeypatch.setenv("CRDT_SORTED_FORM", form)
    case = make_case(seed=4242, n_local=10000, n_new=6384, R=8, per_cs=16384, millis_span=3, counter_span=3,
                     n_ranks=5, neg_mod_frac=0.05, local_rank=1)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False,
                              rank_bound=int(case["rank"].max()) + 1, device_cols=True)
    assert res["plan"]["packed"]


def _cold_bucket_case(seed):
    """Keys spread over the whole of a > 2^20-key table: ~260 cold 4096-key buckets of a few
    hundred records each (no bucket near the 65,536-record split), so every resolve runs the
    unsplit-bucket kernels — the _frame_edge_case keys all sit in bucket 0, which is split."""
    case = make_case(seed=seed, R=24, per_cs=4000, n_local=700_000, n_new=360_000, millis_span=4,
                     counter_span=3, n_ranks=9, tomb_frac=0.15, neg_mod_frac=0.02)
    assert case["n_ids"] > (1 << 20)
    return case


@pytest.mark.parametrize("form_off", ["0", "64", "128", "256", "448", "512", "1024", "2048", "8192", "32768",
                                      "65536"])
def test_sorted_packed_form_switches_cold_buckets(gpu_device, monkeypatch, form_off):
    """Every CRDT_SORTED_FORM switch on records spread over many cold buckets, two levels: the
    unsplit-bucket resolve of each form (the changed-rows-only writes with 13-B final records
    among them) against the oracle."""
    monkeypatch.setenv("CRDT_SORTED_FORM", form_off)
    case = _cold_bucket_case(131)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=case["n_ids"],
                              rank_bound=int(case["rank"].max()) + 1, device_cols=True)
    assert res["plan"]["packed"] and res["plan"]["two_level"], res["plan"]
    assert res["plan"]["key8"] == (form_off not in ("128", "448")), res["plan"]


def _kind_case(kind):
    if kind == "edges":
        return _frame_edge_case(141), (1 << 20) + 3
    if kind == "late_drift":
        return _late_drift_case(142), (1 << 20) + 3
    if kind == "dup":
        return make_case(seed=143, R=40, per_cs=1500, n_local=3000, n_new=1000, millis_span=4, counter_span=3,
                         n_ranks=9, tomb_frac=0.1, dup_frac=0.001, force=[(23, 700, "dup")]), (1 << 20) + 9
    if kind == "send_overflow":
        return make_case(seed=144, R=6, per_cs=2000, n_local=3000, n_new=800, n_ranks=7,
                         c0=((WALL + 10) << 16) | 0xFFFE), (1 << 20) + 1
    if kind == "hot":                                  # every key in bucket 0: split into parts
        return make_case(seed=145, R=120, per_cs=2000, n_local=3000, n_new=1000, millis_span=4, counter_span=3,
                         n_ranks=9, tomb_frac=0.2, neg_mod_frac=0.05), (1 << 20) + 5
    if kind == "cold":
        case = _cold_bucket_case(146)
        return case, case["n_ids"]
    if kind == "one_level":                            # capacity <= 2^20: one partition level, 4-B kj
        return make_case(seed=147, R=50, per_cs=1500, n_local=2500, n_new=1500, millis_span=6, counter_span=3,
                         n_ranks=11, tomb_frac=0.1), None
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["edges", "late_drift", "dup", "send_overflow", "hot", "cold", "one_level"])
def test_sorted_packed_kinds(gpu_device, kind):
    """The packed sorted path with a declared rank bound on frame edges, exceptions raised in recv() (a
    late drift, a duplicate node) and in send(), split hot buckets, cold buckets and one partition level:
    rows, canonical, status and exception fields equal the oracle's."""
    case, cap = _kind_case(kind)
    bound = int(case["rank"].max()) + 1
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=cap, rank_bound=bound,
                              device_cols=True)
    assert res["path"] == "sorted" and res["plan"]["packed"], res["plan"]
    if kind in ("late_drift", "dup", "send_overflow"):
        assert res["status"] != 0, res


@pytest.mark.parametrize("tile", ["16384", "20480"])
@pytest.mark.parametrize("kind", ["edges", "cold", "late_drift"])
def test_sorted_odd_level1_tile(gpu_device, monkeypatch, tile, kind):
    """CRDT_L1_TILE other than the two sizes the scan counts (28672 / 14336) partitions on its
    own tile boundaries, so the scan's fused histogram must not be used — 20,000-record changesets give
    two level-1 tiles at 16384 as at 14336, on different boundaries.  Rows vs the oracle."""
    monkeypatch.setenv("CRDT_L1_TILE", tile)
    case, cap = _kind_case(kind)
    if kind == "edges":
        case = make_case(seed=149, R=70, per_cs=20_000, n_local=300_000, n_new=200_000, millis_span=6,
                         counter_span=3, n_ranks=11, tomb_frac=0.1)
        cap = max(case["n_ids"], (1 << 20) + 3)
    bound = int(case["rank"].max()) + 1
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=cap, rank_bound=bound,
                              device_cols=True)
    assert res["path"] == "sorted" and not res["plan"]["hist_in_scan"], res["plan"]


@pytest.mark.parametrize("L", [44, 45, 46, 47])
def test_sorted_key8_frame_boundary(gpu_device, L):
    """The 1-B key column needs 4 free bits above the packed key (L + K + J <= 60; L / K / J the lt /
    rank / changeset field widths, J = bitlen(min(R, 4096) + 1)): lt spans on both sides of that
    boundary, stretched downwards by old records (no clock effect) — key8 on / off as the frame
    says, same rows as the oracle."""
    R = 2000
    case = make_case(seed=98 + L, R=R, per_cs=60, n_local=2500, n_new=1500, millis_span=4,
                     counter_span=3, n_ranks=9, tomb_frac=0.1)
    rng = np.random.default_rng(L)
    lt = case["lt"].copy()
    hi = int(lt.max())
    pick = np.nonzero(rng.random(len(lt)) < 0.02)[0]
    lt[pick] = hi - rng.integers(0, 1 << (L - 1), len(pick))
    lt[pick[0]] = hi - ((1 << (L - 1)) + 5)                     # lt span has exactly L bits
    case["lt"] = lt
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=(1 << 20) + 17)
    assert res["path"] == "sorted" and res["plan"]["packed"], res["plan"]
    span = int(lt.max()) - int(lt.min())
    assert span.bit_length() == L
    K = (int(case["rank"].max()) - int(case["rank"].min()) + 1).bit_length()
    J = (min(R, 4096) + 1).bit_length()
    assert res["plan"]["key8"] == (L + K + J <= 60), (L, K, J, res["plan"])


@pytest.mark.parametrize("R", [1500, 3000])
def test_sorted_wide_frame_narrow_window(gpu_device, R):
    """A frame too wide for the full 13-bit changeset field (L + K + 13 > 64, L + K <= 54): the
    packed key narrows its window to the changesets that fit (>= 1022 per window, several windows
    per call) and stays packed — same rows as the oracle."""
    case = make_case(seed=77 + R, R=R, per_cs=50, n_local=3000, n_new=1000, millis_span=4,
                     counter_span=3, n_ranks=9, tomb_frac=0.1)
    rng = np.random.default_rng(R)
    lt = case["lt"].copy()
    hi = int(lt.max())
    pick = np.nonzero(rng.random(len(lt)) < 0.02)[0]
    lt[pick] = hi - rng.integers(0, 1 << 48, len(pick))
    lt[pick[0]] = hi - ((1 << 49) + 3)                          # L = 50
    case["lt"] = lt
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=(1 << 20) + 19)
    assert res["path"] == "sorted" and res["plan"]["packed"], res["plan"]


def test_sorted_wide_frame_takes_list_form(gpu_device):
    """Records whose lt span exceeds the packed key (old echoes near lt 0 beside current clocks):
    the packed kernels exit and the list form resolves the window — same rows as the oracle."""
    case = make_case(seed=93, R=30, per_cs=1500, n_local=2500, n_new=1500, millis_span=6, counter_span=3,
                     n_ranks=11, tomb_frac=0.1)
    rng = np.random.default_rng(93)
    old = rng.random(len(case["lt"])) < 0.05
    case["lt"] = np.where(old, rng.integers(1, 1 << 20, len(case["lt"])), case["lt"]).astype(np.int64)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=(1 << 20) + 9)
    assert res["path"] == "sorted" and not res["plan"]["packed"], res["plan"]


@pytest.mark.parametrize("packed", ["1", "0"])
def test_sorted_split_hot_bucket_packed(gpu_device, monkeypatch, packed):
    """The split-bucket parts of the packed form (k_resolve_packed<true> + k_part_carry_packed)
    against the list form's, on the hot-bucket case (4 parts, ties, tombstones)."""
    monkeypatch.setenv("CRDT_PACKED", packed)
    case = make_case(seed=85, R=120, per_cs=2000, n_local=3000, n_new=1000, millis_span=4, counter_span=3,
                     n_ranks=9, tomb_frac=0.2, neg_mod_frac=0.05)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False)
    assert res["path"] == "sorted"


@pytest.mark.parametrize("path", ["gather", "sorted"])
def test_key_out_of_range_stores_nothing(gpu_device, path):
    """A key id >= capacity in a device batch: CRDT_E_KEY_RANGE with no row stored and the
    canonical unchanged, on both store paths (the gather path checks ids before K2, the sorted
    path's resolve skips once its level-1 scatter saw one)."""
    import torch
    from crdt_amd import CrdtNativeError, DeviceTable
    case = make_case(seed=77, R=70, per_cs=1500, n_local=3000, n_new=1000, millis_span=4, counter_span=2,
                     n_ranks=5, tomb_frac=0.1)
    key = case["key"].copy()
    key[len(key) // 2] = case["n_ids"] + 5                      # capacity is n_ids
    t = DeviceTable(0, local_rank=case["local_rank"], capacity=case["n_ids"])
    t.set_merge_path(path)
    if path == "sorted":
        t.set_counts(False)
    loc = case["local"]
    keep = loc["mod"] != ABSENT_MOD
    ids = np.arange(case["n_local"], dtype=np.uint32)[keep]
    t.put_rows(ids, loc["lt"][keep], loc["rank"][keep], loc["val"][keep], loc["mod"][keep])
    t.canonical = case["c0"]
    before = t.read_rows(np.arange(case["n_ids"], dtype=np.uint32))
    cols = [torch.from_numpy(c).cuda() for c in (key, case["lt"], case["rank"], case["val"])]
    with pytest.raises(CrdtNativeError, match="key id out of range"):
        t.merge(*cols, case["offsets"], case["wall"], win_flags=False)
    assert t.last_path() == path
    after = t.read_rows(np.arange(case["n_ids"], dtype=np.uint32))
    for a, b in zip(before, after):
        assert np.array_equal(a, b)
    assert t.canonical == case["c0"]
    t.close()


@pytest.mark.parametrize("shift", [0, 1, 2, 3])
@pytest.mark.parametrize("where", ["first", "middle", "last"])
def test_gather_key_check_any_alignment(gpu_device, shift, where):
    """The gather path's up-front key check reads the keys 16 B at a time between scalar head and tail
    elements: a bad id in the head, the body or the tail of a key column starting at any 4-B offset
    from a 16-B boundary fails the merge with nothing stored; the same columns with good ids merge."""
    import torch
    from crdt_amd import CrdtNativeError, DeviceTable
    n, cap = 4103, 1 << 16
    rng = np.random.default_rng(shift * 7 + len(where))
    base = torch.from_numpy(rng.permutation(cap)[: n + shift].astype(np.int32)).cuda()
    key = base[shift:]                                          # data_ptr() at a 4 * shift offset
    assert key.data_ptr() % 16 == (base.data_ptr() + 4 * shift) % 16
    lt = torch.from_numpy(np.full(n, 5 << 16, np.int64)).cuda()
    rank = torch.ones(n, dtype=torch.int32, device="cuda")
    val = torch.zeros(n, dtype=torch.int32, device="cuda")
    offs = np.array([0, n], np.uint64)
    t = DeviceTable(0, local_rank=0, capacity=cap)
    t.set_merge_path("gather")
    t.canonical = 1 << 16
    res, _ = t.merge(key, lt, rank, val, offs, 1 << 40, win_flags=False)
    assert res["status"] == 0 and res["n_stored"] == 1 and res["n_won"] == n
    t.clear_rows(0, cap)
    i = {"first": 0, "middle": n // 2, "last": n - 1}[where]
    key[i] = cap + 1
    with pytest.raises(CrdtNativeError, match="key id out of range"):
        t.merge(key, lt, rank, val, offs, 1 << 40, win_flags=False)
    lt_r, _, _, mod = t.read_rows(np.arange(cap, dtype=np.uint32))
    assert (mod == ABSENT_MOD).all() or (lt_r == 0).all()
    t.close()


def test_sorted_key_out_of_range(gpu_device):
    from crdt_amd import CrdtNativeError, DeviceTable
    t = DeviceTable(0, local_rank=0, capacity=64)
    t.set_merge_path("sorted")
    with pytest.raises(CrdtNativeError):
        t.merge(np.array([1, 10_000], np.uint32), np.array([5, 6], np.int64), np.array([1, 1], np.uint32),
                np.array([0, 0], np.uint32), np.array([0, 2], np.uint64), 1 << 40, win_flags=False)
    assert t.last_path() == "sorted"


@pytest.mark.parametrize("K,total,R", [(1 << 20, 3_000_000, 64), (1 << 24, 8_000_000, 96)])
@pytest.mark.parametrize("counts", [True, False])
def test_sorted_equals_gather_fanin(gpu_device, K, total, R, counts):
    """Full-table property check at a fan-in shape (Zipf keys, unique per replica, hot head):
    both paths from the same state give the same rows, canonical and counts."""
    import torch

    from crdt_amd import DeviceTable
    from crdt_amd.workload import gen_fanin
    wl = gen_fanin(total=total, R=R, K=K, n_local=K // 2, s=0.8, device="cuda")
    own, loc = wl["owned"], wl["local"]
    out = {}
    for path in ("gather", "sorted"):
        t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
        t.set_merge_path(path)
        t.set_counts(counts)
        t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
        t.canonical = wl["c0"]
        res, _ = t.merge(own["key"], own["lt"], own["rank"], own["val"], wl["owned_offsets"], wl["wall"],
                         win_flags=False)
        assert t.last_path() == path
        rows = t.read_rows(np.arange(wl["capacity"], dtype=np.uint32))
        out[path] = (res, rows)
        t.close()
    (rg, ag), (rs, as_) = out["gather"], out["sorted"]
    for k in RESULT_FIELDS:
        if not counts and k in ("n_present", "n_won"):
            assert rs[k] == (1 << 64) - 1
            continue
        assert rg[k] == rs[k], (k, rg[k], rs[k])
    for a, b in zip(ag, as_):
        assert np.array_equal(a, b)
    torch.cuda.empty_cache()


@pytest.mark.parametrize("inject", [None, "drift", "dup"])
def test_streaming_deltas_one_ctx_vs_oracle(gpu_device, inject):
    """cfg5's shape at small scale on one context: one crdt_merge per delta, so from the second
    call on the scan takes its eager form (the previous call's tiles were mostly above C_0);
    every call's result and win flags, and the final rows, against the C oracle."""
    from crdt_amd import DeviceTable
    from crdt_amd.workload import gen_cfg5
    from oracle.oracle_c import OracleTable
    wl = gen_cfg5(device="cuda", K=200_000, n_delta=40_000, deltas=8, inject=inject, inject_at=(5, 39_000),
                  step_ms=1000)
    np_ = lambda t: t.cpu().numpy()  # noqa: E731
    own = {k: np_(v) for k, v in wl["owned"].items()}
    loc = {k: np_(v) for k, v in wl["local"].items()}
    t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
    o = OracleTable(wl["capacity"], 0, wl["c0"])
    t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
    o.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
    t.canonical = wl["c0"]
    offs = wl["owned_offsets"]
    for d in range(wl["R"]):
        b, e = int(offs[d]), int(offs[d + 1])
        cols = [own[k][b:e] for k in ("key", "lt", "rank", "val")]
        res, fl = t.merge(*cols, np.array([0, e - b], np.uint64), int(wl["walls"][d]))
        ores, ofl = o.merge(cols[0].astype(np.uint32), cols[1], cols[2].astype(np.uint32),
                            cols[3].astype(np.uint32), np.array([0, e - b], np.uint64), int(wl["walls"][d]))
        ores = ores.as_dict()
        for f in RESULT_FIELDS:
            assert res[f] == ores[f], (d, f, res[f], ores[f])
        assert np.array_equal(fl, ofl), d
        if res["status"] != 0:
            break
    lt, rank, val, mod = t.read_rows(np.arange(wl["capacity"], dtype=np.uint32))
    assert np.array_equal(lt, o.rows["lt"]) and np.array_equal(rank, o.rows["rank"])
    assert np.array_equal(val, o.rows["val"]) and np.array_equal(mod, o.rows["mod"])
    assert (res["status"] != 0) == (inject is not None)
    t.close()


def _with_empty_changesets(case, every=3):
    """Empty every changeset j with j % every != 0 (offsets repeat), keeping the rest as they were."""
    offs = case["offsets"].astype(np.int64)
    R = len(offs) - 1
    keep = [j for j in range(R) if j % every == 0]
    idx = np.concatenate([np.arange(offs[j], offs[j + 1]) for j in keep]) if keep else np.zeros(0, np.int64)
    new = [0]
    for j in range(R):
        new.append(new[-1] + (int(offs[j + 1] - offs[j]) if j % every == 0 else 0))
    for k in ("key", "lt", "rank", "val"):
        case[k] = case[k][idx]
    if case.get("millis") is not None:
        case["millis"] = case["millis"][idx]
    case["offsets"] = np.array(new, np.uint64)
    return case


@pytest.mark.parametrize("seed", range(3))
def test_interleaved_empty_changesets(gpu_device, seed):
    """Empty changesets between non-empty ones (zero tiles for them in the scan, the clock's
    W-only steps, K2 skipping them), with an exception after some of them."""
    case = make_case(seed=4200 + seed, R=30, per_cs=400, n_local=3000, n_new=1500, millis_span=30,
                     counter_span=3, n_ranks=7, local_rank=1,
                     force=[(21, 123, "drift")] if seed == 1 else [(27, 5, "dup")] if seed == 2 else [])
    compare_with_oracle(_with_empty_changesets(case))


def test_more_changesets_than_grid_rows(gpu_device):
    """R = 70,000 changesets (> 65,535: the scan's grid.y loops; > the fused clock's limit)."""
    compare_with_oracle(make_case(seed=4300, R=70_000, per_cs=2, n_local=300, n_new=200, millis_span=4000,
                                  counter_span=2, n_ranks=9))


@pytest.mark.parametrize("form_off", ["0", "2048"])
def test_high_water_mark_sequence(gpu_device, monkeypatch, form_off):
    """The table's high-water mark of written rows (crdt_ctx::hw: rows at or above it are the
    never-written fill, so the packed resolve synthesises them instead of reading them) across a
    sequence of stores: put_rows (host and device keys), sorted merges whose rows lie above the
    previous mark, clear_rows reaching the mark, a gather-path merge (mark -> capacity), put_stamped
    — every row and the canonical equal to the C oracle after each step; bit 2048 of
    CRDT_SORTED_FORM reads every row (the same results)."""
    import torch

    from crdt_amd import DeviceTable
    from oracle.oracle_c import OracleTable, new_table
    from tests._cases import WALL
    monkeypatch.setenv("CRDT_SORTED_FORM", form_off)
    cap, NR = (1 << 21) + 37, 9
    rng = np.random.default_rng(4242)
    c0 = (WALL - 5000) << 16
    t = DeviceTable(0, local_rank=0, capacity=cap)
    o = OracleTable(cap, 0, c0)
    t.canonical = c0
    t.set_rank_bound(NR)
    t.set_counts(False)

    def rows_equal(tag):
        lt, rk, val, mod = t.read_rows(np.arange(cap, dtype=np.uint32))
        for f, a in (("lt", lt), ("rank", rk), ("val", val), ("mod", mod)):
            assert np.array_equal(a, o.rows[f]), (tag, f, np.flatnonzero(a != o.rows[f])[:5])
        assert t.canonical == o.canonical, tag

    def put(keys, dev):
        n = len(keys)
        lt = ((WALL - 3000 + rng.integers(0, 64, n)) << 16) | rng.integers(0, 4, n)
        rk = rng.integers(0, NR, n).astype(np.uint32)
        val = rng.integers(0, 1 << 30, n).astype(np.uint32)
        mod = np.full(n, c0, np.int64)
        o.put_rows(keys, lt, rk, val, mod)
        cols = [keys.astype(np.uint32), lt.astype(np.int64), rk, val, mod]
        if dev:
            cols = [torch.from_numpy(c.view(np.int32) if c.dtype == np.uint32 else c).cuda() for c in cols]
        t.put_rows(*cols)

    def batch(R, per, hi):
        keys = [rng.choice(hi, per, replace=False).astype(np.uint32) for _ in range(R)]
        key = np.concatenate(keys)
        n = len(key)
        lt = ((WALL - 2000 + rng.integers(0, 64, n)) << 16) | rng.integers(0, 4, n)
        rk = rng.integers(1, NR, n).astype(np.uint32)
        val = rng.integers(0, 1 << 30, n).astype(np.uint32)
        offs = np.arange(R + 1, dtype=np.uint64) * per
        return key, lt.astype(np.int64), rk, val, offs

    def merge(b, path, dev=True, wall=WALL):
        key, lt, rk, val, offs = b
        t.set_merge_path(path)
        o.merge(key, lt, rk, val, offs, wall)
        cols = [key, lt, rk, val]
        if dev:
            cols = [torch.from_numpy(c.view(np.int32) if c.dtype == np.uint32 else c).cuda() for c in cols]
        res, _ = t.merge(*cols, offs, wall, win_flags=path == "gather")
        assert res["status"] == 0 and t.last_path() == path
        return t.last_plan()

    put(np.arange(3000, dtype=np.uint32), dev=True)                      # mark 3000
    plan = merge(batch(70, 3000, 1_200_000), "sorted")                   # rows up to ~1.2M written
    assert plan["packed"] and plan["high_water"] == (form_off == "0"), plan
    rows_equal("A")
    merge(batch(70, 3000, cap), "sorted")                                 # reads A's rows above 3000
    rows_equal("B")
    t.clear_rows(5000, cap - 5000)                                        # mark back to 5000
    o.rows[5000:] = new_table(cap - 5000)
    plan = merge(batch(66, 2500, cap), "sorted")
    assert plan["high_water"] == (form_off == "0"), plan
    rows_equal("C")
    merge(batch(3, 2000, cap), "gather", dev=False)                       # mark -> capacity
    plan = merge(batch(64, 2000, cap), "sorted")
    assert not plan["high_water"], plan
    rows_equal("D")
    t.clear_rows(0, cap)                                                  # mark 0
    o.rows[:] = new_table(cap)
    put(np.array([7, cap - 40, 1_500_000], np.uint32), dev=False)         # mark cap - 39
    merge(batch(64, 2000, cap), "sorted")
    rows_equal("E")
    t.clear_rows(0, cap)
    o.rows[:] = new_table(cap)
    key = np.array([11, 900_000], np.uint32)
    val = np.array([5, 6], np.uint32)
    r1 = t.put_stamped(key, val, WALL)                                    # mark 900,001
    o.put_stamped(key, val, WALL)
    assert r1["canonical_lt"] == o.canonical
    plan = merge(batch(64, 2000, cap), "sorted")
    assert plan["high_water"] == (form_off == "0"), plan
    rows_equal("F")
    t.close()


def test_high_water_mark_reserve_relayout_remap(gpu_device):
    """The high-water mark across crdt_reserve (new rows are fill above the mark), a relayout to
    32-B rows (the packed resolve then synthesises 32-B-stride fill rows) and crdt_remap_ranks:
    sorted merges after each equal the C oracle."""
    import torch

    from crdt_amd import DeviceTable
    from oracle.oracle_c import OracleTable, new_table
    from tests._cases import WALL
    NR = 7
    rng = np.random.default_rng(777)
    c0 = (WALL - 5000) << 16
    cap0, cap1 = (1 << 20) + 100, (1 << 21) + 3
    t = DeviceTable(0, local_rank=0, capacity=cap0)
    t.canonical = c0
    t.set_rank_bound(NR)
    t.set_counts(False)
    t.set_merge_path("sorted")
    o = OracleTable(cap1, 0, c0)

    def merge(hi, R=64, per=1500):
        keys = [rng.choice(hi, per, replace=False).astype(np.uint32) for _ in range(R)]
        key = np.concatenate(keys)
        n = len(key)
        lt = (((WALL - 2000 + rng.integers(0, 64, n)) << 16) | rng.integers(0, 4, n)).astype(np.int64)
        rk = rng.integers(1, NR, n).astype(np.uint32)
        val = rng.integers(0, 1 << 30, n).astype(np.uint32)
        offs = np.arange(R + 1, dtype=np.uint64) * per
        o.merge(key, lt, rk, val, offs, WALL)
        dev = [torch.from_numpy(c.view(np.int32) if c.dtype == np.uint32 else c).cuda() for c in (key, lt, rk, val)]
        res, _ = t.merge(*dev, offs, WALL, win_flags=False)
        assert res["status"] == 0 and t.last_path() == "sorted"
        return t.last_plan()

    def check(tag):
        n = min(t.capacity, cap1)                     # (reserve may grow past cap1: fill rows)
        lt, rk, val, mod = t.read_rows(np.arange(n, dtype=np.uint32))
        for f, a in (("lt", lt), ("rank", rk), ("val", val), ("mod", mod)):
            assert np.array_equal(a, o.rows[f][:n]), (tag, f)
        assert t.canonical == o.canonical, tag

    keys = np.arange(2000, dtype=np.uint32)
    lt = (((WALL - 3000 + rng.integers(0, 64, 2000)) << 16)).astype(np.int64)
    rk = rng.integers(0, NR, 2000).astype(np.uint32)
    val = rng.integers(0, 1 << 30, 2000).astype(np.uint32)
    mod = np.full(2000, c0, np.int64)
    t.put_rows(keys, lt, rk, val, mod)
    o.put_rows(keys, lt, rk, val, mod)
    assert merge(cap0)["high_water"]
    check("cap0")
    t.reserve(cap1)                                   # grown: rows [cap0, cap1) are fill
    assert t.capacity >= cap1
    assert merge(cap1)["two_level"]
    check("reserve")
    t.set_row_bytes(32)
    t.clear_rows(900_000, t.capacity - 900_000)
    o.rows[900_000:] = new_table(cap1 - 900_000)
    assert merge(cap1)["high_water"]
    check("32-B rows")
    lut = np.array([0, 2, 1, 4, 3, 6, 5], np.uint32)     # ranks permuted (a node id order change)
    t.remap_ranks(t.capacity, lut)
    r = o.rows["rank"]
    sel = r < len(lut)
    r[sel] = lut[r[sel]]
    merge(cap1)
    check("remap")
    t.close()


@pytest.mark.parametrize("form_off", ["0", "131072"])
def test_two_rank_routing_kernel_forms(gpu_device, monkeypatch, form_off):
    """The routing kernels in both forms (vector loads + wave-aggregated slots, and the strided
    one-atomic-per-record form, CRDT_SORTED_FORM bit 131072): 2 ranks over the gloo table, the
    packed wire into the sorted receivers and the 20-B wire into the gather path, vs the oracle."""
    monkeypatch.setenv("CRDT_SORTED_FORM", form_off)
    kw = dict(seed=83, R=70, per_cs=3000, n_local=30_000, n_new=20_000, millis_span=8, counter_span=4,
              n_ranks=71, tomb_frac=0.1)
    run_shard_gpu(kw, 2, "routed", path="sorted", counts=False)
    run_shard_gpu(dict(CASE_SPECS)["drift_late"], 2, "routed")


# ------------------------------------------------------------------ sorted path, flagged form
# Per-record win flags on the sorted path (sorted_path.inc, "win flags"): stable level 2, the
# ordered packed resolve, flags carried back to input order.  Every case against the oracle's
# flags, rows, canonical, exception fields and exact counts (crdt.dart:80-90, map_crdt.dart:33-39).
_TWO = (1 << 20) + 5


def _flagged(case, capacity=None, **kw):
    res = compare_with_oracle(case, path="sorted", flags=True, capacity=capacity, **kw)
    return res


@pytest.mark.parametrize("name", [n for n, _ in CASE_SPECS])
@pytest.mark.parametrize("capacity", [None, _TWO])
def test_flagged_golden_vectors(gpu_device, name, capacity):
    """Every golden case with flags on a forced sorted path: the flagged form whenever the batch's
    frame fits the packed key (else K2), same flags and counts as the golden outputs."""
    case, exp, expected = golden_case(name)
    rows, res, flags = device_run(case, path="sorted", flags=True, capacity=capacity)
    check_rows(*rows, exp)
    assert np.array_equal(flags, exp["flags"])
    for k, v in expected.items():
        assert res[k] == v, (name, k, res[k], v)
    if res["path"] == "sorted":
        assert res["plan"]["flagged"]


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("capacity", [None, _TWO])
def test_flagged_random_small(gpu_device, seed, capacity):
    rng = np.random.default_rng(1000 + seed)
    kw = dict(seed=2000 + seed, R=int(rng.integers(1, 12)), per_cs=int(rng.integers(0, 500)),
              n_local=int(rng.integers(1, 600)), n_new=int(rng.integers(0, 400)),
              millis_span=int(rng.integers(1, 100)), counter_span=int(rng.integers(1, 8)),
              n_ranks=int(rng.integers(2, 40)), tomb_frac=float(rng.random() * 0.5),
              neg_mod_frac=float(rng.random() * 0.1), dup_frac=float(rng.random() * 0.01),
              drift_frac=float(rng.random() * 0.005))
    kw["local_rank"] = int(rng.integers(0, kw["n_ranks"]))
    case = make_case(**kw)
    res = _flagged(case, capacity)
    if case["c0"] >= 0:
        assert res["path"] == "sorted" and res["plan"]["flagged"], res["plan"]


@pytest.mark.parametrize("capacity", [None, (1 << 20) + 7, 1 << 24])
def test_flagged_ties_many_changesets(gpu_device, capacity):
    """300 tie-heavy changesets: equal (lt, rank) across changesets (the earlier one wins, later
    equal records do not), one- and two-level buckets."""
    case = make_case(seed=79, R=300, per_cs=2000, n_local=40_000, n_new=20_000, millis_span=8,
                     counter_span=4, n_ranks=301)
    res = _flagged(case, capacity)
    assert res["path"] == "sorted" and res["plan"]["flagged"] and res["n_won"] > 0


@pytest.mark.parametrize("capacity", [None, _TWO])
def test_flagged_hot_keys_in_one_chunk(gpu_device, capacity):
    """Dozens of records per key in every 2048-record chunk: long in-chunk same-key lists, the
    left-to-right maxima decided inside the chunk."""
    case = make_case(seed=83, R=400, per_cs=60, n_local=50, n_new=30, millis_span=3, counter_span=2,
                     n_ranks=7)
    res = _flagged(case, capacity)
    assert res["path"] == "sorted" and res["plan"]["flagged"]


@pytest.mark.parametrize("capacity", [None, _TWO])
def test_flagged_split_hot_bucket(gpu_device, capacity):
    """240K records in one 4096-key bucket: 4 parts (changeset ranges), each walked from its
    carry-in (row folded with the earlier parts); ties and tombstones across the cuts."""
    case = make_case(seed=85, R=120, per_cs=2000, n_local=3000, n_new=1000, millis_span=4, counter_span=3,
                     n_ranks=9, tomb_frac=0.2, neg_mod_frac=0.05)
    res = _flagged(case, capacity)
    assert res["path"] == "sorted" and res["plan"]["flagged"] and res["n_won"] > 0


def test_flagged_split_buckets_across_blocks(gpu_device):
    buckets = [3, 1023, 1024, 2047, 2048, 4095]
    base = make_case(seed=86, R=40, per_cs=12_000, n_local=18_000, n_new=6 * 4096 - 18_000, millis_span=4,
                     counter_span=3, n_ranks=9, tomb_frac=0.2, neg_mod_frac=0.05)
    case = _spread_case(base, buckets, 1 << 24)
    res = _flagged(case)
    assert res["path"] == "sorted" and res["plan"]["flagged"] and res["n_won"] > 0


def test_flagged_windows_and_late_exception(gpu_device):
    """5000 changesets (two windows), a drift record in changeset 4500: the flags of changesets
    from the stop on stay 0."""
    case = make_case(seed=84, R=5000, per_cs=20, n_local=3000, n_new=2000, millis_span=20,
                     force=[(4500, 7, "drift")])
    res = _flagged(case)
    assert res["status"] == 1 and res["exc_changeset"] == 4500 and res["path"] == "sorted"


@pytest.mark.parametrize("seed", [91, 92])
def test_flagged_frame_edges(gpu_device, seed):
    """Local rows at every edge of the packed frame (below / at / above, ranks outside it, equal
    (lt, rank) with a record), with and without a declared rank bound."""
    case = _frame_edge_case(seed)
    bound = int(case["rank"].max()) + 1
    for cap in (None, (1 << 20) + 3):
        for rb in (0, bound):
            res = _flagged(case, cap, rank_bound=rb)
            assert res["path"] == "sorted" and res["plan"]["flagged"]


@pytest.mark.parametrize("cap", [None, _TWO])
def test_flagged_late_drift(gpu_device, cap):
    case = _late_drift_case(97)
    res = _flagged(case, cap)
    assert res["status"] == 1 and res["exc_changeset"] == 37 and res["plan"]["flagged"]


@pytest.mark.parametrize("counts", [True, False])
def test_flagged_cold_buckets(gpu_device, counts):
    """Records spread thinly over many cold buckets of a > 2^20-key table (unsplit buckets at
    level 2, 14/13-B records), counts on and off (the flagged form always counts)."""
    case = _cold_bucket_case(95)
    rows, res, flags = device_run(case, path="sorted", flags=True, counts=counts, capacity=case["n_ids"])
    orows, ores, oflags = oracle_run(case)
    assert res["plan"]["flagged"] and res["plan"]["key16"]
    assert np.array_equal(flags, oflags)
    for f, a in zip(("lt", "rank", "val", "mod"), rows):
        assert np.array_equal(a, orows[f]), f
    for k in RESULT_FIELDS:
        assert res[k] == ores[k], (k, res[k], ores[k])


def test_flagged_device_columns(gpu_device):
    case = make_case(seed=88, R=90, per_cs=3000, n_local=9000, n_new=4000, millis_span=6, counter_span=3,
                     n_ranks=11, tomb_frac=0.1)
    res = compare_with_oracle(case, path="sorted", flags=True, capacity=_TWO, device_cols=True)
    assert res["plan"]["flagged"]


def test_flagged_key_out_of_range(gpu_device):
    """A key id past the capacity: CRDT_E_KEY_RANGE, nothing stored, every flag 0."""
    from crdt_amd import CrdtNativeError, DeviceTable
    t = DeviceTable(0, local_rank=0, capacity=64)
    t.set_merge_path("sorted")
    with pytest.raises(CrdtNativeError):
        t.merge(np.array([1, 10_000], np.uint32), np.array([5, 6], np.int64), np.array([1, 1], np.uint32),
                np.array([0, 0], np.uint32), np.array([0, 2], np.uint64), 1 << 40, win_flags=True)
    lt, rank, val, mod = t.read_rows(np.arange(64, dtype=np.uint32))
    assert (mod < 0).all()
    t.close()


def test_flagged_switch_off(gpu_device, monkeypatch):
    """CRDT_FLAGS_SORTED=0: a flagged merge takes K2, same results."""
    monkeypatch.setenv("CRDT_FLAGS_SORTED", "0")
    case = make_case(seed=89, R=70, per_cs=1000, n_local=3000, n_new=1000, millis_span=5)
    res = _flagged(case)
    assert res["path"] == "gather" and not res["plan"]["flagged"]


@pytest.mark.parametrize("chk,form", [("0", "134217728"), ("4", "134217728"), ("6", "134217728"), ("6", "0"),
                                      ("6", "4194304"), ("6", "2097152"), ("6", "8388608"), ("6", "14680064"),
                                      ("6", "536870912"), ("6", "268435456"), ("6", "2147483648")])
def test_flagged_back_pass_search_forms(gpu_device, monkeypatch, chk, form):
    """The flag passes: round 5's one-byte staging (CRDT_SORTED_FORM bit 134217728) with its run search without
    checkpoints (CRDT_FBACK_CHK=0), one per 16 staged bytes (4) and one per 64 (6); the default k_flags_back_pre
    (positions loaded first, one checkpoint per 64 staged bytes); the opt-in forms of CRDT_SORTED_FORM: four-byte
    staging with eight-record gathers (4194304), the scatters' XCD tile order (2097152), the split buckets' fold
    and carry-ins on a side stream beside the unsplit buckets' walk (8388608), all three (14680064);
    k_flags_back_pre's level-2 pass in 512-thread workgroups (536870912); the fold and walk over every item slot
    (268435456); the level-1 positions at the input index, not tile-strided (2147483648): split hot bucket, cold
    buckets on the 2-B level-1 key column, a late drift — same flags, rows and counts as the
    oracle."""
    monkeypatch.setenv("CRDT_FBACK_CHK", chk)
    monkeypatch.setenv("CRDT_SORTED_FORM", form)
    case = make_case(seed=85, R=120, per_cs=2000, n_local=3000, n_new=1000, millis_span=4, counter_span=3,
                     n_ranks=9, tomb_frac=0.2, neg_mod_frac=0.05)
    assert _flagged(case, _TWO)["plan"]["flagged"]
    cold = _cold_bucket_case(95)
    rows, res, flags = device_run(cold, path="sorted", flags=True, capacity=cold["n_ids"])
    orows, ores, oflags = oracle_run(cold)
    assert res["plan"]["flagged"] and res["plan"]["key16"] and np.array_equal(flags, oflags)
    for f, a in zip(("lt", "rank", "val", "mod"), rows):
        assert np.array_equal(a, orows[f]), f
    res = _flagged(_late_drift_case(97), _TWO)
    assert res["status"] == 1 and res["plan"]["flagged"]


@pytest.mark.parametrize("K,total,R", [(1 << 20, 3_000_000, 64), (1 << 24, 9_000_000, 96)])
def test_flagged_equals_gather_fanin(gpu_device, K, total, R):
    """A fan-in shape (Zipf keys, unique per replica, hot head split into parts) merged with flags on
    both paths from the same state (auto picks the flagged form): same flags, rows, canonical, counts."""
    import torch

    from crdt_amd import DeviceTable
    from crdt_amd.workload import gen_fanin
    wl = gen_fanin(total=total, R=R, K=K, n_local=K // 2, s=0.8, device="cuda")
    own, loc = wl["owned"], wl["local"]
    out = {}
    auto = total >= (8 << 20)                  # auto takes the flagged form from 64 changesets / 8M records
    for path in ("gather", None):
        t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
        if path or not auto:
            t.set_merge_path(path or "sorted")
        t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
        t.canonical = wl["c0"]
        res, fl = t.merge(own["key"], own["lt"], own["rank"], own["val"], wl["owned_offsets"], wl["wall"],
                          win_flags=True)
        assert t.last_path() == (path or "sorted")
        if not path:
            assert t.last_plan()["flagged"]
        rows = t.read_rows(np.arange(wl["capacity"], dtype=np.uint32))
        out[path] = (res, fl.cpu().numpy(), rows)
        t.close()
    (rg, fg, ag), (rs, fs, as_) = out["gather"], out[None]
    for k in RESULT_FIELDS:
        assert rg[k] == rs[k], (k, rg[k], rs[k])
    assert np.array_equal(fg, fs)
    for a, b in zip(ag, as_):
        assert np.array_equal(a, b)
    torch.cuda.empty_cache()


# ---- the compact form (round 6; sorted_path.inc PackFrame::cb, CRDT_PLAN_COMPACT) --------------------------
def _compact_edge_case(seed, cmax=14, wall=None, explicit_millis=False, millis_span=6):
    """Records whose lt & 0xFFFF reach cmax (14: cb = 4, the top field value 15 reserved), local rows at every
    edge of the compact lt field: counters cmax, cmax + 1 (= the reserved top), cmax + 2 and 0xFFFF at millis
    inside the frame (packed as the top: above every record of their millis, below the next), rows just below /
    above the frame, exact copies of records (equal (lt, rank): local keeps)."""
    from tests._cases import WALL
    case = make_case(seed=seed, R=48, per_cs=2500, n_local=4000, n_new=1500, millis_span=millis_span,
                     counter_span=cmax + 1, base=(WALL if wall is None else wall) - millis_span - 1000,
                     n_ranks=9, local_rank=0, tomb_frac=0.2, wall=WALL if wall is None else wall,
                     explicit_millis=explicit_millis)
    rng = np.random.default_rng(seed)
    lo, hi = int(case["lt"].min()), int(case["lt"].max())
    loc = case["local"]
    n = case["n_local"]
    ms = rng.integers(lo >> 16, (hi >> 16) + 1, n)
    cnt = np.array([0, cmax, cmax + 1, cmax + 2, 0xFFFF], np.int64)[rng.integers(0, 5, n)]
    lt = (ms << 16) + cnt
    edge = rng.random(n)
    lt = np.where(edge < 0.05, lo - 1, np.where(edge > 0.95, hi + 1, lt))
    loc["lt"] = lt.astype(np.int64)
    first = {}
    for x, k in enumerate(case["key"].tolist()):
        first.setdefault(k, x)
    for k in rng.choice(n, n // 10, replace=False):
        if int(k) in first:
            loc["lt"][k] = case["lt"][first[int(k)]]
            loc["rank"][k] = case["rank"][first[int(k)]]
    loc["mod"] = np.where(loc["mod"] >= 0, loc["lt"], loc["mod"])
    vis = loc["mod"] >= 0
    case["c0"] = int(loc["lt"][vis].max())
    return case


@pytest.mark.parametrize("form", ["0", "1048576"])
@pytest.mark.parametrize("variant", ["cmax14", "cmax0", "cmax200", "wide_span", "explicit_millis", "no_fit"])
def test_sorted_compact_form(gpu_device, monkeypatch, form, variant):
    """The compact lt field (CRDT_SORTED_FORM 1048576 switches it off: the 14-B / 13-B records): the same rows,
    canonical and exception fields as the oracle on two-level tables, with local rows at every edge of the
    compact field; and the plan reports which form ran."""
    monkeypatch.setenv("CRDT_SORTED_FORM", form)
    kw = {"cmax14": {}, "cmax0": {"cmax": 0}, "cmax200": {"cmax": 200},
          "wide_span": {"millis_span": 1 << 20}, "explicit_millis": {"explicit_millis": True},
          "no_fit": {"millis_span": 1 << 20, "cmax": 60000}}[variant]     # (no_fit: 20 + 16 bits: the plain field)
    case = _compact_edge_case(77, **kw)
    res = compare_with_oracle(case, path="sorted", flags=False, counts=False, capacity=(1 << 20) + 3,
                              rank_bound=int(case["rank"].max()) + 1, device_cols=True)
    assert res["plan"]["packed"] and res["plan"]["two_level"]
    assert res["plan"]["compact"] == (form == "0" and variant != "no_fit"), res["plan"]


def test_sorted_compact_fanin_equals_oracle(gpu_device):
    """A fan-in shape (gen_fanin: 2^16 ms of clocks, counters < 16 — the bench's) takes the compact form and
    leaves exactly the C oracle's rows; switched off, the same rows."""
    import os

    from crdt_amd import DeviceTable
    from crdt_amd.workload import gen_fanin
    K, total, R = 1 << 22, 3_000_000, 64
    ref, rows = _fanin_reference(K, total, R)
    wl = gen_fanin(total=total, R=R, K=K, n_local=K // 2, s=0.8, device="cuda")
    loc, own = wl["local"], wl["owned"]
    for form in ("0", "1048576"):
        os.environ["CRDT_SORTED_FORM"] = form
        try:
            t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
            t.set_counts(False)
            t.set_merge_path("sorted")
            t.set_rank_bound(R + 1)
            t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
            t.canonical = wl["c0"]
            res, _ = t.merge(own["key"], own["lt"], own["rank"], own["val"], wl["owned_offsets"], wl["wall"],
                             win_flags=False)
            assert t.last_plan()["compact"] == (form == "0"), t.last_plan()
            for f in ("status", "n_stored", "canonical_lt"):
                assert res[f] == ref[f], (form, f)
            for a, b in zip(t.read_rows(np.arange(wl["capacity"], dtype=np.uint32)), rows):
                assert np.array_equal(a, b), form
            t.close()
        finally:
            os.environ.pop("CRDT_SORTED_FORM", None)


@pytest.mark.parametrize("seed", range(48))
def test_random_sweep_sorted_forms(gpu_device, seed):
    """Randomised sweep over the sorted path's round-6 forms at their defaults — compact keys, the step-major scan
    grid, per-kernel item lists, sparse buckets in k_resolve_sparse, and (odd seeds) the flagged form with
    k_flags_back_pre and tile-strided level-1 positions: random table sizes (one or two levels), changeset counts
    and sizes, clock spans (ties to wide frames), node ranks, tombstones, invisible rows, duplicate-node and drift
    records, explicit millis columns — every row, flag and exception field equal to the C oracle's."""
    rng = np.random.default_rng(7000 + seed)
    n_ids = int(rng.integers(2000, 200_000 if seed < 32 else 1_500_000))
    n_local = int(n_ids * rng.uniform(0.3, 0.95))
    kw = dict(seed=8000 + seed, R=int(rng.integers(1, 48)), per_cs=int(rng.integers(100, 20_000 if seed < 32 else 150_000)),
              n_local=n_local, n_new=n_ids - n_local, millis_span=int(rng.choice([1, 8, 300, 70_000])),
              counter_span=int(rng.integers(1, 6)), n_ranks=int(rng.integers(2, 60)),
              tomb_frac=float(rng.choice([0.0, 0.2])), neg_mod_frac=float(rng.choice([0.0, 0.05])),
              dup_frac=float(rng.choice([0.0, 0.0005])), drift_frac=float(rng.choice([0.0, 0.0005])),
              explicit_millis=bool(rng.random() < 0.2))
    kw["local_rank"] = int(rng.integers(0, kw["n_ranks"]))
    case = make_case(**kw)
    flagged = bool(seed % 2)
    capacity = max(n_ids, (1 << 20) + 3) if seed % 3 == 0 else n_ids
    res = compare_with_oracle(case, path="sorted", flags=flagged, counts=flagged, capacity=capacity,
                              rank_bound=int(case["rank"].max()) + 1 if len(case["rank"]) else 0, device_cols=True)
    assert res["path"] == "sorted"
