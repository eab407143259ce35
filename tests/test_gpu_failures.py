"""A rank's local failure inside a collective (sharded) merge fails every rank alike — no rank is left
blocked in a collective its peers will not post (comm_path.inc, "failures agreed over the ranks";
VERDICT r4 item 1).  CRDT_TEST_FAIL="rank:point" makes one rank fail with CRDT_E_NOMEM at a point of the
call: 1 before the gather (staging / the scan), 2 route_l1's preparation (before its count exchange), 3 the
receive area (before the record exchange), 4 the owners' buffers (route_l1: before the record exchange) or
apply (the other ways: after the exchange), 5 the map-side combine's home fold, 6 the owners' apply after the
last exchange (route_l1: its final owner launch).  Every rank must return CRDT_E_NOMEM within the test's timeout, and the same ctxs must
then merge the whole job exactly (rows equal to the C oracle's unsharded merge)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NOMEM = -3
ROUTES = {                      # CRDT_COMBINE, CRDT_ROUTE_L1 (the routing tuner off: the fixed way)
    "route_l1": ("0", "1"),
    "route_l1_head": ("0", "2"),            # with the head fold (its own count exchange after the pieces)
    "route_l1_all": ("0", "3"),             # ... folding every level-1 digit
    "combine": ("2", "1"),
    "records": ("0", "0"),
}


def _fail_worker(rank, world, port, q, K, total, R, route, point, fail_rank, remerge=False):
    import os

    import torch
    import torch.distributed as dist

    from crdt_amd import DeviceTable
    from crdt_amd.device import CrdtNativeError
    from crdt_amd.dist import GlooComm
    from crdt_amd.workload import gen_fanin
    comb, rl1 = ROUTES[route]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CRDT_ENV_DYNAMIC="1", CRDT_ROUTE_TUNE="0",
                      CRDT_COMBINE=comb, CRDT_ROUTE_L1=rl1, CRDT_RL1_SPLIT="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wl = gen_fanin(total=total, R=R, K=K, n_local=K // 2, s=0.8, device="cuda", rank=rank, world=world,
                       route=True)
        t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
        t.set_counts(False)
        t.set_merge_path("sorted")
        loc, home = wl["local"], wl["home"]
        t.comm_init_ops(world, rank, GlooComm(dist))
        out = []
        for inject in (True, False):
            os.environ["CRDT_TEST_FAIL"] = f"{fail_rank}:{point}" if inject else "-1:0"
            if inject or not remerge:
                t.clear_rows(0, wl["capacity"])
                t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
                t.canonical = wl["c0"]
            else:                                   # re-merge on top of the stopped call: its canonical stood
                assert t.canonical == wl["c0"], (t.canonical, wl["c0"])
            try:
                res, _ = t.merge(home["key"], home["lt"], home["rank"], home["val"], wl["home_offsets"], wl["wall"],
                                 win_flags=False)
                st = res["status"]
            except CrdtNativeError as e:
                st, res = e.status, None
            out.append((st, res, t.last_plan()))
        rows = t.read_rows(np.arange(wl["capacity"], dtype=np.uint32))
        q.put((rank, out, rows))
        t.close()
        torch.cuda.empty_cache()
    finally:
        dist.destroy_process_group()


def _run(world, K, total, R, route, point, fail_rank, remerge=False):
    import torch.multiprocessing as mp

    from tests.test_dist_cpu import _free_port
    from tests.test_gpu_parity import _fanin_reference
    ref, rows = _fanin_reference(K, total, R)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, q, K, total, R, route, point, fail_rank,
                                                    remerge)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted([q.get(timeout=240) for _ in range(world)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ((st_fail, _, _), (st_ok, res, plan)), shard in outs:
        assert st_fail == NOMEM, (rank, route, point, st_fail)           # every rank, not only the failing one
        assert st_ok == 0, (rank, st_ok)
        if route.startswith("route_l1"):
            assert plan["route_l1"] and plan["rl1_head"] == (route != "route_l1"), plan
        if route == "combine":
            assert plan["combined"], plan
        for f in ("status", "n_stored", "canonical_lt", "exc_changeset"):
            assert res[f] == ref[f], (rank, f)
        for a, b in zip(shard, rows):
            assert np.array_equal(a, b[rank::world]), rank


@pytest.mark.parametrize("route,point", [("route_l1", 1), ("route_l1", 2), ("route_l1", 3), ("route_l1", 4),
                                         ("route_l1_head", 3), ("route_l1_head", 4), ("route_l1_all", 4),
                                         ("combine", 1), ("combine", 5), ("combine", 3), ("combine", 4),
                                         ("records", 1), ("records", 3), ("records", 4)])
@pytest.mark.parametrize("fail_rank", [0, 1])
def test_two_rank_injected_failure(gpu_device, route, point, fail_rank):
    _run(2, 1 << 22, 2_000_000, 64, route, point, fail_rank)


@pytest.mark.parametrize("route,point", [("route_l1", 1), ("route_l1", 2), ("route_l1", 3), ("route_l1", 4),
                                         ("route_l1_head", 4), ("records", 3)])
def test_eight_rank_injected_failure(gpu_device, route, point):
    """Eight ranks on one GPU (K = 2^24: shards of 2^21 slots, two level-1 digits per owner), rank 5 fails."""
    _run(8, 1 << 24, 4_000_000, 64, route, point, 5)


# ---- point 6: route_l1's owners' apply after the last exchange ------------------------------------
@pytest.mark.parametrize("route", ["route_l1", "route_l1_head"])
@pytest.mark.parametrize("fail_rank", [0, 1])
def test_two_rank_failure_after_last_exchange(gpu_device, route, fail_rank):
    """CRDT_TEST_FAIL point 6: the failing rank skips its final owner launch AFTER every exchange (route_l1 and
    its head fold): every rank returns CRDT_E_NOMEM, the canonical does not move, and the same batch merged
    again on top of the stopped call's rows (no reset) gives the oracle's rows exactly."""
    _run(2, 1 << 22, 2_000_000, 64, route, 6, fail_rank, remerge=True)


# ---- the call's deadline: a stalled or lost peer ------------------------------------------
STALL_S = 6.0                   # the stalled rank sleeps this long at its point
DEADLINE_MS = 2000              # every rank's deadline (crdt_set_comm_timeout; GlooComm bounds each op by it)
COMM = -6


def _stall_worker(rank, world, port, q, K, total, R, route, stall):
    import datetime
    import os
    import time

    import torch.distributed as dist

    from crdt_amd import DeviceTable
    from crdt_amd.device import CrdtNativeError
    from crdt_amd.dist import GlooComm
    from crdt_amd.workload import gen_fanin
    comb, rl1 = ROUTES[route]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CRDT_ENV_DYNAMIC="1", CRDT_ROUTE_TUNE="0",
                      CRDT_COMBINE=comb, CRDT_ROUTE_L1=rl1, CRDT_RL1_SPLIT="1", CRDT_TEST_STALL=stall)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))
    wl = gen_fanin(total=total, R=R, K=K, n_local=K // 2, s=0.8, device="cuda", rank=rank, world=world, route=True)
    t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
    t.set_counts(False)
    t.set_merge_path("sorted")
    loc, home = wl["local"], wl["home"]
    t.comm_init_ops(world, rank, GlooComm(dist))
    t.set_comm_timeout(DEADLINE_MS)
    t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
    t.canonical = wl["c0"]
    dist.barrier()                                   # every rank enters the call together
    out = []
    for _ in range(2):                               # the call, then one more on the aborted ctx
        t0 = time.monotonic()
        try:
            res, _ = t.merge(home["key"], home["lt"], home["rank"], home["val"], wl["home_offsets"], wl["wall"],
                             win_flags=False)
            st = res["status"]
        except CrdtNativeError as e:
            st = e.status
        out.append((st, time.monotonic() - t0, t.comm_state()))
    q.put((rank, out))
    q.close()
    q.join_thread()
    os._exit(0)                                      # (the process group lost a peer: no orderly teardown)


def _run_stall(world, route, point, stall_rank, exit_=False):
    import time

    import torch.multiprocessing as mp

    from tests.test_dist_cpu import _free_port
    stall = f"{stall_rank}:{point}:{-1 if exit_ else int(STALL_S * 1e3)}"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    K, total, R = (1 << 22, 2_000_000, 64) if world == 2 else (1 << 24, 4_000_000, 64)
    procs = [ctx.Process(target=_stall_worker, args=(r, world, port, q, K, total, R, route, stall))
             for r in range(world)]
    for p in procs:
        p.start()
    n_out = world - 1 if exit_ else world
    t0 = time.monotonic()
    outs = sorted([q.get(timeout=240) for _ in range(n_out)], key=lambda o: o[0])
    for p in procs:
        p.join(timeout=60)
    for r, p in enumerate(procs):
        assert p.exitcode == (17 if exit_ and r == stall_rank else 0), (r, p.exitcode)
    assert len(outs) == n_out and time.monotonic() - t0 < 200
    for rank, ((st, el, (state, phase)), (st2, el2, _)) in outs:
        assert st == COMM, (rank, st, phase)                 # every rank: CRDT_E_COMM, none left waiting
        assert state in (1, 2), (rank, state)
        assert phase == "aborted", (rank, phase)
        assert st2 == COMM and el2 < 1.0, (rank, st2, el2)   # the aborted ctx refuses at once
        if rank != stall_rank:
            # a survivor ended at its deadline (or at the transport's error), not when the stalled peer woke
            assert el < STALL_S - 1.0 if not exit_ else el < 20.0, (rank, el)
        else:
            assert el < STALL_S + 20.0, (rank, el)


@pytest.mark.parametrize("point", [1, 2, 3])
def test_two_rank_stalled_peer_deadline(gpu_device, point):
    """Rank 1 stalls 6 s at the gather (1), route_l1's count exchange (2) or before the record exchange (3):
    rank 0 returns CRDT_E_COMM at its 2-s deadline, rank 1 when it wakes; both ctxs refuse the next call."""
    _run_stall(2, "route_l1", point, 1)


@pytest.mark.parametrize("point", [1, 2, 3])
def test_eight_rank_stalled_peer_deadline(gpu_device, point):
    _run_stall(8, "route_l1", point, 5)


@pytest.mark.parametrize("world,point", [(2, 1), (2, 3), (8, 3)])
def test_lost_peer_mid_call(gpu_device, world, point):
    """A rank that exits mid-call (CRDT_TEST_STALL ms < 0: _exit(17) at the point): the survivors return
    CRDT_E_COMM within the deadline instead of waiting forever."""
    _run_stall(world, "route_l1", point, world - 1, exit_=True)


def _rccl_abort_worker(q, K, total, R):
    import os
    import time

    from crdt_amd import DeviceTable
    from crdt_amd.device import CrdtNativeError
    from crdt_amd.workload import gen_fanin
    os.environ.update(CRDT_ENV_DYNAMIC="1", CRDT_TEST_STALL="-1:0:0")    # (switches re-read at every merge)
    wl = gen_fanin(total=total, R=R, K=K, n_local=K // 2, s=0.8, device="cuda")
    t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
    t.set_counts(False)
    loc, own = wl["local"], wl["owned"]

    def merge():
        t.clear_rows(0, wl["capacity"])
        t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
        t.canonical = wl["c0"]
        t0 = time.monotonic()
        try:
            res, _ = t.merge(own["key"], own["lt"], own["rank"], own["val"], wl["owned_offsets"], wl["wall"],
                             win_flags=False)
            st = res["status"]
        except CrdtNativeError as e:
            st = e.status
        return st, time.monotonic() - t0
    out = {}
    t.comm_init_rccl(1, 0, t.comm_unique_id())
    t.set_comm_timeout(1500)
    os.environ["CRDT_TEST_STALL"] = "0:5:4000:d"             # a 4-s device spin behind the final reduction
    out["stalled"] = merge() + (t.comm_state(),)
    os.environ["CRDT_TEST_STALL"] = "-1:0:0"
    out["refused"] = merge()
    t.comm_free()                                            # join a fresh communicator: exact again
    t.comm_init_rccl(1, 0, t.comm_unique_id())
    out["rejoined"] = merge() + (t.comm_state(),)
    out["rows"] = t.read_rows(np.arange(wl["capacity"], dtype=np.uint32))
    q.put(out)
    t.close()


def test_rccl_deadline_abort_single_rank(gpu_device):
    """RCCL's abort path on one rank: a device spin (bounded, 4 s) queued behind the final reduction holds the
    call past its 1.5-s deadline — the host's poll aborts the communicator (nothing of RCCL in flight), the
    call returns CRDT_E_COMM once the stream drained, the ctx refuses the next call, and after crdt_comm_free +
    a new crdt_comm_init_rccl the same merge gives the C oracle's rows."""
    import torch.multiprocessing as mp

    from tests.test_gpu_parity import _fanin_reference
    K, total, R = 1 << 22, 2_000_000, 64
    ref, rows = _fanin_reference(K, total, R)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_abort_worker, args=(q, K, total, R))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    st, el, (state, phase) = out["stalled"]
    assert st == COMM and state == 1 and phase == "aborted", out["stalled"]
    assert 1.4 < el < 15.0, el
    assert out["refused"][0] == COMM and out["refused"][1] < 1.0, out["refused"]
    st, _, (state, _) = out["rejoined"]
    assert st == 0 and state == 0, out["rejoined"]
    for a, b in zip(out["rows"], rows):
        assert np.array_equal(a, b)
