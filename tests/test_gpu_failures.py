"""A rank's local failure inside a collective (sharded) merge fails every rank alike — no rank is left
blocked in a collective its peers will not post (comm_path.inc, "failures agreed over the ranks";
VERDICT r4 item 1).  CRDT_TEST_FAIL="rank:point" makes one rank fail with CRDT_E_NOMEM at a point of the
call: 1 before the gather (staging / the scan), 2 route_l1's preparation (before its count exchange), 3 the
receive area (before the record exchange), 4 the owners' apply (after the exchange), 5 the map-side
combine's home fold.  Every rank must return CRDT_E_NOMEM within the test's timeout, and the same ctxs must
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


def _fail_worker(rank, world, port, q, K, total, R, route, point, fail_rank):
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
            t.clear_rows(0, wl["capacity"])
            t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
            t.canonical = wl["c0"]
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


def _run(world, K, total, R, route, point, fail_rank):
    import torch.multiprocessing as mp

    from tests.test_dist_cpu import _free_port
    from tests.test_gpu_parity import _fanin_reference
    ref, rows = _fanin_reference(K, total, R)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, q, K, total, R, route, point, fail_rank))
             for r in range(world)]
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
