"""One rank's local work in config 4's routed merge, measured on ONE GPU (tools/gpu_r4.sh STAGE=probe).

Rank 0 of an N-rank routed fan-in (gen_fanin(route=True): replica j whole on rank j % N, a shard table of
2^28 / N slots holding rank 0's share of the local map) merges on a ctx joined to a LOOPBACK communicator:
every collective behaves as if all N ranks held rank 0's data — the all-gather repeats rank 0's row, the
reductions leave its words, and the all-to-all hands back, from each peer d, a device copy of exactly the
bytes rank 0 sends to d (on the ctx stream, timed with HIP events: the stand-in for the xGMI exchange, of
the same size as the real one).  Rank 0 thus applies its own part plus, as its "received" records, the
parts it routes to the peers (valid slots of the same distribution): the per-rank volume of the real run.

Modes, alternated in one process (same placement): route_l1 (home records partitioned straight into the
owners' level-1 buckets, owners from level 2 on), route (records routed, owners run the whole sorted
path), combine (map-side fold first).  Prints per mode the merge's device time, the stand-in exchange
time, local work = the difference, and the library's phase split; then checks that the modes leave the
same rows (lt, rank, mod everywhere; val except where two same-slot records carry equal packed keys —
counted and printed).  ENV: N (default 8), STEPS (per mode, default 3), MODES (default all three)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crdt_amd import DeviceTable  # noqa: E402
from crdt_amd.workload import gen_fanin  # noqa: E402
from tests._loopback import LoopbackComm  # noqa: E402

N = int(os.environ.get("N", "8"))
STEPS = int(os.environ.get("STEPS", "3"))
MODES = os.environ.get("MODES", "route_l1,route_l1_head,route_l1_1piece,route_l1_4piece,route,combine").split(",")
os.environ["CRDT_ENV_DYNAMIC"] = "1"
ENV = {"route_l1": {"CRDT_COMBINE": "0", "CRDT_ROUTE_L1": "1", "CRDT_RL1_SPLIT": "1"},
       "route_l1_1piece": {"CRDT_COMBINE": "0", "CRDT_ROUTE_L1": "1", "CRDT_RL1_SPLIT": "0"},
       "route_l1_4piece": {"CRDT_COMBINE": "0", "CRDT_ROUTE_L1": "1", "CRDT_RL1_SPLIT": "4"},
       "route": {"CRDT_COMBINE": "0", "CRDT_ROUTE_L1": "0"},
       "combine": {"CRDT_COMBINE": "2", "CRDT_ROUTE_L1": "1"},
       "route_l1_head": {"CRDT_COMBINE": "0", "CRDT_ROUTE_L1": "2", "CRDT_RL1_SPLIT": "1"},
       "route_l1_all": {"CRDT_COMBINE": "0", "CRDT_ROUTE_L1": "3", "CRDT_RL1_SPLIT": "1"}}

wl = gen_fanin(total=1_000_000_512, R=1024, K=1 << 28, n_local=1 << 27, s=0.8, device="cuda", rank=0, world=N,
               route=True)
home, loc = wl["home"], wl["local"]
cap = wl["capacity"]
t = DeviceTable(0, local_rank=0, capacity=cap)
t.set_counts(False)
comm = LoopbackComm(N)
t.comm_init_ops(N, 0, comm)
t.set_timing(True)
n = int(home["key"].numel())
print(f"N={N}: rank-0 home records {n}, shard slots {cap}", flush=True)
res_t = {m: [] for m in MODES}
rows = {}
for it in range(STEPS + 1):
    for m in MODES:
        os.environ.update(ENV[m])
        t.clear_rows(0, cap)
        t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
        t.canonical = wl["c0"]
        torch.cuda.synchronize()
        ts = time.perf_counter()
        res, _ = t.merge(home["key"], home["lt"], home["rank"], home["val"], wl["home_offsets"], wl["wall"],
                         win_flags=False)
        torch.cuda.synchronize()
        wall_ms = (time.perf_counter() - ts) * 1e3
        xms = comm.exchange_ms()
        xgb = comm.exchange_bytes() / 1e9
        tm = t.timing()
        plan = t.last_plan()
        line = (f"{m:9s} step {it}: wall {wall_ms:.2f} ms, device {tm['total_ms']:.2f}, exchange copy {xms:.2f} "
                f"({xgb:.3f} GB sent; library {tm['sent_bytes'] / 1e9:.3f}), "
                f"local {tm['total_ms'] - xms:.2f} | scan {tm['scan_ms']:.2f} clock {tm['clock_ms']:.2f} "
                f"route {tm['route_ms']:.2f} L1 {tm['part1_ms']:.2f} L2 {tm['part2_ms']:.2f} "
                f"resolve {tm['resolve_ms']:.2f} | route_l1 {plan['route_l1']} head {plan['rl1_head']} "
                f"combined {plan['combined']} "
                f"status {res['status']}")
        print(line, flush=True)
        if it > 0:
            res_t[m].append((tm["total_ms"], xms, xgb))
        if it == STEPS:
            rows[m] = t.read_rows(np.arange(cap, dtype=np.uint32))
for m in MODES:
    v = np.array(res_t[m])
    print(f"mean {m}: device {v[:, 0].mean():.2f} ms, exchange copy {v[:, 1].mean():.2f} ms, "
          f"local work {(v[:, 0] - v[:, 1]).mean():.2f} ms, sent {v[:, 2].mean():.3f} GB", flush=True)
ref = MODES[0]
for m in MODES[1:]:
    a, b = rows[ref], rows[m]
    same = all(np.array_equal(a[i], b[i]) for i in (0, 1, 3))
    dval = int((a[2] != b[2]).sum())
    print(f"rows {ref} vs {m}: lt/rank/mod equal {same}, val differs in {dval} slots", flush=True)
