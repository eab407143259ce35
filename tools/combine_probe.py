"""The map-side combine's local cost at one rank's share of config 4 (tools/gpu_comb_probe.sh).

Rank 0 of an N-rank routed fan-in (gen_fanin(route=True): replica j on rank j % N) merged on a 1-rank
RCCL ctx whose table spans the whole key range, so every record "routes" to itself: with
CRDT_COMBINE=1 the step is the home fold + the owners' apply of the distinct keys, with
CRDT_COMBINE=0 the route scatter + the apply of every record.  Prints both times, the number of
records and of distinct keys (what the combine would send instead), and checks that both leave the
same rows."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crdt_amd import DeviceTable  # noqa: E402
from crdt_amd.workload import gen_fanin  # noqa: E402

os.environ["CRDT_ENV_DYNAMIC"] = "1"
N = int(os.environ.get("N", "2"))
wl = gen_fanin(total=1_000_000_512, R=1024, K=1 << 28, n_local=1 << 27, s=0.8, device="cuda", rank=0, world=N,
               route=True)
home, loc = wl["home"], wl["local"]
n = int(home["key"].numel())
t = DeviceTable(0, local_rank=0, capacity=1 << 28)
t.set_counts(False)
t.set_rank_bound(1025)
t.comm_init_rccl(1, 0, t.comm_unique_id())
out = {}
for it, comb in enumerate(["0", "1", "0", "1", "0", "1"]):
    os.environ["CRDT_COMBINE"] = comb
    t.clear_rows(0, 1 << 28)
    t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
    t.canonical = wl["c0"]
    torch.cuda.synchronize()
    ts = time.perf_counter()
    res, _ = t.merge(home["key"], home["lt"], home["rank"], home["val"], wl["home_offsets"], wl["wall"],
                     win_flags=False)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - ts) * 1e3
    plan = t.last_plan()
    if it >= 2:
        out.setdefault(comb, []).append(ms)
    print(f"combine={comb}: {ms:.2f} ms status {res['status']} combined {plan['combined']}", flush=True)
    if it in (4, 5):
        rows = t.read_rows(np.arange(0, 1 << 28, 997, dtype=np.uint32))
        out["rows" + comb] = rows
for k in ("0", "1"):
    print(f"mean combine={k}: {np.mean(out[k]):.2f} ms", flush=True)
same = all(np.array_equal(a, b) for a, b in zip(out["rows0"], out["rows1"]))
distinct = int(torch.unique(home["key"]).numel())
print(f"N={N} rank-0 home records {n}, distinct keys {distinct} ({n / max(distinct, 1):.2f}x), sampled rows equal: {same}",
      flush=True)
