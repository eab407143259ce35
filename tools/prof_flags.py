"""The 1B fan-in merged with per-record win flags (auto path: the sorted path's flagged form),
STEPS times — run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crdt_amd import DeviceTable  # noqa: E402
from crdt_amd.workload import gen_fanin  # noqa: E402

steps = int(os.environ.get("STEPS", "3"))
wl = gen_fanin(total=1_000_000_512, R=1024, K=1 << 28, n_local=1 << 27, s=0.8, device="cuda")
own, loc = wl["owned"], wl["local"]
t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
t.set_rank_bound(1025)
flags = torch.zeros(wl["total"], dtype=torch.uint8, device="cuda")
for i in range(steps):
    t.clear_rows(0, wl["capacity"])
    t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
    t.canonical = wl["c0"]
    torch.cuda.synchronize()
    ts = time.perf_counter()
    res, _ = t.merge(own["key"], own["lt"], own["rank"], own["val"], wl["owned_offsets"], wl["wall"], win_flags=flags)
    torch.cuda.synchronize()
    print(f"step {i}: {(time.perf_counter() - ts) * 1e3:.2f} ms path {t.last_path()} plan {t.last_plan()} "
          f"won {res['n_won']}", flush=True)
