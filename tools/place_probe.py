"""Within one process: does the level-1 scatter's time follow the partition buffers' placement?
(the process-to-process spread.)  The 1B fan-in of bench.py; the partition buffers are
re-allocated A times (each time a torch filler of a different size is taken from the free pool first, so
the new buffers land on other frames) and STEPS merges are timed on each allocation.  Prints each
allocation's level-1 scatter / step times.  ENV: A (default 5), STEPS (default 3)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crdt_amd import DeviceTable  # noqa: E402
from crdt_amd.workload import gen_fanin  # noqa: E402

A = int(os.environ.get("A", "5"))
STEPS = int(os.environ.get("STEPS", "3"))
t = DeviceTable(0, local_rank=0, capacity=1 << 28)
n = 1_000_000_512
t.reserve_scratch(n)
wl = gen_fanin(total=n, R=1024, K=1 << 28, n_local=1 << 27, s=0.8, device="cuda")
own, loc = wl["owned"], wl["local"]
t.set_counts(False)
t.set_rank_bound(1025)
t.set_timing(True)
fillers = []
for a in range(A):
    if a:
        gb = [3, 7, 1, 5, 2, 6][a % 6]
        fillers.append(torch.empty(gb << 30, dtype=torch.uint8, device="cuda"))
        t.reserve_scratch(n + a * (1 << 22))          # grows: the old buffers go, new ones come
        torch.cuda.synchronize()
    p1 = []
    for s in range(STEPS + 1):
        t.clear_rows(0, wl["capacity"])
        t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
        t.canonical = wl["c0"]
        torch.cuda.synchronize()
        ts = time.perf_counter()
        res, _ = t.merge(own["key"], own["lt"], own["rank"], own["val"], wl["owned_offsets"], wl["wall"],
                         win_flags=False)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - ts) * 1e3
        tm = t.timing()
        if s:
            p1.append((ms, tm["part1_ms"], tm["part2_ms"], tm["resolve_ms"]))
    m = [sum(x[i] for x in p1) / len(p1) for i in range(4)]
    print(f"allocation {a} (fillers {sum(f.numel() for f in fillers) >> 30} GB): step {m[0]:.2f} ms, level-1 "
          f"{m[1]:.2f}, level-2 {m[2]:.2f}, resolve {m[3]:.2f}  | steps {[round(x[0], 2) for x in p1]}", flush=True)
