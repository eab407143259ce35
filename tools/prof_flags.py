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
ab = os.environ.get("AB")                 # e.g. "CRDT_PF_THREADS=1024,512": alternate per step (in-process A/B)
if ab:
    os.environ["CRDT_ENV_DYNAMIC"] = "1"
    ab_var, ab_vals = ab.split("=")[0], ab.split("=")[1].split(",")
wl = gen_fanin(total=1_000_000_512, R=1024, K=1 << 28, n_local=1 << 27, s=0.8, device="cuda")
own, loc = wl["owned"], wl["local"]
t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
t.set_rank_bound(1025)
flags = torch.zeros(wl["total"], dtype=torch.uint8, device="cuda")
times = {}
ref = None                                # the first step's flags: every later step (any A/B value) must equal them
for i in range(steps):
    if ab:
        os.environ[ab_var] = ab_vals[i % len(ab_vals)]
    t.clear_rows(0, wl["capacity"])
    t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
    t.canonical = wl["c0"]
    torch.cuda.synchronize()
    ts = time.perf_counter()
    fl = flags if not (os.environ.get("MIX") and i % 2) else False      # MIX=1: odd steps without flags
    res, _ = t.merge(own["key"], own["lt"], own["rank"], own["val"], wl["owned_offsets"], wl["wall"], win_flags=fl)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - ts) * 1e3
    tag = os.environ.get(ab_var) if ab else ""
    if fl is not False:
        if ref is None:
            ref = (flags.clone(), res["n_won"], res["canonical_lt"])
        elif not (torch.equal(flags, ref[0]) and res["n_won"] == ref[1] and res["canonical_lt"] == ref[2]):
            print(f"step {i} {tag}: FLAGS DIFFER from step 0", flush=True)
            sys.exit(3)
    if i >= (len(ab_vals) if ab else 1):
        times.setdefault(tag, []).append(ms)
    print(f"step {i} {tag}: {ms:.2f} ms path {t.last_path()} flagged {t.last_plan()['flagged']} won {res['n_won']}",
          flush=True)
for k, v in times.items():
    print(f"A/B {k}: mean {sum(v) / len(v):.3f} ms over {len(v)} steps", flush=True)
