"""Diagnostic: cfg5 at full size, one merge call per delta; after each call compare the `modified`
stamp of rows won in that call with R_d = max(C_{d-1}, M_d) (crdt.dart:82,86-87)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from crdt_amd import DeviceTable  # noqa: E402
from crdt_amd.workload import gen_cfg5  # noqa: E402

inject = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "none" else None
deltas = int(sys.argv[2]) if len(sys.argv) > 2 else 12
wl = gen_cfg5(device="cuda", inject=inject, deltas=max(deltas, 38 if inject else deltas))
n, K = wl["n_per_replica"], wl["K"]
t = DeviceTable(0, local_rank=0, capacity=wl["capacity"])
loc, own = wl["local"], wl["owned"]
t.put_rows(loc["slot"], loc["lt"], loc["rank"], loc["val"], loc["mod"])
t.canonical = wl["c0"]
c = wl["c0"]
for d in range(deltas):
    b, e = d * n, (d + 1) * n
    res, _ = t.merge(own["key"][b:e], own["lt"][b:e], own["rank"][b:e], own["val"][b:e],
                     np.array([0, n], np.uint64), int(wl["walls"][d]), win_flags=False)
    m = int(own["lt"][b:e].max().item())
    r = max(c, m)
    # rows whose stored value handle is from this delta: their mod must be R_d
    keys = own["key"][b:e][::997].cpu().numpy().astype(np.uint32)
    lt, rk, val, mod = t.read_rows(keys)
    vals = own["val"][b:e][::997].cpu().numpy().astype(np.uint32)
    mine = (val == vals) & (vals != 0xFFFFFFFF)
    bad = mine & (mod != r)
    print(f"delta {d}: status {res['status']} canon {res['canonical_lt']} M {m} C_prev {c} R {r} "
          f"won-sample {int(mine.sum())} bad {int(bad.sum())}"
          + (f" e.g. mod {mod[bad][:3]} (R - mod {r - mod[bad][:3]})" if bad.any() else ""), flush=True)
    c = max(r + 1, int(wl["walls"][d]) << 16)
    if res["status"]:
        break
