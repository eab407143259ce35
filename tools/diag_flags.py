"""Diagnostic: the flagged sorted form vs the oracle's flags on one case, under form switches."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests._cases import make_case, oracle_run  # noqa: E402
from tests.test_gpu_parity import device_run  # noqa: E402

case = make_case(seed=79, R=300, per_cs=2000, n_local=40_000, n_new=20_000, millis_span=8,
                 counter_span=4, n_ranks=301)
orows, ores, oflags = oracle_run(case)
offs = case["offsets"].astype(np.int64)
for env in ["", "CRDT_SORTED_FORM=65536", "CRDT_XCD_MAP=0", "CRDT_SORTED_FORM=1024"]:
    for k in ("CRDT_SORTED_FORM", "CRDT_XCD_MAP"):
        os.environ.pop(k, None)
    if env:
        k, v = env.split("=")
        os.environ[k] = v
    for cap in (None, (1 << 20) + 7, 1 << 24):
        rows, res, fl = device_run(case, path="sorted", flags=True, capacity=cap)
        bad = np.nonzero(fl != oflags)[0]
        js = np.searchsorted(offs, bad, side="right") - 1
        print(f"{env or 'default':24s} cap={cap} flagged={res['plan']['flagged']} mismatches={len(bad)} "
              f"(1->0 {int(((fl == 0) & (oflags == 1)).sum())}, 0->1 {int(((fl == 1) & (oflags == 0)).sum())}) "
              f"n_won {res['n_won']} vs {ores['n_won']} n_present {res['n_present']} vs {ores['n_present']}",
              flush=True)
        if len(bad):
            print("   first idx", bad[:8].tolist(), "changesets", js[:8].tolist(), "keys",
                  case["key"][bad[:8]].tolist(), flush=True)
