"""Generates tests/golden/merge_golden.npz from the object-level Python oracle.

The oracle (oracle/crdt_oracle.py) is pinned by the reference's known-answer
tests (tests/test_oracle_kat.py).  Each case of tests/_cases.CASE_SPECS is
replayed as R sequential MapCrdt.merge() calls on real Hlc/Record objects and
the final per-key rows, win flags, canonical and exception are recorded in the
columnar layout.  Re-run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.crdt_oracle import (ClockDriftException, DuplicateNodeException, Hlc, MapCrdt,  # noqa: E402
                                OverflowException, Record)
from tests._cases import ABSENT_MOD, CASE_SPECS, NULL, make_case  # noqa: E402

UINT64_MAX = (1 << 64) - 1


def node(r):
    return f"n{r:04d}"


def key(i):
    return f"k{i:06d}"


def run_python_oracle(case):
    lr = case["local_rank"]
    loc = case["local"]
    seed = {}
    for i in range(case["n_local"]):
        if loc["mod"][i] == ABSENT_MOD:
            continue
        v = None if loc["val"][i] == NULL else int(loc["val"][i])
        seed[key(i)] = Record(Hlc.from_logical_time(int(loc["lt"][i]), node(int(loc["rank"][i]))), v,
                              Hlc.from_logical_time(int(loc["mod"][i]), node(lr)))
    c = MapCrdt(node(lr), seed)
    c._canonical_time = Hlc.from_logical_time(case["c0"], node(lr))
    offs = case["offsets"]
    n = int(offs[-1])
    flags = np.zeros(n, np.uint8)
    out = {"status": 0, "n_stored": 0, "exc_changeset": 0, "exc_index": UINT64_MAX, "drift_ms": 0,
           "counter": 0, "n_present": 0, "n_won": 0}
    for j in range(len(offs) - 1):
        b, e = int(offs[j]), int(offs[j + 1])
        remote = {}
        for x in range(b, e):
            lt = int(case["lt"][x])
            ms = int(case["millis"][x]) if case["millis"] is not None else lt >> 16
            h = Hlc(ms, lt - (ms << 16), node(int(case["rank"][x])))
            assert h.logical_time == lt
            v = None if case["val"][x] == NULL else int(case["val"][x])
            remote[key(int(case["key"][x]))] = Record(h, v, Hlc(0, 0, node(lr)))
        keys_in_order = list(remote.keys())
        try:
            c.merge(remote, case["wall"])
        except (ClockDriftException, DuplicateNodeException, OverflowException) as ex:
            out["exc_changeset"] = j
            if c.trace["phase"] == "recv":
                out["exc_index"] = c.trace["index"]
                out["n_stored"] = j
            else:
                out["n_stored"] = j + 1
                out["n_present"] += c.trace["present"]
                for x, k in enumerate(keys_in_order):
                    flags[b + x] = k in remote
            if isinstance(ex, ClockDriftException):
                out["status"], out["drift_ms"] = 1, ex.drift
            elif isinstance(ex, DuplicateNodeException):
                out["status"] = 2
            else:
                out["status"], out["counter"] = 3, ex.counter
            break
        out["n_stored"] = j + 1
        out["n_present"] += c.trace["present"]
        for x, k in enumerate(keys_in_order):
            flags[b + x] = k in remote
    out["n_won"] = int(flags.sum())
    out["canonical_lt"] = c.canonical_time.logical_time
    rows = {"lt": np.zeros(case["n_ids"], np.int64), "rank": np.zeros(case["n_ids"], np.uint32),
            "val": np.zeros(case["n_ids"], np.uint32), "mod": np.full(case["n_ids"], ABSENT_MOD, np.int64)}
    exists = np.zeros(case["n_ids"], np.uint8)
    for k, r in c._map.items():
        i = int(k[1:])
        exists[i] = 1
        rows["lt"][i] = r.hlc.logical_time
        rows["rank"][i] = int(r.hlc.node_id[1:])
        rows["val"][i] = NULL if r.value is None else r.value
        rows["mod"][i] = r.modified.logical_time
    return rows, exists, flags, out


def main():
    arrays, meta = {}, {}
    for ci, (name, kw) in enumerate(CASE_SPECS):
        case = make_case(**kw)
        rows, exists, flags, out = run_python_oracle(case)
        p = f"{name}__"
        for f in ("key", "lt", "rank", "val", "offsets"):
            arrays[p + f] = case[f]
        if case["millis"] is not None:
            arrays[p + "millis"] = case["millis"]
        for f in ("lt", "rank", "val", "mod"):
            arrays[p + "local_" + f] = case["local"][f]
            arrays[p + "exp_" + f] = rows[f]
        arrays[p + "exp_exists"] = exists
        arrays[p + "exp_flags"] = flags
        meta[name] = {"n_ids": case["n_ids"], "n_local": case["n_local"], "local_rank": case["local_rank"],
                      "c0": case["c0"], "wall": case["wall"], "expected": out}
    here = os.path.dirname(os.path.abspath(__file__))
    np.savez_compressed(os.path.join(here, "merge_golden.npz"), **arrays)
    with open(os.path.join(here, "merge_golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print({k: v["expected"]["status"] for k, v in meta.items()})


if __name__ == "__main__":
    main()
