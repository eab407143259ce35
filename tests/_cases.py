"""Seeded synthetic merge cases in the columnar layout (test helper).

A case = a local row table + canonical + R changesets + wall.  Knobs force the
edge cases the reference semantics has: ties on (lt, rank), tombstones,
negative ``modified`` (invisible rows), duplicate-node and drift records, and
canonicals that make ``send`` fail (drift / counter overflow).
"""
from __future__ import annotations

import numpy as np

NULL = 0xFFFFFFFF
ABSENT_MOD = np.frombuffer(b"\x80" * 8, dtype="<i8")[0]
WALL = 1_700_000_000_000


def make_case(seed: int, n_local: int = 200, n_new: int = 100, R: int = 3, per_cs: int = 80,
              n_ranks: int = 6, local_rank: int = 0, millis_span: int = 50, counter_span: int = 4,
              tomb_frac: float = 0.1, neg_mod_frac: float = 0.0, absent_frac: float = 0.0,
              dup_frac: float = 0.0, drift_frac: float = 0.0, c0: int | None = None,
              wall: int = WALL, explicit_millis: bool = False, base: int | None = None,
              force=()) -> dict:
    rng = np.random.default_rng(seed)
    base = wall - 1000 if base is None else base
    n_ids = n_local + n_new
    # ---- local rows
    lt = ((base + rng.integers(0, millis_span, n_local)) << 16) + rng.integers(0, counter_span, n_local)
    rank = rng.integers(0, n_ranks, n_local).astype(np.uint32)
    val = rng.integers(0, 1 << 20, n_local).astype(np.uint32)
    val[rng.random(n_local) < tomb_frac] = NULL
    mod = lt + rng.integers(0, 5, n_local)
    mod[rng.random(n_local) < neg_mod_frac] = -(1 << 20)
    absent = rng.random(n_local) < absent_frac
    mod[absent] = ABSENT_MOD
    local = {"lt": lt.astype(np.int64), "rank": rank, "val": val, "mod": mod.astype(np.int64)}
    if c0 is None:
        vis = mod >= 0
        c0 = int(lt[vis].max()) if vis.any() else 0
    # ---- changesets (distinct keys each)
    keys, lts, ranks, vals, millis = [], [], [], [], []
    offsets = [0]
    for j in range(R):
        n = min(per_cs, n_ids)
        k = rng.choice(n_ids, size=n, replace=False).astype(np.uint32)
        l = ((base + rng.integers(0, millis_span, n)) << 16) + rng.integers(0, counter_span, n)
        r = rng.integers(0, n_ranks, n).astype(np.uint32)
        r[r == local_rank] = (local_rank + 1) % n_ranks       # foreign by default
        dup = rng.random(n) < dup_frac
        r[dup] = local_rank
        v = rng.integers(0, 1 << 20, n).astype(np.uint32)
        v[rng.random(n) < tomb_frac] = NULL
        ms = l >> 16
        if explicit_millis:       # Hlc(millis, counter > 0xFFFF): lt carries into millis (hlc.dart:16)
            odd = rng.random(n) < 0.2
            ms = np.where(odd, ms - 1, ms)
        drift = rng.random(n) < drift_frac
        ms = np.where(drift, wall + 60001 + rng.integers(0, 10, n), ms)
        l = np.where(drift, (ms << 16) + rng.integers(0, counter_span, n), l)
        for (fj, fi, kind) in force:   # make record fi of changeset fj a raising record-setter
            if fj == j and fi < n:
                top = max(int(l.max()), int(c0), *(int(x.max()) for x in lts if len(x))) + 1
                if j > 0:                    # canonical is >= wall << 16 after the first send()
                    top = max(top, ((wall + 1) << 16) + j)
                if kind == "dup":
                    r[fi] = local_rank
                    l[fi] = top
                    ms[fi] = top >> 16
                else:
                    ms[fi] = max(wall + 60001, (top >> 16) + 1)
                    l[fi] = ms[fi] << 16
        keys.append(k); lts.append(l.astype(np.int64)); ranks.append(r); vals.append(v)
        millis.append(ms.astype(np.int64))
        offsets.append(offsets[-1] + n)
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
    case = {
        "n_ids": n_ids, "n_local": n_local, "local": local, "local_rank": local_rank, "c0": int(c0),
        "wall": int(wall), "key": cat(keys, np.uint32), "lt": cat(lts, np.int64),
        "rank": cat(ranks, np.uint32), "val": cat(vals, np.uint32),
        "offsets": np.array(offsets, np.uint64), "millis": None,
    }
    if explicit_millis:
        case["millis"] = cat(millis, np.int64)
    return case


def oracle_run(case, faithful=False):
    """Run the C restatement on a case; returns (table rows, result dict, flags)."""
    from oracle.oracle_c import OracleTable
    t = OracleTable(case["n_ids"], case["local_rank"], case["c0"])
    n_local = case["n_local"]
    loc = case["local"]
    keep = loc["mod"] != ABSENT_MOD
    ids = np.arange(n_local, dtype=np.uint32)[keep]
    t.put_rows(ids, loc["lt"][keep], loc["rank"][keep], loc["val"][keep], loc["mod"][keep])
    res, flags = t.merge(case["key"], case["lt"], case["rank"], case["val"], case["offsets"], case["wall"],
                         millis=case["millis"])
    return t.rows, res.as_dict(), flags


CASE_SPECS = [
    # name, kwargs — every knob the semantics has, at sizes the oracle finishes instantly
    ("r1_basic", dict(seed=1, R=1, per_cs=150)),
    ("r1_ties", dict(seed=2, R=1, per_cs=250, millis_span=2, counter_span=1, n_ranks=3)),
    ("r4_ties", dict(seed=3, R=4, per_cs=120, millis_span=3, counter_span=2, n_ranks=4)),
    ("r8_tombstones", dict(seed=4, R=8, per_cs=60, tomb_frac=0.5)),
    ("neg_mod", dict(seed=5, R=3, neg_mod_frac=0.3)),
    ("absent_rows", dict(seed=6, R=3, absent_frac=0.3)),
    ("dup_node", dict(seed=7, R=4, dup_frac=0.02, c0=0, force=[(2, 17, "dup")])),
    ("dup_first_record", dict(seed=20, R=2, force=[(0, 0, "dup")])),
    ("drift_last_record", dict(seed=21, R=3, force=[(1, 79, "drift")])),
    ("dup_late", dict(seed=17, R=6, dup_frac=0.004, base=WALL + 100, millis_span=400)),
    ("drift_late", dict(seed=18, R=6, drift_frac=0.003, base=WALL + 100, millis_span=400)),
    ("dup_and_drift", dict(seed=19, R=5, dup_frac=0.01, drift_frac=0.01, base=WALL - 200,
                           millis_span=600, c0=0)),
    ("drift", dict(seed=8, R=4, drift_frac=0.01)),
    ("dup_old_echo", dict(seed=9, R=3, dup_frac=0.3, c0=(WALL + 5000) << 16)),
    ("send_overflow", dict(seed=10, R=2, c0=((WALL + 10) << 16) | 0xFFFF)),
    ("send_drift", dict(seed=11, R=2, c0=(WALL + 70000) << 16)),
    ("explicit_millis", dict(seed=12, R=3, explicit_millis=True, drift_frac=0.005)),
    ("empty_changesets", dict(seed=13, R=5, per_cs=0)),
    ("r32_small", dict(seed=14, R=32, per_cs=20, n_local=50, n_new=30, millis_span=4)),
    ("local_rank_mid", dict(seed=15, R=3, local_rank=3, n_ranks=7, dup_frac=0.01)),
    ("c0_negative", dict(seed=16, R=2, c0=-(1 << 30), base=-2000, wall=WALL)),
]
