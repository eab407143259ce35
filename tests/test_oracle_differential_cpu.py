"""Differential property test of the two oracle restatements on random small batches: the columnar C oracle
(oracle/merge_oracle.c — the checker every GPU parity test and the bench's parity leg compare against) and the
object-level Python restatement of the reference (oracle/crdt_oracle.py, pinned by the reference's KATs,
tests/test_oracle_kat.py), each merge of R changesets run as R sequential Crdt.merge calls (crdt.dart:77-94).
The committed golden vectors (tests/test_golden_cpu.py) cover fixed cases; this draws new ones — ties across
changesets (few millis / counters, few node ranks), tombstones, invisible local rows, duplicate-node and drift
records, forced raising records — and requires the same rows, win flags, canonical and exception fields."""
from __future__ import annotations

import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from tests._cases import make_case, oracle_run
from tests.golden.make_golden import run_python_oracle
from tests.test_golden_cpu import check_rows

_kw = st.fixed_dictionaries({
    "seed": st.integers(0, 2 ** 31 - 1),
    "R": st.integers(1, 6),
    "per_cs": st.integers(0, 50),
    "n_local": st.integers(1, 60),
    "n_new": st.integers(0, 30),
    "millis_span": st.integers(1, 12),
    "counter_span": st.integers(1, 4),
    "n_ranks": st.integers(2, 7),
    "tomb_frac": st.sampled_from([0.0, 0.2, 0.5]),
    "neg_mod_frac": st.sampled_from([0.0, 0.1]),
    "dup_frac": st.sampled_from([0.0, 0.0, 0.02]),
    "drift_frac": st.sampled_from([0.0, 0.0, 0.02]),
    "explicit_millis": st.booleans(),
})


@settings(max_examples=120, deadline=None)
@given(kw=_kw, local_rank=st.integers(0, 6), force=st.sampled_from([(), "dup", "drift"]))
def test_c_oracle_equals_object_oracle(kw, local_rank, force):
    kw = dict(kw)
    kw["local_rank"] = local_rank % kw["n_ranks"]
    if force:
        kw["force"] = [(kw["R"] - 1, 0, force)]
    case = make_case(**kw)
    rows, res, flags = oracle_run(case)
    prow, exists, pflags, pout = run_python_oracle(case)
    exp = {"lt": prow["lt"], "rank": prow["rank"], "val": prow["val"], "mod": prow["mod"], "exists": exists}
    check_rows(rows["lt"], rows["rank"], rows["val"], rows["mod"], exp)
    assert np.array_equal(flags, pflags)
    for k, v in pout.items():
        assert res[k] == v, (k, res[k], v)
