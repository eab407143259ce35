"""The columnar C restatement (oracle/merge_oracle.c) reproduces every golden
vector produced by the object-level Python oracle (itself pinned by the
reference KATs), bit for bit: rows, win flags, canonical, exception fields."""
import json
import os

import numpy as np
import pytest

from tests._cases import ABSENT_MOD, CASE_SPECS, make_case, oracle_run

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = np.load(os.path.join(HERE, "golden", "merge_golden.npz"))
META = json.load(open(os.path.join(HERE, "golden", "merge_golden.json")))


def golden_case(name):
    m = META[name]
    p = name + "__"
    case = {"n_ids": m["n_ids"], "n_local": m["n_local"], "local_rank": m["local_rank"], "c0": m["c0"],
            "wall": m["wall"], "key": GOLD[p + "key"], "lt": GOLD[p + "lt"], "rank": GOLD[p + "rank"],
            "val": GOLD[p + "val"], "offsets": GOLD[p + "offsets"],
            "millis": GOLD[p + "millis"] if p + "millis" in GOLD else None,
            "local": {f: GOLD[p + "local_" + f] for f in ("lt", "rank", "val", "mod")}}
    exp = {f: GOLD[p + "exp_" + f] for f in ("lt", "rank", "val", "mod", "exists", "flags")}
    return case, exp, m["expected"]


def check_rows(rows_lt, rows_rank, rows_val, rows_mod, exp):
    ex = exp["exists"].astype(bool)
    assert np.array_equal(rows_lt[ex], exp["lt"][ex])
    assert np.array_equal(rows_rank[ex], exp["rank"][ex])
    assert np.array_equal(rows_val[ex], exp["val"][ex])
    assert np.array_equal(rows_mod[ex], exp["mod"][ex])
    assert np.all(rows_mod[~ex] < 0), "rows the reference never stored must stay absent"


@pytest.mark.parametrize("name", [n for n, _ in CASE_SPECS])
def test_c_oracle_matches_golden(name):
    case, exp, expected = golden_case(name)
    rows, res, flags = oracle_run(case)
    check_rows(rows["lt"], rows["rank"], rows["val"], rows["mod"], exp)
    assert np.array_equal(flags, exp["flags"])
    for k, v in expected.items():
        assert res[k] == v, (k, res[k], v)


def test_golden_is_current():
    """The committed fixtures are exactly what the generator produces."""
    for name, kw in CASE_SPECS:
        case = make_case(**kw)
        g, _, _ = golden_case(name)
        for f in ("key", "lt", "rank", "val", "offsets"):
            assert np.array_equal(case[f], g[f]), (name, f)


def test_faithful_mode_same_results():
    """The cost-mirroring mode (map copy per merge, clock read per record) changes nothing."""
    from oracle.oracle_c import OracleTable
    case = make_case(seed=99, R=4)
    r1, s1, f1 = oracle_run(case)
    t = OracleTable(case["n_ids"], case["local_rank"], case["c0"])
    loc = case["local"]
    t.put_rows(np.arange(case["n_local"], dtype=np.uint32), loc["lt"], loc["rank"], loc["val"], loc["mod"])
    res, f2 = t.merge(case["key"], case["lt"], case["rank"], case["val"], case["offsets"], case["wall"],
                      faithful=True)
    assert res.as_dict() == s1 and np.array_equal(f1, f2) and np.array_equal(t.rows, r1)


def test_absent_pattern():
    assert ABSENT_MOD < 0


@pytest.mark.parametrize("name", [n for n, _ in CASE_SPECS])
def test_omp_baseline_equals_sequential(name):
    """oracle/merge_omp.c (the multi-core CPU baseline) == or_merge on every case."""
    from oracle.oracle_c import OracleTable
    from tests._cases import ABSENT_MOD, oracle_run
    case = make_case(**dict(CASE_SPECS)[name])
    orows, ores, oflags = oracle_run(case)
    t = OracleTable(case["n_ids"], case["local_rank"], case["c0"])
    loc = case["local"]
    keep = loc["mod"] != ABSENT_MOD
    ids = np.arange(case["n_local"], dtype=np.uint32)[keep]
    t.put_rows(ids, loc["lt"][keep], loc["rank"][keep], loc["val"][keep], loc["mod"][keep])
    res, flags = t.merge_omp(case["key"], case["lt"], case["rank"], case["val"], case["offsets"], case["wall"],
                             millis=case["millis"], threads=4)
    assert res.as_dict() == ores
    assert np.array_equal(flags, oflags)
    for f in ("lt", "rank", "val", "mod"):
        assert np.array_equal(t.rows[f], orows[f]), f
