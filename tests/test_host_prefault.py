"""The parallel decoder's page population (MADV_POPULATE_WRITE on the ordered pass's reserved
columns, crdt_host.cpp `prefault`) changes no output: columns, ids and node list equal the run
with CRDT_HOST_PREFAULT=0, on a document large enough (> 4 MB) to take the parallel path."""
import os

import numpy as np

from crdt_amd import hostlib
from crdt_amd.intern import KeyIndex


def _doc(n, seed=3):
    rng = np.random.default_rng(seed)
    lt = ((1_735_689_600_000 + rng.integers(0, 1 << 20, n)) << 16) + rng.integers(0, 16, n)
    node = rng.integers(0, 5, n).astype(np.uint32)
    hlcs = hostlib.hlc_strings(lt, node, [f"n{i}" for i in range(5)])
    keys = rng.integers(0, n // 2, n)                     # repeated keys: first position, last record
    return "{" + ",".join(f'"k{keys[i]}":{{"hlc":"{hlcs[i]}","value":{i}}}' for i in range(n)) + "}"


def _decode(doc, mode):
    old = os.environ.get("CRDT_HOST_PREFAULT")
    os.environ["CRDT_HOST_PREFAULT"] = mode
    try:
        return hostlib.decode(doc, KeyIndex().native)
    finally:
        if old is None:
            del os.environ["CRDT_HOST_PREFAULT"]
        else:
            os.environ["CRDT_HOST_PREFAULT"] = old


def test_prefault_changes_no_output():
    doc = _doc(120_000)
    assert len(doc) > 4 << 20
    a, b = _decode(doc, "1"), _decode(doc, "0")
    for c in ("key_id", "lt", "node", "val_off", "val_len"):
        assert np.array_equal(a[c], b[c]), c
    assert a["nodes"] == b["nodes"]
    assert len(a["key_id"]) == len(np.unique(a["key_id"]))
