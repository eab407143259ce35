"""Node-id order under Dart's String.compareTo (UTF-16 code units, hlc.dart:158-161) — property checks of the
host-side ranking (crdt_amd.intern.NodeRanks, whose ranks the packed key and the gather path compare on the
GPU) against the oracle's restatement (oracle/crdt_oracle.py dart_compare), over node ids built to stress where
UTF-16 order differs from code-point / UTF-8 order: astral characters (surrogate pairs D800-DBFF) against BMP
characters above them (U+E000-U+FFFF), common prefixes, combining marks and the empty string.  The reference has
no test of non-ASCII node order (parity unpinned there); this pins the restatement's rule.
CPU only; the GPU side of the same rule is tests/test_gpu_api.py::test_node_ids_ordered_by_utf16_not_utf8."""
from __future__ import annotations

from hypothesis import given, settings
from hypothesis import strategies as st

from crdt_amd.intern import NodeRanks
from oracle.crdt_oracle import dart_compare

# characters where the orders disagree: astral (emoji, CJK ext. B, the last plane) vs high BMP (private use,
# halfwidth/fullwidth forms, U+FFFD, U+FFFF) and ASCII / Latin / combining marks for prefixes and ties
_CHARS = ["a", "b", "Z", "~", "\u00e9", "\u0301", "\u6f22", "\ue000", "\uff5e", "\ufffd", "\uffff",
          "\U0001F600", "\U0001F601", "\U00020000", "\U0010FFFF"]
_ids = st.lists(st.sampled_from(_CHARS), min_size=0, max_size=4).map("".join)


@settings(max_examples=300, deadline=None)
@given(batches=st.lists(st.lists(_ids, min_size=1, max_size=6), min_size=1, max_size=4))
def test_node_ranks_follow_utf16_order_across_batches(batches):
    """Registered batch by batch (existing ranks move when a smaller id arrives: register() returns the
    old -> new table), the ranks always order every pair as dart_compare does, and the table maps every old
    rank to the same id's new rank."""
    nr = NodeRanks()
    seen: list[str] = []
    for batch in batches:
        before = {n: nr.rank(n) for n in seen}
        lut = nr.register(batch)
        for n in batch:
            if n not in seen:
                seen.append(n)
        if lut is not None:
            for n, r in before.items():
                assert lut[r] == nr.rank(n)
        else:
            for n, r in before.items():
                assert nr.rank(n) == r
        for a in seen:
            for b in seen:
                ra, rb = nr.rank(a), nr.rank(b)
                assert (ra > rb) - (ra < rb) == dart_compare(a, b), (a, b)
    assert sorted(nr.rank(n) for n in seen) == list(range(len(seen)))


def test_utf16_order_differs_from_code_point_order_where_expected():
    """The cases the property test is built around, spelled out: an astral character sorts before a high BMP one
    in UTF-16 (its lead surrogate D83D < E000) although its code point is larger."""
    nr = NodeRanks()
    ids = ["\U0001F600", "\uffff", "\ue000", "\U0010FFFF", "a", ""]
    nr.register(ids)
    order = sorted(ids, key=nr.rank)
    assert order == ["", "a", "\U0001F600", "\U0010FFFF", "\ue000", "\uffff"]
    assert sorted(order) != order                       # Python's code-point order disagrees
