"""Pins the CPU oracle (oracle/crdt_oracle.py) to the reference's own known-answer tests.

Transliterated from /root/reference/test/hlc_test.dart (all groups),
test/map_crdt_test.dart (Seed, Merge, Serialization, Delta subsets, Delta sync)
and test/crdt_test.dart (Basic, Watch).  Wall-clock reads of the reference
(``DateTime.now()``) are replaced by explicit ``wall`` values chosen so every
assertion means what the original test means.
"""
import pytest

from oracle.crdt_oracle import (ClockDriftException, CrdtJson, DuplicateNodeException, Hlc, MapCrdt,
                                OverflowException, Record, dart_compare, iso_from_millis,
                                millis_from_iso)

MILLIS = 1000000000000                       # hlc_test.dart:4
ISO = "2001-09-09T01:46:40.000Z"             # hlc_test.dart:5
LT = 65536000000000066                       # hlc_test.dart:6
WALL = 1700000000000


# ----------------------------------------------------------- hlc_test.dart
class TestConstructors:
    hlc = Hlc(MILLIS, 0x42, "abc")

    def test_default(self):                                  # :13-17
        assert (self.hlc.millis, self.hlc.counter, self.hlc.node_id) == (MILLIS, 0x42, "abc")

    def test_microseconds(self):                             # :19-21
        assert Hlc(MILLIS * 1000, 0x42, "abc") == self.hlc

    def test_zero(self):                                     # :28-30
        assert Hlc.zero("abc") == Hlc(0, 0, "abc")

    def test_from_date(self):                                # :32-34
        assert Hlc(millis_from_iso(ISO), 0, "abc") == Hlc(MILLIS, 0, "abc")

    def test_logical_time(self):                             # :36-38
        assert Hlc.from_logical_time(LT, "abc") == self.hlc

    def test_parse(self):                                    # :40-42
        assert Hlc.parse(f"{ISO}-0042-abc") == self.hlc


class TestStringOps:
    def test_to_string(self):                                # :46-49
        assert str(Hlc.parse(f"{ISO}-0042-abc")) == f"{ISO}-0042-abc"

    def test_parse(self):                                    # :51-53
        assert Hlc.parse(f"{ISO}-0042-abc") == Hlc(MILLIS, 0x42, "abc")

    def test_int_node_parse(self):                           # :57-60
        assert Hlc.parse(f"{ISO}-0042-1", int) == Hlc(MILLIS, 0x42, 1)

    def test_int_node_to_string(self):                       # :62-65
        assert str(Hlc(MILLIS, 0x42, 1)) == f"{ISO}-0042-1"


class TestComparison:
    def test_equality(self):                                 # :69-75
        a, b = Hlc.parse(f"{ISO}-0042-abc"), Hlc.parse(f"{ISO}-0042-abc")
        assert a == b and a <= b and a >= b

    def test_different_node_ids(self):                       # :77-81
        assert Hlc.parse(f"{ISO}-0042-abc") != Hlc.parse(f"{ISO}-0042-abcd")

    def test_less_than_millis(self):                         # :83-88
        a, b = Hlc(MILLIS, 0x42, "abc"), Hlc(MILLIS + 1, 0, "abc")
        assert a < b and a <= b

    def test_less_than_counter(self):                        # :90-95
        a, b = Hlc.parse(f"{ISO}-0042-abc"), Hlc.parse(f"{ISO}-0043-abc")
        assert a < b and a <= b

    def test_less_than_node_id(self):                        # :97-102
        a, b = Hlc.parse(f"{ISO}-0042-abc"), Hlc.parse(f"{ISO}-0042-abb")
        assert a > b and a >= b

    def test_fail_less_than_if_equal(self):                  # :104-108
        assert not (Hlc.parse(f"{ISO}-0042-abc") < Hlc.parse(f"{ISO}-0042-abc"))

    def test_fail_less_than_disagree(self):                  # :110-114
        assert not (Hlc(MILLIS + 1, 0, "abc") < Hlc(MILLIS, 0x42, "abc"))

    def test_more_than_millis(self):                         # :116-121
        a, b = Hlc(MILLIS + 1, 0x42, "abc"), Hlc(MILLIS, 0, "abc")
        assert a > b and a >= b

    def test_more_than_node(self):                           # :130-135
        a, b = Hlc(MILLIS, 0x42, "abc"), Hlc(MILLIS, 0x42, "abb")
        assert a > b and a >= b

    def test_compare(self):                                  # :137-148
        h = Hlc(MILLIS, 0x42, "abc")
        assert h.compare_to(Hlc(MILLIS, 0x42, "abc")) == 0
        assert h.compare_to(Hlc(MILLIS + 1, 0x42, "abc")) == -1
        assert h.compare_to(Hlc(MILLIS, 0x43, "abc")) == -1
        assert h.compare_to(Hlc(MILLIS, 0x42, "abd")) == -1
        assert h.compare_to(Hlc(MILLIS - 1, 0x42, "abc")) == 1
        assert h.compare_to(Hlc(MILLIS, 0x41, "abc")) == 1
        assert h.compare_to(Hlc(MILLIS, 0x42, "abb")) == 1


class TestLogicalTime:
    def test_stability(self):                                # :152-155
        assert Hlc.from_logical_time(LT, "abc").logical_time == LT

    def test_as_logical_time(self):                          # :157-160
        assert Hlc.parse(f"{ISO}-0042-abc").logical_time == LT

    def test_constants(self):                                # :4-7 (checked in SURVEY §4)
        assert (MILLIS << 16) + 0x42 == LT
        assert iso_from_millis(MILLIS) == ISO


class TestSend:
    def test_higher_canonical(self):                         # :183-190
        h = Hlc(MILLIS + 1, 0x42, "abc")
        s = Hlc.send(h, MILLIS)
        assert s != h and s.millis == h.millis and s.counter == 0x43 and s.node_id == h.node_id

    def test_equal_canonical(self):                          # :192-199
        h = Hlc(MILLIS, 0x42, "abc")
        s = Hlc.send(h, MILLIS)
        assert s != h and s.millis == MILLIS and s.counter == 0x43

    def test_lower_canonical(self):                          # :201-208
        h = Hlc(MILLIS - 1, 0x42, "abc")
        s = Hlc.send(h, MILLIS)
        assert s != h and s.millis == MILLIS and s.counter == 0

    def test_drift(self):                                    # :210-213
        with pytest.raises(ClockDriftException) as e:
            Hlc.send(Hlc(MILLIS + 60001, 0, "abc"), MILLIS)
        assert e.value.drift == 60001
        assert str(e.value) == "Clock drift of 60001 ms exceeds maximum (60000)"

    def test_overflow(self):                                 # :215-218
        with pytest.raises(OverflowException) as e:
            Hlc.send(Hlc(MILLIS, 0xFFFF, "abc"), MILLIS)
        assert e.value.counter == 0x10000


class TestReceive:
    canonical = Hlc.parse(f"{ISO}-0042-abc")

    def test_higher_canonical(self):                         # :224-228
        assert Hlc.recv(self.canonical, Hlc(MILLIS - 1, 0x42, "abcd"), MILLIS) == self.canonical

    def test_same_remote_time(self):                         # :230-234
        r = Hlc(MILLIS, 0x42, "abcd")
        assert Hlc.recv(self.canonical, r, MILLIS) == Hlc(r.millis, r.counter, self.canonical.node_id)

    def test_higher_remote_time(self):                       # :236-240
        r = Hlc(MILLIS + 1, 0, "abcd")
        assert Hlc.recv(self.canonical, r, MILLIS) == Hlc(r.millis, r.counter, self.canonical.node_id)

    def test_higher_wall(self):                              # :242-246
        r = Hlc.parse(f"{ISO}-0000-abcd")
        assert Hlc.recv(self.canonical, r, MILLIS + 1) == self.canonical

    def test_skip_node_check_lower(self):                    # :248-251
        assert Hlc.recv(self.canonical, Hlc(MILLIS - 1, 0x42, "abc"), MILLIS) == self.canonical

    def test_skip_node_check_same(self):                     # :253-256
        assert Hlc.recv(self.canonical, Hlc(MILLIS, 0x42, "abc"), MILLIS) == self.canonical

    def test_fail_on_node_id(self):                          # :258-261
        with pytest.raises(DuplicateNodeException) as e:
            Hlc.recv(self.canonical, Hlc(MILLIS + 1, 0, "abc"), MILLIS)
        assert str(e.value) == "Duplicate node: abc"

    def test_fail_on_drift(self):                            # :263-266
        with pytest.raises(ClockDriftException):
            Hlc.recv(self.canonical, Hlc(MILLIS + 60001, 0x42, "abcd"), MILLIS)


def test_string_compare_is_utf16_code_unit_order():
    assert dart_compare("nodeB", "nodeA") == 1               # map_crdt_test.dart:59-63
    assert dart_compare("abc", "abcd") == -1
    # U+FF5E (one code unit) sorts after U+1F600 (surrogate pair D83D...) in UTF-16
    assert dart_compare("～", "\U0001F600") == 1


# ------------------------------------------------------- map_crdt_test.dart
def hlc_now(node="abc", wall=WALL):
    return Hlc(wall, 0, node)


class TestSeed:                                              # :17-31
    def test_seed_item(self):
        c = MapCrdt("abc", {"x": Record(hlc_now(), 1, hlc_now())})
        assert c.get("x") == 1
        assert c.canonical_time.logical_time == 0           # ctor refreshes before seeding

    def test_seed_and_put(self):
        c = MapCrdt("abc", {"x": Record(hlc_now(), 1, hlc_now())})
        c.put("x", 2, WALL)
        assert c.get("x") == 2


class TestMerge:                                             # :33-103
    def setup_method(self):
        self.c = MapCrdt("abc")

    def test_merge_older(self):
        self.c.put("x", 2, WALL)
        self.c.merge({"x": Record(Hlc(MILLIS - 1, 0, "xyz"), 1, hlc_now())}, WALL)
        assert self.c.get("x") == 2

    def test_merge_very_old(self):
        self.c.put("x", 2, WALL)
        self.c.merge({"x": Record(Hlc(0, 0, "xyz"), 1, hlc_now())}, WALL)
        assert self.c.get("x") == 2

    def test_merge_newer(self):
        self.c.put("x", 1, WALL)
        self.c.merge({"x": Record(Hlc(WALL + 1, 0, "xyz"), 2, hlc_now())}, WALL + 1)
        assert self.c.get("x") == 2

    def test_disambiguate_using_node_id(self):
        self.c.merge({"x": Record(Hlc(MILLIS, 0, "nodeA"), 1, hlc_now())}, WALL)
        self.c.merge({"x": Record(Hlc(MILLIS, 0, "nodeB"), 2, hlc_now())}, WALL)
        assert self.c.get("x") == 2

    def test_merge_same(self):
        self.c.put("x", 2, WALL)
        ts = self.c.get_record("x").hlc
        self.c.merge({"x": Record(ts, 1, hlc_now())}, WALL)
        assert self.c.get("x") == 2

    def test_merge_older_newer_counter(self):
        self.c.put("x", 2, WALL)
        self.c.merge({"x": Record(Hlc(MILLIS - 1, 2, "xyz"), 1, hlc_now())}, WALL)
        assert self.c.get("x") == 2

    def test_merge_same_newer_counter(self):
        self.c.put("x", 1, WALL)
        ts = Hlc(self.c.get_record("x").hlc.millis, 2, "xyz")
        self.c.merge({"x": Record(ts, 2, hlc_now())}, WALL)
        assert self.c.get("x") == 2

    def test_merge_new_item(self):
        m = {"x": Record(Hlc(WALL, 0, "xyz"), 2, hlc_now())}
        self.c.merge(m, WALL)
        assert self.c.record_map() == m

    def test_merge_deleted_item(self):
        self.c.put("x", 1, WALL)
        self.c.merge({"x": Record(Hlc(WALL + 1, 0, "xyz"), None, hlc_now())}, WALL + 1)
        assert self.c.is_deleted("x") is True

    def test_update_hlc_on_merge(self):
        self.c.put("x", 1, WALL)
        self.c.merge({"y": Record(Hlc(MILLIS - 1, 0, "xyz"), 2, hlc_now())}, WALL)
        assert self.c.values == [1, 2]


class TestSerialization:                                     # :105-201 (the codec pins)
    def test_to_map(self):
        c = MapCrdt("abc", {"x": Record(Hlc(MILLIS, 0, "abc"), 1, hlc_now())})
        assert c.record_map() == {"x": Record(Hlc(MILLIS, 0, "abc"), 1, hlc_now())}

    def test_json_encode_string_key(self):
        c = MapCrdt("abc", {"x": Record(Hlc(MILLIS, 0, "abc"), 1, hlc_now())})
        assert c.to_json() == f'{{"x":{{"hlc":"{ISO}-0000-abc","value":1}}}}'

    def test_json_encode_int_key(self):
        c = MapCrdt("abc", {1: Record(Hlc(MILLIS, 0, "abc"), 1, hlc_now())})
        assert c.to_json() == f'{{"1":{{"hlc":"{ISO}-0000-abc","value":1}}}}'

    def test_json_encode_custom_node_id(self):
        c = MapCrdt("abc", {"x": Record(Hlc(MILLIS, 0, 1), 0, hlc_now())})
        assert c.to_json() == f'{{"x":{{"hlc":"{ISO}-0000-1","value":0}}}}'

    def test_json_decode_string_key(self):
        c = MapCrdt("abc")
        m = CrdtJson.decode(f'{{"x":{{"hlc":"{ISO}-0000-abc","value":1}}}}', hlc_now(), WALL)
        c.put_records(m)
        assert c.record_map() == {"x": Record(Hlc(MILLIS, 0, "abc"), 1, hlc_now())}

    def test_json_decode_int_key(self):
        c = MapCrdt("abc")
        m = CrdtJson.decode(f'{{"1":{{"hlc":"{ISO}-0000-abc","value":1}}}}', hlc_now(), WALL,
                            key_decoder=int)
        c.put_records(m)
        assert c.record_map() == {1: Record(Hlc(MILLIS, 0, "abc"), 1, hlc_now())}

    def test_json_decode_custom_node_id(self):
        c = MapCrdt("abc")
        m = CrdtJson.decode(f'{{"x":{{"hlc":"{ISO}-0000-1","value":0}}}}', hlc_now(), WALL,
                            node_id_decoder=int)
        c.put_records(m)
        assert c.record_map() == {"x": Record(Hlc(MILLIS, 0, 1), 0, hlc_now())}


class TestDeltaSubsets:                                      # :203-235
    h1, h2, h3 = Hlc(MILLIS, 0, "abc"), Hlc(MILLIS + 1, 0, "abc"), Hlc(MILLIS + 2, 0, "abc")

    def setup_method(self):
        self.c = MapCrdt("abc", {"x": Record(self.h1, 1, self.h1), "y": Record(self.h2, 2, self.h2)})

    def test_null(self):
        assert len(self.c.record_map()) == 2

    def test_since_h1(self):
        assert len(self.c.record_map(self.h1)) == 2

    def test_since_h2(self):
        assert len(self.c.record_map(self.h2)) == 1

    def test_since_h3(self):
        assert len(self.c.record_map(self.h3)) == 0


def _sync(local, remote, wall):                              # map_crdt_test.dart:273-279
    time = local.canonical_time
    remote.merge(local.record_map(), wall)
    local.merge(remote.record_map(time), wall)


class TestDeltaSync:                                         # :237-270
    def setup_method(self):
        self.a, self.b, self.c = MapCrdt("a"), MapCrdt("b"), MapCrdt("c")
        self.a.put("x", 1, WALL)
        self.b.put("x", 2, WALL + 100)

    def test_in_order(self):
        _sync(self.a, self.c, WALL + 200)
        _sync(self.b, self.c, WALL + 200)
        assert (self.a.get("x"), self.b.get("x"), self.c.get("x")) == (1, 2, 2)

    def test_reverse_order(self):
        _sync(self.b, self.c, WALL + 200)
        _sync(self.a, self.c, WALL + 200)
        _sync(self.b, self.c, WALL + 200)
        assert (self.a.get("x"), self.b.get("x"), self.c.get("x")) == (2, 2, 2)


# ---------------------------------------------------------- crdt_test.dart
class TestBasic:                                             # crdt_test.dart:12-93
    def setup_method(self):
        self.c = MapCrdt("abc")

    def test_node_id(self):
        assert self.c.node_id == "abc"

    def test_empty(self):
        assert self.c.is_empty and self.c.length == 0 and self.c.map == {} and self.c.keys == []

    def test_one_record(self):
        self.c.put("x", 1, WALL)
        assert (not self.c.is_empty, self.c.length, self.c.map, self.c.keys, self.c.values) == \
            (True, 1, {"x": 1}, ["x"], [1])

    def test_empty_after_delete(self):
        self.c.put("x", 1, WALL)
        self.c.delete("x", WALL)
        assert self.c.is_empty and self.c.map == {}

    def test_update_existing(self):
        self.c.put("x", 1, WALL)
        self.c.put("x", 2, WALL)
        assert self.c.get("x") == 2

    def test_put_many(self):
        self.c.put_all({"x": 2, "y": 3}, WALL)
        assert (self.c.get("x"), self.c.get("y")) == (2, 3)

    def test_delete_value(self):
        self.c.put("x", 1, WALL)
        self.c.put("y", 2, WALL)
        self.c.delete("x", WALL)
        assert self.c.is_deleted("x") is True and self.c.is_deleted("y") is False
        assert self.c.get("x") is None and self.c.get("y") == 2

    def test_clear(self):
        self.c.put("x", 1, WALL)
        self.c.put("y", 2, WALL)
        self.c.clear(WALL)
        assert self.c.is_deleted("x") and self.c.is_deleted("y")

    def test_watch_all(self):                                # crdt_test.dart:98-113
        self.c.put("x", 1, WALL)
        self.c.put("y", 2, WALL)
        assert self.c.events == [("x", 1), ("y", 2)]


# ------------------------------------------- source-only semantics (unpinned by tests)
class TestMergeStampAndCanonical:
    """crdt.dart:82,86-87,93: every winner gets the canonical after the WHOLE recv loop;
    the canonical then advances by one send()."""

    def test_uniform_modified_stamp_and_send(self):
        c = MapCrdt("local")
        m = {"a": Record(Hlc(WALL - 5, 3, "r1"), 1, hlc_now()),
             "b": Record(Hlc(WALL - 2, 1, "r1"), 2, hlc_now())}
        c.merge(m, WALL)
        stamp = Hlc(WALL - 2, 1, "local").logical_time
        assert c.get_record("a").modified.logical_time == stamp
        assert c.get_record("b").modified.logical_time == stamp
        assert c.canonical_time.logical_time == Hlc(WALL, 0, "x").logical_time   # send: wall ahead

    def test_recv_failure_leaves_map_untouched(self):
        c = MapCrdt("local")
        m = {"a": Record(Hlc(WALL - 5, 0, "r1"), 1, hlc_now()),
             "b": Record(Hlc(WALL + 60001, 0, "r1"), 2, hlc_now())}
        with pytest.raises(ClockDriftException):
            c.merge(m, WALL)
        assert len(m) == 2 and c.record_map() == {}
        assert c.canonical_time.logical_time == Hlc(WALL - 5, 0, "x").logical_time
