"""The drop-in API on the GPU, written like the reference's own tests
(test/map_crdt_test.dart, test/crdt_test.dart), plus randomized operation
sequences checked against the object-level oracle."""
import json

import numpy as np
import pytest

from crdt_amd import (ClockDriftException, CrdtJson, DuplicateNodeException, Hlc, MapCrdt,
                      OverflowException, Record)

pytestmark = pytest.mark.gpu

MILLIS = 1000000000000
ISO = "2001-09-09T01:46:40.000Z"
WALL = 1700000000000


def hlc_now(node="abc", wall=WALL):
    return Hlc(wall, 0, node)


def crdt(node="abc", seed=None):
    return MapCrdt(node, seed, clock=lambda: WALL)


class TestBasic:                                     # crdt_test.dart:12-93
    def test_node_id(self, gpu_device):
        assert crdt().nodeId == "abc"

    def test_empty(self, gpu_device):
        c = crdt()
        assert c.isEmpty and c.length == 0 and c.map == {} and c.keys == [] and c.values == []

    def test_one_record(self, gpu_device):
        c = crdt()
        c.put("x", 1)
        assert (c.isEmpty, c.length, c.map, c.keys, c.values) == (False, 1, {"x": 1}, ["x"], [1])

    def test_empty_after_deleted(self, gpu_device):
        c = crdt()
        c.put("x", 1)
        c.delete("x")
        assert c.isEmpty and c.length == 0 and c.map == {}

    def test_update_existing(self, gpu_device):
        c = crdt()
        c.put("x", 1)
        c.put("x", 2)
        assert c.get("x") == 2

    def test_put_many(self, gpu_device):
        c = crdt()
        c.putAll({"x": 2, "y": 3})
        assert (c.get("x"), c.get("y")) == (2, 3)

    def test_delete_value(self, gpu_device):
        c = crdt()
        c.put("x", 1)
        c.put("y", 2)
        c.delete("x")
        assert c.isDeleted("x") is True and c.isDeleted("y") is False
        assert c.get("x") is None and c.get("y") == 2

    def test_clear(self, gpu_device):
        c = crdt()
        c.put("x", 1)
        c.put("y", 2)
        c.clear()
        assert c.isDeleted("x") and c.isDeleted("y") and c.get("x") is None

    def test_watch(self, gpu_device):               # crdt_test.dart:98-130
        c = crdt()
        w_all, w_y = c.watch(), c.watch(key="y")
        c.put("x", 1)
        c.put("y", 2)
        assert w_all.events == [("x", 1), ("y", 2)] and w_y.events == [("y", 2)]


class TestSeed:                                      # map_crdt_test.dart:17-31
    def test_seed_item(self, gpu_device):
        c = crdt(seed={"x": Record(hlc_now(), 1, hlc_now())})
        assert c.get("x") == 1 and c.canonicalTime.logicalTime == 0

    def test_seed_and_put(self, gpu_device):
        c = crdt(seed={"x": Record(hlc_now(), 1, hlc_now())})
        c.put("x", 2)
        assert c.get("x") == 2


class TestMerge:                                     # map_crdt_test.dart:33-103
    def test_merge_older(self, gpu_device):
        c = crdt()
        c.put("x", 2)
        c.merge({"x": Record(Hlc(MILLIS - 1, 0, "xyz"), 1, hlc_now())})
        assert c.get("x") == 2

    def test_merge_very_old(self, gpu_device):
        c = crdt()
        c.put("x", 2)
        c.merge({"x": Record(Hlc(0, 0, "xyz"), 1, hlc_now())})
        assert c.get("x") == 2

    def test_merge_newer(self, gpu_device):
        c = crdt()
        c.put("x", 1)
        c.merge({"x": Record(Hlc(WALL + 1, 0, "xyz"), 2, hlc_now())}, wall=WALL + 1)
        assert c.get("x") == 2

    def test_disambiguate_using_node_id(self, gpu_device):
        c = crdt()
        c.merge({"x": Record(Hlc(MILLIS, 0, "nodeA"), 1, hlc_now())})
        c.merge({"x": Record(Hlc(MILLIS, 0, "nodeB"), 2, hlc_now())})
        assert c.get("x") == 2

    def test_merge_same(self, gpu_device):
        c = crdt()
        c.put("x", 2)
        ts = c.getRecord("x").hlc
        c.merge({"x": Record(ts, 1, hlc_now())})
        assert c.get("x") == 2

    def test_merge_older_newer_counter(self, gpu_device):
        c = crdt()
        c.put("x", 2)
        c.merge({"x": Record(Hlc(MILLIS - 1, 2, "xyz"), 1, hlc_now())})
        assert c.get("x") == 2

    def test_merge_same_newer_counter(self, gpu_device):
        c = crdt()
        c.put("x", 1)
        c.merge({"x": Record(Hlc(c.getRecord("x").hlc.millis, 2, "xyz"), 2, hlc_now())})
        assert c.get("x") == 2

    def test_merge_new_item(self, gpu_device):
        c = crdt()
        m = {"x": Record(Hlc(WALL, 0, "xyz"), 2, hlc_now())}
        c.merge(m)
        assert c.recordMap() == m

    def test_merge_deleted_item(self, gpu_device):
        c = crdt()
        c.put("x", 1)
        c.merge({"x": Record(Hlc(WALL + 1, 0, "xyz"), None, hlc_now())}, wall=WALL + 1)
        assert c.isDeleted("x") is True

    def test_update_hlc_on_merge(self, gpu_device):
        c = crdt()
        c.put("x", 1)
        c.merge({"y": Record(Hlc(MILLIS - 1, 0, "xyz"), 2, hlc_now())})
        assert c.values == [1, 2]

    def test_merge_mutates_map_to_winners(self, gpu_device):   # crdt.dart:80-85
        c = crdt()
        c.put("x", 5)
        m = {"x": Record(Hlc(0, 0, "xyz"), 1, hlc_now()), "y": Record(Hlc(1, 0, "xyz"), 2, hlc_now())}
        c.merge(m)
        assert list(m) == ["y"]

    def test_duplicate_node_raises_and_leaves_state(self, gpu_device):
        c = crdt()
        c.put("x", 1)
        before = c.canonicalTime
        m = {"y": Record(Hlc(WALL + 5, 0, "abc"), 2, hlc_now())}
        with pytest.raises(DuplicateNodeException) as e:
            c.merge(m)
        assert str(e.value) == "Duplicate node: abc"
        assert c.get("y") is None and not c.containsKey("y") and list(m) == ["y"]
        assert c.canonicalTime == before

    def test_drift_raises(self, gpu_device):
        c = crdt()
        with pytest.raises(ClockDriftException) as e:
            c.merge({"y": Record(Hlc(WALL + 60001, 0, "q"), 2, hlc_now())})
        assert e.value.drift == 60001

    def test_send_overflow_after_store(self, gpu_device):
        """Hlc.send raises after putRecords (crdt.dart:90-93): the record stays stored and the
        canonical stays at the received clock."""
        c = crdt()
        with pytest.raises(OverflowException) as e:
            c.merge({"z": Record(Hlc(WALL, 0xFFFF, "q"), 3, hlc_now())}, wall=WALL)
        assert e.value.counter == 0x10000
        assert c.get("z") == 3
        assert c.canonicalTime.logicalTime == (WALL << 16) + 0xFFFF


class TestSerialization:                            # map_crdt_test.dart:105-201
    def test_json_encode(self, gpu_device):
        hlcNow = hlc_now()
        c = crdt(seed={"x": Record(Hlc(MILLIS, 0, "abc"), 1, hlcNow)})
        assert c.toJson() == f'{{"x":{{"hlc":"{ISO}-0000-abc","value":1}}}}'
        c2 = MapCrdt("abc", {1: Record(Hlc(MILLIS, 0, "abc"), 1, hlcNow)})
        assert c2.toJson() == f'{{"1":{{"hlc":"{ISO}-0000-abc","value":1}}}}'

    def test_json_decode_put_records(self, gpu_device):
        c = crdt()
        c.putRecords(CrdtJson.decode(f'{{"x":{{"hlc":"{ISO}-0000-abc","value":1}}}}', hlc_now()))
        assert c.recordMap() == {"x": Record(Hlc(MILLIS, 0, "abc"), 1, hlc_now())}

    def test_merge_json_example(self, gpu_device):   # example/crdt_example.dart
        c = crdt("node_id")
        c.put("a", 1)
        remote = json.dumps({"a": {"hlc": str(Hlc(WALL + 1, 0, "another_nodeId")), "value": 2}})
        c.mergeJson(remote, wall=WALL + 1)
        assert c.get("a") == 2


class TestDeltaSync:                                 # map_crdt_test.dart:203-279
    def test_delta_subsets(self, gpu_device):
        h1, h2, h3 = Hlc(MILLIS, 0, "abc"), Hlc(MILLIS + 1, 0, "abc"), Hlc(MILLIS + 2, 0, "abc")
        c = crdt(seed={"x": Record(h1, 1, h1), "y": Record(h2, 2, h2)})
        assert [len(c.recordMap(modifiedSince=h)) for h in (None, h1, h2, h3)] == [2, 2, 1, 0]

    @staticmethod
    def _sync(local, remote, wall):
        time = local.canonicalTime
        remote.merge(local.recordMap(), wall=wall)
        local.merge(remote.recordMap(modifiedSince=time), wall=wall)

    def test_in_order_and_reverse(self, gpu_device):
        for order in ("in", "reverse"):
            a, b, cc = MapCrdt("a"), MapCrdt("b"), MapCrdt("c")
            a.put("x", 1, wall=WALL)
            b.put("x", 2, wall=WALL + 100)
            if order == "in":
                self._sync(a, cc, WALL + 200)
                self._sync(b, cc, WALL + 200)
                assert (a.get("x"), b.get("x"), cc.get("x")) == (1, 2, 2)
            else:
                self._sync(b, cc, WALL + 200)
                self._sync(a, cc, WALL + 200)
                self._sync(b, cc, WALL + 200)
                assert (a.get("x"), b.get("x"), cc.get("x")) == (2, 2, 2)


def _random_ops_vs_oracle(seed, n_ops=40):
    from oracle import crdt_oracle as O
    rng = np.random.default_rng(seed)
    nodes = ["local", "a", "m", "zz", "b0", "~"]
    dev, ora = MapCrdt("local"), O.MapCrdt("local")
    wall = WALL
    for _ in range(n_ops):
        wall += int(rng.integers(0, 3))
        op = rng.integers(0, 5)
        try:
            if op == 0:
                k, v = f"k{rng.integers(0, 30)}", int(rng.integers(0, 100))
                e1 = e2 = None
                try:
                    dev.put(k, v, wall=wall)
                except Exception as ex:  # noqa: BLE001
                    e1 = type(ex).__name__
                try:
                    ora.put(k, v, wall)
                except Exception as ex:  # noqa: BLE001
                    e2 = type(ex).__name__
                assert e1 == e2
            else:
                R = int(rng.integers(1, 4))
                css_d, css_o = [], []
                for _ in range(R):
                    keys = rng.choice(40, int(rng.integers(0, 15)), replace=False)
                    cs_d, cs_o = {}, {}
                    for k in keys:
                        ms = wall + int(rng.integers(-50, 8)) + (60001 if rng.random() < 0.01 else 0)
                        node = nodes[int(rng.integers(0, len(nodes)))] if rng.random() < 0.97 else "local"
                        cnt = int(rng.integers(0, 3))
                        val = None if rng.random() < 0.15 else int(rng.integers(0, 1000))
                        cs_d[f"k{k}"] = Record(Hlc(ms, cnt, node), val, Hlc(0, 0, "local"))
                        cs_o[f"k{k}"] = O.Record(O.Hlc(ms, cnt, node), val, O.Hlc(0, 0, "local"))
                    css_d.append(cs_d)
                    css_o.append(cs_o)
                e1 = e2 = None
                try:
                    dev.mergeAll(css_d, wall=wall)
                except Exception as ex:  # noqa: BLE001
                    e1 = (type(ex).__name__, str(ex))
                try:
                    for cs in css_o:
                        ora.merge(cs, wall)
                except Exception as ex:  # noqa: BLE001
                    e2 = (type(ex).__name__, str(ex))
                assert e1 == e2
                for a, b in zip(css_d, css_o):
                    assert list(a) == list(b)           # same removeWhere mutation
        finally:
            pass
        rm_d, rm_o = dev.recordMap(), ora.record_map()
        assert list(rm_d) == list(rm_o)                 # same LinkedHashMap order
        for k in rm_o:
            assert rm_d[k].hlc.logicalTime == rm_o[k].hlc.logical_time
            assert rm_d[k].hlc.nodeId == rm_o[k].hlc.node_id
            assert rm_d[k].value == rm_o[k].value
            assert rm_d[k].modified.logicalTime == rm_o[k].modified.logical_time
        assert dev.canonicalTime.logicalTime == ora.canonical_time.logical_time


@pytest.mark.parametrize("seed", range(6))
def test_random_operation_sequences(gpu_device, seed):
    _random_ops_vs_oracle(seed)


# ------------------------------------------------------ native mergeJson ingest
def _json_ops_vs_oracle(seed, n_ops=30, force_python=False):
    """mergeJson through libcrdt_host.so (or the Python decoder) against the oracle's
    merge_json: same state, same exceptions, same watch events."""
    from oracle import crdt_oracle as O
    rng = np.random.default_rng(seed)
    nodes = ["local", "a", "m-x", "zz", "b0", "ü", ""]
    dev, ora = MapCrdt("local"), O.MapCrdt("local")
    if force_python:
        dev._native_ingest = lambda: False
    w = dev.watch()
    wall = WALL
    paths = set()
    for _ in range(n_ops):
        wall += int(rng.integers(0, 3))
        if rng.random() < 0.25:
            k, v = f"k{rng.integers(0, 30)}", int(rng.integers(0, 100))
            e1 = e2 = None
            try:
                dev.put(k, v, wall=wall)
            except Exception as ex:  # noqa: BLE001
                e1 = type(ex).__name__
            try:
                ora.put(k, v, wall)
            except Exception as ex:  # noqa: BLE001
                e2 = type(ex).__name__
            assert e1 == e2
        else:
            recs = {}
            for k in rng.choice(40, int(rng.integers(0, 15)), replace=False):
                ms = wall + int(rng.integers(-50, 8)) + (60001 if rng.random() < 0.01 else 0)
                node = nodes[int(rng.integers(0, len(nodes)))] if rng.random() < 0.97 else "local"
                val = None if rng.random() < 0.15 else [int(rng.integers(0, 1000)), {"s": "é"}]
                recs[f"k{k}"] = O.Record(O.Hlc(ms, int(rng.integers(0, 3)), node), val, O.Hlc(0, 0, "local"))
            doc = O.CrdtJson.encode(recs)
            e1 = e2 = None
            try:
                dev.mergeJson(doc, wall=wall)
            except Exception as ex:  # noqa: BLE001
                e1 = (type(ex).__name__, str(ex))
            paths.add(getattr(dev, "last_ingest", None))
            try:
                ora.merge_json(doc, wall)
            except Exception as ex:  # noqa: BLE001
                e2 = (type(ex).__name__, str(ex))
            assert e1 == e2
        rm_d, rm_o = dev.recordMap(), ora.record_map()
        assert list(rm_d) == list(rm_o)
        for k in rm_o:
            assert rm_d[k].hlc.logicalTime == rm_o[k].hlc.logical_time
            assert rm_d[k].hlc.nodeId == rm_o[k].hlc.node_id
            assert rm_d[k].value == rm_o[k].value
            assert rm_d[k].modified.logicalTime == rm_o[k].modified.logical_time
        assert dev.canonicalTime.logicalTime == ora.canonical_time.logical_time
    assert [(k, v) for k, v in w] == list(ora.events)
    # export: native toJson (device compaction + libcrdt_host encode) == the oracle's
    for since in (None, O.Hlc(WALL + 3, 0, "local"), O.Hlc(wall + 50, 0, "local")):
        mine = None if since is None else Hlc(since.millis, since.counter, since.node_id)
        assert dev.toJson(modifiedSince=mine) == ora.to_json(modified_since=since)
        assert dev.last_export == "native"
    return paths


@pytest.mark.parametrize("seed", range(4))
def test_merge_json_native_ingest_vs_oracle(gpu_device, seed):
    assert _json_ops_vs_oracle(seed) == {"native"}


def test_merge_json_python_decoder_vs_oracle(gpu_device):
    assert _json_ops_vs_oracle(11, force_python=True) == {"python"}


def _cfg1_docs(n_keys=10_000, seed=0xC0FFEE01):
    """configs[0]: node_a local (putAll of every key, then a put per key), node_b's
    10k-record JSON with 50 % key overlap; millis = base + U[0,2000), counter U[0,4)."""
    from oracle import crdt_oracle as O
    rng = np.random.default_rng(seed)
    base = 1_735_689_600_000
    keys = [f"k{i:05d}" for i in range(n_keys)]
    remote_keys = keys[: n_keys // 2] + [f"k{i:05d}" for i in range(n_keys, n_keys + n_keys // 2)]
    recs = {}
    for k in remote_keys:
        recs[k] = O.Record(O.Hlc(base + int(rng.integers(0, 2000)), int(rng.integers(0, 4)), "node_b"),
                           int(rng.integers(0, 1 << 30)), O.Hlc(0, 0, "node_b"))
    return base, keys, O.CrdtJson.encode(recs)


def test_cfg1_merge_json_10k_keys_vs_oracle(gpu_device):
    from oracle import crdt_oracle as O
    base, keys, doc = _cfg1_docs()
    dev, ora = MapCrdt("node_a"), O.MapCrdt("node_a")
    dev.putAll({k: 0 for k in keys}, wall=base)
    ora.put_all({k: 0 for k in keys}, base)
    for i, k in enumerate(keys[::7]):
        dev.put(k, i, wall=base + 1 + i % 1500)
        ora.put(k, i, base + 1 + i % 1500)
    wall = base + 10_000
    dev.mergeJson(doc, wall=wall)
    ora.merge_json(doc, wall)
    assert dev.last_ingest == "native"
    rm_d, rm_o = dev.recordMap(), ora.record_map()
    assert list(rm_d) == list(rm_o) and len(rm_o) == 15_000
    for k in rm_o:
        assert (rm_d[k].hlc.logicalTime, rm_d[k].hlc.nodeId, rm_d[k].value, rm_d[k].modified.logicalTime) == \
            (rm_o[k].hlc.logical_time, rm_o[k].hlc.node_id, rm_o[k].value, rm_o[k].modified.logical_time)
    assert dev.canonicalTime.logicalTime == ora.canonical_time.logical_time
    assert dev.toJson() == ora.to_json()


# ------------------------------------------------------------ native toJson export
def test_to_json_native_export_vs_restatement(gpu_device):
    """MapCrdt.toJson through crdt_modified_since + crdt_json_encode against the Python
    restatement (Crdt.toJson over recordMap): raw mergeJson values kept verbatim or re-encoded
    (whitespace, floats, escapes, repeated keys), put() values, tombstones, escaped keys and
    node ids, an Hlc outside the columnar form, modifiedSince."""
    from crdt_amd.crdt import Crdt
    c = MapCrdt("lo\"cal")
    c.put("plain", {"a": [1, 2, None]}, wall=WALL)
    c.put("flt", 1.5, wall=WALL)
    c.put("tab\tkey", "é\n", wall=WALL)
    c.putRecord("odd", Record(Hlc(WALL, 0x1FFFF, "z"), 3, Hlc(WALL, 0, "lo\"cal")))   # counter > 0xFFFF
    texts = ['{"a":1}', '{"a": 1}', '1.0', '"\\u00e9"', '{"k":1,"k":2}', 'null', '[true,false]', '-0', '1e3',
             '12345678901234567890']
    doc = "{" + ",".join(f'"r{i}":{{"hlc":"{Hlc(WALL + 1, i, "n" + str(i % 3))}","value":{t}}}'
                         for i, t in enumerate(texts)) + "}"
    c.mergeJson(doc, wall=WALL + 1)
    assert c.last_ingest == "native"
    c.mergeJson('{"sur":{"hlc":"%s","value":"\\ud83d\\ude00"}}' % Hlc(WALL + 1, 0, "n"), wall=WALL + 1)
    c.delete("plain", wall=WALL + 2)
    for since in (None, Hlc(WALL + 1, 0, "x"), Hlc(WALL + 2, 0, "x"), Hlc(WALL + 9, 0, "x")):
        want = Crdt.toJson(c, modifiedSince=since)
        got = c.toJson(modifiedSince=since)
        assert c.last_export == "native"
        assert got == want, (since, got, want)
    assert json.loads(c.toJson())["r3"]["value"] == "é"


def test_to_json_encoders_and_int_keys_take_restatement(gpu_device):
    c = MapCrdt("a")
    c.put(7, "x", wall=WALL)
    assert c.toJson() == f'{{"7":{{"hlc":"{Hlc(WALL, 0, "a")}","value":"x"}}}}'
    assert c.last_export == "python"
    s = MapCrdt("a")
    s.put("k", 1, wall=WALL)
    assert s.toJson(valueEncoder=lambda k, v: v + 1) == f'{{"k":{{"hlc":"{Hlc(WALL, 0, "a")}","value":2}}}}'
    assert s.last_export == "python"
    assert s.toJson() == f'{{"k":{{"hlc":"{Hlc(WALL, 0, "a")}","value":1}}}}'
    assert s.last_export == "native"


# ------------------------------------------------------------ parity edges (round 2)
def _state_equal(dev, ora):
    rm_d, rm_o = dev.recordMap(), ora.record_map()
    assert list(rm_d) == list(rm_o)
    for k in rm_o:
        assert (rm_d[k].hlc.logicalTime, rm_d[k].hlc.nodeId, rm_d[k].value, rm_d[k].modified.logicalTime) == \
            (rm_o[k].hlc.logical_time, rm_o[k].hlc.node_id, rm_o[k].value, rm_o[k].modified.logical_time), k
    assert dev.canonicalTime.logicalTime == ora.canonical_time.logical_time


@pytest.mark.parametrize("via", ["merge", "mergeJson"])
@pytest.mark.parametrize("first", ["\U0001F600", "～"])
def test_node_ids_ordered_by_utf16_not_utf8(gpu_device, via, first):
    """hlc.dart:158-161 breaks (lt) ties with String.compareTo: UTF-16 code units.  '😀' (U+1F600,
    surrogates D83D DE00) sorts BEFORE '～' (U+FF5E) in UTF-16 but after it in UTF-8 bytes and in
    code points; the same keys at the same lt from both nodes must resolve like the oracle."""
    from oracle import crdt_oracle as O
    second = "～" if first == "\U0001F600" else "\U0001F600"
    dev, ora = MapCrdt("local"), O.MapCrdt("local")
    for node in (first, second):
        recs = {f"k{i}": O.Record(O.Hlc(WALL - 10, i % 3, node), f"{node}{i}", O.Hlc(0, 0, "local")) for i in range(12)}
        if via == "merge":
            dev.merge({k: Record(Hlc(r.hlc.millis, r.hlc.counter, node), r.value, Hlc(0, 0, "local"))
                       for k, r in recs.items()}, wall=WALL)
        else:
            dev.mergeJson(O.CrdtJson.encode(recs), wall=WALL)
        ora.merge(recs, WALL) if via == "merge" else ora.merge_json(O.CrdtJson.encode(recs), WALL)
    _state_equal(dev, ora)
    assert {r.hlc.nodeId for r in dev.recordMap().values()} == {"～"}     # the UTF-16 larger one


def test_parsed_counter_over_0xffff_roundtrip(gpu_device):
    """An Hlc whose counter exceeds 0xFFFF (Hlc.parse of a wider hex counter, hlc.dart:39-46; lt =
    (millis << 16) + counter carries into millis, hlc.dart:16): merged, exported with toJson
    (Hlc.toString keeps millis and counter, hlc.dart:102-104), merged again into a fresh replica."""
    from oracle import crdt_oracle as O
    doc_in = '{"a":{"hlc":"%s-1FFFF-zz","value":1},"b":{"hlc":"%s-0003-zz","value":2}}' % (
        O.iso_from_millis(WALL - 5), O.iso_from_millis(WALL - 5))
    dev, ora = MapCrdt("local"), O.MapCrdt("local")
    dev.mergeJson(doc_in, wall=WALL)
    ora.merge_json(doc_in, WALL)
    _state_equal(dev, ora)
    out_d, out_o = dev.toJson(), ora.to_json()
    assert out_d == out_o and "-1FFFF-zz" in out_d
    dev2, ora2 = MapCrdt("other"), O.MapCrdt("other")
    dev2.mergeJson(out_d, wall=WALL)
    ora2.merge_json(out_o, WALL)
    _state_equal(dev2, ora2)
    assert dev2.toJson() == ora2.to_json()


@pytest.mark.parametrize("drift_at", [1, 2, 5])
def test_batch_with_wide_counter_then_normal_records(gpu_device, drift_at):
    """A changeset whose FIRST record is an Hlc with counter 0x1FFFF, followed by canonical-form
    records, one of them drifting (millis = wall + 60001): the device's millis column must hold
    every record's Hlc.millis (it was built from a half-filled lt column)."""
    from oracle import crdt_oracle as O
    dev, ora = MapCrdt("local"), O.MapCrdt("local")
    cs_d, cs_o = {}, {}
    for i in range(8):
        if i == 0:
            ms, cnt = WALL - 3, 0x1FFFF
        elif i == drift_at:
            ms, cnt = WALL + 60_001, 0
        else:
            ms, cnt = WALL - 1, i
        cs_d[f"k{i}"] = Record(Hlc(ms, cnt, "peer"), i, Hlc(0, 0, "local"))
        cs_o[f"k{i}"] = O.Record(O.Hlc(ms, cnt, "peer"), i, O.Hlc(0, 0, "local"))
    e1 = e2 = None
    try:
        dev.mergeAll([{"x": Record(Hlc(WALL - 9, 0, "peer"), 0, Hlc(0, 0, "local"))}, cs_d], wall=WALL)
    except Exception as ex:  # noqa: BLE001
        e1 = (type(ex).__name__, str(ex))
    try:
        ora.merge({"x": O.Record(O.Hlc(WALL - 9, 0, "peer"), 0, O.Hlc(0, 0, "local"))}, WALL)
        ora.merge(cs_o, WALL)
    except Exception as ex:  # noqa: BLE001
        e2 = (type(ex).__name__, str(ex))
    assert e1 == e2 and e1 is not None and e1[0] == "ClockDriftException"
    _state_equal(dev, ora)


@pytest.mark.parametrize("seed", [0, 1])
def test_merge_all_bulk_sorted_vs_oracle(gpu_device, seed):
    """MapCrdt.mergeAllBulk on the sorted path (order-free form, forced: the batch is small):
    recordMap (hlc, value, modified), canonical and the exception equal the oracle's sequential
    merges and MapCrdt.mergeAll's — ties on (lt, node) across changesets, tombstones, new and
    seeded keys, a drift in a late changeset for seed 1."""
    import random
    from oracle import crdt_oracle as O
    rnd = random.Random(seed)
    nodes = ["n%d" % k for k in range(6)]
    seed_o = {f"k{i}": O.Record(O.Hlc(WALL - 500 + rnd.randrange(8), rnd.randrange(3), rnd.choice(nodes)), i,
                                O.Hlc(WALL - 400, 0, "local")) for i in range(300)}
    css_o = []
    for j in range(70):
        cs = {}
        for x, i in enumerate(rnd.sample(range(600), 90)):
            ms = WALL - 300 + rnd.randrange(6)
            if seed == 1 and j == 55 and x == 40:
                ms = WALL + 60_001
            cs[f"k{i}"] = O.Record(O.Hlc(ms, rnd.randrange(3), rnd.choice(nodes)),
                                   None if rnd.random() < 0.1 else j * 1000 + i, O.Hlc(0, 0, "local"))
        css_o.append(cs)

    def to_dev(cs):
        return {k: Record(Hlc(r.hlc.millis, r.hlc.counter, r.hlc.node_id), r.value,
                          Hlc(r.modified.millis, r.modified.counter, r.modified.node_id)) for k, r in cs.items()}

    results = []
    for form in ("bulk", "all", "oracle"):
        if form == "oracle":
            m = O.MapCrdt("local", seed_o)
        else:
            m = MapCrdt("local", to_dev(seed_o))
            m._table.set_merge_path("sorted" if form == "bulk" else "gather")
        exc = None
        try:
            if form == "oracle":
                for cs in css_o:
                    m.merge(dict(cs), WALL)
            elif form == "bulk":
                m.mergeAllBulk([to_dev(cs) for cs in css_o], wall=WALL)
            else:
                m.mergeAll([to_dev(cs) for cs in css_o], wall=WALL)
        except Exception as ex:  # noqa: BLE001
            exc = type(ex).__name__
        if form == "bulk":
            assert m._table.last_path() == "sorted"
        results.append((m, exc))
    (bulk, e_b), (allm, e_a), (ora, e_o) = results
    assert e_b == e_a == e_o
    assert (e_o is not None) == (seed == 1)
    _state_equal(bulk, ora)
    _state_equal(allm, ora)


def test_c_abi_from_a_plain_c_host(gpu_device):
    """tests/c/abi_golden.c (built by build()): the library loaded by a C program with no Python
    or torch in it — golden cases through crdt_merge (gather + flags, sorted, a 1-rank sharded
    ctx over a loopback crdt_comm_ops table written in C, and sorted on 32-B rows with a declared
    rank bound), every row compared bit for bit."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tests", "c", "abi_golden")
    assert os.path.exists(exe), "build() compiles tests/c/abi_golden"
    env = {k: v for k, v in os.environ.items() if not k.startswith("PYTHON")}
    out = subprocess.run([exe, os.path.join(root, "tests", "golden", "abi_cases.bin")], capture_output=True,
                         text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "all equal" in out.stdout
