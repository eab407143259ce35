"""Native export (libcrdt_host.so: crdt_json_encode / crdt_json_canonical / crdt_json_split,
include/crdt_host.h) against the Python restatement of CrdtJson.encode + Record.toJson +
Hlc.toString (crdt_amd/crdt_json.py, crdt_amd/hlc.py; crdt_json.dart:8-17, record.dart:28-31,
hlc.dart:101-104).  CPU only; the device-backed MapCrdt.toJson is in test_gpu_api.py."""
import json

import numpy as np
import pytest

from crdt_amd import hostlib
from crdt_amd.crdt_json import CrdtJson, _default
from crdt_amd.hlc import Hlc
from crdt_amd.intern import NULL_HANDLE, KeyIndex, ValueStore
from crdt_amd.record import Record

pytestmark = pytest.mark.skipif(not hostlib.available(), reason="libcrdt_host.so not built")


def dumps(o):
    return json.dumps(o, separators=(",", ":"), ensure_ascii=False, default=_default)


def _canon(texts):
    bufs = [t.encode("utf-8", "surrogatepass") for t in texts]
    buf = b"".join(bufs)
    off = np.zeros(len(bufs), np.uint64)
    off[1:] = np.cumsum([len(b) for b in bufs])[:-1]
    return hostlib.canonical(buf, off, np.array([len(b) for b in bufs], np.uint32))


YES = ['1', '-5', '0', '12345678901234567890123', 'true', 'false', 'null', '""', '"abc"', '"a\\"b"',
       '"back\\\\slash"', '"\\n\\r\\t\\b\\f"', '"\\u0001\\u001f"', '"é漢字😀"', '"\x7f"', '[]', '{}', '[1,2,[3]]',
       '{"a":1,"b":{"c":[true,null]}}', '{"":0}', '"/"']
NO = ['1.0', '1e5', '-0', '1E2', ' 1', '[1, 2]', '{"a": 1}', '"\\/"', '"\\u00e9"', '"\\u000a"', '"\\u001F"',
      '{"a":1,"a":2}', '"\\ud83d\\ude00"', 'NaN', 'Infinity', '01', '[1,]', '"abc', '', '{"a":1}x']


@pytest.mark.parametrize("t", YES)
def test_canonical_accepts_dumps_form(t):
    assert dumps(json.loads(t)) == t
    assert _canon([t])[0] == 1


@pytest.mark.parametrize("t", NO)
def test_canonical_rejects_what_dumps_rewrites(t):
    assert _canon([t])[0] == 0


def _random_value(rng, depth=0):
    r = rng.random()
    if depth > 3 or r < 0.3:
        return rng.choice([None, True, False, int(rng.integers(-10**12, 10**12)), "s", "é\"\\\n\x01",
                           "漢字😀", "", 1.5, -0.0, 1e-7, 10**30])
    if r < 0.6:
        return [_random_value(rng, depth + 1) for _ in range(int(rng.integers(0, 4)))]
    return {rng.choice(["a", "b", "é", "k\"", "\t", ""]) + str(int(rng.integers(0, 3))): _random_value(rng, depth + 1)
            for _ in range(int(rng.integers(0, 4)))}


def test_canonical_is_sound_on_random_values():
    rng = np.random.default_rng(11)
    texts = []
    for _ in range(3000):
        t = dumps(_random_value(rng))
        texts.append(t)
        # whitespace / escape perturbations of the same value
        texts.append(t.replace(",", ", ", 1))
        texts.append(t.replace("\\n", "\\u000a"))
        texts.append(t.replace("é", "\\u00e9"))
    ok = _canon(texts)
    for t, f in zip(texts, ok):
        if f:
            assert dumps(json.loads(t)) == t, t
    # every float-free dumps output is recognised

    def has_float(v):
        if isinstance(v, float):
            return True
        if isinstance(v, list):
            return any(has_float(x) for x in v)
        if isinstance(v, dict):
            return any(has_float(x) for x in v.values())
        return False
    for t, f in zip(texts[::4], ok[::4]):
        assert bool(f) != has_float(json.loads(t)), t


def test_split_array_spans():
    rng = np.random.default_rng(12)
    vals = [_random_value(rng) for _ in range(2000)]
    text = dumps(vals).encode("utf-8", "surrogatepass")
    off, ln = hostlib.split_array(text, len(vals))
    for v, o, n in zip(vals, off.tolist(), ln.tolist()):
        assert text[o:o + n].decode("utf-8", "surrogatepass") == dumps(v)
    off, ln = hostlib.split_array(b"[]", 0)
    assert len(off) == 0
    with pytest.raises(hostlib.Fallback):
        hostlib.split_array(b"[1,2]", 3)
    with pytest.raises(hostlib.Fallback):
        hostlib.split_array(dumps([float("nan")]).encode(), 1)


def _python_doc(keys, lt, node, node_ids, values, hlc_override=None):
    m = {}
    for i, k in enumerate(keys):
        h = hlc_override[i] if hlc_override and i in hlc_override else Hlc.fromLogicalTime(int(lt[i]), node_ids[node[i]])
        m[k] = Record(h, values[i], h)
    return CrdtJson.encode(m)


def test_encode_matches_restatement():
    rng = np.random.default_rng(13)
    ki = KeyIndex()
    names = ["k", "é", "漢字", "a\"b", "back\\slash", "tab\t", "😀", "nl\n", "\x01ctl", "\x7f"]
    keys = [names[i % len(names)] + str(i) for i in range(5000)]
    ids = np.array([ki.intern(k) for k in keys], np.uint32)
    node_ids = ["node_a", "", "a-b-c", "ünï", "q\"uote", "ctl\x02", 17]
    n = len(keys)
    lt = ((rng.integers(-60_000_000_000_000, 140_000_000_000_000, n)) << 16) + rng.integers(0, 0x10000, n)
    node = rng.integers(0, len(node_ids), n).astype(np.uint32)
    values = [_random_value(rng) for _ in range(n)]
    for i in range(0, n, 7):
        values[i] = None
    vs = ValueStore()
    handles = np.array([vs.put(v) for v in values], np.uint32)
    ptr, ln, keep = vs.texts(handles, dumps)
    override = {3: Hlc(5, 0x1FFFF, "x"), 10: Hlc(1_700_000_000_000, -3, "neg")}
    got = hostlib.encode(ki.native, ids, lt, node, node_ids, ptr, ln,
                         {r: str(h) for r, h in override.items()})
    assert got == _python_doc(keys, lt, node, node_ids, values, override)
    # row order is the caller's; a subset
    sub = np.arange(0, n, 3)
    got = hostlib.encode(ki.native, ids[sub], lt[sub], node[sub], node_ids, ptr[sub], ln[sub])
    assert got == _python_doc([keys[i] for i in sub], lt[sub], node[sub], node_ids, [values[i] for i in sub])
    assert hostlib.encode(ki.native, ids[:0], lt[:0], node[:0], node_ids, ptr[:0], ln[:0]) == "{}"


def test_encode_year_out_of_range_falls_back():
    ki = KeyIndex()
    i = ki.intern("k")
    with pytest.raises(hostlib.Fallback):
        hostlib.encode(ki.native, np.array([i], np.uint32), np.array([(-100_000_000_000_000 << 16)], np.int64),
                       np.zeros(1, np.uint32), ["n"], np.zeros(1, np.uint64), np.zeros(1, np.uint32))


def test_value_texts_reuse_raw_spans_and_match_dumps():
    rng = np.random.default_rng(14)
    vs = ValueStore()
    raw_texts = ['{"a":1}', '{"a": 1}', '1.5', '"é"', '"\\u00e9"', '[1,2]', 'null', '{"x":{"y":[true]}}', '-0', '7']
    buf = "".join(raw_texts).encode()
    lens = np.array([len(t.encode()) for t in raw_texts], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    lens[6] = 0                                                  # null span -> tombstone handle
    raw_h = vs.put_raw(buf, offs, lens)
    py_h = np.array([vs.put(_random_value(rng)) for _ in range(50)], np.uint32)
    vs.get(int(raw_h[0]))                                        # decoded: its Python object is exported
    vs.release(int(raw_h[9]))
    h2 = vs.put({"reused": True})                                # takes the freed raw handle
    handles = np.concatenate([raw_h[:9], py_h, [NULL_HANDLE, h2]]).astype(np.uint32)
    ptr, ln, keep = vs.texts(handles, dumps)
    import ctypes
    for h, p, n in zip(handles.tolist(), ptr.tolist(), ln.tolist()):
        if h == NULL_HANDLE:
            assert n == 0
            continue
        txt = ctypes.string_at(p, n).decode("utf-8", "surrogatepass")
        assert txt == dumps(vs.get(h)), (h, txt)
    # the canonical raw spans were not decoded to produce their text
    vs2 = ValueStore()
    hh = vs2.put_raw(buf, offs, lens)
    vs2.texts(hh, dumps)
    assert vs2._rawflag[int(hh[5])] == 1 and vs2._rawflag[int(hh[1])] == 0


def test_release_many_equals_release_loop():
    rng = np.random.default_rng(15)
    stores = [ValueStore(), ValueStore()]
    buf = b"".join(b'{"a":%d}' % i for i in range(500))
    lens = np.full(500, 7, np.uint32)
    lens[np.arange(500) >= 10] = [len(b'{"a":%d}' % i) for i in range(10, 500)]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    for vs in stores:
        vs.put_raw(buf, offs, lens)
        for i in range(300):
            vs.put(i)
        for h in range(0, 500, 7):
            vs.get(h)                                   # some raw values decoded
    drop = rng.choice(800, 400, replace=False).astype(np.uint32)
    drop = np.concatenate([drop, [NULL_HANDLE]]).astype(np.uint32)
    stores[0].release_many(drop)
    for h in drop.tolist():
        stores[1].release(h) if h != NULL_HANDLE else None
    a, b = stores
    assert a._values == b._values and bytes(a._rawflag) == bytes(b._rawflag)
    assert sorted(a._free) == sorted(b._free)
    assert [x[3] for x in a._raw] == [x[3] for x in b._raw]
    assert [x[0] is None for x in a._raw] == [x[0] is None for x in b._raw]


def test_parallel_export_equals_sequential(monkeypatch):
    """crdt_json_encode / crdt_json_canonical split over threads give the same bytes / flags."""
    rng = np.random.default_rng(16)
    ki = KeyIndex()
    keys = [f"k{i}\t{'é' * (i % 3)}" for i in range(3000)]
    ids = np.array([ki.intern(k) for k in keys], np.uint32)
    n = len(keys)
    lt = (rng.integers(0, 100_000_000_000_000, n) << 16) + rng.integers(0, 0x10000, n)
    node = rng.integers(0, 3, n).astype(np.uint32)
    vs = ValueStore()
    handles = np.array([vs.put(_random_value(rng)) for _ in range(n)], np.uint32)
    texts = [dumps(_random_value(rng)) for _ in range(n)]
    monkeypatch.setenv("CRDT_HOST_THREADS", "1")
    ptr, ln, keep = vs.texts(handles, dumps)
    want = hostlib.encode(ki.native, ids, lt, node, ["a", "b\"", "c"], ptr, ln)
    want_ok = _canon(texts)
    monkeypatch.setenv("CRDT_HOST_THREADS", "7")
    monkeypatch.setenv("CRDT_HOST_MIN_CHUNK", "100")
    assert hostlib.encode(ki.native, ids, lt, node, ["a", "b\"", "c"], ptr, ln) == want
    assert np.array_equal(_canon(texts), want_ok)
    bad = lt.copy()
    bad[2500] = -100_000_000_000_000 << 16                        # year < 0 in a later chunk
    with pytest.raises(hostlib.Fallback):
        hostlib.encode(ki.native, ids, bad, node, ["a", "b\"", "c"], ptr, ln)
