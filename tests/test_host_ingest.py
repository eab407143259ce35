"""Native host ingest (libcrdt_host.so, include/crdt_host.h) against the Python
restatement of CrdtJson.decode / Record.fromJson / Hlc.parse / Hlc.toString
(crdt_amd/crdt_json.py, crdt_amd/hlc.py, themselves pinned by the reference KATs in
test_oracle_kat.py).  CPU only."""
import ctypes
import json
import os
import re
import subprocess

import numpy as np
import pytest

from crdt_amd import hostlib
from crdt_amd.crdt_json import CrdtJson
from crdt_amd.hlc import Hlc, iso_from_millis
from crdt_amd.intern import NULL_HANDLE, KeyIndex, ValueStore

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WALL = 1_700_000_000_000

pytestmark = pytest.mark.skipif(not hostlib.available(), reason="libcrdt_host.so not built")


def test_library_exports_every_header_symbol():
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "crdt_host.h")).read(), flags=re.S)
    declared = set(re.findall(r"^\s*(?:int|void|uint64_t|uint32_t|crdt_keys\*|const char\*)\s+(crdt_\w+)\s*\(", txt, flags=re.M))
    assert declared == set(hostlib.SIGNATURES), declared ^ set(hostlib.SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", hostlib.LIB_PATH], capture_output=True, text=True).stdout
    assert declared <= set(re.findall(r" T (crdt_\w+)", out))
    assert ctypes.CDLL(hostlib.LIB_PATH).crdt_host_abi_version() == 2


def _native_records(dec, keys: KeyIndex):
    ks = keys.keys
    out = {}
    for i in range(len(dec["key_id"])):
        o, ln = int(dec["val_off"][i]), int(dec["val_len"][i])
        v = None if ln == 0 else json.loads(dec["buf"][o:o + ln])
        out[ks[int(dec["key_id"][i])]] = (int(dec["lt"][i]), dec["nodes"][int(dec["node"][i])], v)
    return out


def _python_records(js):
    m = CrdtJson.decode(js, Hlc(0, 0, "local"), millis=WALL)
    return {k: (r.hlc.logicalTime, r.hlc.nodeId, r.value) for k, r in m.items()}


def _random_doc(rng, n, n_nodes=5, dup_frac=0.05):
    nodes = [f"node-{i}" for i in range(n_nodes)] + ["", "a-b-c", "ünï-ñode", "漢字", "x y"]
    keys = []
    parts = []
    for i in range(n):
        if keys and rng.random() < dup_frac:
            k = keys[int(rng.integers(len(keys)))]
        else:
            k = f"k{i}" if rng.random() < 0.7 else rng.choice(["é", "漢字", "a\"b", "back\\slash", "tab\t", "😀", "nl\n"]) + str(i)
            keys.append(k)
        ms = int(rng.integers(-2_000_000_000_000, 4_000_000_000_000))
        counter = int(rng.integers(0, 0x10000))
        node = nodes[int(rng.integers(len(nodes)))]
        hlc = str(Hlc(ms, counter, node))
        if rng.random() < 0.2:
            hlc = hlc[:25] + hlc[25:29].lower() + hlc[29:]
        r = rng.random()
        if r < 0.15:
            val = None
        elif r < 0.3:
            val = {"nested": [1, 2.5, {"x": "y"}], "s": "é\u0001"}
        elif r < 0.5:
            val = int(rng.integers(-1 << 60, 1 << 60))
        elif r < 0.6:
            val = [True, False, None, 1e300, -0.0]
        else:
            val = f"v{i}"
        rec = {"hlc": hlc, "value": val}
        if rng.random() < 0.05:
            rec = {"hlc": hlc}                           # missing value -> tombstone
        if rng.random() < 0.05:
            rec = {"extra": 1, "value": val, "hlc": hlc, "more": [1]}
        parts.append((k, rec))
    # serialise by hand so duplicate keys really appear twice in the text
    body = ",".join(json.dumps(k, ensure_ascii=bool(rng.random() < 0.5)) + ":" +
                    json.dumps(r, ensure_ascii=bool(rng.random() < 0.5), separators=(",", ":") if rng.random() < 0.5
                               else (", ", ": ")) for k, r in parts)
    return "{" + body + "}"


@pytest.mark.parametrize("seed", range(6))
def test_decode_matches_restatement(seed):
    rng = np.random.default_rng(seed)
    js = _random_doc(rng, int(rng.integers(0, 400)))
    keys = KeyIndex()
    keys.intern("k0")                                  # a pre-existing key keeps its id
    dec = hostlib.decode(js, keys.native)
    assert _native_records(dec, keys) == _python_records(js)
    # new keys were appended in first-occurrence order
    py = list(_python_records(js).keys())
    assert keys.keys[1:] == [k for k in py if k != "k0"][:len(keys) - 1]


def test_decode_edge_values():
    hl = str(Hlc(WALL, 0x1F, "n"))
    js = json.dumps({"a": {"hlc": hl, "value": None}, "b": {"hlc": hl, "value": 0}, "c": {"hlc": hl, "value": ""},
                     "d": {"hlc": hl, "value": []}, "e": {"hlc": hl, "value": {}}, "f": {"value": "x", "hlc": hl}})
    keys = KeyIndex()
    assert _native_records(hostlib.decode(js, keys.native), keys) == _python_records(js)
    js = '{}'
    assert len(hostlib.decode(js, KeyIndex().native)["key_id"]) == 0
    # duplicate field inside a record: last wins; duplicate top-level key: first position, last record
    h2 = str(Hlc(WALL + 5, 2, "m"))
    js = '{"x": {"hlc": "%s", "hlc": "%s", "value": 1}, "y": {"hlc": "%s", "value": 2}, "x": {"hlc": "%s", "value": 3}}' % (
        hl, h2, hl, hl)
    keys = KeyIndex()
    dec = hostlib.decode(js, keys.native)
    assert keys.keys == ["x", "y"] and _native_records(dec, keys) == _python_records(js)


def test_iso_field_normalisation_matches_restatement():
    """DateTime.parse normalises out-of-range fields (month 13, day 00, hour 24, ...)."""
    for iso in ["2021-13-01T00:00:00.000Z", "2021-00-31T24:60:60.999Z", "0000-01-01T00:00:00.000Z",
                "9999-12-31T23:59:59.999Z", "2020-02-30T12:00:00.000Z", "1969-12-31T23:59:59.999Z",
                "2000-99-99T99:99:99.999Z"]:
        js = json.dumps({"k": {"hlc": iso + "-00FF-nd", "value": 1}})
        keys = KeyIndex()
        assert _native_records(hostlib.decode(js, keys.native), keys) == _python_records(js), iso


@pytest.mark.parametrize("doc", [
    '{"k": {"hlc": "2021-01-01T00:00:00.000Z-0001-a:b", "value": 1}}',          # ':' in node id
    '{"k": {"hlc": "2021-01-01T00:00:00.000Z-1F-n", "value": 1}}',              # 2-digit counter
    '{"k": {"hlc": "2021-01-01T00:00:00Z-0001-n", "value": 1}}',                # other ISO form
    '{"k": {"hlc": "2021-01-01 00:00:00.000Z-0001-n", "value": 1}}',
    '{"k": {"hlc": "+2021-01-01T00:00:00.000Z-0001-n", "value": 1}}',
    '{"k": {"value": 1}}',                                                       # no hlc
    '{"k": {"hlc": 5, "value": 1}}',                                             # hlc not a string
    '{"k": [1, 2]}',                                                             # record not an object
    '{"k": {"hlc": "2021-01-01T00:00:00.000Z-0001-n", "value": NaN}}',          # Python-only literal
    '{"\\ud800": {"hlc": "2021-01-01T00:00:00.000Z-0001-n", "value": 1}}',      # lone surrogate
])
def test_outside_fast_path_falls_back(doc):
    keys = KeyIndex()
    keys.intern("pre")
    with pytest.raises(hostlib.Fallback):
        hostlib.decode(doc, keys.native)
    assert keys.keys == ["pre"] and len(keys) == 1                # nothing interned


@pytest.mark.parametrize("doc", ['{"k": {"hlc": "2021-01-01T00:00:00.000Z-0001-n", "value": 1}',
                                 '{"k" {}}', '[1]', '{"k": {"hlc": "x\u0001", "value": 1}}', '{} x', ''])
def test_malformed_json_is_an_error(doc):
    keys = KeyIndex()
    with pytest.raises((ValueError, hostlib.Fallback)):
        hostlib.decode(doc, keys.native)
    assert len(keys) == 0


def test_key_index_native_and_python_modes():
    k = KeyIndex()
    assert k.native is not None
    ids = [k.intern(x) for x in ["a", "b", "a", "漢", "\ud800"]]
    assert ids == [0, 1, 0, 2, 3] and len(k) == 4
    assert k.get("漢") == 2 and k.get("zz") is None and k.get(7) is None
    k.truncate(2)
    assert k.keys == ["a", "b"] and k.get("漢") is None
    assert k.intern(7) == 2 and k.native is None                 # first non-string key: Python mode
    assert k.get("b") == 1 and k.get(7) == 2 and k.keys == ["a", "b", 7]


def test_value_store_raw_batches():
    vs = ValueStore()
    h0 = vs.put("python")
    buf = b'[1,2] "s" {"a":null} 3.5'
    hs = vs.put_raw(buf, np.array([0, 6, 0, 10, 21]), np.array([5, 3, 0, 10, 3]))
    assert hs[2] == NULL_HANDLE
    assert [vs.get(int(h)) for h in hs] == [[1, 2], "s", None, {"a": None}, 3.5]
    vs.release(int(hs[0]))
    assert vs.put("reuse") == int(hs[0]) and vs.get(h0) == "python"
    vs.compact([h0])
    assert len(vs) == 1


@pytest.mark.parametrize("seed", range(3))
def test_hlc_format_matches_to_string(seed):
    rng = np.random.default_rng(seed)
    n = 500
    ms = rng.integers(-62_000_000_000_000, (1 << 47) - 1, n)     # |millis| < 2^47: lt fits int64
    counter = rng.integers(0, 0x10000, n)
    lt = (ms << 16) + counter
    nodes = ["n", "", "ünï", "a-b", "😀"]
    node = rng.integers(0, len(nodes), n).astype(np.uint32)
    got = hostlib.hlc_strings(lt, node, nodes)
    exp = [str(Hlc.fromLogicalTime(int(lt[i]), nodes[int(node[i])])) for i in range(n)]
    assert got == exp
    with pytest.raises(hostlib.Fallback):                         # year 10000+: Dart's +YYYYYY form
        hostlib.hlc_strings(np.array([-(63_000_000_000_000 << 16)]), np.array([0], np.uint32), ["n"])
    assert iso_from_millis(-63_000_000_000_000).startswith("-0")


# ------------------------------------------------------- parallel decode (large documents)
def _decode_with(js, threads, par_min, pre=("k0",)):
    old = {k: os.environ.get(k) for k in ("CRDT_HOST_THREADS", "CRDT_HOST_PAR_MIN")}
    os.environ["CRDT_HOST_THREADS"] = str(threads)
    os.environ["CRDT_HOST_PAR_MIN"] = str(par_min)
    try:
        keys = KeyIndex()
        for k in pre:
            keys.intern(k)
        try:
            dec = hostlib.decode(js, keys.native)
        except hostlib.Fallback:
            return "fallback", list(keys.keys)
        except ValueError:
            return "json", list(keys.keys)
        cols = {k: np.asarray(v).tolist() for k, v in dec.items() if k not in ("buf", "nodes")}
        return cols, dec["nodes"], list(keys.keys)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _adversarial_doc(rng, n):
    """Records whose strings hold the `},"` split pattern, whitespace between tokens, escapes."""
    hl = [str(Hlc(WALL + i, i % 7, f"n{i % 5}")) for i in range(50)]
    parts = []
    for i in range(n):
        k = rng.choice(["k%d" % i, 'q},"%d' % i, "e\\u00e9%d" % i, "k%d" % (i // 3)])
        v = rng.choice(['"},\\"x\\":{\\"hlc\\":\\""', '{"a": "},\\"b\\": 1"}', "[1, 2]", "null", '"plain"',
                        '{"z":{"y":[{},{"x":"},"}]}}'])
        ws = rng.choice(["", " ", "\n  "])
        parts.append(f'{ws}"{k}"{ws}:{ws}{{"hlc":{ws}"{hl[i % 50]}",{ws}"value":{ws}{v}}}{ws}')
    return "{" + ",".join(parts) + "}"


@pytest.mark.parametrize("seed", range(8))
def test_parallel_decode_equals_sequential(seed):
    rng = np.random.default_rng(100 + seed)
    js = _random_doc(rng, int(rng.integers(200, 1500))) if seed % 2 else _adversarial_doc(rng, int(rng.integers(200, 1500)))
    want = _decode_with(js, 1, 1 << 60)
    for threads in (2, 3, 7, 16):
        assert _decode_with(js, threads, 0) == want, threads
    if want[0] not in ("fallback", "json"):
        keys = KeyIndex()
        keys.intern("k0")
        assert _native_records(hostlib.decode(js, keys.native), keys) == _python_records(js)


@pytest.mark.parametrize("where", [0.1, 0.5, 0.9])
def test_parallel_decode_errors_match_sequential(where):
    rng = np.random.default_rng(7)
    js = _random_doc(rng, 800, dup_frac=0.0)
    cut = int(len(js) * where)
    i = js.index('"hlc"', cut)
    bad_hlc = js[:i] + '"hlc":"2021-01-01T00:00:00Z-0001-n","x' + js[i + 5:]     # fallback form
    broken = js[:cut] + "}{" + js[cut:]                                          # malformed
    for doc in (bad_hlc, broken, js[:-1], js + " x"):
        want = _decode_with(doc, 1, 1 << 60)
        for threads in (2, 5, 16):
            assert _decode_with(doc, threads, 0) == want
