"""Host-side logic of the product (no GPU): the Hlc mirror against the same
reference KATs, interning / rank order / remap tables, the JSON codec, and the
C-ABI library: it loads and exports exactly what include/crdt_merge.h declares."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from crdt_amd import _capi
from crdt_amd.crdt_json import CrdtJson
from crdt_amd.hlc import (ClockDriftException, DuplicateNodeException, Hlc, OverflowException,
                          iso_from_millis, millis_from_iso)
from crdt_amd.intern import NULL_HANDLE, KeyIndex, NodeRanks, ValueStore
from crdt_amd.record import Record

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MILLIS = 1000000000000
ISO = "2001-09-09T01:46:40.000Z"
LT = 65536000000000066


# ------------------------------------------------------------------ Hlc mirror
def test_hlc_constants_and_codec():                       # hlc_test.dart:4-43
    h = Hlc(MILLIS, 0x42, "abc")
    assert h.logicalTime == LT
    assert Hlc(MILLIS * 1000, 0x42, "abc") == h
    assert Hlc.fromLogicalTime(LT, "abc") == h
    assert Hlc.parse(f"{ISO}-0042-abc") == h
    assert str(h) == f"{ISO}-0042-abc"
    assert Hlc.parse(f"{ISO}-0042-1", int) == Hlc(MILLIS, 0x42, 1)
    assert h.pack() == "00cre66i9s001uabc"                 # hlc_test.dart:7,170-173
    u = Hlc.unpack("00cre66i9s001uabc")
    assert (u.millis, u.counter, u.nodeId) == (MILLIS, 0x42, "abc")


def test_hlc_compare_send_recv():                         # hlc_test.dart:137-267
    h = Hlc(MILLIS, 0x42, "abc")
    assert h.compareTo(Hlc(MILLIS, 0x42, "abd")) == -1 and h.compareTo(Hlc(MILLIS, 0x42, "abb")) == 1
    assert Hlc.send(Hlc(MILLIS + 1, 0x42, "abc"), millis=MILLIS).counter == 0x43
    assert Hlc.send(Hlc(MILLIS - 1, 0x42, "abc"), millis=MILLIS).counter == 0
    with pytest.raises(ClockDriftException):
        Hlc.send(Hlc(MILLIS + 60001, 0, "abc"), millis=MILLIS)
    with pytest.raises(OverflowException):
        Hlc.send(Hlc(MILLIS, 0xFFFF, "abc"), millis=MILLIS)
    c = Hlc.parse(f"{ISO}-0042-abc")
    assert Hlc.recv(c, Hlc(MILLIS - 1, 0x42, "abcd"), millis=MILLIS) == c
    assert Hlc.recv(c, Hlc(MILLIS, 0x42, "abc"), millis=MILLIS) == c
    with pytest.raises(DuplicateNodeException):
        Hlc.recv(c, Hlc(MILLIS + 1, 0, "abc"), millis=MILLIS)
    with pytest.raises(ClockDriftException):
        Hlc.recv(c, Hlc(MILLIS + 60001, 0x42, "abcd"), millis=MILLIS)


def test_iso_matches_oracle():
    from oracle.crdt_oracle import iso_from_millis as o_iso, millis_from_iso as o_parse
    rng = np.random.default_rng(0)
    for ms in list(rng.integers(-(10 ** 14), 10 ** 14, 500)) + [0, -1, 253402300799999, 253402300800000]:
        ms = int(ms)
        assert iso_from_millis(ms) == o_iso(ms)
        assert millis_from_iso(iso_from_millis(ms)) == ms == o_parse(o_iso(ms))
    for s in ["2001-09-09T01:46:40Z", "2001-09-09 01:46:40.1234567+02:00", "20010909T014640", "2001-13-01"]:
        assert millis_from_iso(s) == o_parse(s)


# ------------------------------------------------------------------ interning
def test_node_ranks_follow_dart_string_order_and_remap():
    nr = NodeRanks()
    assert nr.register(["m", "z"]) is None
    lut = nr.register(["a"])                              # sorts first: every rank moves
    assert lut == [1, 2] and nr.rank("a") == 0
    assert nr.register(["zz"]) is None                     # sorts last: nothing moves
    from oracle.crdt_oracle import dart_compare
    names = ["abc", "abd", "abcd", "ab", "\U0001F600", "～", "Z", "a"]
    nr2 = NodeRanks()
    nr2.register(names)
    for a in names:
        for b in names:
            assert (nr2.rank(a) > nr2.rank(b)) - (nr2.rank(a) < nr2.rank(b)) == dart_compare(a, b)


def test_key_index_truncate_and_values():
    k = KeyIndex()
    assert [k.intern(x) for x in "abcab"] == [0, 1, 2, 0, 1]
    k.truncate(1)
    assert k.get("b") is None and k.intern("c") == 1
    v = ValueStore()
    assert v.put(None) == NULL_HANDLE
    h = v.put({"x": 1})
    v.release(h)
    assert v.put(5) == h and v.get(h) == 5


def test_crdt_json_roundtrip():
    m = {"x": Record(Hlc(MILLIS, 0, "abc"), 1, Hlc(0, 0, "abc")), 1: Record(Hlc(MILLIS, 2, "q"), None, None)}
    js = CrdtJson.encode(m)
    assert js == f'{{"x":{{"hlc":"{ISO}-0000-abc","value":1}},"1":{{"hlc":"{ISO}-0002-q","value":null}}}}'
    back = CrdtJson.decode(js, Hlc(0, 0, "abc"), millis=MILLIS)
    assert back == {"x": m["x"], "1": m[1]}


# ------------------------------------------------------------------ C-ABI library
def _header_functions():
    txt = open(os.path.join(ROOT, "include", "crdt_merge.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"^\s*(?:int|void|const char\*)\s+(crdt_\w+)\s*\(", txt, flags=re.M))


def test_library_exports_every_header_symbol():
    lib = _capi.load()
    declared = _header_functions()
    assert declared == set(_capi.SIGNATURES), declared ^ set(_capi.SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (crdt_\w+)", out))
    assert declared <= exported, declared - exported
    for name in declared:
        assert getattr(lib, name) is not None
    assert lib.crdt_abi_version() == _capi.ABI_VERSION == 5
    assert _capi.status_string(1) == "clock drift"


def test_library_has_gfx950_code_object():
    data = open(_capi.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_abi_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of the header structs have the C compiler's sizes and offsets."""
    src = tmp_path / "sz.c"
    fields = {"crdt_result": _capi.CrdtResult, "crdt_batch": _capi.CrdtBatch, "crdt_timing": _capi.CrdtTiming}
    lines = ['#include "crdt_merge.h"', "#include <stdio.h>", "#include <stddef.h>", "int main(void){"]
    for cname, cls in fields.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src.write_text("\n".join(lines))
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    for cname, cls in fields.items():
        assert int(got[cname]) == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(cls, f).offset, (cname, f)
    from oracle.oracle_c import OrResult
    assert ctypes.sizeof(OrResult) == ctypes.sizeof(_capi.CrdtResult)


def test_no_device_means_loud_failure():
    """On a box with no GPU the product refuses to run (no CPU fallback)."""
    if _capi.device_count() > 0:
        pytest.skip("a GPU is visible")
    from crdt_amd import CrdtNativeError, MapCrdt
    with pytest.raises(CrdtNativeError):
        MapCrdt("abc")


def test_product_never_imports_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "crdt_amd")):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, flags=re.M), f


def test_workload_generators_cpu():
    """Invariants of the BASELINE.json generators (run on CPU torch at small sizes)."""
    import torch
    from crdt_amd.workload import gen_cfg3, gen_cfg5
    wl = gen_cfg5(device="cpu", K=10_007, n_delta=1000, deltas=6, inject="drift", inject_at=(3, 499))
    own, offs = wl["owned"], wl["owned_offsets"]
    for d in range(6):
        k = own["key"][int(offs[d]):int(offs[d + 1])]
        assert torch.unique(k).numel() == k.numel() and int(k.min()) >= 0 and int(k.max()) < 10_007
    assert np.all(np.diff(wl["walls"]) > 0)
    frac = float((own["val"] == -1).double().mean())
    assert 0.07 < frac < 0.13
    assert int(own["lt"][3 * 1000 + 499]) >> 16 == int(wl["walls"][3]) + 60_001
    wl3 = gen_cfg3(device="cpu", total=20_000, K=50_000, R=16)
    assert torch.unique(wl3["owned"]["lt"]).numel() <= 32
    o3 = wl3["owned_offsets"]
    for j in range(16):
        k = wl3["owned"]["key"][int(o3[j]):int(o3[j + 1])]
        assert torch.unique(k).numel() == k.numel()


def test_iso_edge_strings_match_independent_oracle():
    """The oracle's date maths (datetime ordinals + 400-year shifts, a hand-written scanner) is
    independent of crdt_amd/hlc.py's (civil-from-days, regular expression): they must agree on
    DateTime's whole range and on the grammar's edges, errors included."""
    from oracle.crdt_oracle import iso_from_millis as o_iso, millis_from_iso as o_parse
    rng = np.random.default_rng(7)
    edges = [8640000000000000, -8640000000000000, -62135596800001, -62135596800000, 253402300800000]
    for ms in [int(x) for x in rng.integers(-8640000000000000, 8640000000000000, 3000)] + edges:
        assert iso_from_millis(ms) == o_iso(ms)
        assert millis_from_iso(o_iso(ms)) == ms
    strings = ["2001-09-09T01:46:40Z", "20010909T014640", "+002001-01-01", "-0001-12-31T23:59:59.999Z",
               "2020-02-31", "2001-13-01", "2001-09-09T01:46", "2001-09-09T01", "2001-09-09T0146Z",
               "2001-09-09T01:46:40,5-0130", "2001-09-09T01:46:40 Z", "275760-09-13T00:00:00Z",
               "-271821-04-20T00:00:00Z", "2001-9-09", "abc", "2001-09-09T", "2001-09-09T01:4",
               "2001-09-09T01:46:40.", "1234567-01-01", "275760-09-13T00:00:00.001Z"]
    for s in strings:
        got = []
        for f in (millis_from_iso, o_parse):
            try:
                got.append(f(s))
            except ValueError:
                got.append("error")
        assert got[0] == got[1], (s, got)
