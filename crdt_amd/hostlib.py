"""ctypes binding of ``include/crdt_host.h`` (``crdt_amd/libcrdt_host.so``).

The native host half of sync: key interning, ``CrdtJson.decode`` of the wire format into
integer columns, batch ``Hlc.toString``, and ``CrdtJson.encode`` of a record map (export).  CPU code (g++), no GPU.  It decodes
the format the reference writes; for anything else it answers ``Fallback`` and the
caller uses the Python restatement (``crdt_json.py`` / ``hlc.py``), so results do not
depend on which decoder ran.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libcrdt_host.so")

OK, FALLBACK, E_INVALID, E_JSON, E_NOMEM = 0, 1, -1, -2, -3

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_INT = ctypes.c_int

SIGNATURES = {
    "crdt_host_abi_version": (_INT, []),
    "crdt_keys_create": (_P, []),
    "crdt_keys_destroy": (None, [_P]),
    "crdt_keys_size": (_U64, [_P]),
    "crdt_keys_find": (_INT, [_P, ctypes.c_char_p, _U64, _P]),
    "crdt_keys_intern": (_INT, [_P, ctypes.c_char_p, _U64, _P, _P]),
    "crdt_keys_export": (_INT, [_P, _U64, _U64, _P, _U64, _P]),
    "crdt_keys_bytes": (_U64, [_P, _U64, _U64]),
    "crdt_keys_truncate": (_INT, [_P, _U64]),
    "crdt_keys_clear": (_INT, [_P]),
    "crdt_json_decode": (_INT, [ctypes.c_char_p, _U64, _P, _P]),
    "crdt_decoded_free": (None, [_P]),
    "crdt_decoded_count": (_U64, [_P]),
    "crdt_decoded_node_count": (_U32, [_P]),
    "crdt_decoded_columns": (_INT, [_P, _P, _P, _P, _P, _P]),
    "crdt_decoded_node_bytes": (_U64, [_P]),
    "crdt_decoded_nodes": (_INT, [_P, _P, _U64, _P]),
    "crdt_hlc_format": (_INT, [_P, _P, _U64, _P, _P, _P, _U64, _P]),
    "crdt_json_encode": (_INT, [_P, _P, _P, _P, _P, _P, _P, _P, _U64, _P, _P, _U32, _P]),
    "crdt_text_data": (_P, [_P]),
    "crdt_text_size": (_U64, [_P]),
    "crdt_text_free": (None, [_P]),
    "crdt_json_canonical": (_INT, [_P, _P, _P, _U64, _P]),
    "crdt_json_split": (_INT, [_P, _U64, _U64, _P, _P]),
}


class Fallback(Exception):
    """Input outside the native fast path: decode it with the Python restatement."""


_lib = None
_missing = False


def load():
    """The host library, or None when it was not built (the Python restatement then runs)."""
    global _lib, _missing
    if _lib is not None or _missing:
        return _lib
    if not os.path.exists(LIB_PATH):
        _missing = True
        return None
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def available() -> bool:
    return load() is not None


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def utf8(s: str) -> bytes:
    return s.encode("utf-8", "surrogatepass")


class NativeKeys:
    """Owner of a ``crdt_keys`` table (UTF-8 key string <-> dense id)."""

    def __init__(self):
        self._lib = load()
        self._h = self._lib.crdt_keys_create()
        if not self._h:
            raise MemoryError("crdt_keys_create")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and self._lib is not None:
            self._lib.crdt_keys_destroy(h)

    def __len__(self):
        return int(self._lib.crdt_keys_size(self._h))

    def find(self, b: bytes):
        v = ctypes.c_uint32(0)
        return v.value if self._lib.crdt_keys_find(self._h, b, len(b), ctypes.byref(v)) == 0 else None

    def intern(self, b: bytes) -> int:
        v = ctypes.c_uint32(0)
        st = self._lib.crdt_keys_intern(self._h, b, len(b), ctypes.byref(v), None)
        if st != OK:
            raise MemoryError(f"crdt_keys_intern: {st}")
        return v.value

    def export(self, first: int, count: int) -> list:
        if count <= 0:
            return []
        nb = int(self._lib.crdt_keys_bytes(self._h, first, count))
        buf = ctypes.create_string_buffer(max(nb, 1))
        offs = np.zeros(count + 1, np.uint64)
        st = self._lib.crdt_keys_export(self._h, first, count, buf, nb, _ptr(offs))
        if st != OK:
            raise RuntimeError(f"crdt_keys_export: {st}")
        raw = buf.raw[:nb]
        o = offs.tolist()
        return [raw[o[i]:o[i + 1]].decode("utf-8", "surrogatepass") for i in range(count)]

    def truncate(self, n: int):
        self._lib.crdt_keys_truncate(self._h, n)

    def clear(self):
        self._lib.crdt_keys_clear(self._h)


def decode(js, keys: NativeKeys) -> dict:
    """``CrdtJson.decode`` fast path: {key_id, lt, node, val_off, val_len, nodes, buf}.

    Interns the document's keys into ``keys`` (new ids appended).  Raises ``Fallback``
    when the document is outside the fast path and ``ValueError`` for malformed JSON."""
    lib = load()
    if isinstance(js, str):
        try:
            buf = js.encode("utf-8")
        except UnicodeEncodeError:          # lone surrogates: the Python decoder handles them
            raise Fallback("surrogates") from None
    else:
        buf = bytes(js)
    out = ctypes.c_void_p(None)
    st = lib.crdt_json_decode(buf, len(buf), keys._h, ctypes.byref(out))
    if st == FALLBACK:
        raise Fallback("format")
    if st == E_JSON:
        raise ValueError("FormatException: malformed JSON")
    if st != OK:
        raise RuntimeError(f"crdt_json_decode: {st}")
    d = out.value
    try:
        n = int(lib.crdt_decoded_count(d))
        key_id = np.empty(n, np.uint32)
        lt = np.empty(n, np.int64)
        node = np.empty(n, np.uint32)
        val_off = np.empty(n, np.uint64)
        val_len = np.empty(n, np.uint32)
        lib.crdt_decoded_columns(d, _ptr(key_id), _ptr(lt), _ptr(node), _ptr(val_off), _ptr(val_len))
        nn = int(lib.crdt_decoded_node_count(d))
        nb = int(lib.crdt_decoded_node_bytes(d))
        nbuf = ctypes.create_string_buffer(max(nb, 1))
        noffs = np.zeros(nn + 1, np.uint64)
        lib.crdt_decoded_nodes(d, nbuf, nb, _ptr(noffs))
        raw = nbuf.raw[:nb]
        o = noffs.tolist()
        nodes = [raw[o[i]:o[i + 1]].decode("utf-8") for i in range(nn)]
    finally:
        lib.crdt_decoded_free(d)
    return {"key_id": key_id, "lt": lt, "node": node, "val_off": val_off, "val_len": val_len, "nodes": nodes,
            "buf": buf}


def hlc_strings(lt: np.ndarray, node: np.ndarray, node_ids: list) -> list:
    """``Hlc.fromLogicalTime(lt, node_ids[node]).toString()`` for a batch (hlc.dart:101-104);
    raises ``Fallback`` for years outside 0000..9999."""
    lib = load()
    n = len(lt)
    if n == 0:
        return []
    enc = [utf8(str(x)) for x in node_ids]
    nbuf = b"".join(enc)
    noffs = np.zeros(len(enc) + 1, np.uint64)
    np.cumsum([len(e) for e in enc], out=noffs[1:])
    lt = np.ascontiguousarray(lt, np.int64)
    node = np.ascontiguousarray(node, np.uint32)
    cap = 30 * n + (int(np.sum(np.diff(noffs)[node])) if len(enc) else 0)
    out = ctypes.create_string_buffer(max(cap, 1))
    ooffs = np.zeros(n + 1, np.uint64)
    st = lib.crdt_hlc_format(_ptr(lt), _ptr(node), n, nbuf, _ptr(noffs), out, cap, _ptr(ooffs))
    if st == FALLBACK:
        raise Fallback("year")
    if st != OK:
        raise RuntimeError(f"crdt_hlc_format: {st}")
    raw = out.raw[:int(ooffs[-1])]
    o = ooffs.tolist()
    return [raw[o[i]:o[i + 1]].decode("utf-8", "surrogatepass") for i in range(n)]


def address(b: bytes) -> int:
    """Address of a bytes object's buffer (valid while the object lives)."""
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value or 0


def canonical(buf: bytes, off: np.ndarray, length: np.ndarray) -> np.ndarray:
    """uint8 flags: span k of buf is what json.dumps(json.loads(span)) writes (exportable as is)."""
    lib = load()
    off = np.ascontiguousarray(off, np.uint64)
    length = np.ascontiguousarray(length, np.uint32)
    ok = np.zeros(len(off), np.uint8)
    if len(off):
        st = lib.crdt_json_canonical(buf, _ptr(off), _ptr(length), len(off), _ptr(ok))
        if st != OK:
            raise RuntimeError(f"crdt_json_canonical: {st}")
    return ok


def split_array(text: bytes, count: int):
    """(off, len) of the ``count`` elements of the JSON array ``text``; raises Fallback."""
    lib = load()
    off = np.zeros(count, np.uint64)
    ln = np.zeros(count, np.uint32)
    st = lib.crdt_json_split(text, len(text), count, _ptr(off), _ptr(ln))
    if st == FALLBACK:
        raise Fallback("split")
    if st != OK:
        raise RuntimeError(f"crdt_json_split: {st}")
    return off, ln


def encode(keys: NativeKeys, key_id, lt, node, node_ids: list, val_ptr, val_len, hlc_text: dict | None = None) -> str:
    """``CrdtJson.encode`` of rows (key_id, Hlc.fromLogicalTime(lt, node_ids[node]), value text at
    val_ptr / val_len, 0 = null); ``hlc_text`` {row: str} overrides a row's hlc.  Raises Fallback
    for years outside 0000..9999."""
    lib = load()
    n = len(key_id)
    key_id = np.ascontiguousarray(key_id, np.uint32)
    lt = np.ascontiguousarray(lt, np.int64)
    node = np.ascontiguousarray(node, np.uint32)
    val_ptr = np.ascontiguousarray(val_ptr, np.uint64)
    val_len = np.ascontiguousarray(val_len, np.uint32)
    enc = [utf8(str(x)) for x in node_ids]
    nbuf = b"".join(enc) or b"\0"
    noffs = np.zeros(len(enc) + 1, np.uint64)
    np.cumsum([len(e) for e in enc], out=noffs[1:])
    keep = []
    hp = hl = None
    if hlc_text:
        hp = np.zeros(n, np.uint64)
        hl = np.zeros(n, np.uint32)
        for row, txt in hlc_text.items():
            b = utf8(txt)
            keep.append(b)
            hp[row] = address(b)
            hl[row] = len(b)
    out = ctypes.c_void_p(None)
    st = lib.crdt_json_encode(keys._h, _ptr(key_id), _ptr(lt), _ptr(node), _ptr(hp) if hp is not None else None,
                              _ptr(hl) if hl is not None else None, _ptr(val_ptr), _ptr(val_len), n, nbuf,
                              _ptr(noffs), len(enc), ctypes.byref(out))
    if st == FALLBACK:
        raise Fallback("year")
    if st != OK:
        raise RuntimeError(f"crdt_json_encode: {st}")
    t = out.value
    try:
        raw = ctypes.string_at(lib.crdt_text_data(t), int(lib.crdt_text_size(t)))
    finally:
        lib.crdt_text_free(t)
    return raw.decode("utf-8", "surrogatepass")
