"""TEST INFRASTRUCTURE ONLY — ctypes binding of the columnar C restatement.

Used by tests/ (as the bit-exact checker), __graft_entry__.smoke() and the
``cpu_baseline`` leg of bench.py.  Never imported by the product package.
See ``merge_oracle.c`` for the reference lines each function follows.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")

ROW_DTYPE = np.dtype([("lt", "<i8"), ("rank", "<u4"), ("val", "<u4"), ("mod", "<i8"), ("aux", "<i8")])
assert ROW_DTYPE.itemsize == 32

ABSENT_MOD = np.int64(np.frombuffer(b"\x80" * 8, dtype="<i8")[0])


class OrResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("n_stored", ctypes.c_uint32),
                ("exc_changeset", ctypes.c_uint32), ("pad", ctypes.c_uint32),
                ("exc_index", ctypes.c_uint64), ("canonical_lt", ctypes.c_int64),
                ("drift_ms", ctypes.c_int64), ("counter", ctypes.c_int64),
                ("n_present", ctypes.c_uint64), ("n_won", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "pad"}


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.or_merge.argtypes = [P, ctypes.c_uint64, P, ctypes.c_uint32, P, P, P, P, P, P,
                               ctypes.c_uint32, ctypes.c_int64, P, ctypes.c_int, P]
        L.or_merge.restype = ctypes.c_int
        L.or_merge_omp.argtypes = L.or_merge.argtypes
        L.or_merge_omp.restype = ctypes.c_int
        L.or_put_stamped.argtypes = [P, ctypes.c_uint64, P, ctypes.c_uint32, P, P, ctypes.c_uint64,
                                     ctypes.c_int64, P]
        L.or_put_stamped.restype = ctypes.c_int
        L.or_refresh.argtypes = [P, ctypes.c_uint64]
        L.or_refresh.restype = ctypes.c_int64
        L.or_modified_since.argtypes = [P, ctypes.c_uint64, ctypes.c_int64, P]
        L.or_modified_since.restype = ctypes.c_uint64
        L.or_clear_rows.argtypes = [P, ctypes.c_uint64, ctypes.c_uint64]
        L.or_send_scalar.argtypes = [ctypes.c_int64, ctypes.c_int64, P, P, P]
        L.or_send_scalar.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def new_table(capacity: int) -> np.ndarray:
    t = np.empty(capacity, dtype=ROW_DTYPE)
    t.view(np.uint8)[:] = 0x80
    return t


class OracleTable:
    """A columnar replica state checked by the C restatement."""

    def __init__(self, capacity: int, local_rank: int, canonical: int = 0):
        self.rows = new_table(capacity)
        self.local_rank = local_rank
        self._canon = np.array([canonical], dtype=np.int64)

    @property
    def canonical(self) -> int:
        return int(self._canon[0])

    @canonical.setter
    def canonical(self, v: int):
        self._canon[0] = v

    def put_rows(self, key, lt, rank, val, mod):
        key = np.asarray(key, dtype=np.uint32)
        self.rows["lt"][key] = lt
        self.rows["rank"][key] = rank
        self.rows["val"][key] = val
        self.rows["mod"][key] = mod
        self.rows["aux"][key] = 0

    def merge_omp(self, key, lt, rank, val, offsets, wall, millis=None, threads=0, want_flags=True):
        """oracle/merge_omp.c: the optimised multi-core baseline (same results as merge())."""
        key = np.ascontiguousarray(key, dtype=np.uint32)
        lt = np.ascontiguousarray(lt, dtype=np.int64)
        rank = np.ascontiguousarray(rank, dtype=np.uint32)
        val = np.ascontiguousarray(val, dtype=np.uint32)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        millis = None if millis is None else np.ascontiguousarray(millis, dtype=np.int64)
        flags = np.zeros(int(offsets[-1]), dtype=np.uint8) if want_flags else None
        res = OrResult()
        st = lib().or_merge_omp(_p(self.rows), len(self.rows), _p(self._canon), self.local_rank,
                                _p(key), _p(lt), _p(rank), _p(val), _p(millis), _p(offsets),
                                len(offsets) - 1, wall, _p(flags), int(threads), ctypes.byref(res))
        if st < 0:
            raise ValueError(f"oracle error {st}")
        return res, flags

    def merge(self, key, lt, rank, val, offsets, wall, millis=None, faithful=False, want_flags=True):
        key = np.ascontiguousarray(key, dtype=np.uint32)
        lt = np.ascontiguousarray(lt, dtype=np.int64)
        rank = np.ascontiguousarray(rank, dtype=np.uint32)
        val = np.ascontiguousarray(val, dtype=np.uint32)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        millis = None if millis is None else np.ascontiguousarray(millis, dtype=np.int64)
        flags = np.zeros(int(offsets[-1]), dtype=np.uint8) if want_flags else None
        res = OrResult()
        st = lib().or_merge(_p(self.rows), len(self.rows), _p(self._canon), self.local_rank,
                            _p(key), _p(lt), _p(rank), _p(val), _p(millis), _p(offsets),
                            len(offsets) - 1, wall, _p(flags), int(faithful), ctypes.byref(res))
        assert st == res.status or st < 0
        if st < 0:
            raise ValueError(f"oracle error {st}")
        return res, flags

    def put_stamped(self, key, val, wall):
        key = np.ascontiguousarray(key, dtype=np.uint32)
        val = np.ascontiguousarray(val, dtype=np.uint32)
        res = OrResult()
        lib().or_put_stamped(_p(self.rows), len(self.rows), _p(self._canon), self.local_rank,
                             _p(key), _p(val), len(key), wall, ctypes.byref(res))
        return res

    def refresh(self, n_rows: int) -> int:
        return int(lib().or_refresh(_p(self.rows), n_rows))

    def modified_since(self, n_rows: int, since: int) -> np.ndarray:
        out = np.empty(n_rows, dtype=np.uint32)
        n = lib().or_modified_since(_p(self.rows), n_rows, since, _p(out))
        return out[:n]


def send_scalar(c: int, wall: int):
    out = ctypes.c_int64()
    drift = ctypes.c_int64()
    counter = ctypes.c_int64()
    st = lib().or_send_scalar(c, wall, ctypes.byref(out), ctypes.byref(drift), ctypes.byref(counter))
    return st, out.value, drift.value, counter.value
