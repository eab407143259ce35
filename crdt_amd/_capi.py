"""ctypes binding of ``include/crdt_merge.h`` (``crdt_amd/libcrdt_mi355x.so``).

The shared library is the only compute path: if it is missing, or there is no
gfx950 device, every operation raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CRDT_LIB_PATH") or os.path.join(_HERE, "libcrdt_mi355x.so")   # override: profiling builds

CRDT_OK = 0
CRDT_CLOCK_DRIFT = 1
CRDT_DUPLICATE_NODE = 2
CRDT_OVERFLOW = 3
CRDT_E_INVALID = -1
CRDT_E_HIP = -2
CRDT_E_NOMEM = -3
CRDT_E_KEY_RANGE = -4
CRDT_E_NO_DEVICE = -5
CRDT_E_COMM = -6

CRDT_MEM_HOST = 0
CRDT_MEM_DEVICE = 1
CRDT_NULL_VALUE = 0xFFFFFFFF


class CrdtBatch(ctypes.Structure):
    _fields_ = [("key_id", ctypes.c_void_p), ("lt", ctypes.c_void_p), ("rank", ctypes.c_void_p),
                ("val", ctypes.c_void_p), ("millis", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("n_changesets", ctypes.c_uint32), ("mem", ctypes.c_int32)]


class CrdtResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("n_stored", ctypes.c_uint32),
                ("exc_changeset", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("exc_index", ctypes.c_uint64), ("canonical_lt", ctypes.c_int64),
                ("drift_ms", ctypes.c_int64), ("counter", ctypes.c_int64),
                ("n_present", ctypes.c_uint64), ("n_won", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved"}


class CrdtTiming(ctypes.Structure):
    _fields_ = [("scan_ms", ctypes.c_double), ("clock_ms", ctypes.c_double),
                ("apply_ms", ctypes.c_double), ("apply_launches", ctypes.c_uint32),
                ("apply_total", ctypes.c_uint32), ("total_ms", ctypes.c_double),
                ("route_ms", ctypes.c_double), ("part1_ms", ctypes.c_double), ("part2_ms", ctypes.c_double),
                ("resolve_ms", ctypes.c_double), ("part1_records", ctypes.c_uint64),
                ("sent_bytes", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


# crdt_comm_ops callbacks (include/crdt_merge.h)
ALL_REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32,
                                 ctypes.c_void_p)
ALL_GATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                 ctypes.c_void_p)
ALL_TO_ALL_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p),
                                 ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint32),
                                 ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p)


class CrdtCommOps(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("mem", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("all_reduce_i64", ALL_REDUCE_FN), ("all_gather_i64", ALL_GATHER_FN),
                ("all_to_all_v", ALL_TO_ALL_FN)]


COMM_ID_BYTES = 128
ABI_VERSION = 5                            # include/crdt_merge.h CRDT_ABI_VERSION

_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_INT = ctypes.c_int

# name -> (restype, argtypes); exactly the entry points include/crdt_merge.h declares
SIGNATURES = {
    "crdt_abi_version": (_INT, []),
    "crdt_status_string": (ctypes.c_char_p, [_INT]),
    "crdt_device_count": (_INT, [_P]),
    "crdt_create": (_INT, [_INT, _U32, _U64, _P]),
    "crdt_destroy": (None, [_P]),
    "crdt_reserve": (_INT, [_P, _U64]),
    "crdt_capacity": (_INT, [_P, _P]),
    "crdt_set_local_rank": (_INT, [_P, _U32]),
    "crdt_get_canonical": (_INT, [_P, _P]),
    "crdt_set_canonical": (_INT, [_P, _I64]),
    "crdt_put_rows": (_INT, [_P, _P, _P, _P, _P, _P, _U64, _I32]),
    "crdt_read_rows": (_INT, [_P, _P, _U64, _P, _P, _P, _P, _I32]),
    "crdt_modified_since": (_INT, [_P, _U64, _I64, _P, _P]),
    "crdt_clear_rows": (_INT, [_P, _U64, _U64]),
    "crdt_remap_ranks": (_INT, [_P, _U64, _P, _U32]),
    "crdt_put_stamped": (_INT, [_P, _P, _P, _U64, _I64, _I32, _P]),
    "crdt_refresh_canonical": (_INT, [_P, _U64, _P]),
    "crdt_merge": (_INT, [_P, _P, _I64, _P, _P]),
    "crdt_comm_unique_id": (_INT, [_P]),
    "crdt_comm_init_rccl": (_INT, [_P, _U32, _U32, _P]),
    "crdt_comm_init_ops": (_INT, [_P, _U32, _U32, _P]),
    "crdt_comm_info": (_INT, [_P, _P, _P]),
    "crdt_comm_free": (_INT, [_P]),
    "crdt_set_presharded": (_INT, [_P, _INT]),
    "crdt_set_comm_timeout": (_INT, [_P, _U32]),
    "crdt_comm_state": (_INT, [_P, _P, _P]),
    "crdt_set_merge_path": (_INT, [_P, _INT]),
    "crdt_set_counts": (_INT, [_P, _INT]),
    "crdt_set_rank_bound": (_INT, [_P, _U32]),
    "crdt_reserve_scratch": (_INT, [_P, _U64]),
    "crdt_set_row_bytes": (_INT, [_P, _U32]),
    "crdt_last_plan": (_INT, [_P, _P]),
    "crdt_route_tune_info": (_INT, [_P, _P, _P]),
    "crdt_place_info": (_INT, [_P, _P, _P, _P, _P]),
    "crdt_last_path": (_INT, [_P, _P]),
    "crdt_set_timing": (_INT, [_P, _INT]),
    "crdt_get_timing": (_INT, [_P, _P]),
}


class NativeLibraryMissing(RuntimeError):
    pass


_lib = None


def load():
    """Load the gfx950 library (raises loudly if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64 (same SONAME
    # libamdhip64.so.7).  Loaded first, it is the one our library binds to; loaded after us
    # it would bring a second runtime whose device enumeration then fails.
    if os.environ.get("CRDT_AMD_NO_TORCH") != "1" and "torch" not in sys.modules:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.crdt_abi_version() != ABI_VERSION:      # struct layouts below are ABI_VERSION's
        raise NativeLibraryMissing(f"{LIB_PATH} has ABI {lib.crdt_abi_version()}, the bindings ABI {ABI_VERSION}:"
                                   " rebuild it")
    _lib = lib
    return lib


def status_string(status: int) -> str:
    return load().crdt_status_string(status).decode()


def device_count() -> int:
    n = ctypes.c_int(0)
    load().crdt_device_count(ctypes.byref(n))
    return n.value
