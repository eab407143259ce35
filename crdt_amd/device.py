"""``DeviceTable``: one replica's row table on one MI355X, over the C-ABI.

Columns may be numpy arrays (host memory, staged by the library) or torch
tensors already resident on the GPU (zero-copy: their device pointers are
passed straight through, ``CRDT_MEM_DEVICE``).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _capi
from ._capi import CrdtBatch, CrdtResult, CrdtTiming


class CrdtNativeError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = _capi.status_string(status) if status else "ok"
        super().__init__(f"{what}: {msg} ({status})" if what else f"{msg} ({status})")


def _is_torch(a) -> bool:
    return type(a).__module__.startswith("torch")


_NP_TYPES = {"u4": np.uint32, "i8": np.int64, "u1": np.uint8}
# torch dtypes a device column of each kind may have (same element width; the kernels
# reinterpret the bits, so int32 carries uint32 ids / handles)
_TORCH_KINDS = {"u4": ("int32", "uint32"), "i8": ("int64",), "u1": ("uint8", "bool")}


def check_device_tensor(t, kind: str, device: int, name: str = "tensor"):
    """A GPU tensor handed to the library by pointer: contiguous, of the kind's element width
    and on the ctx's device (the kernels index it by element; a wrong width reads past its end)."""
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    dt = str(t.dtype).replace("torch.", "")
    if dt not in _TORCH_KINDS[kind]:
        raise ValueError(f"{name}: dtype {dt} where {'/'.join(_TORCH_KINDS[kind])} is expected")
    if t.device.index is not None and device is not None and t.device.index != device:
        raise ValueError(f"{name} is on cuda:{t.device.index}, the table on cuda:{device}")


def torch_ready(t):
    """The library reads device columns on its own HIP stream, but torch produced them on torch's
    current stream (asynchronously): that stream's pending work on the tensor's device is finished
    before the pointer is handed over (the C-ABI's contract: resident columns are ready when a crdt_*
    call starts; the call itself returns only when its stream is done, so outputs need nothing)."""
    import torch
    torch.cuda.current_stream(t.device).synchronize()


class _Cols:
    """Normalises a set of columns to one memory kind and keeps them alive."""

    def __init__(self, device=None, **cols):
        self.keep = []
        self.mem = None
        self.ptrs = {}
        for name, (arr, kind) in cols.items():
            if arr is None:
                self.ptrs[name] = None
                continue
            if _is_torch(arr):
                if not arr.is_cuda:
                    arr = arr.numpy()
                else:
                    check_device_tensor(arr, kind, device, f"column {name}")
                    if not self.keep or not _is_torch(self.keep[0]):
                        torch_ready(arr)
                    mem = _capi.CRDT_MEM_DEVICE
                    self._set_mem(mem)
                    self.keep.append(arr)
                    self.ptrs[name] = ctypes.c_void_p(arr.data_ptr())
                    continue
            a = np.ascontiguousarray(arr, dtype=_NP_TYPES[kind])
            self._set_mem(_capi.CRDT_MEM_HOST)
            self.keep.append(a)
            self.ptrs[name] = a.ctypes.data_as(ctypes.c_void_p)
        if self.mem is None:
            self.mem = _capi.CRDT_MEM_HOST

    def _set_mem(self, mem):
        if self.mem is None:
            self.mem = mem
        elif self.mem != mem:
            raise ValueError("all columns of one call must live in the same memory (host or device)")


class DeviceTable:
    """Rows ``{lt, rank, val, mod}`` indexed by key id, plus the canonical clock."""

    def __init__(self, device: int = 0, local_rank: int = 0, capacity: int = 1024):
        self._lib = _capi.load()
        self._ctx = ctypes.c_void_p()
        st = self._lib.crdt_create(device, local_rank, max(int(capacity), 16), ctypes.byref(self._ctx))
        if st != 0:
            raise CrdtNativeError(st, "crdt_create")
        self.device = device
        self._local_rank = local_rank

    # ---------------------------------------------------------------- lifecycle
    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            self._lib.crdt_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _dptr(self, t, kind: str, name: str):
        """Device pointer of a GPU tensor argument after the width / device checks."""
        check_device_tensor(t, kind, self.device, name)
        torch_ready(t)
        return ctypes.c_void_p(t.data_ptr())

    def _check(self, st: int, what: str):
        if st < 0:
            raise CrdtNativeError(st, what)
        return st

    @property
    def capacity(self) -> int:
        v = ctypes.c_uint64()
        self._check(self._lib.crdt_capacity(self._ctx, ctypes.byref(v)), "crdt_capacity")
        return v.value

    def reserve(self, capacity: int):
        if capacity > self.capacity:
            cap = max(int(capacity), 2 * self.capacity)
            self._check(self._lib.crdt_reserve(self._ctx, cap), "crdt_reserve")

    @property
    def canonical(self) -> int:
        v = ctypes.c_int64()
        self._check(self._lib.crdt_get_canonical(self._ctx, ctypes.byref(v)), "crdt_get_canonical")
        return v.value

    @canonical.setter
    def canonical(self, lt: int):
        self._check(self._lib.crdt_set_canonical(self._ctx, int(lt)), "crdt_set_canonical")

    @property
    def local_rank(self) -> int:
        return self._local_rank

    @local_rank.setter
    def local_rank(self, r: int):
        self._check(self._lib.crdt_set_local_rank(self._ctx, int(r)), "crdt_set_local_rank")
        self._local_rank = int(r)

    # ---------------------------------------------------------------------- SPI
    def put_rows(self, key, lt, rank, val, mod):
        c = _Cols(self.device, key=(key, "u4"), lt=(lt, "i8"), rank=(rank, "u4"), val=(val, "u4"), mod=(mod, "i8"))
        n = len(key)
        p = c.ptrs
        self._check(self._lib.crdt_put_rows(self._ctx, p["key"], p["lt"], p["rank"], p["val"], p["mod"],
                                            n, c.mem), "crdt_put_rows")

    def read_rows(self, key):
        key = np.ascontiguousarray(key, dtype=np.uint32)
        n = len(key)
        lt = np.empty(n, np.int64)
        rank = np.empty(n, np.uint32)
        val = np.empty(n, np.uint32)
        mod = np.empty(n, np.int64)
        if n:
            P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
            self._check(self._lib.crdt_read_rows(self._ctx, P(key), n, P(lt), P(rank), P(val), P(mod),
                                                 _capi.CRDT_MEM_HOST), "crdt_read_rows")
        return lt, rank, val, mod

    def modified_since(self, n_rows: int, since: int) -> np.ndarray:
        out = np.empty(max(n_rows, 1), np.uint32)
        n = ctypes.c_uint64()
        self._check(self._lib.crdt_modified_since(self._ctx, n_rows, int(since),
                                                  out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(n)),
                    "crdt_modified_since")
        return out[:n.value]

    def clear_rows(self, first: int, count: int):
        self._check(self._lib.crdt_clear_rows(self._ctx, first, count), "crdt_clear_rows")

    def remap_ranks(self, n_rows: int, old_to_new):
        lut = np.ascontiguousarray(old_to_new, dtype=np.uint32)
        self._check(self._lib.crdt_remap_ranks(self._ctx, n_rows, lut.ctypes.data_as(ctypes.c_void_p),
                                               len(lut)), "crdt_remap_ranks")

    def refresh_canonical(self, n_rows: int) -> int:
        v = ctypes.c_int64()
        self._check(self._lib.crdt_refresh_canonical(self._ctx, n_rows, ctypes.byref(v)),
                    "crdt_refresh_canonical")
        return v.value

    # ---------------------------------------------------------------- Crdt API
    def put_stamped(self, key, val, wall: int) -> dict:
        c = _Cols(self.device, key=(key, "u4"), val=(val, "u4"))
        res = CrdtResult()
        self._check(self._lib.crdt_put_stamped(self._ctx, c.ptrs["key"], c.ptrs["val"], len(key), int(wall),
                                               c.mem, ctypes.byref(res)), "crdt_put_stamped")
        return res.as_dict()

    def _batch(self, key, lt, rank, val, offsets, millis):
        c = _Cols(self.device, key=(key, "u4"), lt=(lt, "i8"), rank=(rank, "u4"), val=(val, "u4"), millis=(millis, "i8"))
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        c.keep.append(offs)
        b = CrdtBatch(c.ptrs["key"], c.ptrs["lt"], c.ptrs["rank"], c.ptrs["val"], c.ptrs["millis"],
                      offs.ctypes.data_as(ctypes.c_void_p), len(offs) - 1, c.mem)
        return b, c, offs

    def merge(self, key, lt, rank, val, offsets, wall: int, millis=None, win_flags=True):
        """R sequential merges (one per changeset); returns (result dict, win flags or None).

        ``win_flags``: True -> a host uint8 array is returned; a torch uint8 CUDA tensor
        -> filled in place (device batches); False/None -> not produced."""
        b, c, offs = self._batch(key, lt, rank, val, offsets, millis)
        n = int(offs[-1])
        flags_arr = None
        fptr = None
        if win_flags is True:
            if c.mem == _capi.CRDT_MEM_DEVICE:
                import torch
                flags_arr = torch.zeros(max(n, 1), dtype=torch.uint8, device=c.keep[0].device)
                torch_ready(flags_arr)                  # (its zero fill must not land after the merge)
                fptr = ctypes.c_void_p(flags_arr.data_ptr())
            else:
                flags_arr = np.zeros(max(n, 1), np.uint8)
                fptr = flags_arr.ctypes.data_as(ctypes.c_void_p)
        elif win_flags is not None and win_flags is not False:
            flags_arr = win_flags
            if _is_torch(win_flags):
                fptr = self._dptr(win_flags, "u1", "win_flags")
            else:
                if win_flags.dtype != np.uint8 or not win_flags.flags.c_contiguous or len(win_flags) < n:
                    raise ValueError("win_flags must be a contiguous uint8 array of one entry per record")
                fptr = win_flags.ctypes.data_as(ctypes.c_void_p)
        res = CrdtResult()
        st = self._lib.crdt_merge(self._ctx, ctypes.byref(b), int(wall), fptr, ctypes.byref(res))
        if st == _capi.CRDT_E_COMM and getattr(self, "_comm", None) is not None and self._comm.error is not None:
            raise CrdtNativeError(st, f"crdt_merge (communicator: {self._comm.error!r})")
        self._check(st, "crdt_merge")
        if flags_arr is not None and win_flags is True:
            flags_arr = flags_arr[:n]
        return res.as_dict(), flags_arr

    # ------------------------------------------ key-sharded replica (comm_path.inc)
    def comm_unique_id(self) -> bytes:
        """crdt_comm_unique_id: the 128 bytes rank 0 hands every rank (RCCL)."""
        buf = (ctypes.c_uint8 * _capi.COMM_ID_BYTES)()
        self._check(self._lib.crdt_comm_unique_id(buf), "crdt_comm_unique_id")
        return bytes(buf)

    def comm_init_rccl(self, n_ranks: int, rank: int, uid: bytes):
        buf = (ctypes.c_uint8 * _capi.COMM_ID_BYTES).from_buffer_copy(uid)
        self._check(self._lib.crdt_comm_init_rccl(self._ctx, n_ranks, rank, buf), "crdt_comm_init_rccl")

    def comm_init_ops(self, n_ranks: int, rank: int, comm):
        """Join a communicator given as a crdt_comm_ops table (``comm.ops()``, e.g. dist.GlooComm)."""
        self._comm = comm                      # the callbacks must outlive the ctx's use of them
        ops = comm.ops()
        st = self._lib.crdt_comm_init_ops(self._ctx, n_ranks, rank, ctypes.byref(ops))
        self._check(st, "crdt_comm_init_ops")
        ms = getattr(self, "_comm_timeout_ms", None)       # (a deadline set before: the transport's bound too)
        if ms is not None and hasattr(comm, "timeout") and comm.timeout is None:
            comm.timeout = ms / 1e3 if ms else None

    def set_comm_timeout(self, ms: int):
        """crdt_set_comm_timeout: a collective merge's deadline in ms (0 = none).  A host transport given
        to comm_init_ops that has a ``timeout`` of its own (dist.GlooComm) gets the same bound per operation."""
        self._check(self._lib.crdt_set_comm_timeout(self._ctx, int(ms)), "crdt_set_comm_timeout")
        self._comm_timeout_ms = int(ms)
        comm = getattr(self, "_comm", None)
        if comm is not None and hasattr(comm, "timeout"):
            comm.timeout = ms / 1e3 if ms else None

    def comm_state(self) -> tuple[int, str]:
        """crdt_comm_state: (0 usable / 1 aborted at the deadline / 2 aborted on a transport error, the phase
        the current or last collective merge is or was in).  Callable from another thread during a merge."""
        st, ph = ctypes.c_int32(), ctypes.c_char_p()
        self._check(self._lib.crdt_comm_state(self._ctx, ctypes.byref(st), ctypes.byref(ph)), "crdt_comm_state")
        return st.value, (ph.value or b"").decode()

    def comm_info(self) -> tuple[int, int]:
        n, r = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self._lib.crdt_comm_info(self._ctx, ctypes.byref(n), ctypes.byref(r)), "crdt_comm_info")
        return n.value, r.value

    def comm_free(self):
        self._check(self._lib.crdt_comm_free(self._ctx), "crdt_comm_free")

    def set_presharded(self, on: bool):
        """True: batches hold only records this rank owns, with key = slot (no record exchange)."""
        self._check(self._lib.crdt_set_presharded(self._ctx, 1 if on else 0), "crdt_set_presharded")

    # ---------------------------------------------------------------- timing
    PATHS = {"auto": 0, "gather": 1, "sorted": 2}

    def set_counts(self, exact: bool):
        """crdt_set_counts: per-record n_present / n_won; False lets the sorted path fold each
        bucket in any order (same rows / canonical / status; both counts reported as 2^64 - 1)."""
        self._check(self._lib.crdt_set_counts(self._ctx, 1 if exact else 0), "crdt_set_counts")

    def set_row_bytes(self, row_bytes: int):
        """crdt_set_row_bytes: 24-B rows (default; sorted-path fan-ins) or 32-B rows (gather-path
        streaming). Same results."""
        self._check(self._lib.crdt_set_row_bytes(self._ctx, int(row_bytes)), "crdt_set_row_bytes")

    def reserve_scratch(self, n_records: int):
        """crdt_reserve_scratch: size the sorted path's partition buffers up front."""
        self._check(self._lib.crdt_reserve_scratch(self._ctx, int(n_records)), "crdt_reserve_scratch")

    def set_rank_bound(self, bound: int):
        """crdt_set_rank_bound: every later rank is < bound (0: no promise).  The sorted path then
        needs no pass over the ranks for its packed key's frame."""
        self._check(self._lib.crdt_set_rank_bound(self._ctx, int(bound)), "crdt_set_rank_bound")

    def set_merge_path(self, path: str):
        """'auto' | 'gather' | 'sorted' (crdt_set_merge_path): the strategy of later merges."""
        self._check(self._lib.crdt_set_merge_path(self._ctx, self.PATHS[path]), "crdt_set_merge_path")

    def last_path(self) -> str:
        v = ctypes.c_int(0)
        self._check(self._lib.crdt_last_path(self._ctx, ctypes.byref(v)), "crdt_last_path")
        return {1: "gather", 2: "sorted"}[v.value]

    PLAN_FLAGS = {"sorted": 1, "packed": 2, "two_level": 4, "hist_in_scan": 8, "key8": 16, "key16": 32,
                  "high_water": 64, "anchored": 128, "wire_packed": 256, "own_in_place": 512,
                  "flagged": 1024, "ordered": 2048,
                  "combined": 4096, "route_l1": 8192, "route_tuned": 16384, "rl1_head": 262144,
                  "compact": 524288}

    def last_plan(self) -> dict:
        """crdt_last_plan: how the last merge ran ({'sorted': bool, 'packed': ..., ...})."""
        v = ctypes.c_uint32(0)
        self._check(self._lib.crdt_last_plan(self._ctx, ctypes.byref(v)), "crdt_last_plan")
        plan = {k: bool(v.value & b) for k, b in self.PLAN_FLAGS.items()}
        plan["rl1_pieces"] = (v.value >> 15) & 7                # route_l1's pipelined pieces (0: not route_l1)
        return plan

    def place_info(self) -> dict:
        """crdt_place_info: the level-1 placement tuner ({'candidates': n, 'kept': index or None while the
        trials run, 'merges_used': the warm-up + two merges per candidate so far, 'level1_ms': each candidate's
        timed level-1 scatter, the faster of its two trials})."""
        n, kept, done = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
        ms = (ctypes.c_float * 4)()
        self._check(self._lib.crdt_place_info(self._ctx, ctypes.byref(n), ctypes.byref(kept), ctypes.byref(done), ms),
                    "crdt_place_info")
        return {"candidates": n.value, "kept": kept.value if kept.value >= 0 else None, "merges_used": done.value,
                "level1_ms": [round(float(m), 3) for m in ms[:max(n.value, 0)]]}

    TUNE_WAYS = ("route_l1", "combine", "route_l1_4", "route_l1_1", "route_l1_head")

    def route_tune(self) -> dict:
        """crdt_route_tune_info: the sharded fan-in routing the ctx measured ({'best': None while the
        trials run, else 'route_l1' (2 pipelined pieces) / 'combine' / 'route_l1_4' (4) / 'route_l1_1' (1) /
        'route_l1_head' (2 pieces, the owners' first digit folded at the sender); '<way>_ms': each way's timed
        call, max over ranks, None if not yet})."""
        best = ctypes.c_int32(0)
        us = (ctypes.c_int64 * 5)()
        self._check(self._lib.crdt_route_tune_info(self._ctx, ctypes.byref(best), us), "crdt_route_tune_info")
        out = {"best": self.TUNE_WAYS[best.value] if 0 <= best.value < len(self.TUNE_WAYS) else None}
        for w, u in zip(self.TUNE_WAYS, us):
            out[f"{w}_ms"] = u / 1e3 if u >= 0 else None
        return out

    def set_timing(self, enable: bool):
        self._check(self._lib.crdt_set_timing(self._ctx, int(bool(enable))), "crdt_set_timing")

    def timing(self) -> dict:
        t = CrdtTiming()
        self._check(self._lib.crdt_get_timing(self._ctx, ctypes.byref(t)), "crdt_get_timing")
        return t.as_dict()
