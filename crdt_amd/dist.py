"""Key-sharded multi-GPU replicas: one process per GPU, the exchanges inside the library.

A ``DeviceTable`` joined to a communicator is shard ``rank`` of ``n_ranks`` of ONE
replica: it owns keys ``key % n_ranks`` at slot ``key // n_ranks``, and its ``merge``
is collective — the library (``crdt_amd/csrc/comm_path.inc``) scans the rank's parts,
all-gathers the part maxima, reduces the first exception, routes every record to its
owner in one grouped all-to-all and applies what the rank owns (include/crdt_merge.h,
"key-sharded multi-GPU").  This module only wires communicators:

* ``attach_rccl(table, dist)``: RCCL over xGMI.  Rank 0 draws the 128-byte unique id,
  ``torch.distributed`` broadcasts it, every rank joins (``crdt_comm_init_rccl``).
* ``GlooComm``: a host-staged ``crdt_comm_ops`` table over a ``torch.distributed`` gloo
  group (tests: several ranks sharing one GPU, or no RCCL at all).  Its Python methods
  are the same three operations; ``tests/_phase_model.py`` drives them on CPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _capi

REDUCE_SUM, REDUCE_MAX, REDUCE_MIN = 0, 1, 2


def attach_rccl(table, dist) -> None:
    """Join ``table`` to an RCCL communicator spanning the ``torch.distributed`` world."""
    world, rank = dist.get_world_size(), dist.get_rank()
    uid = [table.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    table.comm_init_rccl(world, rank, uid[0])


class GlooComm:
    """``crdt_comm_ops`` (CRDT_MEM_HOST) over a torch.distributed gloo process group."""

    def __init__(self, dist, group=None, timeout: float | None = None):
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._ops = None
        self.error = None
        # seconds one operation may take (None: the process group's own timeout).  The library cannot
        # interrupt a host callback, so a host transport bounds its own operations (include/crdt_merge.h,
        # crdt_set_comm_timeout); DeviceTable.set_comm_timeout sets it to the library's deadline
        self.timeout = timeout

    def _wait(self, works) -> None:
        """Wait for gloo works, all of them within ``timeout`` seconds (a lost or stalled peer raises)."""
        import datetime
        import time
        if self.timeout is None:
            for w in works:
                w.wait()
            return
        end = time.monotonic() + self.timeout
        for w in works:
            left = max(end - time.monotonic(), 1e-3)
            w.wait(timeout=datetime.timedelta(seconds=left))

    # ---- the three operations, on numpy arrays ----------------------------------------
    def all_reduce(self, words: np.ndarray, op: int) -> None:
        import torch
        t = torch.from_numpy(words)
        red = {REDUCE_SUM: self.dist.ReduceOp.SUM, REDUCE_MAX: self.dist.ReduceOp.MAX,
               REDUCE_MIN: self.dist.ReduceOp.MIN}[op]
        self._wait([self.dist.all_reduce(t, op=red, group=self.group, async_op=True)])

    def all_gather(self, send: np.ndarray, recv: np.ndarray) -> None:
        import torch
        n = len(send)
        outs = [torch.from_numpy(recv[r * n:(r + 1) * n]) for r in range(self.world)]
        self._wait([self.dist.all_gather(outs, torch.from_numpy(np.ascontiguousarray(send)), group=self.group,
                                         async_op=True)])

    def all_to_all_v(self, send_cols, recv_cols, elem_bytes, sc, sd, rc, rd) -> None:
        """Byte columns; to peer d: elements [sd[d], + sc[d]) of every column, from it [rd[d], + rc[d])."""
        import torch
        reqs = []
        for d in range(self.world):
            if d == self.rank:
                continue
            for s, r, eb in zip(send_cols, recv_cols, elem_bytes):
                if sc[d]:
                    reqs.append(self.dist.isend(torch.from_numpy(s[sd[d] * eb:(sd[d] + sc[d]) * eb]), d,
                                                group=self.group))
                if rc[d]:
                    reqs.append(self.dist.irecv(torch.from_numpy(r[rd[d] * eb:(rd[d] + rc[d]) * eb]), d,
                                                group=self.group))
        self._wait(reqs)

    # ---- the C table -------------------------------------------------------------------
    def ops(self) -> _capi.CrdtCommOps:
        """The callbacks the library calls (host pointers: the library stages device words)."""
        if self._ops is not None:
            return self._ops

        def arr(p, n, dtype=np.int64):
            if n == 0:
                return np.zeros(0, dtype)
            return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dtype))),
                                         shape=(int(n),))

        def guard(fn):
            def call(*a):
                try:
                    fn(*a)
                    return 0
                except Exception as e:  # noqa: BLE001 -- reported as CRDT_E_COMM by the library
                    self.error = e
                    return 1
            return call

        def _ar(user, words, n, op, stream):
            self.all_reduce(arr(words, n), op)

        def _ag(user, send, recv, n, stream):
            self.all_gather(arr(send, n), arr(recv, n * self.world))

        def _a2a(user, n_cols, send, recv, eb, sc, sd, rc, rd, stream):
            G = self.world
            ebs = [eb[k] for k in range(n_cols)]
            scs, sds = [sc[d] for d in range(G)], [sd[d] for d in range(G)]
            rcs, rds = [rc[d] for d in range(G)], [rd[d] for d in range(G)]
            ns = max([sds[d] + scs[d] for d in range(G)] + [0])
            nr = max([rds[d] + rcs[d] for d in range(G)] + [0])
            sb = [arr(send[k], ns * ebs[k], np.uint8) for k in range(n_cols)]
            rb = [arr(recv[k], nr * ebs[k], np.uint8) for k in range(n_cols)]
            self.all_to_all_v(sb, rb, ebs, scs, sds, rcs, rds)

        self._cbs = (_capi.ALL_REDUCE_FN(guard(_ar)), _capi.ALL_GATHER_FN(guard(_ag)),
                     _capi.ALL_TO_ALL_FN(guard(_a2a)))
        self._ops = _capi.CrdtCommOps(None, _capi.CRDT_MEM_HOST, 0, *self._cbs)
        return self._ops


def route_by_owner(key, offsets, world: int):
    """Stable split of a columnar batch by owner rank ``key % world``.

    Returns, per rank, (row indices in iteration order, per-changeset offsets): the
    pre-sharded layout (``set_presharded``), where each rank ingests only what it owns."""
    key = np.asarray(key)
    offsets = np.asarray(offsets, dtype=np.uint64)
    owner = key % world
    out = []
    R = len(offsets) - 1
    cs = np.repeat(np.arange(R), np.diff(offsets).astype(np.int64))
    for r in range(world):
        idx = np.nonzero(owner == r)[0]
        counts = np.bincount(cs[idx], minlength=R)
        out.append((idx, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)))
    return out


def home_part(offsets, world: int, rank: int):
    """Rows of the changesets homed on ``rank`` (j % world == rank, whole) and the per-changeset
    offsets of that part (the other changesets' parts empty): the routed layout."""
    offs = np.asarray(offsets, np.int64)
    R = len(offs) - 1
    sel = np.concatenate([np.arange(offs[j], offs[j + 1]) for j in range(R) if j % world == rank] or
                         [np.zeros(0, np.int64)]).astype(np.int64)
    hc = np.where(np.arange(R) % world == rank, np.diff(offs), 0)
    return sel, np.concatenate([[0], np.cumsum(hc)]).astype(np.uint64)
