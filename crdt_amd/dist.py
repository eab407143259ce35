"""Key-sharded multi-GPU merge: one process per GPU, torch.distributed (RCCL).

Keys are owned by rank ``key % G`` (local slot ``key // G``); changeset j is
*homed* on rank ``j % G``, which holds its full (lt, rank) columns in iteration
order and runs its canonical-clock scan.  The only cross-rank exchange is
three small all-reduces of int64 words:

  1. MAX over the per-changeset maxima M_j            (R words)
  2. MIN over the first-exception key                 (1 word)
  3. MAX over that exception's details                (3 words)

after which every rank knows the same stop point, stamps R_j and final
canonical, and applies the records it owns.  No record crosses the fabric in
this path (records are routed to their owner at ingest, see ``route_by_owner``).
"""
from __future__ import annotations

import numpy as np


def sharded_merge(table, home, owned, wall: int, d_maxima, d_event, all_reduce_max, all_reduce_min,
                  win_flags=None) -> dict:
    """Run one batched merge across ranks.

    ``table`` exposes the phase API of ``DeviceTable`` (merge_scan / merge_clock /
    merge_resolve / merge_apply); ``home`` / ``owned`` are column tuples
    ``(key, lt, rank, val, offsets, millis)`` with the same number of changesets on
    every rank; ``all_reduce_max`` / ``all_reduce_min`` reduce an int64 tensor in place.
    """
    table.merge_scan(home, wall, d_maxima)
    all_reduce_max(d_maxima)
    table.merge_clock(home, wall, d_maxima, d_event)
    all_reduce_min(d_event[:1])
    table.merge_resolve(home, d_event)
    all_reduce_max(d_event[1:])
    return table.merge_apply(owned, wall, d_event, win_flags=win_flags)


def torch_reducers(dist):
    """all-reduce helpers over torch.distributed (``nccl`` = RCCL on ROCm, or ``gloo``)."""
    import torch
    host_staged = dist.get_backend() == "gloo"      # gloo reduces host tensors

    def _reduce(t, op):
        if t.is_cuda and host_staged:
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op)
        if t.is_cuda:
            torch.cuda.synchronize()

    return (lambda t: _reduce(t, dist.ReduceOp.MAX)), (lambda t: _reduce(t, dist.ReduceOp.MIN))


def route_by_owner(key, offsets, world: int):
    """Stable split of a columnar batch by owner rank ``key % world``.

    Returns, per rank, (row indices in iteration order, per-changeset offsets).
    Host-side helper for ingest (the interner already visits every record)."""
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


def home_mask(R: int, world: int, rank: int) -> np.ndarray:
    return (np.arange(R) % world) == rank
