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


def sharded_merge_parts(table, part, wall: int, index_base, d_maxima, d_event, all_gather, all_reduce_max,
                        all_reduce_min, rank: int, win_flags=None) -> dict:
    """Batched merge when changeset j is the concatenation, in rank order, of the parts
    the ranks own (weak-scaling layout: every rank generates / ingests its own part).

    ``index_base[j]`` = records of changeset j held by lower ranks (host, from one
    all-gather of the per-rank counts).  Collectives: all-gather of the R per-part maxima
    (the global M_j is their max; the exception scan of this part starts from the max
    of the lower ranks' parts), then the same MIN / MAX event reductions as
    ``sharded_merge``.
    """
    import torch
    table.merge_scan(part, wall, d_maxima)
    g = all_gather(d_maxima)                                     # [G, R]
    prefix = torch.full_like(d_maxima, torch.iinfo(torch.int64).min)
    if rank > 0:
        prefix.copy_(g[:rank].max(dim=0).values)
    d_maxima.copy_(g.max(dim=0).values)
    if d_maxima.is_cuda:                     # torch's stream -> the library's stream
        torch.cuda.synchronize()
    table.merge_clock(part, wall, d_maxima, d_event, d_prefix_max=prefix, index_base=index_base)
    all_reduce_min(d_event[:1])
    table.merge_resolve(part, d_event)
    all_reduce_max(d_event[1:])
    return table.merge_apply(part, wall, d_event, win_flags=win_flags)


def route_plan(counts_all, rank: int):
    """Send / receive layout of the routed protocol from the all-gathered count matrices.

    counts_all[s, j, d] = records of changeset j that rank s holds and rank d owns.
    Send columns: owner-major, then changeset order (chunk (j, d) at send_base[j, d]).
    Receive columns: source-major (the all-to-all), so changeset j sits at
    [seg_begin[j], seg_end[j]) provided a single source holds it (home layout)."""
    counts_all = np.asarray(counts_all, dtype=np.int64)
    G, R, _ = counts_all.shape
    mine = counts_all[rank]                                   # [R, G] my sends
    send_split = mine.sum(axis=0)                             # per owner
    dst_base = np.concatenate([[0], np.cumsum(send_split)[:-1]])
    send_base = dst_base[None, :] + np.cumsum(mine, axis=0) - mine
    recv = counts_all[:, :, rank]                             # [G(src), R]
    recv_split = recv.sum(axis=1)
    src_base = np.concatenate([[0], np.cumsum(recv_split)[:-1]])
    within = np.cumsum(recv, axis=1) - recv                   # offset of changeset j inside src s's chunk
    holders = (counts_all.sum(axis=2) > 0)                    # [G, R]
    if (holders.sum(axis=0) > 1).any():
        raise ValueError("routed protocol: every changeset must be held by one rank (home layout)")
    src = np.argmax(holders, axis=0)                          # holder of j (0 when empty: count 0 anyway)
    jj = np.arange(R)
    seg_begin = src_base[src] + within[src, jj]
    seg_end = seg_begin + recv[src, jj]
    return (send_base.astype(np.uint64), send_split, recv_split, seg_begin.astype(np.uint64),
            seg_end.astype(np.uint64))


def sharded_merge_routed(table, home, wall: int, d_maxima, d_event, all_reduce_max, all_reduce_min,
                         all_gather, all_to_all, rank: int, world: int, alloc, win_flags=None) -> dict:
    """Batched merge when changeset j arrives whole on its home rank (north star
    config 4): the clock / exception phases of ``sharded_merge`` on the home columns, then the
    home rank partitions its records by owner (``key % world``, slot ``key // world``), RCCL
    all-to-all moves them, and each owner applies changeset j from its receive segment.

    ``home`` = (key, lt, rank, val, offsets, millis) with all R changesets (non-home ones empty);
    ``alloc(n, kind)`` returns a torch buffer ("u4" -> int32, "i8" -> int64, "u1" -> uint8);
    ``all_to_all(out, inp, out_splits, in_splits)``; ``win_flags`` (optional torch uint8, sized like
    the home batch) receives the flags back on the home rank."""
    table.merge_scan(home, wall, d_maxima)
    all_reduce_max(d_maxima)
    table.merge_clock(home, wall, d_maxima, d_event)
    all_reduce_min(d_event[:1])
    table.merge_resolve(home, d_event)
    all_reduce_max(d_event[1:])
    counts = table.route_count(home, world)                   # [R, G]
    import torch
    dev_counts = torch.from_numpy(counts.astype(np.int64).reshape(-1))
    if d_maxima.is_cuda:
        dev_counts = dev_counts.to(d_maxima.device)
    counts_all = all_gather(dev_counts).cpu().numpy().reshape(world, counts.shape[0], world)
    send_base, send_split, recv_split, seg_begin, seg_end = route_plan(counts_all, rank)
    ns, nr = int(send_split.sum()), int(recv_split.sum())
    s_cols = (alloc(ns, "u4"), alloc(ns, "i8"), alloc(ns, "u4"), alloc(ns, "u4"))
    perm = alloc(ns, "i8") if win_flags is not None else None
    table.route_scatter(home, world, send_base, *s_cols, out_perm=perm)
    r_cols = (alloc(nr, "u4"), alloc(nr, "i8"), alloc(nr, "u4"), alloc(nr, "u4"))
    for o, i in zip(r_cols, s_cols):
        all_to_all(o, i, recv_split.tolist(), send_split.tolist())
    r_flags = alloc(nr, "u1") if win_flags is not None else None
    res = table.merge_apply_segments(r_cols, seg_begin, seg_end, wall, d_event, win_flags=r_flags)
    res["n_sent"], res["n_recv"] = ns, nr
    if win_flags is not None:
        s_flags = alloc(ns, "u1")
        all_to_all(s_flags, r_flags, send_split.tolist(), recv_split.tolist())
        win_flags[perm] = s_flags
    return res


def torch_alloc(device):
    """Buffer factory for sharded_merge_routed."""
    import torch
    kinds = {"u4": torch.int32, "i8": torch.int64, "u1": torch.uint8}
    return lambda n, kind: torch.empty(int(n), dtype=kinds[kind], device=device)


def torch_all_to_all(dist):
    """all_to_all_single with split sizes (host-staged on gloo)."""
    import torch
    host_staged = dist.get_backend() == "gloo"

    def _a2a(out, inp, out_splits, in_splits):
        if host_staged and out.is_cuda:
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
            out.copy_(o)
            torch.cuda.synchronize()
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits)
            if out.is_cuda:
                torch.cuda.synchronize()

    return _a2a


def torch_all_gather(dist):
    """all-gather of an int64 vector into a [G, n] tensor (host-staged on gloo)."""
    import torch
    host_staged = dist.get_backend() == "gloo"

    def _gather(t):
        world = dist.get_world_size()
        if not host_staged:
            out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t.contiguous())
            return out.view(world, -1)
        src = t.cpu() if t.is_cuda else t
        out = [torch.empty_like(src) for _ in range(world)]
        dist.all_gather(out, src)
        g = torch.stack(out)
        if t.is_cuda:
            g = g.to(t.device)
            torch.cuda.synchronize()
        return g

    return _gather


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
