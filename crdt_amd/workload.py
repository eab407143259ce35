"""Synthetic columnar workloads for the BASELINE.json configurations.

Generated directly in HBM with torch (plumbing only: the merge itself never
touches torch).  Deterministic for a seed on a given device type.

fanin (configs[3], the metric's workload): R replicas x n records, keys Zipf(s)
over K ids, unique inside each replica; a local table pre-populated with the
first ``n_local`` ids.  Keys are sharded over G ranks by ``key % G`` (slot =
key // G); changeset j is "homed" on rank ``j % G`` (the rank that runs its
canonical-clock scan).

cfg2 (configs[1]): one 10M-record changeset against a 10M-key table, ~50%
overlap (5M existing ids + 5M new ids).

cfg3 (configs[2]): the fan-in generator at 100M keys / 100M records / 1024
replicas, Zipf(1.0), millis over 8 values and counters over 4 (heavy
(millis, counter) ties, decided by the node rank).

cfg5 (configs[4]): streaming — a 100M-key table, 100 deltas of 10M records,
one merge call per delta (advancing wall clock), 10% tombstones, optional
drift / duplicate-node injection at (delta 37, position 4,999,999).
"""
from __future__ import annotations

import numpy as np
import torch

NULL = 0xFFFFFFFF
BASE_MILLIS = 1_735_689_600_000          # 2025-01-01T00:00:00Z


def _zipf_keys(n: int, rows: int, K: int, s: float, gen: torch.Generator, device) -> torch.Tensor:
    """[rows, n] int64 keys, strictly increasing along each row (unique per replica).

    Stratified inverse-CDF sampling of a continuous Zipf(s) over [1, K+1), then
    key'_i = i + cummax(key_i - i) forces strict increase (the dense head of the
    distribution becomes "every hot key once per replica")."""
    i = torch.arange(n, device=device, dtype=torch.float64)
    u = (i.unsqueeze(0) + torch.rand(rows, n, device=device, dtype=torch.float64, generator=gen)) / n
    a = 1.0 - s
    if abs(a) < 1e-9:
        x = torch.exp(u * np.log(K + 1.0))
    else:
        x = torch.pow(1.0 + u * ((K + 1.0) ** a - 1.0), 1.0 / a)
    key = (torch.floor(x) - 1).clamp_(0, K - 1).to(torch.int64)
    del x, u
    ii = torch.arange(n, device=device, dtype=torch.int64).unsqueeze(0)
    y = torch.cummax(key - ii, dim=1).values
    key = y + ii
    key = torch.minimum(key, (K - n) + ii)           # leave room at the top: still strictly increasing
    return key


def gen_fanin(total: int = 1_000_000_000, R: int = 1024, K: int = 1 << 28, n_local: int = 1 << 27,
              s: float = 0.8, seed: int = 0xC0FFEE04, device="cuda", order: str = "shuffled",
              rank: int = 0, world: int = 1, chunk: int = 64, millis_span: int = 1 << 16,
              counter_span: int = 16, route: bool = False, census: bool = False) -> dict:
    """``route``: records are NOT pre-split by owner — this rank keeps the full changesets it is
    home to (``home`` gets key and val too, ``owned`` is empty) for the routed protocol.
    ``census``: also count U_touch of SURVEY §8(d) for this rank's slots — the distinct keys of
    the whole batch that it owns and that are present in the local map (``u_touch``)."""
    dev = torch.device(device)
    n = -(-total // R)                                   # records per replica (ceil)
    wall = BASE_MILLIS + millis_span + 1000
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    own = {"key": [], "lt": [], "rank": [], "val": []}
    own_counts = np.zeros(R, np.int64)
    home = {"lt": [], "rank": []}
    home_counts = np.zeros(R, np.int64)
    seen = torch.zeros(-(-K // world), dtype=torch.bool, device=dev) if census else None
    for j0 in range(0, R, chunk):
        rows = min(chunk, R - j0)
        key = _zipf_keys(n, rows, K, s, gen, dev)
        if census:
            kk = key[(key % world) == rank] if world > 1 else key.reshape(-1)
            seen[kk // world] = True
            del kk
        if order == "shuffled":
            rnd = torch.rand(rows, n, device=dev, generator=gen)
            if route and world > 1:                      # only this rank's home replicas are kept: shuffle
                hr = [r_ for r_ in range(rows) if (j0 + r_) % world == rank]     # those (same draws)
                if hr:
                    hi = torch.tensor(hr, device=dev)
                    key[hi] = torch.gather(key[hi], 1, torch.argsort(rnd[hi], dim=1))
            else:
                key = torch.gather(key, 1, torch.argsort(rnd, dim=1))
            del rnd
        ms = BASE_MILLIS + torch.randint(0, millis_span, (rows, n), device=dev, generator=gen)
        cnt = torch.randint(0, counter_span, (rows, n), device=dev, generator=gen)
        lt = (ms << 16) + cnt
        del ms, cnt
        jj = torch.arange(j0, j0 + rows, device=dev, dtype=torch.int64).unsqueeze(1)
        rk = (jj + 1).expand(rows, n)                    # replica j has node rank j + 1 (local = 0)
        val = ((jj << 20) | torch.arange(n, device=dev, dtype=torch.int64).unsqueeze(0)) & 0x7FFFFFFF
        for r_ in range(rows):
            j = j0 + r_
            if world > 1 and j % world == rank:
                home["lt"].append(lt[r_].clone())
                home["rank"].append(rk[r_].to(torch.int32))
                if route:
                    home.setdefault("key", []).append(key[r_].to(torch.int32))
                    home.setdefault("val", []).append(val.expand(rows, n)[r_].to(torch.int32))
                home_counts[j] = n
            if route:
                continue
            if world == 1:
                m = slice(None)
                k_own = key[r_]
            else:
                m = (key[r_] % world) == rank
                k_own = key[r_][m] // world
            own["key"].append(k_own.to(torch.int32))
            own["lt"].append(lt[r_][m])
            own["rank"].append(rk[r_][m].to(torch.int32))
            own["val"].append(val.expand(rows, n)[r_][m].to(torch.int32))
            own_counts[j] = own["key"][-1].numel()
        del key, lt, rk, val
    cat = lambda xs: torch.cat(xs) if xs else torch.zeros(0, device=dev, dtype=torch.int32)  # noqa: E731
    owned = {k: cat(v) for k, v in own.items()}
    if route:
        owned["lt"] = owned["lt"].to(torch.int64)
    del own
    if world == 1:                                       # one rank is home to every changeset
        homed = {"lt": owned["lt"], "rank": owned["rank"]}
        home_counts = own_counts
    else:
        homed = {k: cat(v) for k, v in home.items()}
    # ---- local table: ids [0, n_local), owned slots only
    slots_total = -(-K // world)
    lids = torch.arange(rank, n_local, world, device=dev, dtype=torch.int64)
    lgen = torch.Generator(device=dev)
    lgen.manual_seed(seed ^ 0x5EED)
    nl = lids.numel()
    # local rows use the same generator on every rank: draw for all ids then pick this shard
    l_ms = BASE_MILLIS + torch.randint(0, millis_span, (n_local,), device=dev, generator=lgen)
    l_cnt = torch.randint(0, counter_span, (n_local,), device=dev, generator=lgen)
    l_rank = torch.randint(0, R + 1, (n_local,), device=dev, generator=lgen)
    l_lt_all = (l_ms << 16) + l_cnt
    c0 = int(l_lt_all.max().item())                    # refreshCanonicalTime() of the full replica
    u_touch = int(seen[:nl].sum().item()) if census else None
    del seen
    local = {"slot": (lids // world).to(torch.int32), "lt": l_lt_all[lids].contiguous(),
             "rank": l_rank[lids].to(torch.int32), "val": (lids & 0x7FFFFFFF).to(torch.int32),
             "mod": l_lt_all[lids].contiguous()}
    del l_ms, l_cnt, l_rank, l_lt_all
    return {
        "owned": {k: v.contiguous() for k, v in owned.items()},
        "owned_offsets": np.concatenate([[0], np.cumsum(own_counts)]).astype(np.uint64),
        "home": {k: v.contiguous() for k, v in homed.items()},
        "home_offsets": np.concatenate([[0], np.cumsum(home_counts)]).astype(np.uint64),
        "local": local, "n_local_rows": nl, "capacity": slots_total, "c0": c0, "wall": wall,
        "R": R, "n_per_replica": n, "total": n * R, "K": K, "n_local": n_local, "world": world, "rank": rank,
        "u_touch": u_touch,
    }


def gen_cfg2(n_local: int = 10_000_000, n_remote: int = 10_000_000, overlap: float = 0.5,
             seed: int = 0xC0FFEE02, device="cuda", millis_span: int = 1 << 20) -> dict:
    """configs[1]: one changeset; ~overlap of its keys already exist locally."""
    dev = torch.device(device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    n_old = int(n_remote * overlap)
    n_new = n_remote - n_old
    old = torch.randperm(n_local, device=dev, generator=gen)[:n_old]
    new = torch.arange(n_local, n_local + n_new, device=dev)
    key = torch.cat([old, new])
    key = key[torch.randperm(n_remote, device=dev, generator=gen)]
    # new ids must appear in first-seen order (interning): renumber them along the stream
    is_new = key >= n_local
    key[is_new] = n_local + torch.arange(int(is_new.sum().item()), device=dev)
    ms = BASE_MILLIS + torch.randint(0, millis_span, (n_remote,), device=dev, generator=gen)
    lt = (ms << 16) + torch.randint(0, 16, (n_remote,), device=dev, generator=gen)
    l_ms = BASE_MILLIS + torch.randint(0, millis_span, (n_local,), device=dev, generator=gen)
    l_lt = (l_ms << 16) + torch.randint(0, 16, (n_local,), device=dev, generator=gen)
    owned = {"key": key.to(torch.int32), "lt": lt, "rank": torch.ones(n_remote, device=dev, dtype=torch.int32),
             "val": torch.arange(1, n_remote + 1, device=dev, dtype=torch.int32)}
    local = {"slot": torch.arange(n_local, device=dev, dtype=torch.int32), "lt": l_lt,
             "rank": torch.zeros(n_local, device=dev, dtype=torch.int32),
             "val": torch.arange(n_local, device=dev, dtype=torch.int32), "mod": l_lt.clone()}
    offs = np.array([0, n_remote], np.uint64)
    return {"owned": owned, "owned_offsets": offs, "home": {"lt": lt, "rank": owned["rank"]},
            "home_offsets": offs, "local": local, "n_local_rows": n_local, "capacity": n_local + n_new,
            "c0": int(l_lt.max().item()), "wall": BASE_MILLIS + millis_span + 1000, "R": 1,
            "n_per_replica": n_remote, "total": n_remote, "K": n_local + n_new, "n_local": n_local,
            "world": 1, "rank": 0}


def gen_cfg3(device="cuda", total: int = 100_000_000, K: int = 100_000_000, R: int = 1024) -> dict:
    """configs[2]: SURVEY §8(d) cfg3 (seed 0xC0FFEE03)."""
    wl = gen_fanin(total=total, R=R, K=K, n_local=K, s=1.0, seed=0xC0FFEE03, device=device,
                   millis_span=8, counter_span=4)
    return wl


def _affine(K: int, gen: torch.Generator, dev) -> tuple[int, int]:
    """(a, b) with gcd(a, K) = 1: i -> (a*i + b) mod K is a bijection of [0, K)."""
    while True:
        a = int(torch.randint(1, K, (1,), device=dev, generator=gen).item()) | 1
        if np.gcd(a, K) == 1:
            return a, int(torch.randint(0, K, (1,), device=dev, generator=gen).item())


def gen_cfg5(device="cuda", K: int = 100_000_000, n_delta: int = 10_000_000, deltas: int = 100,
             tomb: float = 0.1, inject: str | None = None, inject_at: tuple[int, int] = (37, 4_999_999),
             seed: int = 0xC0FFEE05, peers: int = 16, step_ms: int = 1000, rank: int = 0,
             world: int = 1) -> dict:
    """configs[4]: ``deltas`` merge calls of ``n_delta`` records each against a K-key table.

    Delta d comes from peer ``1 + d % peers`` (local node rank 0), keys = an affine bijection of
    [0, K) restricted to the first n_delta points (unique within the delta), millis in
    [base + d*step_ms, base + (d+1)*step_ms), wall_d = base + (d+1)*step_ms + 500.
    ``inject``: None, "drift" (millis = wall + 60_001) or "dup" (local rank, newest lt) at
    ``inject_at`` = (delta, position).

    ``world`` > 1 (configs[4] on N GPUs, one key-sharded replica): every delta is split into
    ``world`` contiguous parts, part r on rank r (so the concatenation in rank order is the delta in
    its own order: the parts protocol of include/crdt_merge.h), keys stay global ids (the library
    routes them to their owner ``key % world``); ``home`` / ``home_offsets`` hold this rank's parts,
    one changeset per delta, and the local table holds this rank's shard (slot = key // world)."""
    assert n_delta <= K
    dev = torch.device(device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    cut = [(n_delta * r) // world for r in range(world + 1)]          # part r of a delta: [cut[r], cut[r+1])
    mine = cut[rank + 1] - cut[rank]
    n = mine * deltas
    key = torch.empty(n, dtype=torch.int32, device=dev)
    lt = torch.empty(n, dtype=torch.int64, device=dev)
    rank_c = torch.empty(n, dtype=torch.int32, device=dev)
    val = torch.empty(n, dtype=torch.int32, device=dev)
    walls = np.zeros(deltas, np.int64)
    aff = []
    i = torch.arange(n_delta, device=dev, dtype=torch.int64)
    part = slice(cut[rank], cut[rank + 1])
    for d in range(deltas):
        a, b = _affine(K, gen, dev)
        aff.append((a, b))
        sl = slice(d * mine, (d + 1) * mine)
        walls[d] = BASE_MILLIS + (d + 1) * step_ms + 500
        k_d = ((i * a + b) % K).to(torch.int32)
        ms = BASE_MILLIS + d * step_ms + torch.randint(0, step_ms, (n_delta,), device=dev, generator=gen)
        lt_d = (ms << 16) + torch.randint(0, 16, (n_delta,), device=dev, generator=gen)
        r_d = torch.full((n_delta,), 1 + d % peers, dtype=torch.int32, device=dev)
        v = (d * n_delta + i + 1).to(torch.int32)
        v[torch.rand(n_delta, device=dev, generator=gen) < tomb] = -1          # NULL handle 0xFFFFFFFF
        if inject and d == inject_at[0]:
            pi = inject_at[1]
            if inject == "drift":
                lt_d[pi] = (walls[d] + 60_001) << 16
            elif inject == "dup":
                lt_d[pi] = (walls[d] + 1) << 16
                r_d[pi] = 0
            else:
                raise ValueError(inject)
        key[sl], lt[sl], rank_c[sl], val[sl] = k_d[part], lt_d[part], r_d[part], v[part]
        del k_d, ms, lt_d, r_d, v
    lgen = torch.Generator(device=dev)
    lgen.manual_seed(seed ^ 0x5EED)
    # local rows: clocks over [base - span/2, base + 0.3 span) — the early deltas compete with them,
    # and the canonical is below delta 37's wall clock, so the injected record is a recv() advance
    span = deltas * step_ms
    l_ms = BASE_MILLIS - span // 2 + torch.randint(0, span // 2 + (3 * span) // 10, (K,), device=dev,
                                                   generator=lgen)
    l_lt = (l_ms << 16) + torch.randint(0, 16, (K,), device=dev, generator=lgen)
    del l_ms
    c0 = int(l_lt.max().item())
    lids = torch.arange(rank, K, world, device=dev, dtype=torch.int64)
    local = {"slot": (lids // world).to(torch.int32), "lt": l_lt[lids].contiguous(),
             "rank": torch.zeros(len(lids), device=dev, dtype=torch.int32),
             "val": lids.to(torch.int32), "mod": l_lt[lids].contiguous()}
    del l_lt
    offs = (np.arange(deltas + 1, dtype=np.uint64) * mine)
    cols = {"key": key, "lt": lt, "rank": rank_c, "val": val}
    out = {"local": local, "n_local_rows": len(lids), "capacity": -(-K // world), "c0": c0, "wall": int(walls[0]),
           "walls": walls, "per_call": True, "affine": aff, "R": deltas, "n_per_replica": n_delta,
           "total": n_delta * deltas, "K": K, "n_local": K, "world": world, "rank": rank}
    if world == 1:
        out.update(owned=cols, owned_offsets=offs, home={"lt": lt, "rank": rank_c}, home_offsets=offs)
    else:
        out.update(owned={}, owned_offsets=None, home=cols, home_offsets=offs)
    return out
