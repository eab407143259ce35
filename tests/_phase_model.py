"""TEST INFRASTRUCTURE — numpy model of the device phase algebra.

Implements the DeviceTable phase API (merge_scan / merge_clock / merge_resolve /
merge_apply) with the same batched algebra the HIP kernels use
(crdt_amd/csrc/crdt_merge.hip K3a-K3d, K2): per-changeset maxima, the
prefix-max canonical recurrence C_j = max(R_j + 1, W), candidate-tile exception
search, stop point, sequential apply.  Used to test the multi-rank protocol of
crdt_amd/dist.py on CPU (gloo), and, being an independent restatement of the
batched algebra, checked against the sequential C oracle.
"""
import numpy as np

SHIFT = 16
MAXC = 0xFFFF
DRIFT = 60000
I64MIN = np.iinfo(np.int64).min
I64MAX = np.iinfo(np.int64).max
LOW = (1 << 40) - 1


def _np(t):
    """numpy view of a numpy array or a CPU torch tensor (shared memory)."""
    return t.numpy() if hasattr(t, "numpy") else t


def _send_fails(r, wall):
    m, c = r >> SHIFT, r & MAXC
    mn = max(m, wall)
    cn = c + 1 if m == mn else 0
    if mn - wall > DRIFT:
        return 1, mn - wall, 0
    if cn > MAXC:
        return 3, 0, cn
    return 0, 0, 0


class PhaseModel:
    def __init__(self, capacity, local_rank, canonical):
        absent8 = np.frombuffer(b"\x80" * 8, "<i8")[0]          # the device's 0x80 fill pattern
        self.lt = np.full(capacity, absent8, np.int64)
        self.rank = np.full(capacity, 0x80808080, np.uint32)
        self.val = np.full(capacity, 0x80808080, np.uint32)
        self.mod = np.full(capacity, absent8, np.int64)
        self.local_rank = local_rank
        self.canonical = canonical

    def put_rows(self, key, lt, rank, val, mod):
        self.lt[key], self.rank[key], self.val[key], self.mod[key] = lt, rank, val, mod

    # K3a
    def merge_scan(self, home, wall, d_max):
        _, lt, _, _, offs, _ = home
        offs = np.asarray(offs, np.int64)
        for j in range(len(offs) - 1):
            seg = lt[offs[j]:offs[j + 1]]
            d_max[j] = int(seg.max()) if len(seg) else I64MIN

    # K3b + K3c
    def merge_clock(self, home, wall, d_max, d_ev, d_prefix_max=None, index_base=None):
        _, lt, rank, _, offs, millis = home
        offs = np.asarray(offs, np.int64)
        R = len(offs) - 1
        W = wall << SHIFT
        c = self.canonical
        self.Cprev, self.R, self.C = [], [], []
        first_send = None
        for j in range(R):
            m = int(d_max[j])
            r = c if m == I64MIN else max(c, m)
            self.Cprev.append(c)
            self.R.append(r)
            if first_send is None and _send_fails(r, wall)[0]:
                first_send = j
            c = max(r + 1, W)
            self.C.append(c)
        ev = I64MAX if first_send is None else (first_send << 40) | LOW
        self.cands = {}
        for j in range(R):                       # home changesets only have records here
            p = self.Cprev[j]
            if d_prefix_max is not None:
                p = max(p, int(d_prefix_max[j]))
            ib = 0 if index_base is None else int(index_base[j])
            for x in range(offs[j], offs[j + 1]):
                v = int(lt[x])
                ms = int(millis[x]) if millis is not None else v >> SHIFT
                dup = int(rank[x]) == self.local_rank
                if (dup or ms - wall > DRIFT) and v > p:
                    key = (j << 40) | (x - offs[j] + ib)
                    self.cands[key] = (p, 2 if dup else 1, ms)
                    ev = min(ev, key)
                    break
                p = max(p, v)
        d_ev[0] = ev

    def merge_resolve(self, home, d_ev):
        ev = int(d_ev[0])
        d_ev[1], d_ev[2], d_ev[3] = I64MIN, 0, I64MIN
        if ev in self.cands:
            d_ev[1], d_ev[2], d_ev[3] = self.cands[ev]

    # routing (k_route_count / k_route_scatter): owner d = key % G, slot = key // G
    def route_count(self, batch, G):
        key, _, _, _, offs, _ = batch
        offs = np.asarray(offs, np.int64)
        out = np.zeros((len(offs) - 1, G), np.uint64)
        for j in range(len(offs) - 1):
            out[j] = np.bincount(np.asarray(key[offs[j]:offs[j + 1]], np.int64) % G, minlength=G)
        return out

    def route_scatter(self, batch, G, send_base, o_slot, o_lt, o_rank, o_val, out_perm=None):
        key, lt, rank, val, offs, _ = batch
        offs = np.asarray(offs, np.int64)
        o = [_np(o_slot).view(np.uint32), _np(o_lt), _np(o_rank).view(np.uint32), _np(o_val).view(np.uint32)]
        perm = None if out_perm is None else _np(out_perm)
        cur = np.asarray(send_base, np.int64).copy()
        for j in range(len(offs) - 1):
            for x in range(offs[j], offs[j + 1]):            # (the device order inside a chunk differs)
                d = int(key[x]) % G
                at = cur[j, d]
                cur[j, d] += 1
                o[0][at], o[1][at], o[2][at], o[3][at] = int(key[x]) // G, lt[x], rank[x], val[x]
                if perm is not None:
                    perm[at] = x

    def merge_apply_segments(self, cols, seg_begin, seg_end, wall, d_ev, win_flags=None):
        key, lt, rank, val = (_np(c) for c in cols)
        fl = None if win_flags is None else _np(win_flags)
        return self._apply(key.view(np.uint32), lt, rank.view(np.uint32), val.view(np.uint32),
                           np.asarray(seg_begin, np.int64), np.asarray(seg_end, np.int64), wall, d_ev, fl)

    # K3d + K2
    def merge_apply(self, owned, wall, d_ev, win_flags=None):
        key, lt, rank, val, offs, _ = owned
        offs = np.asarray(offs, np.int64)
        return self._apply(key, lt, rank, val, offs[:-1], offs[1:], wall, d_ev, win_flags)

    def _apply(self, key, lt, rank, val, begin, end, wall, d_ev, win_flags):
        R = len(begin)
        ev = int(d_ev[0])
        res = dict(status=0, n_stored=R, exc_changeset=0, exc_index=(1 << 64) - 1, drift_ms=0, counter=0,
                   n_present=0, n_won=0)
        if ev == I64MAX:
            stop, canon = R, (self.C[-1] if R else self.canonical)
        else:
            j, low = ev >> 40, ev & LOW
            res["exc_changeset"] = j
            if low == LOW:
                stop, canon = j + 1, self.R[j]
                st, drift, cnt = _send_fails(self.R[j], wall)
                res.update(status=st, drift_ms=drift, counter=cnt)
            else:
                stop, canon = j, int(d_ev[1])
                res.update(status=int(d_ev[2]), exc_index=low)
                if res["status"] == 1:
                    res["drift_ms"] = int(d_ev[3]) - wall
        res["n_stored"] = stop
        for j in range(stop):
            for x in range(begin[j], end[j]):
                k = int(key[x])
                present = self.mod[k] >= 0
                win = (not present) or lt[x] > self.lt[k] or (lt[x] == self.lt[k] and rank[x] > self.rank[k])
                res["n_present"] += int(present)
                if win:
                    self.lt[k], self.rank[k], self.val[k], self.mod[k] = lt[x], rank[x], val[x], self.R[j]
                    res["n_won"] += 1
                    if win_flags is not None:
                        win_flags[x] = 1
        self.canonical = canon
        res["canonical_lt"] = canon
        return res
