"""TEST INFRASTRUCTURE — numpy model of a sharded replica's crdt_merge.

``ShardModel.merge`` follows crdt_amd/csrc/comm_path.inc::merge_sharded step by step —
part scan, all-gather of the part maxima and counts, the prefix-max canonical
recurrence C_j = max(R_j + 1, W) (K3b), the candidate exception scan from each part's
predecessors (K3c), MIN / MAX event reductions, the owner-count exchange, the grouped
record exchange, the segmented sequential apply (K2) and the SUM of the counts — with
the collectives issued through ``crdt_amd.dist.GlooComm``'s Python methods, so the
CPU tests (gloo, world size 2 and 3) exercise the protocol and the communicator the
GPU library is driven with, and, being an independent restatement of the batched
algebra, check it against the sequential C oracle.
"""
import numpy as np

SHIFT = 16
MAXC = 0xFFFF
DRIFT = 60000
I64MIN = np.iinfo(np.int64).min
I64MAX = np.iinfo(np.int64).max
LOW = (1 << 40) - 1


def _send_fails(r, wall):
    m, c = r >> SHIFT, r & MAXC
    mn = max(m, wall)
    cn = c + 1 if m == mn else 0
    if mn - wall > DRIFT:
        return 1, mn - wall, 0
    if cn > MAXC:
        return 3, 0, cn
    return 0, 0, 0


class ShardModel:
    """Slot-indexed rows of shard ``rank`` of ``n_ranks`` (the device's 0x80 fill = absent)."""

    def __init__(self, capacity, local_rank, canonical, n_ranks=1, rank=0):
        absent8 = np.frombuffer(b"\x80" * 8, "<i8")[0]
        self.lt = np.full(capacity, absent8, np.int64)
        self.rank = np.full(capacity, 0x80808080, np.uint32)
        self.val = np.full(capacity, 0x80808080, np.uint32)
        self.mod = np.full(capacity, absent8, np.int64)
        self.local_rank = local_rank
        self.canonical = canonical
        self.G, self.me = n_ranks, rank

    def put_rows(self, key, lt, rank, val, mod):
        self.lt[key], self.rank[key], self.val[key], self.mod[key] = lt, rank, val, mod

    def merge(self, key, lt, rank, val, offsets, wall, comm, millis=None, win_flags=None, presharded=False):
        G, me = self.G, self.me
        offs = np.asarray(offsets, np.int64)
        R = len(offs) - 1
        key = np.asarray(key, np.uint32)
        # 1-2: part maxima and counts, all-gathered
        gsend = np.empty(2 * R, np.int64)
        for j in range(R):
            seg = lt[offs[j]:offs[j + 1]]
            gsend[j] = int(seg.max()) if len(seg) else I64MIN
            gsend[R + j] = len(seg)
        grecv = np.empty(2 * R * G, np.int64)
        comm.all_gather(gsend, grecv)
        g = grecv.reshape(G, 2 * R)
        M = g[:, :R].max(axis=0)
        pbase = g[:me, :R].max(axis=0) if me else np.full(R, I64MIN, np.int64)
        ibase = g[:me, R:].sum(axis=0) if me else np.zeros(R, np.int64)
        # 3: canonical recurrence (K3b) and the first send() failure
        W = wall << SHIFT
        c = self.canonical
        Cprev, Rj, Cj = [], [], []
        ev = I64MAX
        for j in range(R):
            m = int(M[j])
            r = c if m == I64MIN else max(c, m)
            Cprev.append(c)
            Rj.append(r)
            if ev == I64MAX and _send_fails(r, wall)[0]:
                ev = (j << 40) | LOW
            c = max(r + 1, W)
            Cj.append(c)
        # exception scan of this part from its predecessors (K3c)
        cands = {}
        for j in range(R):
            p = max(Cprev[j], int(pbase[j]))
            for x in range(offs[j], offs[j + 1]):
                v = int(lt[x])
                ms = int(millis[x]) if millis is not None else v >> SHIFT
                dup = int(rank[x]) == self.local_rank
                if (dup or ms - wall > DRIFT) and v > p:
                    k = (j << 40) | (x - offs[j] + int(ibase[j]))
                    cands[k] = (p, 2 if dup else 1, ms)
                    ev = min(ev, k)
                    break
                p = max(p, v)
        w = np.array([ev], np.int64)
        comm.all_reduce(w, 2)                                       # MIN
        ev = int(w[0])
        det = np.array(cands.get(ev, (I64MIN, 0, I64MIN)), np.int64)
        comm.all_reduce(det, 1)                                     # MAX
        res = dict(status=0, exc_changeset=0, exc_index=(1 << 64) - 1, drift_ms=0, counter=0)
        if ev == I64MAX:
            stop, canon = R, (Cj[-1] if R else self.canonical)
        else:
            j, low = ev >> 40, ev & LOW
            res["exc_changeset"] = j
            if low == LOW:
                stop, canon = j + 1, Rj[j]
                st, drift, cnt = _send_fails(Rj[j], wall)
                res.update(status=st, drift_ms=drift, counter=cnt)
            else:
                stop, canon = j, int(det[0])
                res.update(status=int(det[1]), exc_index=low)
                if res["status"] == 1:
                    res["drift_ms"] = int(det[2]) - wall
        res["n_stored"] = stop
        # 4: route (owner-major send columns, changeset order, stable inside a chunk)
        n = int(offs[-1])
        if presharded:
            cols = (key, np.asarray(lt, np.int64), np.asarray(rank, np.uint32), np.asarray(val, np.uint32))
            segs = [(int(offs[j]), int(offs[j + 1]), j) for j in range(R)]
            perm = None
        else:
            owner = (key % G).astype(np.int64)
            cs = np.repeat(np.arange(R), np.diff(offs))
            cnt = np.zeros((G, R), np.int64)
            np.add.at(cnt, (owner, cs), 1)
            rcnt = np.zeros((G, R), np.int64)
            rcnt[me] = cnt[me]
            sc = [0 if d == me else R for d in range(G)]
            disp = [d * R for d in range(G)]
            comm.all_to_all_v([cnt.reshape(-1).view(np.uint8)], [rcnt.reshape(-1).view(np.uint8)], [8],
                              sc, disp, sc, disp)
            perm = np.lexsort((np.arange(n), cs, owner))            # owner, then changeset, then position
            sc = cnt.sum(axis=1)
            sd = np.concatenate([[0], np.cumsum(sc)[:-1]])
            rc = rcnt.sum(axis=1)
            rd = np.concatenate([[0], np.cumsum(rc)[:-1]])
            nr = int(rc.sum())
            send = [(key[perm] // G).astype(np.uint32), np.asarray(lt, np.int64)[perm],
                    np.asarray(rank, np.uint32)[perm], np.asarray(val, np.uint32)[perm]]
            recv = [np.zeros(nr, a.dtype) for a in send]
            for s, r in zip(send, recv):                            # own chunk: a local copy
                r[rd[me]:rd[me] + rc[me]] = s[sd[me]:sd[me] + sc[me]]
            sc0, rc0 = sc.copy(), rc.copy()
            sc0[me] = rc0[me] = 0
            comm.all_to_all_v([a.view(np.uint8) for a in send], [a.view(np.uint8) for a in recv], [4, 8, 4, 4],
                              sc0.tolist(), sd.tolist(), rc0.tolist(), rd.tolist())
            cols = tuple(recv)
            run = rd.copy()
            segs = []
            for j in range(R):
                for s in range(G):
                    k = int(rcnt[s, j])
                    if k:
                        segs.append((int(run[s]), int(run[s]) + k, j))
                        run[s] += k
        # 5: sequential apply of the owned records, changeset by changeset (K2)
        ks, ls, rs, vs = cols
        rflags = np.zeros(len(ks), np.uint8)
        npres = nwon = err = 0
        for b, e, j in segs:
            if j >= stop:
                continue
            for x in range(b, e):
                k = int(ks[x])
                if k >= len(self.lt):
                    err = 1
                    continue
                present = self.mod[k] >= 0
                win = (not present) or ls[x] > self.lt[k] or (ls[x] == self.lt[k] and rs[x] > self.rank[k])
                npres += int(present)
                if win:
                    self.lt[k], self.rank[k], self.val[k], self.mod[k] = ls[x], rs[x], vs[x], Rj[j]
                    nwon += 1
                    rflags[x] = 1
        tot = np.array([npres, nwon, err, 0], np.int64)
        comm.all_reduce(tot, 0)                                     # SUM
        res.update(n_present=int(tot[0]), n_won=int(tot[1]))
        if tot[2]:
            res["status"] = -4
        self.canonical = canon
        res["canonical_lt"] = canon
        # win flags back to the ranks that sent the records
        if win_flags is not None:
            if presharded:
                win_flags[:] = rflags
            else:
                sflags = np.zeros(n, np.uint8)
                sflags[sd[me]:sd[me] + sc[me]] = rflags[rd[me]:rd[me] + rc[me]]
                comm.all_to_all_v([rflags], [sflags], [1], rc0.tolist(), rd.tolist(), sc0.tolist(), sd.tolist())
                win_flags[perm] = sflags
        return res
