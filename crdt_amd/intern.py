"""Host-side interning: keys -> dense ids, node ids -> order-preserving ranks,
values -> uint32 handles.  The north star keeps string work on the host; the
device only ever sees the integer columns these tables produce.
"""
from __future__ import annotations

import bisect

from .hlc import node_sort_key

NULL_HANDLE = 0xFFFFFFFF


class KeyIndex:
    """Key <-> dense id in first-committed order, so id order is the
    LinkedHashMap insertion order of ``MapCrdt._map`` (map_crdt.dart:10).

    String keys live in the native table of ``libcrdt_host.so`` (``hostlib.NativeKeys``),
    which the native JSON decoder interns into directly; ``keys`` (id -> key) is filled
    lazily from it.  The first non-string key (``MapCrdt<K, V>`` with any ``K``) moves the
    index to a Python dict for good; so does a missing host library."""

    def __init__(self):
        from . import hostlib
        self._native = hostlib.NativeKeys() if hostlib.available() else None
        self._ids: dict = {}
        self._list: list = []

    @property
    def native(self):
        """The native table while every key is a string, else None."""
        return self._native

    def __len__(self):
        return len(self._native) if self._native is not None else len(self._list)

    @property
    def keys(self) -> list:
        if self._native is not None and len(self._list) < len(self._native):
            self._list.extend(self._native.export(len(self._list), len(self._native) - len(self._list)))
        return self._list

    def _to_python(self):
        keys = self.keys
        self._ids = {k: i for i, k in enumerate(keys)}
        self._native = None

    def get(self, key):
        if self._native is not None:
            if not isinstance(key, str):
                return None
            from .hostlib import utf8
            return self._native.find(utf8(key))
        return self._ids.get(key)

    def intern(self, key) -> int:
        if self._native is not None:
            if isinstance(key, str):
                from .hostlib import utf8
                i = self._native.intern(utf8(key))
                if i == len(self._list):
                    self._list.append(key)
                return i
            self._to_python()
        i = self._ids.get(key)
        if i is None:
            i = len(self._list)
            self._ids[key] = i
            self._list.append(key)
        return i

    def truncate(self, n: int):
        """Forget ids >= n (keys first seen in changesets that were not stored)."""
        if self._native is not None:
            self._native.truncate(n)
        else:
            for k in self._list[n:]:
                del self._ids[k]
        del self._list[n:]

    def clear(self):
        if self._native is not None:
            self._native.clear()
        self._ids.clear()
        self._list.clear()


class NodeRanks:
    """Node id <-> rank under Dart ``compareTo`` order (hlc.dart:160).

    Ranks are positions in the sorted list of every node id seen.  Inserting a
    node id that sorts before an existing one shifts ranks: ``register``
    returns the old->new table so the device rows can be re-ranked
    (``crdt_remap_ranks``)."""

    def __init__(self):
        self._sorted_keys: list = []
        self._nodes: list = []
        self._rank: dict = {}
        self._kind = None

    def __len__(self):
        return len(self._nodes)

    @property
    def kind(self):
        """'str' or 'int' once a node id is registered, else None."""
        return self._kind

    def rank(self, node_id) -> int:
        return self._rank[node_id]

    def node(self, rank: int):
        return self._nodes[rank]

    def _check_kind(self, node_id):
        kind = "str" if isinstance(node_id, str) else "int"
        if self._kind is None:
            self._kind = kind
        elif self._kind != kind:
            raise TypeError("node ids of one replica must all be String or all int")

    def register(self, node_ids) -> list | None:
        """Add node ids; returns an old->new rank table if existing ranks moved."""
        new = [n for n in set(node_ids) if n not in self._rank]
        if not new:
            return None
        for n in new:
            self._check_kind(n)
        old_nodes = list(self._nodes)
        moved = False
        for n in sorted(new, key=node_sort_key):
            k = node_sort_key(n)
            pos = bisect.bisect_left(self._sorted_keys, k)
            if pos < len(self._sorted_keys):
                moved = True
            self._sorted_keys.insert(pos, k)
            self._nodes.insert(pos, n)
        self._rank = {n: i for i, n in enumerate(self._nodes)}
        if not moved:
            return None
        return [self._rank[n] for n in old_nodes]


_RAW = object()            # handle whose value is still raw JSON text (decoded on first get)


class ValueStore:
    """Value <-> uint32 handle; ``None`` (tombstone) is ``NULL_HANDLE``.

    ``put_raw`` registers a batch of JSON value spans (from the native decoder) without
    building Python objects: such a value is ``json.loads``-ed on its first ``get``, and
    ``texts`` exports it without ever decoding it when its span is already in dumps form."""

    def __init__(self):
        self._values: list = []
        self._free: list = []
        self._rawflag = bytearray()         # per handle: 1 = still raw JSON text
        self._raw_start: list = []          # sorted first handles of raw batches
        self._raw: list = []                # [buf, off, len, live, canonical flags] per batch

    def __len__(self):
        return len(self._values) - len(self._free)

    def put(self, value) -> int:
        if value is None:
            return NULL_HANDLE
        if self._free:
            h = self._free.pop()
            self._values[h] = value
            self._rawflag[h] = 0
            return h
        h = len(self._values)
        if h >= NULL_HANDLE:
            raise MemoryError("value handle space exhausted")
        self._values.append(value)
        self._rawflag.append(0)
        return h

    def put_raw(self, buf: bytes, off, length):
        """Handles for the JSON texts buf[off[i] : off[i] + length[i]]; length 0 = null."""
        import numpy as np
        length = np.asarray(length)
        out = np.full(len(length), NULL_HANDLE, np.uint32)
        nz = np.flatnonzero(length)
        m = len(nz)
        if m == 0:
            return out
        h0 = len(self._values)
        if h0 + m >= NULL_HANDLE:
            raise MemoryError("value handle space exhausted")
        self._values.extend([_RAW] * m)
        self._rawflag.extend(b"\x01" * m)
        self._raw_start.append(h0)
        self._raw.append([buf, np.asarray(off)[nz].astype(np.int64), length[nz].astype(np.int64), m, None])
        out[nz] = np.arange(h0, h0 + m, dtype=np.uint32)
        return out

    def _batch(self, h: int) -> int:
        return bisect.bisect_right(self._raw_start, h) - 1

    def _retire_raw(self, h: int):
        b = self._raw[self._batch(h)]
        b[3] -= 1
        if b[3] == 0:                       # every value of the batch decoded or freed
            b[0] = b[1] = b[2] = None

    def get(self, handle: int):
        if handle == NULL_HANDLE:
            return None
        v = self._values[handle]
        if v is _RAW:
            import json
            bi = self._batch(handle)
            buf, off, ln = self._raw[bi][:3]
            k = handle - self._raw_start[bi]
            v = json.loads(buf[off[k]:off[k] + ln[k]])
            self._values[handle] = v
            self._rawflag[handle] = 0
            self._retire_raw(handle)
        return v

    def release(self, handle: int):
        if handle != NULL_HANDLE:
            if self._values[handle] is _RAW:
                self._retire_raw(handle)
            self._values[handle] = None
            self._rawflag[handle] = 0
            self._free.append(handle)

    def release_many(self, handles):
        """release() of many handles at once (vectorised: a merge can drop millions of losers)."""
        import numpy as np
        h = np.asarray(handles, np.int64)
        h = h[h != NULL_HANDLE]
        if len(h) == 0:
            return
        if len(h) < 64:
            for x in h.tolist():
                self.release(x)
            return
        h = np.unique(h)
        flags = np.frombuffer(bytes(self._rawflag), np.uint8)
        raw = h[flags[h] == 1]
        if len(raw):                                    # live-count bookkeeping of raw batches
            starts = np.asarray(self._raw_start, np.int64)
            bi = np.searchsorted(starts, raw, side="right") - 1
            for b, cnt in zip(*np.unique(bi, return_counts=True)):
                batch = self._raw[int(b)]
                batch[3] -= int(cnt)
                if batch[3] == 0:
                    batch[0] = batch[1] = batch[2] = None
        vals = self._values
        for x in h.tolist():
            vals[x] = None
        rf = self._rawflag
        for x in raw.tolist():
            rf[x] = 0
        self._free.extend(h.tolist())

    def compact(self, live_handles):
        """Free every handle not in ``live_handles``."""
        live = set(int(h) for h in live_handles)
        free = set(self._free)
        for h in range(len(self._values)):
            if h not in live and h not in free:
                self.release(h)

    def clear(self):
        self._values.clear()
        self._free.clear()
        self._rawflag.clear()
        self._raw_start.clear()
        self._raw.clear()

    def texts(self, handles, dumps):
        """JSON texts of the values of ``handles`` for the native encoder: (ptr, len, keepalive).

        A still-raw value whose input span is already what ``dumps`` writes is passed as that
        span (never decoded); every other value is encoded by one ``dumps`` of the list of them,
        which the native splitter cuts into elements.  len 0 = null (tombstone).  Raises
        ``hostlib.Fallback`` when that list does not split (NaN / Infinity ...)."""
        import numpy as np
        from . import hostlib
        h = np.asarray(handles, np.uint32)
        n = len(h)
        ptr = np.zeros(n, np.uint64)
        ln = np.zeros(n, np.uint32)
        keep = []
        rows = np.flatnonzero(h != NULL_HANDLE)
        if len(rows) == 0:
            return ptr, ln, keep
        hv = h[rows].astype(np.int64)
        raw = np.frombuffer(bytes(self._rawflag), np.uint8)[hv].astype(bool)
        other = rows[~raw]
        if raw.any():
            rr, rh = rows[raw], hv[raw]
            starts = np.asarray(self._raw_start, np.int64)
            bi = np.searchsorted(starts, rh, side="right") - 1
            slow = []
            for b in np.unique(bi):
                sel = bi == b
                batch = self._raw[int(b)]
                buf, boff, blen = batch[0], batch[1], batch[2]
                if batch[4] is None:                        # canonical flags, once per batch
                    batch[4] = hostlib.canonical(buf, boff, blen).astype(bool)
                k = rh[sel] - int(starts[b])
                good = batch[4][k]
                base = hostlib.address(buf)
                keep.append(buf)
                ptr[rr[sel][good]] = base + boff[k[good]].astype(np.uint64)
                ln[rr[sel][good]] = blen[k[good]].astype(np.uint32)
                slow.append(rr[sel][~good])
            if slow:
                other = np.sort(np.concatenate([other] + slow))
        if len(other):
            objs = [self.get(int(x)) for x in h[other]]
            text = dumps(objs).encode("utf-8", "surrogatepass")
            off, el = hostlib.split_array(text, len(objs))
            keep.append(text)
            ptr[other] = hostlib.address(text) + off
            ln[other] = el
            # a value that dumps to nothing cannot exist; length 0 stays reserved for null
        return ptr, ln, keep
