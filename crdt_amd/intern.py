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
    LinkedHashMap insertion order of ``MapCrdt._map`` (map_crdt.dart:10)."""

    def __init__(self):
        self.ids: dict = {}
        self.keys: list = []

    def __len__(self):
        return len(self.keys)

    def get(self, key):
        return self.ids.get(key)

    def intern(self, key) -> int:
        i = self.ids.get(key)
        if i is None:
            i = len(self.keys)
            self.ids[key] = i
            self.keys.append(key)
        return i

    def truncate(self, n: int):
        """Forget ids >= n (keys first seen in changesets that were not stored)."""
        for k in self.keys[n:]:
            del self.ids[k]
        del self.keys[n:]

    def clear(self):
        self.ids.clear()
        self.keys.clear()


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


class ValueStore:
    """Value <-> uint32 handle; ``None`` (tombstone) is ``NULL_HANDLE``."""

    def __init__(self):
        self._values: list = []
        self._free: list = []

    def __len__(self):
        return len(self._values) - len(self._free)

    def put(self, value) -> int:
        if value is None:
            return NULL_HANDLE
        if self._free:
            h = self._free.pop()
            self._values[h] = value
            return h
        h = len(self._values)
        if h >= NULL_HANDLE:
            raise MemoryError("value handle space exhausted")
        self._values.append(value)
        return h

    def get(self, handle: int):
        return None if handle == NULL_HANDLE else self._values[handle]

    def release(self, handle: int):
        if handle != NULL_HANDLE:
            self._values[handle] = None
            self._free.append(handle)

    def compact(self, live_handles):
        """Free every handle not in ``live_handles``."""
        live = set(int(h) for h in live_handles)
        free = set(self._free)
        for h in range(len(self._values)):
            if h not in live and h not in free:
                self._values[h] = None
                self._free.append(h)

    def clear(self):
        self._values.clear()
        self._free.clear()
