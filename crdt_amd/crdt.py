"""``Crdt`` / ``MapCrdt`` — drop-in mirror of ``lib/src/crdt.dart`` and
``lib/src/map_crdt.dart`` whose storage and merge live on an MI355X.

The public surface keeps the reference's names and argument meanings
(``put``, ``putAll``, ``delete``, ``get``, ``merge``, ``mergeJson``,
``canonicalTime``, ``refreshCanonicalTime``, ``toJson``, ``recordMap``,
``watch``, ...).  Every clock read takes an optional ``wall`` (ms since epoch);
by default ``self.clock()`` = the host wall clock, as ``DateTime.now()`` is in
the reference.  ``mergeAll`` is the batched extension: R sequential merges in
one device call (the hot path of the benchmark).
"""
from __future__ import annotations

import numpy as np

from . import _capi
from .crdt_json import CrdtJson
from .device import CrdtNativeError, DeviceTable
from .hlc import (ClockDriftException, DuplicateNodeException, Hlc, OverflowException, now_millis)
from .intern import NULL_HANDLE, KeyIndex, NodeRanks, ValueStore
from .record import Record


class Watch:
    """A subscription to change events (``Stream<MapEntry<K, V?>>``, map_crdt.dart:47-49)."""

    def __init__(self, key=None, has_key=False):
        self.key = key
        self._has_key = has_key
        self.events: list = []

    def _offer(self, key, value):
        if not self._has_key or key == self.key:
            self.events.append((key, value))

    def __iter__(self):
        return iter(self.events)

    def __len__(self):
        return len(self.events)


class Crdt:
    """Abstract ``Crdt<K, V>`` (crdt.dart:7-170): the API over a storage SPI."""

    # ---- views (crdt.dart:13-29) ----
    @property
    def isEmpty(self) -> bool:
        return len(self.map) == 0

    @property
    def length(self) -> int:
        return len(self.map)

    @property
    def map(self) -> dict:
        return {k: r.value for k, r in self.recordMap().items() if not r.isDeleted}

    @property
    def keys(self) -> list:
        return list(self.map.keys())

    @property
    def values(self) -> list:
        return list(self.map.values())

    def get(self, key):                                                 # crdt.dart:36
        r = self.getRecord(key)
        return None if r is None else r.value

    def delete(self, key, wall: int | None = None):                     # crdt.dart:58
        self.put(key, None, wall=wall)

    def isDeleted(self, key):                                           # crdt.dart:62
        r = self.getRecord(key)
        return None if r is None else r.isDeleted

    def clear(self, purge: bool = False, wall: int | None = None):      # crdt.dart:67-73
        if purge:
            self.purge()
        else:
            self.putAll({k: None for k in self.map}, wall=wall)

    def mergeJson(self, js: str, keyDecoder=None, valueDecoder=None, wall: int | None = None):
        wall = self._wall(wall)                                         # crdt.dart:100-109
        if keyDecoder is None and valueDecoder is None and self._native_ingest():
            from . import hostlib
            n0 = len(self._keys)
            try:
                dec = hostlib.decode(js, self._keys.native)             # libcrdt_host.so
            except (hostlib.Fallback, ValueError):
                dec = None                                              # the restatement decides
            if dec is not None:
                self.last_ingest = "native"
                return self._merge_decoded(dec, n0, wall)
        self.last_ingest = "python"
        m = CrdtJson.decode(js, self.canonicalTime, keyDecoder=keyDecoder, valueDecoder=valueDecoder,
                            millis=wall)
        self.merge(m, wall=wall)

    def _native_ingest(self) -> bool:
        return False

    def toJson(self, modifiedSince: Hlc | None = None, keyEncoder=None, valueEncoder=None) -> str:
        return CrdtJson.encode(self.recordMap(modifiedSince=modifiedSince),           # crdt.dart:127-135
                               keyEncoder=keyEncoder, valueEncoder=valueEncoder)

    def __str__(self):
        return str(self.recordMap())

    def _wall(self, wall):
        return self.clock() if wall is None else int(wall)


class MapCrdt(Crdt):
    """``MapCrdt<K, V>`` (map_crdt.dart:9-53) with its map on the GPU.

    ``MapCrdt(nodeId, seed)`` keeps the reference's constructor quirk: the
    canonical clock is refreshed on the still-empty map (crdt.dart:31-33) before
    the seed is added (map_crdt.dart:16-18), so it starts at 0.
    """

    def __init__(self, nodeId, seed: dict | None = None, *, device: int = 0, capacity: int = 1024,
                 clock=None):
        self.nodeId = nodeId
        self.clock = clock or now_millis
        self._keys = KeyIndex()
        self._nodes = NodeRanks()
        self._values = ValueStore()
        self._hlc_override: dict = {}     # key id -> Hlc not in canonical (millis, counter) form
        self._mod_override: dict = {}     # key id -> modified Hlc with a foreign node / odd form
        self._watches: list = []
        self._rank_bound = 0
        self._nodes.register([nodeId])
        self._table = DeviceTable(device, local_rank=self._nodes.rank(nodeId), capacity=capacity)
        self._table.set_rank_bound(len(self._nodes))
        self._rank_bound = len(self._nodes)
        self.refreshCanonicalTime()
        if seed:
            self._store(list(seed.items()), notify=False)

    # ------------------------------------------------------------ internals
    def _register_nodes(self, node_ids):
        lut = self._nodes.register(node_ids)
        if lut is not None:
            self._table.remap_ranks(len(self._keys), lut)
            self._table.local_rank = self._nodes.rank(self.nodeId)
        if len(self._nodes) != self._rank_bound:      # ranks are dense: 0 .. len - 1
            self._rank_bound = len(self._nodes)
            self._table.set_rank_bound(self._rank_bound)

    def _reserve(self):
        if len(self._keys) > self._table.capacity:
            self._table.reserve(len(self._keys))

    def _emit(self, key, value):
        for w in self._watches:
            w._offer(key, value)

    def _note_overrides(self, kid: int, hlc: Hlc, modified: Hlc | None):
        if hlc.is_canonical_form:
            self._hlc_override.pop(kid, None)
        else:
            self._hlc_override[kid] = hlc
        if modified is None or (modified.nodeId == self.nodeId and modified.is_canonical_form):
            self._mod_override.pop(kid, None)
        else:
            self._mod_override[kid] = modified

    def _store(self, items, notify: bool):
        """putRecord(s) (map_crdt.dart:27-39): rows stored verbatim."""
        if not items:
            return
        self._register_nodes([r.hlc.nodeId for _, r in items])
        n = len(items)
        kid = np.empty(n, np.uint32)
        lt = np.empty(n, np.int64)
        rank = np.empty(n, np.uint32)
        val = np.empty(n, np.uint32)
        mod = np.empty(n, np.int64)
        for i, (k, r) in enumerate(items):
            kid[i] = self._keys.intern(k)
            lt[i] = r.hlc.logicalTime
            rank[i] = self._nodes.rank(r.hlc.nodeId)
            val[i] = self._values.put(r.value)
            mod[i] = r.modified.logicalTime
            self._note_overrides(int(kid[i]), r.hlc, r.modified)
        self._reserve()
        self._table.put_rows(kid, lt, rank, val, mod)
        if notify:
            for k, r in items:
                self._emit(k, r.value)
        self._maybe_compact()

    def _maybe_compact(self):
        if len(self._values) > 2 * max(4096, len(self._keys)):
            _, _, val, _ = self._table.read_rows(np.arange(len(self._keys), dtype=np.uint32))
            self._values.compact(val[val != NULL_HANDLE])

    def _raise_for(self, res: dict):
        st = res["status"]
        if st == _capi.CRDT_CLOCK_DRIFT:
            raise ClockDriftException(res["drift_ms"], 0)
        if st == _capi.CRDT_DUPLICATE_NODE:
            raise DuplicateNodeException(str(self.nodeId))
        if st == _capi.CRDT_OVERFLOW:
            raise OverflowException(res["counter"])

    def _make_record(self, kid: int, lt: int, rank: int, val: int, mod: int) -> Record:
        hlc = self._hlc_override.get(kid) or Hlc.fromLogicalTime(int(lt), self._nodes.node(int(rank)))
        modified = self._mod_override.get(kid) or Hlc.fromLogicalTime(int(mod), self.nodeId)
        return Record(hlc, self._values.get(int(val)), modified)

    # ------------------------------------------------------------ SPI
    def containsKey(self, key) -> bool:                                 # map_crdt.dart:21
        return self._keys.get(key) is not None

    def getRecord(self, key):                                           # map_crdt.dart:24
        kid = self._keys.get(key)
        if kid is None:
            return None
        lt, rank, val, mod = self._table.read_rows(np.array([kid], np.uint32))
        return self._make_record(kid, lt[0], rank[0], val[0], mod[0])

    def putRecord(self, key, record: Record):                           # map_crdt.dart:27-30
        self._store([(key, record)], notify=True)

    def putRecords(self, records: dict):                                # map_crdt.dart:33-39
        self._store(list(records.items()), notify=True)

    def recordMap(self, modifiedSince: Hlc | None = None) -> dict:      # map_crdt.dart:42-45
        since = modifiedSince.logicalTime if modifiedSince is not None else 0
        ids = self._table.modified_since(len(self._keys), since)
        if len(ids) == 0:
            return {}
        lt, rank, val, mod = self._table.read_rows(ids)
        keys = self._keys.keys
        return {keys[int(i)]: self._make_record(int(i), lt[x], rank[x], val[x], mod[x])
                for x, i in enumerate(ids)}

    def toJson(self, modifiedSince: Hlc | None = None, keyEncoder=None, valueEncoder=None) -> str:
        """crdt.dart:127-135 over recordMap (map_crdt.dart:42-45).  String keys and no encoders:
        the rows come from the device compaction (crdt_modified_since) and the document is
        assembled natively (hostlib.encode) — keys from the native table, Hlc.toString of the
        columns, raw input values reused when already in dumps form — so no Record is built.
        Anything else, or a Fallback from the native side, runs the restatement."""
        if keyEncoder is None and valueEncoder is None and self._keys.native is not None:
            from . import hostlib
            try:
                return self._native_export(modifiedSince)
            except hostlib.Fallback:
                pass
        self.last_export = "python"
        return super().toJson(modifiedSince, keyEncoder=keyEncoder, valueEncoder=valueEncoder)

    def _native_export(self, modifiedSince: Hlc | None) -> str:
        import json

        from . import hostlib
        from .crdt_json import _default
        since = modifiedSince.logicalTime if modifiedSince is not None else 0
        ids = self._table.modified_since(len(self._keys), since)
        if len(ids) == 0:
            self.last_export = "native"
            return "{}"
        lt, rank, val, _ = self._table.read_rows(ids)
        hlc_text = None
        if self._hlc_override:
            pos = {int(k): x for x, k in enumerate(ids.tolist())} if len(self._hlc_override) > 64 else None
            for kid, h in self._hlc_override.items():
                row = pos.get(kid) if pos is not None else (
                    int(np.searchsorted(ids, kid)) if kid <= int(ids[-1]) else None)
                if row is not None and row < len(ids) and int(ids[row]) == kid:
                    hlc_text = hlc_text or {}
                    hlc_text[row] = str(h)

        def dumps(objs):
            return json.dumps(objs, separators=(",", ":"), ensure_ascii=False, default=_default)

        ptr, ln, keep = self._values.texts(val, dumps)
        nodes = [self._nodes.node(r) for r in range(len(self._nodes))]
        out = hostlib.encode(self._keys.native, ids, lt, rank, nodes, ptr, ln, hlc_text)
        del keep
        self.last_export = "native"
        return out

    def watch(self, key=None, **kw) -> Watch:                           # map_crdt.dart:47-49
        w = Watch(key, has_key=("key" in kw) or key is not None)
        self._watches.append(w)
        return w

    def purge(self):                                                    # map_crdt.dart:52
        self._table.clear_rows(0, len(self._keys))
        self._keys.clear()
        self._values.clear()
        self._hlc_override.clear()
        self._mod_override.clear()

    # ------------------------------------------------------------ clock
    @property
    def canonicalTime(self) -> Hlc:                                     # crdt.dart:11
        return Hlc.fromLogicalTime(self._table.canonical, self.nodeId)

    def refreshCanonicalTime(self):                                     # crdt.dart:114-121
        self._table.refresh_canonical(len(self._keys))

    # ------------------------------------------------------------ writes
    def put(self, key, value, wall: int | None = None):                 # crdt.dart:39-43
        self.putAll({key: value}, wall=wall)

    def putAll(self, values: dict, wall: int | None = None):          # crdt.dart:46-54
        if not values:
            return
        wall = self._wall(wall)
        n0 = len(self._keys)
        items = list(values.items())
        kid = np.array([self._keys.intern(k) for k, _ in items], np.uint32)
        handles = np.array([self._values.put(v) for _, v in items], np.uint32)
        self._reserve()
        res = self._table.put_stamped(kid, handles, wall)
        if res["status"] != 0:
            self._keys.truncate(n0)
            for h in handles:
                self._values.release(int(h))
            self._raise_for(res)
        for i in kid:
            self._hlc_override.pop(int(i), None)
            self._mod_override.pop(int(i), None)
        for k, v in items:
            self._emit(k, v)
        self._maybe_compact()

    # ------------------------------------------------------------ merge
    def _native_ingest(self) -> bool:
        return self._keys.native is not None and self._nodes.kind in (None, "str")

    def _merge_decoded(self, dec: dict, n0: int, wall: int):
        """merge() of one natively decoded CrdtJson document (crdt.dart:77-94 on columns):
        keys already interned (ids >= n0 are new), values still raw JSON text."""
        kid, lt, nodes = dec["key_id"], dec["lt"], dec["nodes"]
        n = len(kid)
        self._register_nodes(nodes)
        lut = np.array([self._nodes.rank(x) for x in nodes], np.uint32)
        rank = lut[dec["node"]] if n else np.zeros(0, np.uint32)
        val = self._values.put_raw(dec["buf"], dec["val_off"], dec["val_len"])
        self._reserve()
        res, flags = self._table.merge(kid, lt, rank, val, np.array([0, n], np.uint64), wall)
        won = flags[:n].astype(bool) if res["n_stored"] else np.zeros(n, bool)
        if not res["n_stored"]:
            self._keys.truncate(n0)                    # keys of an unstored changeset never entered
        self._values.release_many(val[~won & (val != NULL_HANDLE)])
        if won.any() and (self._hlc_override or self._mod_override):
            for k in kid[won].tolist():                 # canonical-form Hlc, modified by this node
                self._hlc_override.pop(k, None)
                self._mod_override.pop(k, None)
        if won.any() and self._watches:
            keys = self._keys.keys
            for x in np.flatnonzero(won).tolist():
                self._emit(keys[int(kid[x])], self._values.get(int(val[x])))
        self._maybe_compact()
        self._raise_for(res)
        return res

    def merge(self, remoteRecords: dict, wall: int | None = None):    # crdt.dart:77-94
        self.mergeAll([remoteRecords], wall=wall)

    def mergeAllBulk(self, changesets, wall: int | None = None):
        """The catch-up form of ``mergeAll``: the same R sequential merges (rows, canonical clock,
        exceptions), but the merged maps are not cut down to their winners (``removeWhere``,
        crdt.dart:80-85) and no ``watch()`` event is emitted, so no per-record outcome is needed and
        the device may take the sorted path's order-free form.  Mirrors
        ``GpuMapCrdt.mergeAllBulk`` (dart/lib/src/gpu_map_crdt.dart).  A batch that needs per-record
        host bookkeeping — an Hlc outside the (millis << 16) + counter form, or a key whose stored
        Hlc / modified is kept on the host — runs as ``mergeAll``."""
        wall = self._wall(wall)
        changesets = list(changesets)
        R = len(changesets)
        if R == 0:
            return
        if self._hlc_override or self._mod_override or any(
                not r.hlc.is_canonical_form for cs in changesets for r in cs.values()):
            keyed = set(self._hlc_override) | set(self._mod_override)
            if any(not r.hlc.is_canonical_form for cs in changesets for r in cs.values()) or any(
                    self._keys.get(k) in keyed for cs in changesets for k in cs):
                self.mergeAll([dict(cs) for cs in changesets], wall=wall)   # (copies: maps untouched)
                return
        self._register_nodes([r.hlc.nodeId for cs in changesets for r in cs.values()])
        n_total = sum(len(cs) for cs in changesets)
        kid = np.empty(n_total, np.uint32)
        lt = np.empty(n_total, np.int64)
        rank = np.empty(n_total, np.uint32)
        val = np.empty(n_total, np.uint32)
        offsets = np.zeros(R + 1, np.uint64)
        newid_start = []
        i = 0
        for j, cs in enumerate(changesets):
            newid_start.append(len(self._keys))
            for key, rec in cs.items():
                kid[i] = self._keys.intern(key)
                lt[i] = rec.hlc.logicalTime
                rank[i] = self._nodes.rank(rec.hlc.nodeId)
                val[i] = self._values.put(rec.value)
                i += 1
            offsets[j + 1] = i
        newid_start.append(len(self._keys))
        self._reserve()
        self._table.set_counts(False)
        try:
            res, _ = self._table.merge(kid, lt, rank, val, offsets, wall, win_flags=False)
        except CrdtNativeError:
            self._keys.truncate(newid_start[0])
            self._values.release_many(val)
            raise
        finally:
            self._table.set_counts(True)
        stop = res["n_stored"]
        self._keys.truncate(newid_start[stop])
        self._values.release_many(val[int(offsets[stop]):])       # changesets never stored
        # the stored changesets' losing handles are unknown here: the next compaction frees them
        self._maybe_compact()
        self._raise_for(res)
        return res

    def mergeAll(self, changesets, wall: int | None = None):
        """``for m in changesets: merge(m)`` as ONE device call (R sequential merges)."""
        wall = self._wall(wall)
        changesets = list(changesets)
        R = len(changesets)
        if R == 0:
            return
        self._register_nodes([r.hlc.nodeId for cs in changesets for r in cs.values()])
        n_total = sum(len(cs) for cs in changesets)
        kid = np.empty(n_total, np.uint32)
        lt = np.empty(n_total, np.int64)
        rank = np.empty(n_total, np.uint32)
        val = np.empty(n_total, np.uint32)
        odd = []                  # (index, Hlc.millis) of Hlcs outside the (millis << 16) + counter form
        offsets = np.zeros(R + 1, np.uint64)
        newid_start = []
        items = []
        i = 0
        for j, cs in enumerate(changesets):
            newid_start.append(len(self._keys))
            for key, rec in cs.items():
                h = rec.hlc
                kid[i] = self._keys.intern(key)
                lt[i] = h.logicalTime
                rank[i] = self._nodes.rank(h.nodeId)
                val[i] = self._values.put(rec.value)
                if not h.is_canonical_form:
                    odd.append((i, h.millis))
                items.append((key, rec))
                i += 1
            offsets[j + 1] = i
        newid_start.append(len(self._keys))
        millis = None
        if odd:                   # built from the COMPLETE lt column, then the odd Hlcs patched in
            millis = lt >> 16
            for x, ms in odd:
                millis[x] = ms
        self._reserve()
        try:
            res, flags = self._table.merge(kid, lt, rank, val, offsets, wall, millis=millis)
        except CrdtNativeError:
            # the library refused the call (nothing stored on a single context, include/crdt_merge.h):
            # forget the keys and value handles this batch interned
            self._keys.truncate(newid_start[0])
            for x in range(n_total):
                self._values.release(int(val[x]))
            raise
        stop = res["n_stored"]
        # keys first seen in changesets that were not stored never entered the map
        self._keys.truncate(newid_start[stop])
        stored_end = int(offsets[stop])
        for x in range(n_total):
            if x >= stored_end or not flags[x]:
                self._values.release(int(val[x]))
        # the reference mutates each merged Map to its winners (removeWhere, crdt.dart:80-85)
        for j in range(stop):
            cs = changesets[j]
            b = int(offsets[j])
            for x, key in enumerate(list(cs.keys())):
                if not flags[b + x]:
                    del cs[key]
            for key, rec in cs.items():
                k = self._keys.get(key)
                self._note_overrides(k, rec.hlc, None)
                self._emit(key, rec.value)
        self._maybe_compact()
        self._raise_for(res)
        return res
