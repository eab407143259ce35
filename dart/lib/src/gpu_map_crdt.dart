// GpuMapCrdt — a drop-in for MapCrdt (lib/src/map_crdt.dart:9-53) whose records live on an
// MI355X and whose merge runs there (include/crdt_merge.h through dart:ffi).
//
// It mirrors crdt_amd/crdt.py (the Python twin the GPU tests drive): keys become dense ids in
// first-committed order (so id order is the LinkedHashMap insertion order of MapCrdt._map),
// node ids become ranks in Dart String.compareTo order (hlc.dart:160), values become uint32
// handles (0xFFFFFFFF = null, the tombstone of record.dart:17).
//
// Crdt keeps its clock in the library-private `_canonicalTime` (crdt.dart:9), which a subclass
// in another library cannot assign.  This class therefore keeps the canonical clock on the
// device and overrides every member that reads or writes `_canonicalTime`: canonicalTime,
// put, putAll, merge, mergeJson and refreshCanonicalTime (crdt.dart:11, 39-58, 77-121); the
// base constructor's refreshCanonicalTime() call (crdt.dart:31-33) lands in the override.
import 'dart:async';
import 'dart:collection';
import 'dart:convert';
import 'dart:ffi';
import 'dart:typed_data';

import 'package:crdt/crdt.dart';
import 'package:ffi/ffi.dart';

import 'ffi_bindings.dart';

/// Dart String.compareTo order is UTF-16 code-unit order; node ids of other types use their
/// own Comparable order (hlc.dart:160).
int _compareNodes(dynamic a, dynamic b) => (a as Comparable).compareTo(b);

class _NodeRanks {
  final List<dynamic> sorted = [];
  final Map<dynamic, int> rankOf = {};

  /// Registers node ids; returns the old -> new rank table when existing ranks moved.
  List<int>? register(Iterable<dynamic> nodes) {
    final fresh = <dynamic>{};
    for (final n in nodes) {
      if (!rankOf.containsKey(n)) fresh.add(n);
    }
    if (fresh.isEmpty) return null;
    final old = List<dynamic>.of(sorted);
    sorted
      ..addAll(fresh)
      ..sort(_compareNodes);
    rankOf.clear();
    for (var i = 0; i < sorted.length; ++i) {
      rankOf[sorted[i]] = i;
    }
    final lut = [for (final n in old) rankOf[n]!];
    for (var i = 0; i < lut.length; ++i) {
      if (lut[i] != i) return lut;
    }
    return null; // only appended after every existing rank
  }

  int rank(dynamic node) => rankOf[node]!;
  dynamic node(int rank) => sorted[rank];
}

class _ValueStore<V> {
  final List<V?> _values = [];
  final List<int> _free = [];

  int put(V? v) {
    if (v == null) return crdtNullValue;
    if (_free.isNotEmpty) {
      final h = _free.removeLast();
      _values[h] = v;
      return h;
    }
    _values.add(v);
    return _values.length - 1;
  }

  V? get(int h) => h == crdtNullValue ? null : _values[h];

  void release(int h) {
    if (h == crdtNullValue) return;
    _values[h] = null;
    _free.add(h);
  }

  /// Handles in use (the store's live size).
  int get length => _values.length - _free.length;

  /// Frees every handle not in [live] (the value handles the device table still holds) and
  /// rebuilds the free list: bulk merges keep every stored handle, losers included.
  void compact(Iterable<int> live) {
    final keep = List<bool>.filled(_values.length, false);
    for (final h in live) {
      if (h != crdtNullValue && h < keep.length) keep[h] = true;
    }
    _free.clear();
    for (var h = 0; h < _values.length; ++h) {
      if (!keep[h]) {
        _values[h] = null;
        _free.add(h);
      }
    }
  }

  void clear() {
    _values.clear();
    _free.clear();
  }
}

class GpuMapCrdt<K, V> extends Crdt<K, V> {
  GpuMapCrdt(this.nodeId,
      [Map<K, Record<V>> seed = const {}, int device = 0, int capacity = 1024, String? library,
      String? hostLibrary])
      : _lib = CrdtLib.open(library ?? 'libcrdt_mi355x.so'),
        _device = device,
        _initialCapacity = capacity,
        _hostPath = hostLibrary,
        _nRanks = 1,
        _shardRank = 0,
        _commId = null,
        _commTimeoutMs = 0 {
    // (the base constructor has already run refreshCanonicalTime() on the empty map: 0)
    if (seed.isNotEmpty) _store(seed, notify: false); // map_crdt.dart:16-18: no clock refresh
  }

  /// One key shard of a replica spread over [nRanks] GPUs, one process per GPU (include/crdt_merge.h,
  /// "key-sharded multi-GPU", in its pre-sharded form: crdt_set_presharded).  The application owns the
  /// partition of the key space (e.g. a hash of the key modulo nRanks) and hands every process only the
  /// records of the keys it owns — so keys, node ids and values are interned per process exactly as in
  /// a single GpuMapCrdt, and no value handle crosses processes.  The shards join one RCCL
  /// communicator (rank 0 draws [commId] with [commUniqueId], the application passes the 128 bytes to
  /// every process) and their merges are COLLECTIVE: every rank calls merge / mergeAll / mergeAllBulk /
  /// mergeJson together with its part of each changeset (changeset j = the parts in rank order, a
  /// legal iteration order), and the library all-gathers the part maxima and reduces the first
  /// exception, so every shard applies the same changesets and keeps the same canonical clock as the
  /// whole replica would (crdt.dart:77-94).  getRecord / containsKey / recordMap / watch see this
  /// shard's keys.  Local writes (put, putAll, putRecord(s), purge) would advance one shard's clock
  /// alone, so they throw here.  No reference counterpart: the reference is one process
  /// (example/crdt_example.dart:21-25).
  GpuMapCrdt.sharded(this.nodeId,
      {required int nRanks,
      required int rank,
      required Uint8List commId,
      int device = 0,
      int capacity = 1024,
      int commTimeoutMs = 300000,
      String? library,
      String? hostLibrary})
      : _lib = CrdtLib.open(library ?? 'libcrdt_mi355x.so'),
        _device = device,
        _initialCapacity = capacity,
        _hostPath = hostLibrary,
        _nRanks = nRanks,
        _shardRank = rank,
        _commId = commId,
        _commTimeoutMs = commTimeoutMs {
    if (commId.length != crdtCommIdBytes) throw ArgumentError.value(commId.length, 'commId', 'must be 128 bytes');
    _c; // join the communicator now: every rank constructs its shard together
  }

  /// The 128-byte RCCL unique id rank 0 draws for [GpuMapCrdt.sharded] (crdt_comm_unique_id).
  static Uint8List commUniqueId([String? library]) {
    final lib = CrdtLib.open(library ?? 'libcrdt_mi355x.so');
    final p = calloc<Uint8>(crdtCommIdBytes);
    try {
      final st = lib.commUniqueId(p);
      if (st != crdtOk) throw StateError('crdt_comm_unique_id: ${lib.statusString(st).cast<Utf8>().toDartString()}');
      return Uint8List.fromList(p.asTypedList(crdtCommIdBytes));
    } finally {
      calloc.free(p);
    }
  }

  final int _nRanks;
  final int _shardRank;
  final int _commTimeoutMs; // a collective merge's deadline in ms (crdt_set_comm_timeout; 0: none)
  final Uint8List? _commId;
  bool get _sharded => _commId != null;

  void _localOnly(String what) {
    if (_sharded) throw UnsupportedError('$what on a key shard: local writes belong to a single-replica GpuMapCrdt');
  }

  @override
  final dynamic nodeId;

  final CrdtLib _lib;
  final int _device;
  final int _initialCapacity;
  final String? _hostPath;
  CrdtHostLib? _hostLib;
  bool _hostTried = false;

  CrdtHostLib? get _host {
    if (!_hostTried) {
      _hostTried = true;
      _hostLib = CrdtHostLib.tryOpen(_hostPath ?? 'libcrdt_host.so');
    }
    return _hostLib;
  }
  Pointer<Void> _ctx = nullptr;
  final _keyIds = <K, int>{};
  final _keys = <K>[];
  final _nodes = _NodeRanks();
  final _values = _ValueStore<V>();
  final _hlcOverride = <int, Hlc>{}; // key id -> Hlc not in (millis << 16) + counter form
  final _modOverride = <int, Hlc>{}; // key id -> modified Hlc with a foreign node id
  final _controller = StreamController<MapEntry<K, V?>>.broadcast();

  // ------------------------------------------------------------------ device context
  Pointer<Void> get _c {
    if (_ctx == nullptr) {
      _nodes.register([nodeId]);
      final out = calloc<Pointer<Void>>();
      try {
        _check(_lib.create(_device, _nodes.rank(nodeId), _initialCapacity, out), 'crdt_create');
        _ctx = out.value;
        _check(_lib.setRankBound(_ctx, _nodes.sorted.length), 'crdt_set_rank_bound');
        if (_commId != null) {
          final id = calloc<Uint8>(crdtCommIdBytes);
          try {
            id.asTypedList(crdtCommIdBytes).setAll(0, _commId!);
            _check(_lib.commInitRccl(_ctx, _nRanks, _shardRank, id), 'crdt_comm_init_rccl');
            _check(_lib.setCommTimeout(_ctx, _commTimeoutMs), 'crdt_set_comm_timeout');
            _check(_lib.setPresharded(_ctx, 1), 'crdt_set_presharded'); // key ids are this shard's slots
          } finally {
            calloc.free(id);
          }
        }
      } finally {
        calloc.free(out);
      }
    }
    return _ctx;
  }

  void close() {
    if (_ctx != nullptr && _sharded) _lib.commFree(_ctx);
    if (_ctx != nullptr) _lib.destroy(_ctx);
    _ctx = nullptr;
    _controller.close();
  }

  void _check(int st, String what) {
    if (st < 0) {
      throw StateError('$what: ${_lib.statusString(st).cast<Utf8>().toDartString()} ($st)');
    }
  }

  void _rethrow(Pointer<CrdtResult> r) {
    switch (r.ref.status) {
      case crdtClockDrift: // drift = millisTs - millisWall (hlc.dart:167)
        throw ClockDriftException(r.ref.driftMs, 0);
      case crdtDuplicateNode:
        throw DuplicateNodeException(nodeId.toString());
      case crdtOverflow:
        throw OverflowException(r.ref.counter);
    }
  }

  void _registerNodes(Iterable<dynamic> nodes) {
    final c = _c;
    final before = _nodes.sorted.length;
    final lut = _nodes.register(nodes);
    // ranks are dense (0 .. nodes - 1): the bound lets the sorted path skip reading ranks
    if (_nodes.sorted.length != before) _check(_lib.setRankBound(c, _nodes.sorted.length), 'crdt_set_rank_bound');
    if (lut == null) return;
    final p = calloc<Uint32>(lut.length);
    try {
      p.asTypedList(lut.length).setAll(0, lut);
      _check(_lib.remapRanks(c, _keys.length, p, lut.length), 'crdt_remap_ranks');
    } finally {
      calloc.free(p);
    }
    _check(_lib.setLocalRank(c, _nodes.rank(nodeId)), 'crdt_set_local_rank');
  }

  int _intern(K key) => _keyIds.putIfAbsent(key, () {
        _keys.add(key);
        return _keys.length - 1;
      });

  void _truncateKeys(int n) {
    for (var i = n; i < _keys.length; ++i) {
      _keyIds.remove(_keys[i]);
    }
    _keys.removeRange(n, _keys.length);
  }

  void _reserve() {
    final cap = calloc<Uint64>();
    try {
      _check(_lib.capacity(_c, cap.cast()), 'crdt_capacity');
      if (_keys.length > cap.value) {
        final want = _keys.length > 2 * cap.value ? _keys.length : 2 * cap.value;
        _check(_lib.reserve(_c, want), 'crdt_reserve');
      }
    } finally {
      calloc.free(cap);
    }
  }

  static bool _canonicalForm(Hlc h) => h.counter <= 0xFFFF && h.counter >= 0;

  void _noteOverrides(int kid, Hlc hlc, Hlc? modified) {
    if (_canonicalForm(hlc)) {
      _hlcOverride.remove(kid);
    } else {
      _hlcOverride[kid] = hlc;
    }
    if (modified == null || (modified.nodeId == nodeId && _canonicalForm(modified))) {
      _modOverride.remove(kid);
    } else {
      _modOverride[kid] = modified;
    }
  }

  Record<V> _makeRecord(int kid, int lt, int rank, int val, int mod) => Record<V>(
      _hlcOverride[kid] ?? Hlc.fromLogicalTime(lt, _nodes.node(rank)),
      _values.get(val),
      _modOverride[kid] ?? Hlc.fromLogicalTime(mod, nodeId));

  /// putRecord(s) (map_crdt.dart:27-39): rows stored verbatim, no clock update.
  void _store(Map<K, Record<V>> items, {required bool notify}) {
    if (items.isEmpty) return;
    _registerNodes(items.values.map((r) => r.hlc.nodeId));
    final n = items.length;
    final kid = calloc<Uint32>(n), rank = calloc<Uint32>(n), val = calloc<Uint32>(n);
    final lt = calloc<Int64>(n), mod = calloc<Int64>(n);
    try {
      var i = 0;
      items.forEach((k, r) {
        final id = _intern(k);
        kid[i] = id;
        lt[i] = r.hlc.logicalTime;
        rank[i] = _nodes.rank(r.hlc.nodeId);
        val[i] = _values.put(r.value);
        mod[i] = r.modified.logicalTime;
        _noteOverrides(id, r.hlc, r.modified);
        ++i;
      });
      _reserve();
      _check(_lib.putRows(_c, kid, lt, rank, val, mod, n, crdtMemHost), 'crdt_put_rows');
    } finally {
      calloc.free(kid);
      calloc.free(rank);
      calloc.free(val);
      calloc.free(lt);
      calloc.free(mod);
    }
    if (notify) items.forEach((k, r) => _controller.add(MapEntry(k, r.value)));
    _maybeCompact();
  }

  /// Mirrors MapCrdt._maybe_compact (crdt_amd/crdt.py): once the value store holds more than
  /// twice as many handles as there are keys, the handles still referenced by the table are
  /// read back (crdt_read_rows of every key id) and every other handle is freed.
  void _maybeCompact() {
    final nKeys = _keys.length;
    if (_values.length <= 2 * (nKeys > 4096 ? nKeys : 4096)) return;
    final ids = calloc<Uint32>(nKeys == 0 ? 1 : nKeys), val = calloc<Uint32>(nKeys == 0 ? 1 : nKeys);
    try {
      for (var i = 0; i < nKeys; ++i) {
        ids[i] = i;
      }
      _check(_lib.readRows(_c, ids, nKeys, nullptr, nullptr, val, nullptr, crdtMemHost), 'crdt_read_rows');
      _values.compact(val.asTypedList(nKeys == 0 ? 1 : nKeys).take(nKeys));
    } finally {
      calloc.free(ids);
      calloc.free(val);
    }
  }

  // --------------------------------------------------------------------------- SPI
  @override
  bool containsKey(K key) => _keyIds.containsKey(key); // map_crdt.dart:21

  @override
  Record<V>? getRecord(K key) {
    // map_crdt.dart:24
    final id = _keyIds[key];
    if (id == null) return null;
    final k = calloc<Uint32>(), lt = calloc<Int64>(), mod = calloc<Int64>();
    final rank = calloc<Uint32>(), val = calloc<Uint32>();
    try {
      k.value = id;
      _check(_lib.readRows(_c, k, 1, lt, rank, val, mod, crdtMemHost), 'crdt_read_rows');
      return _makeRecord(id, lt.value, rank.value, val.value, mod.value);
    } finally {
      calloc.free(k);
      calloc.free(lt);
      calloc.free(mod);
      calloc.free(rank);
      calloc.free(val);
    }
  }

  @override
  void putRecord(K key, Record<V> value) {
    _localOnly('putRecord');
    _store({key: value}, notify: true); // map_crdt.dart:27-30
  }

  @override
  void putRecords(Map<K, Record<V>> recordMap) {
    _localOnly('putRecords');
    _store(recordMap, notify: true); // map_crdt.dart:33-39
  }

  @override
  Map<K, Record<V>> recordMap({Hlc? modifiedSince}) {
    // map_crdt.dart:42-45: rows whose modified.logicalTime >= since, in insertion (id) order
    final out = LinkedHashMap<K, Record<V>>();
    final nRows = _keys.length;
    if (nRows == 0) return out;
    final ids = calloc<Uint32>(nRows), nOut = calloc<Uint64>();
    try {
      _check(_lib.modifiedSince(_c, nRows, modifiedSince?.logicalTime ?? 0, ids, nOut), 'crdt_modified_since');
      final m = nOut.value;
      if (m == 0) return out;
      final lt = calloc<Int64>(m), mod = calloc<Int64>(m);
      final rank = calloc<Uint32>(m), val = calloc<Uint32>(m);
      try {
        _check(_lib.readRows(_c, ids, m, lt, rank, val, mod, crdtMemHost), 'crdt_read_rows');
        for (var x = 0; x < m; ++x) {
          final id = ids[x];
          out[_keys[id]] = _makeRecord(id, lt[x], rank[x], val[x], mod[x]);
        }
      } finally {
        calloc.free(lt);
        calloc.free(mod);
        calloc.free(rank);
        calloc.free(val);
      }
    } finally {
      calloc.free(ids);
      calloc.free(nOut);
    }
    return out;
  }

  @override
  Stream<MapEntry<K, V?>> watch({K? key}) =>
      _controller.stream.where((event) => key == null || key == event.key); // map_crdt.dart:47-49

  @override
  void purge() {
    // map_crdt.dart:52
    _localOnly('purge');
    _check(_lib.clearRows(_c, 0, _keys.length), 'crdt_clear_rows');
    _keyIds.clear();
    _keys.clear();
    _values.clear();
    _hlcOverride.clear();
    _modOverride.clear();
  }

  // ------------------------------------------------------------------------ clock
  @override
  Hlc get canonicalTime {
    // crdt.dart:11
    final p = calloc<Int64>();
    try {
      _check(_lib.getCanonical(_c, p.cast()), 'crdt_get_canonical');
      return Hlc.fromLogicalTime(p.value, nodeId);
    } finally {
      calloc.free(p);
    }
  }

  @override
  void refreshCanonicalTime() {
    // crdt.dart:114-121 on the device: max lt over the rows recordMap() keeps, 0 when empty
    final p = calloc<Int64>();
    try {
      _check(_lib.refreshCanonical(_c, _keys.length, p), 'crdt_refresh_canonical');
    } finally {
      calloc.free(p);
    }
  }

  // ------------------------------------------------------------------------ writes
  @override
  void put(K key, V? value) => putAll({key: value}); // crdt.dart:39-43: one send(), one record

  @override
  void putAll(Map<K, V?> values) {
    // crdt.dart:46-54: ONE Hlc.send for the call, every record {C, value, C}
    if (values.isEmpty) return;
    _localOnly('putAll');
    final n0 = _keys.length;
    final n = values.length;
    final kid = calloc<Uint32>(n), val = calloc<Uint32>(n);
    final res = calloc<CrdtResult>();
    try {
      var i = 0;
      final handles = <int>[];
      values.forEach((k, v) {
        kid[i] = _intern(k);
        val[i] = _values.put(v);
        handles.add(val[i]);
        ++i;
      });
      _reserve();
      final st = _lib.putStamped(_c, kid, val, n, DateTime.now().millisecondsSinceEpoch, crdtMemHost, res);
      if (st != crdtOk) {
        _truncateKeys(n0);
        handles.forEach(_values.release);
        _check(st, 'crdt_put_stamped');
        _rethrow(res);
      }
      for (var x = 0; x < n; ++x) {
        _hlcOverride.remove(kid[x]);
        _modOverride.remove(kid[x]);
      }
    } finally {
      calloc.free(kid);
      calloc.free(val);
      calloc.free(res);
    }
    values.forEach((k, v) => _controller.add(MapEntry(k, v)));
    _maybeCompact();
  }

  // ------------------------------------------------------------------------ merge
  @override
  void merge(Map<K, Record<V>> remoteRecords) => mergeAll([remoteRecords]); // crdt.dart:77-94

  @override
  void mergeJson(String json, {KeyDecoder<K>? keyDecoder, ValueDecoder<V>? valueDecoder}) {
    // crdt.dart:100-109.  Without decoders the document is decoded by libcrdt_host.so's
    // crdt_json_decode (JSON parse, Hlc.parse and key interning in C++, as MapCrdt.mergeJson of
    // crdt_amd/crdt.py does); input outside its fast path, or no host library, falls back to
    // CrdtJson.decode, so the map merged is the same either way.
    final native = keyDecoder == null && valueDecoder == null ? _decodeNative(json) : null;
    merge(native ??
        CrdtJson.decode<K, V>(json, canonicalTime, keyDecoder: keyDecoder, valueDecoder: valueDecoder));
  }

  /// CrdtJson.decode (crdt_json.dart:19-37) through crdt_json_decode: the document's keys in their
  /// order (a repeated key keeps its first position and its last record, as jsonDecode does), each
  /// Hlc from its logical time and node id (Hlc.parse, hlc.dart:39-46), each value jsonDecode-d from
  /// its span.  The `modified` placeholder (crdt_json.dart:23-24) never survives merge.  Null: fall back.
  Map<K, Record<V>>? _decodeNative(String json) {
    final host = _host;
    if (host == null || '' is! K) return null; // keys are the document's strings (`key as K`)
    final bytes = utf8.encode(json);
    final src = calloc<Uint8>(bytes.isEmpty ? 1 : bytes.length);
    final keys = host.keysCreate();
    final out = calloc<Pointer<Void>>();
    try {
      src.asTypedList(bytes.length).setAll(0, bytes);
      final st = host.jsonDecode(src, bytes.length, keys, out);
      if (st == crdtHostFallback) return null;
      if (st == crdtHostEJson) throw FormatException('crdt_json_decode: malformed JSON');
      if (st != crdtHostOk) throw StateError('crdt_json_decode: $st');
      final d = out.value;
      try {
        final n = host.decodedCount(d);
        final nk = host.keysSize(keys);
        final kb = host.keysBytes(keys, 0, nk);
        final kbuf = calloc<Uint8>(kb == 0 ? 1 : kb), koff = calloc<Uint64>(nk + 1);
        final nn = host.decodedNodeCount(d), nb = host.decodedNodeBytes(d);
        final nbuf = calloc<Uint8>(nb == 0 ? 1 : nb), noff = calloc<Uint64>(nn + 1);
        final m = n == 0 ? 1 : n;
        final kid = calloc<Uint32>(m), node = calloc<Uint32>(m), vlen = calloc<Uint32>(m);
        final lt = calloc<Int64>(m), voff = calloc<Uint64>(m);
        try {
          if (host.keysExport(keys, 0, nk, kbuf, kb, koff) != crdtHostOk ||
              host.decodedNodes(d, nbuf, nb, noff) != crdtHostOk ||
              host.decodedColumns(d, kid, lt, node, voff, vlen) != crdtHostOk) {
            return null;
          }
          final kt = kbuf.asTypedList(kb == 0 ? 1 : kb), nt = nbuf.asTypedList(nb == 0 ? 1 : nb);
          final keyStr = [for (var i = 0; i < nk; ++i) utf8.decode(kt.sublist(koff[i], koff[i + 1]))];
          final nodes = <dynamic>[for (var i = 0; i < nn; ++i) utf8.decode(nt.sublist(noff[i], noff[i + 1]))];
          final modified = canonicalTime;
          final result = <K, Record<V>>{};
          for (var i = 0; i < n; ++i) {
            final dynamic value =
                vlen[i] == 0 ? null : jsonDecode(utf8.decode(bytes.sublist(voff[i], voff[i] + vlen[i])));
            result[keyStr[kid[i]] as K] =
                Record<V>(Hlc<dynamic>.fromLogicalTime(lt[i], nodes[node[i]]), value as V?, modified);
          }
          return result;
        } finally {
          for (final p in <Pointer>[kbuf, koff, nbuf, noff, kid, node, vlen, lt, voff]) {
            calloc.free(p);
          }
        }
      } finally {
        host.decodedFree(d);
      }
    } finally {
      host.keysDestroy(keys);
      calloc.free(src);
      calloc.free(out);
    }
  }

  /// `for (m in changesets) merge(m)` as ONE device call: R sequential merges batched
  /// (the hot path; crdt_merge applies them with the reference's exact stop semantics).
  void mergeAll(List<Map<K, Record<V>>> changesets, {bool winners = true}) {
    final R = changesets.length;
    if (R == 0) return;
    _registerNodes([for (final cs in changesets) for (final r in cs.values) r.hlc.nodeId]);
    final n = changesets.fold<int>(0, (s, cs) => s + cs.length);
    final kid = calloc<Uint32>(n == 0 ? 1 : n), rank = calloc<Uint32>(n == 0 ? 1 : n);
    final val = calloc<Uint32>(n == 0 ? 1 : n), lt = calloc<Int64>(n == 0 ? 1 : n);
    final offsets = calloc<Uint64>(R + 1), flags = calloc<Uint8>(n == 0 ? 1 : n);
    final batch = calloc<CrdtBatch>(), res = calloc<CrdtResult>();
    Pointer<Int64> millis = nullptr;
    final newIdStart = <int>[];
    try {
      final odd = <int, int>{}; // record index -> Hlc.millis outside the lt form (counter > 0xFFFF)
      var i = 0;
      for (var j = 0; j < R; ++j) {
        newIdStart.add(_keys.length);
        changesets[j].forEach((k, r) {
          kid[i] = _intern(k);
          lt[i] = r.hlc.logicalTime;
          rank[i] = _nodes.rank(r.hlc.nodeId);
          val[i] = _values.put(r.value);
          if (!_canonicalForm(r.hlc)) odd[i] = r.hlc.millis;
          ++i;
        });
        offsets[j + 1] = i;
      }
      newIdStart.add(_keys.length);
      if (odd.isNotEmpty) {
        // the complete lt column first, then the odd ones patched in
        millis = calloc<Int64>(n);
        for (var x = 0; x < n; ++x) {
          millis[x] = lt[x] >> 16;
        }
        odd.forEach((x, ms) => millis[x] = ms);
      }
      _reserve();
      batch.ref
        ..keyId = kid
        ..lt = lt
        ..rank = rank
        ..val = val
        ..millis = millis
        ..offsets = offsets
        ..nChangesets = R
        ..mem = crdtMemHost;
      final st = _lib.merge(_c, batch, DateTime.now().millisecondsSinceEpoch, winners ? flags : nullptr, res);
      if (st < 0) {
        // the library refused the call (nothing stored on a single context, crdt_merge.h): forget
        // the keys and value handles this batch interned, as MapCrdt.mergeAll does (crdt.py)
        _truncateKeys(newIdStart[0]);
        for (var x = 0; x < n; ++x) {
          _values.release(val[x]);
        }
        _check(st, 'crdt_merge');
      }
      final stop = res.ref.nStored;
      _truncateKeys(newIdStart[stop]); // keys first seen in changesets never stored
      final storedEnd = offsets[stop];
      if (!winners) {                  // bulk form: no per-record outcome; the stored changesets'
        for (var x = storedEnd; x < n; ++x) {   // handles stay referenced (losers unknown until
          _values.release(val[x]);              // the next compaction), the unstored ones are released
        }
        _maybeCompact();
        _rethrow(res);
        return;
      }
      final won = Uint8List.fromList(flags.asTypedList(n == 0 ? 1 : n));
      for (var x = 0; x < n; ++x) {
        if (x >= storedEnd || won[x] == 0) _values.release(val[x]);
      }
      // removeWhere (crdt.dart:80-85): every stored changeset keeps only its winners
      for (var j = 0; j < stop; ++j) {
        final cs = changesets[j];
        final b = offsets[j];
        var x = 0;
        final losers = <K>[];
        for (final k in cs.keys) {
          if (won[b + x] == 0) losers.add(k);
          ++x;
        }
        losers.forEach(cs.remove);
        cs.forEach((k, r) {
          _noteOverrides(_keyIds[k]!, r.hlc, null);
          _controller.add(MapEntry(k, r.value)); // map_crdt.dart:36-38
        });
      }
      _maybeCompact();
      _rethrow(res); // after the partial state is committed, like the reference
    } finally {
      calloc.free(kid);
      calloc.free(rank);
      calloc.free(val);
      calloc.free(lt);
      calloc.free(offsets);
      calloc.free(flags);
      calloc.free(batch);
      calloc.free(res);
      if (millis != nullptr) calloc.free(millis);
    }
  }

  /// A bulk catch-up merge that needs neither the removeWhere side effect nor watch()
  /// events: no win flags, per-record counts off, so crdt_merge may take the sorted path in
  /// its order-free form (same rows, canonical and exceptions; DESIGN.md §5.2).
  ///
  /// A batch that needs per-record host bookkeeping — an Hlc outside the (millis << 16) + counter
  /// form, or a key whose stored Hlc / modified is kept on the host — runs as [mergeAll] on copies
  /// of the maps (mirrors MapCrdt.mergeAllBulk in crdt_amd/crdt.py).
  void mergeAllBulk(List<Map<K, Record<V>>> changesets) {
    bool hostKept(K k) {
      final id = _keyIds[k];
      return id != null && (_hlcOverride.containsKey(id) || _modOverride.containsKey(id));
    }

    final needsHost = changesets.any((cs) => cs.entries.any((e) => !_canonicalForm(e.value.hlc) || hostKept(e.key)));
    if (needsHost) {
      mergeAll([for (final cs in changesets) Map<K, Record<V>>.of(cs)]);
      return;
    }
    _check(_lib.setCounts(_c, 0), 'crdt_set_counts');
    try {
      mergeAll(changesets, winners: false);
    } finally {
      _check(_lib.setCounts(_c, 1), 'crdt_set_counts');
    }
  }
}
