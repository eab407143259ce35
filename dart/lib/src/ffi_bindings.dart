// dart:ffi bindings of include/crdt_merge.h (libcrdt_mi355x.so): the structs and the entry
// points GpuMapCrdt calls.  Field order and widths follow the header exactly
// (tests/test_host_cpu.py checks the same layout against the C compiler for the ctypes side).
import 'dart:ffi';

const int crdtOk = 0;
const int crdtClockDrift = 1; // ClockDriftException   hlc.dart:164-171
const int crdtDuplicateNode = 2; // DuplicateNodeException hlc.dart:182-189
const int crdtOverflow = 3; // OverflowException      hlc.dart:173-180
const int crdtMemHost = 0;
const int crdtMemDevice = 1;
const int crdtNullValue = 0xFFFFFFFF;
const int crdtPathAuto = 0, crdtPathGather = 1, crdtPathSorted = 2;

/// crdt_batch: R changesets concatenated column-wise (changeset j = rows [offsets[j], offsets[j+1])).
class CrdtBatch extends Struct {
  external Pointer<Uint32> keyId;
  external Pointer<Int64> lt;
  external Pointer<Uint32> rank;
  external Pointer<Uint32> val;
  external Pointer<Int64> millis; // nullptr: millis = lt >> 16
  external Pointer<Uint64> offsets; // host memory, [nChangesets + 1]
  @Uint32()
  external int nChangesets;
  @Int32()
  external int mem;
}

/// crdt_result: outcome of a merge / put call.
class CrdtResult extends Struct {
  @Int32()
  external int status;
  @Uint32()
  external int nStored;
  @Uint32()
  external int excChangeset;
  @Uint32()
  external int reserved;
  @Uint64()
  external int excIndex;
  @Int64()
  external int canonicalLt;
  @Int64()
  external int driftMs;
  @Int64()
  external int counter;
  @Uint64()
  external int nPresent;
  @Uint64()
  external int nWon;
}

typedef _CreateC = Int32 Function(Int32, Uint32, Uint64, Pointer<Pointer<Void>>);
typedef _CreateD = int Function(int, int, int, Pointer<Pointer<Void>>);
typedef _DestroyC = Void Function(Pointer<Void>);
typedef _DestroyD = void Function(Pointer<Void>);
typedef _CtxU64C = Int32 Function(Pointer<Void>, Uint64);
typedef _CtxU64D = int Function(Pointer<Void>, int);
typedef _CtxU32C = Int32 Function(Pointer<Void>, Uint32);
typedef _CtxIntC = Int32 Function(Pointer<Void>, Int32);
typedef _CtxIntD = int Function(Pointer<Void>, int);
typedef _CtxPtrC = Int32 Function(Pointer<Void>, Pointer<Void>);
typedef _CtxPtrD = int Function(Pointer<Void>, Pointer<Void>);
typedef _SetCanonC = Int32 Function(Pointer<Void>, Int64);
typedef _PutRowsC = Int32 Function(Pointer<Void>, Pointer<Uint32>, Pointer<Int64>, Pointer<Uint32>,
    Pointer<Uint32>, Pointer<Int64>, Uint64, Int32);
typedef _PutRowsD = int Function(Pointer<Void>, Pointer<Uint32>, Pointer<Int64>, Pointer<Uint32>,
    Pointer<Uint32>, Pointer<Int64>, int, int);
typedef _ReadRowsC = Int32 Function(Pointer<Void>, Pointer<Uint32>, Uint64, Pointer<Int64>, Pointer<Uint32>,
    Pointer<Uint32>, Pointer<Int64>, Int32);
typedef _ReadRowsD = int Function(Pointer<Void>, Pointer<Uint32>, int, Pointer<Int64>, Pointer<Uint32>,
    Pointer<Uint32>, Pointer<Int64>, int);
typedef _ModSinceC = Int32 Function(Pointer<Void>, Uint64, Int64, Pointer<Uint32>, Pointer<Uint64>);
typedef _ModSinceD = int Function(Pointer<Void>, int, int, Pointer<Uint32>, Pointer<Uint64>);
typedef _ClearC = Int32 Function(Pointer<Void>, Uint64, Uint64);
typedef _ClearD = int Function(Pointer<Void>, int, int);
typedef _RemapC = Int32 Function(Pointer<Void>, Uint64, Pointer<Uint32>, Uint32);
typedef _RemapD = int Function(Pointer<Void>, int, Pointer<Uint32>, int);
typedef _PutStampedC = Int32 Function(
    Pointer<Void>, Pointer<Uint32>, Pointer<Uint32>, Uint64, Int64, Int32, Pointer<CrdtResult>);
typedef _PutStampedD = int Function(
    Pointer<Void>, Pointer<Uint32>, Pointer<Uint32>, int, int, int, Pointer<CrdtResult>);
typedef _RefreshC = Int32 Function(Pointer<Void>, Uint64, Pointer<Int64>);
typedef _RefreshD = int Function(Pointer<Void>, int, Pointer<Int64>);
typedef _MergeC = Int32 Function(
    Pointer<Void>, Pointer<CrdtBatch>, Int64, Pointer<Uint8>, Pointer<CrdtResult>);
typedef _MergeD = int Function(Pointer<Void>, Pointer<CrdtBatch>, int, Pointer<Uint8>, Pointer<CrdtResult>);
typedef _StatusStrC = Pointer<Uint8> Function(Int32);
typedef _StatusStrD = Pointer<Uint8> Function(int);
// key-sharded multi-GPU (include/crdt_merge.h, "key-sharded multi-GPU")
typedef _CommIdC = Int32 Function(Pointer<Uint8>);
typedef _CommIdD = int Function(Pointer<Uint8>);
typedef _CommInitC = Int32 Function(Pointer<Void>, Uint32, Uint32, Pointer<Uint8>);
typedef _CommInitD = int Function(Pointer<Void>, int, int, Pointer<Uint8>);
typedef _CommInfoC = Int32 Function(Pointer<Void>, Pointer<Uint32>, Pointer<Uint32>);
typedef _CommInfoD = int Function(Pointer<Void>, Pointer<Uint32>, Pointer<Uint32>);
typedef _CtxOnlyC = Int32 Function(Pointer<Void>);
typedef _CtxOnlyD = int Function(Pointer<Void>);

const int crdtCommIdBytes = 128;
/// include/crdt_merge.h CRDT_ABI_VERSION: the struct layouts above are this version's.
const int crdtAbiVersion = 5;
typedef _AbiC = Int32 Function();
typedef _AbiD = int Function();

/// The library's entry points, looked up once.
class CrdtLib {
  CrdtLib(DynamicLibrary lib)
      : create = lib.lookupFunction<_CreateC, _CreateD>('crdt_create'),
        destroy = lib.lookupFunction<_DestroyC, _DestroyD>('crdt_destroy'),
        reserve = lib.lookupFunction<_CtxU64C, _CtxU64D>('crdt_reserve'),
        capacity = lib.lookupFunction<_CtxPtrC, _CtxPtrD>('crdt_capacity'),
        setLocalRank = lib.lookupFunction<_CtxU32C, _CtxIntD>('crdt_set_local_rank'),
        getCanonical = lib.lookupFunction<_CtxPtrC, _CtxPtrD>('crdt_get_canonical'),
        setCanonical = lib.lookupFunction<_SetCanonC, _CtxIntD>('crdt_set_canonical'),
        putRows = lib.lookupFunction<_PutRowsC, _PutRowsD>('crdt_put_rows'),
        readRows = lib.lookupFunction<_ReadRowsC, _ReadRowsD>('crdt_read_rows'),
        modifiedSince = lib.lookupFunction<_ModSinceC, _ModSinceD>('crdt_modified_since'),
        clearRows = lib.lookupFunction<_ClearC, _ClearD>('crdt_clear_rows'),
        remapRanks = lib.lookupFunction<_RemapC, _RemapD>('crdt_remap_ranks'),
        putStamped = lib.lookupFunction<_PutStampedC, _PutStampedD>('crdt_put_stamped'),
        refreshCanonical = lib.lookupFunction<_RefreshC, _RefreshD>('crdt_refresh_canonical'),
        merge = lib.lookupFunction<_MergeC, _MergeD>('crdt_merge'),
        setMergePath = lib.lookupFunction<_CtxIntC, _CtxIntD>('crdt_set_merge_path'),
        setCounts = lib.lookupFunction<_CtxIntC, _CtxIntD>('crdt_set_counts'),
        setRankBound = lib.lookupFunction<_CtxU32C, _CtxIntD>('crdt_set_rank_bound'),
        statusString = lib.lookupFunction<_StatusStrC, _StatusStrD>('crdt_status_string'),
        commUniqueId = lib.lookupFunction<_CommIdC, _CommIdD>('crdt_comm_unique_id'),
        commInitRccl = lib.lookupFunction<_CommInitC, _CommInitD>('crdt_comm_init_rccl'),
        commInfo = lib.lookupFunction<_CommInfoC, _CommInfoD>('crdt_comm_info'),
        commFree = lib.lookupFunction<_CtxOnlyC, _CtxOnlyD>('crdt_comm_free'),
        setPresharded = lib.lookupFunction<_CtxIntC, _CtxIntD>('crdt_set_presharded'),
        setCommTimeout = lib.lookupFunction<_CtxU32C, _CtxIntD>('crdt_set_comm_timeout');

  /// Opens the library and refuses one built against another ABI (crdt_timing / crdt_result layouts).
  factory CrdtLib.open([String path = 'libcrdt_mi355x.so']) {
    final lib = DynamicLibrary.open(path);
    final abi = lib.lookupFunction<_AbiC, _AbiD>('crdt_abi_version')();
    if (abi != crdtAbiVersion) {
      throw StateError('$path has C-ABI $abi, these bindings expect $crdtAbiVersion');
    }
    return CrdtLib(lib);
  }

  final _CreateD create;
  final _DestroyD destroy;
  final _CtxU64D reserve;
  final _CtxPtrD capacity;
  final _CtxIntD setLocalRank;
  final _CtxPtrD getCanonical;
  final _CtxIntD setCanonical;
  final _PutRowsD putRows;
  final _ReadRowsD readRows;
  final _ModSinceD modifiedSince;
  final _ClearD clearRows;
  final _RemapD remapRanks;
  final _PutStampedD putStamped;
  final _RefreshD refreshCanonical;
  final _MergeD merge;
  final _CtxIntD setMergePath;
  final _CtxIntD setCounts;
  final _CtxIntD setRankBound;
  final _StatusStrD statusString;
  final _CommIdD commUniqueId;
  final _CommInitD commInitRccl;
  final _CommInfoD commInfo;
  final _CtxOnlyD commFree;
  /// crdt_set_comm_timeout: a collective merge's deadline (ms; 0 = none) — past it the communicator is
  /// aborted and the merge throws (CRDT_E_COMM) instead of waiting forever on a lost peer.
  final _CtxIntD setCommTimeout;
  final _CtxIntD setPresharded;
}

// ---------------------------------------------------------------------------------------------
// dart:ffi bindings of include/crdt_host.h (libcrdt_host.so, no GPU code): the native CrdtJson.decode
// that GpuMapCrdt.mergeJson uses (crdt.dart:100-109, crdt_json.dart:19-37), as crdt_amd/hostlib.py does.
const int crdtHostOk = 0;
const int crdtHostFallback = 1; // valid input outside the fast path: decode it with CrdtJson.decode
const int crdtHostEJson = -2; // malformed JSON: jsonDecode would throw FormatException

typedef _KeysCreateC = Pointer<Void> Function();
typedef _KeysDestroyC = Void Function(Pointer<Void>);
typedef _KeysDestroyD = void Function(Pointer<Void>);
typedef _KeysSizeC = Uint64 Function(Pointer<Void>);
typedef _KeysSizeD = int Function(Pointer<Void>);
typedef _KeysBytesC = Uint64 Function(Pointer<Void>, Uint64, Uint64);
typedef _KeysBytesD = int Function(Pointer<Void>, int, int);
typedef _KeysExportC = Int32 Function(Pointer<Void>, Uint64, Uint64, Pointer<Uint8>, Uint64, Pointer<Uint64>);
typedef _KeysExportD = int Function(Pointer<Void>, int, int, Pointer<Uint8>, int, Pointer<Uint64>);
typedef _DecodeC = Int32 Function(Pointer<Uint8>, Uint64, Pointer<Void>, Pointer<Pointer<Void>>);
typedef _DecodeD = int Function(Pointer<Uint8>, int, Pointer<Void>, Pointer<Pointer<Void>>);
typedef _DecNodeCountC = Uint32 Function(Pointer<Void>);
typedef _DecColumnsC = Int32 Function(
    Pointer<Void>, Pointer<Uint32>, Pointer<Int64>, Pointer<Uint32>, Pointer<Uint64>, Pointer<Uint32>);
typedef _DecColumnsD = int Function(
    Pointer<Void>, Pointer<Uint32>, Pointer<Int64>, Pointer<Uint32>, Pointer<Uint64>, Pointer<Uint32>);
typedef _DecNodesC = Int32 Function(Pointer<Void>, Pointer<Uint8>, Uint64, Pointer<Uint64>);
typedef _DecNodesD = int Function(Pointer<Void>, Pointer<Uint8>, int, Pointer<Uint64>);

class CrdtHostLib {
  CrdtHostLib(DynamicLibrary lib)
      : keysCreate = lib.lookupFunction<_KeysCreateC, _KeysCreateC>('crdt_keys_create'),
        keysDestroy = lib.lookupFunction<_KeysDestroyC, _KeysDestroyD>('crdt_keys_destroy'),
        keysSize = lib.lookupFunction<_KeysSizeC, _KeysSizeD>('crdt_keys_size'),
        keysBytes = lib.lookupFunction<_KeysBytesC, _KeysBytesD>('crdt_keys_bytes'),
        keysExport = lib.lookupFunction<_KeysExportC, _KeysExportD>('crdt_keys_export'),
        jsonDecode = lib.lookupFunction<_DecodeC, _DecodeD>('crdt_json_decode'),
        decodedFree = lib.lookupFunction<_KeysDestroyC, _KeysDestroyD>('crdt_decoded_free'),
        decodedCount = lib.lookupFunction<_KeysSizeC, _KeysSizeD>('crdt_decoded_count'),
        decodedNodeCount = lib.lookupFunction<_DecNodeCountC, _KeysSizeD>('crdt_decoded_node_count'),
        decodedColumns = lib.lookupFunction<_DecColumnsC, _DecColumnsD>('crdt_decoded_columns'),
        decodedNodeBytes = lib.lookupFunction<_KeysSizeC, _KeysSizeD>('crdt_decoded_node_bytes'),
        decodedNodes = lib.lookupFunction<_DecNodesC, _DecNodesD>('crdt_decoded_nodes');

  /// The host library, or null when it cannot be opened (mergeJson then decodes in Dart).
  static CrdtHostLib? tryOpen([String path = 'libcrdt_host.so']) {
    try {
      return CrdtHostLib(DynamicLibrary.open(path));
    } catch (_) {
      return null;
    }
  }

  final _KeysCreateC keysCreate;
  final _KeysDestroyD keysDestroy;
  final _KeysSizeD keysSize;
  final _KeysBytesD keysBytes;
  final _KeysExportD keysExport;
  final _DecodeD jsonDecode;
  final _KeysDestroyD decodedFree;
  final _KeysSizeD decodedCount;
  final _KeysSizeD decodedNodeCount;
  final _DecColumnsD decodedColumns;
  final _KeysSizeD decodedNodeBytes;
  final _DecNodesD decodedNodes;
}
