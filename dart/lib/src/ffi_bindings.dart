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
        statusString = lib.lookupFunction<_StatusStrC, _StatusStrD>('crdt_status_string');

  factory CrdtLib.open([String path = 'libcrdt_mi355x.so']) => CrdtLib(DynamicLibrary.open(path));

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
}
