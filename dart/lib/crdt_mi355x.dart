/// GPU-backed MapCrdt (include/crdt_merge.h over dart:ffi).  Re-exports the reference API
/// (package:crdt, lib/crdt.dart:3-7) so `import 'package:crdt_mi355x/crdt_mi355x.dart'` is
/// the only import a MapCrdt user changes.
library crdt_mi355x;

export 'package:crdt/crdt.dart';

export 'src/gpu_map_crdt.dart';
