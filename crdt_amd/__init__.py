"""crdt_amd — MI355X-native MapCrdt merge hot path (drop-in for Dart ``crdt`` v4.0.2).

Public names mirror the reference barrel ``lib/crdt.dart:3-7``.
"""
from .crdt import Crdt, MapCrdt, Watch
from .crdt_json import CrdtJson
from .device import CrdtNativeError, DeviceTable
from .hlc import ClockDriftException, DuplicateNodeException, Hlc, OverflowException
from .record import Record

__all__ = ["Crdt", "MapCrdt", "Watch", "CrdtJson", "DeviceTable", "CrdtNativeError", "Hlc", "Record",
           "ClockDriftException", "DuplicateNodeException", "OverflowException"]
