"""``Record<V>`` — mirror of ``lib/src/record.dart:12-39``."""
from __future__ import annotations

from .hlc import Hlc


class Record:
    __slots__ = ("hlc", "value", "modified")

    def __init__(self, hlc: Hlc, value, modified: Hlc):
        self.hlc = hlc
        self.value = value
        self.modified = modified

    @property
    def isDeleted(self) -> bool:                                      # record.dart:17
        return self.value is None

    @classmethod
    def fromJson(cls, key, m: dict, modified: Hlc, valueDecoder=None, nodeIdDecoder=None):
        hlc = Hlc.parse(m["hlc"], nodeIdDecoder)                      # record.dart:21-26
        v = m.get("value")
        value = v if valueDecoder is None or v is None else valueDecoder(key, v)
        return cls(hlc, value, modified)

    def toJson(self, key, valueEncoder=None) -> dict:                  # record.dart:28-31
        return {"hlc": self.hlc.toJson(),
                "value": self.value if valueEncoder is None else valueEncoder(key, self.value)}

    def __eq__(self, other):                                          # record.dart:33-35
        return isinstance(other, Record) and self.hlc == other.hlc and self.value == other.value

    def __hash__(self):
        return hash(str(self.hlc))

    def __repr__(self):
        return f"Record({self.hlc}, {self.value!r})"
