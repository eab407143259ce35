"""``CrdtJson`` — mirror of ``lib/src/crdt_json.dart:5-38`` (host-side codec)."""
from __future__ import annotations

import json

from .hlc import Hlc
from .record import Record


def _default(o):
    to_json = getattr(o, "toJson", None)
    if callable(to_json):                 # dart:convert calls toJson() on objects
        return to_json()
    raise TypeError(f"Converting object to an encodable object failed: {o!r}")


class CrdtJson:
    @staticmethod
    def encode(record_map: dict, keyEncoder=None, valueEncoder=None) -> str:   # crdt_json.dart:8-17
        out = {}
        for k, r in record_map.items():
            out[str(k) if keyEncoder is None else keyEncoder(k)] = r.toJson(k, valueEncoder=valueEncoder)
        return json.dumps(out, separators=(",", ":"), ensure_ascii=False, default=_default)

    @staticmethod
    def decode(js: str, canonicalTime: Hlc, keyDecoder=None, valueDecoder=None, nodeIdDecoder=None,
               millis: int | None = None) -> dict:                            # crdt_json.dart:19-37
        now = Hlc.now(canonicalTime.nodeId, millis)
        modified = canonicalTime if canonicalTime >= now else now
        out = {}
        for k, v in json.loads(js).items():
            key = k if keyDecoder is None else keyDecoder(k)
            out[key] = Record.fromJson(k, v, modified, valueDecoder=valueDecoder, nodeIdDecoder=nodeIdDecoder)
        return out
