"""Hybrid Logical Clock — host-side mirror of ``lib/src/hlc.dart``.

Scalar clock arithmetic stays on the host (one ``send`` per merge/put call);
the batched ``recv`` of a merge runs on the GPU (``crdt_merge.hip`` K3a-K3d).
Names and semantics follow the reference class ``Hlc<T>`` (hlc.dart:11-162);
the optional ``millis`` arguments are the reference's own clock-injection
parameters (hlc.dart:51,80).
"""
from __future__ import annotations

import random
import re
import time

SHIFT = 16                      # hlc.dart:3
MAX_COUNTER = 0xFFFF            # hlc.dart:4
MAX_DRIFT = 60000               # hlc.dart:5
_M64 = (1 << 64) - 1


def wrap64(x: int) -> int:
    """Dart VM int: two's-complement 64-bit wrap."""
    x &= _M64
    return x - (1 << 64) if x >> 63 else x


def _tdiv(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def now_millis() -> int:
    return time.time_ns() // 1_000_000


# --------------------------------------------------------------- node-id order
def node_sort_key(node_id):
    """Sort key reproducing Dart ``compareTo`` for String (UTF-16 code units) and int node ids."""
    if isinstance(node_id, str):
        return node_id.encode("utf-16-be", "surrogatepass")
    if isinstance(node_id, int) and not isinstance(node_id, bool):
        return node_id
    raise TypeError(f"node id must be String or int, got {type(node_id).__name__}")


def compare_node_ids(a, b) -> int:
    if type(a) is not type(b) and not (isinstance(a, int) and isinstance(b, int)):
        raise TypeError(f"cannot compare {type(a).__name__} with {type(b).__name__}")
    ka, kb = node_sort_key(a), node_sort_key(b)
    return (ka > kb) - (ka < kb)


# ------------------------------------------------------------ ISO-8601 (UTC)
def _days_from_civil(y: int, m: int, d: int) -> int:
    y -= m <= 2
    era = y // 400
    yoe = y - era * 400
    doy = (153 * ((m + 9) % 12) + 2) // 5 + d - 1
    return era * 146097 + yoe * 365 + yoe // 4 - yoe // 100 + doy - 719468


def _civil_from_days(z: int):
    z += 719468
    era = z // 146097
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    m = mp + 3 if mp < 10 else mp - 9
    return yoe + era * 400 + (m <= 2), m, doy - (153 * mp + 2) // 5 + 1


_MAX_MS = 8_640_000_000_000_000
_ISO_RE = re.compile(
    r"^([+-]?\d{4,6})-?(\d\d)-?(\d\d)"
    r"(?:[ T](\d\d)(?::?(\d\d)(?::?(\d\d)(?:[.,](\d+))?)?)?"
    r"( ?[zZ]| ?([-+])(\d\d)(?::?(\d\d))?)?)?$")
_FAST_ISO = re.compile(r"^(\d{4})-(\d\d)-(\d\d)T(\d\d):(\d\d):(\d\d)\.(\d{3})Z$")


def iso_from_millis(ms: int) -> str:
    """``DateTime.fromMillisecondsSinceEpoch(ms, isUtc: true).toIso8601String()``."""
    if abs(ms) > _MAX_MS:
        raise ValueError(f"Invalid time value {ms}")
    days, rem = divmod(ms, 86_400_000)
    y, mo, d = _civil_from_days(days)
    h, rem = divmod(rem, 3_600_000)
    mi, rem = divmod(rem, 60_000)
    s, milli = divmod(rem, 1000)
    if -9999 <= y <= 9999:
        ys = ("-" if y < 0 else "") + str(abs(y)).rjust(4, "0")
    else:
        ys = ("-" if y < 0 else "+") + str(abs(y)).rjust(6, "0")
    return f"{ys}-{mo:02d}-{d:02d}T{h:02d}:{mi:02d}:{s:02d}.{milli:03d}Z"


def millis_from_iso(s: str) -> int:
    """``DateTime.parse(s).millisecondsSinceEpoch``; zone-less strings are read as UTC."""
    f = _FAST_ISO.match(s)
    if f:
        y, mo, d, h, mi, sec, milli = (int(g) for g in f.groups())
        if 1 <= mo <= 12:
            return ((_days_from_civil(y, mo, d) * 24 + h) * 60 + mi) * 60_000 + sec * 1000 + milli
    m = _ISO_RE.match(s)
    if not m:
        raise ValueError(f"Invalid date format {s}")
    year, month, day = int(m.group(1)), int(m.group(2)), int(m.group(3))
    hour, minute, second = int(m.group(4) or 0), int(m.group(5) or 0), int(m.group(6) or 0)
    micros = int((m.group(7) + "000000")[:6]) if m.group(7) else 0
    mz = month - 1
    year += mz // 12
    mz %= 12
    days = _days_from_civil(year, mz + 1, 1) + day - 1
    us = ((((days * 24 + hour) * 60 + minute) * 60) + second) * 1_000_000 + micros
    if m.group(8) is not None and m.group(9) is not None:
        sign = -1 if m.group(9) == "-" else 1
        us -= sign * (int(m.group(10)) * 60 + int(m.group(11) or 0)) * 60_000_000
    ms = _tdiv(us, 1000)
    if abs(ms) > _MAX_MS:
        raise ValueError(f"Time out of range {s}")
    return ms


# ------------------------------------------------------------------ exceptions
class ClockDriftException(Exception):
    """hlc.dart:164-171"""

    def __init__(self, millis_ts: int, millis_wall: int | None = None):
        self.drift = wrap64(millis_ts - millis_wall) if millis_wall is not None else millis_ts
        super().__init__(str(self))

    def __str__(self):
        return f"Clock drift of {self.drift} ms exceeds maximum ({MAX_DRIFT})"


class OverflowException(Exception):
    """hlc.dart:173-180"""

    def __init__(self, counter: int):
        self.counter = counter
        super().__init__(str(self))

    def __str__(self):
        return f"Timestamp counter overflow: {self.counter}"


class DuplicateNodeException(Exception):
    """hlc.dart:182-189"""

    def __init__(self, node_id: str):
        self.nodeId = node_id
        super().__init__(str(self))

    def __str__(self):
        return f"Duplicate node: {self.nodeId}"


# ------------------------------------------------------------------------ Hlc
class Hlc:
    """``Hlc<T>`` (hlc.dart:11-162)."""

    __slots__ = ("millis", "counter", "nodeId")

    def __init__(self, millis: int, counter: int, nodeId):
        # hlc.dart:18-23: microseconds are detected and converted to millis
        self.millis = millis if millis < 0x0001000000000000 else _tdiv(millis, 1000)
        self.counter = counter
        self.nodeId = nodeId

    @property
    def logicalTime(self) -> int:                                    # hlc.dart:16
        return wrap64(wrap64(self.millis << SHIFT) + self.counter)

    @property
    def is_canonical_form(self) -> bool:
        """True when (millis, counter) round-trips through logicalTime."""
        lt = self.logicalTime
        return (lt >> SHIFT) == self.millis and (lt & MAX_COUNTER) == self.counter

    @classmethod
    def zero(cls, nodeId):                                           # hlc.dart:25
        return cls(0, 0, nodeId)

    @classmethod
    def fromDate(cls, millis_since_epoch: int, nodeId):              # hlc.dart:33
        return cls(millis_since_epoch, 0, nodeId)

    @classmethod
    def now(cls, nodeId, millis: int | None = None):                # hlc.dart:35
        return cls(now_millis() if millis is None else millis, 0, nodeId)

    @classmethod
    def fromLogicalTime(cls, logicalTime: int, nodeId):              # hlc.dart:37
        return cls(logicalTime >> SHIFT, logicalTime & MAX_COUNTER, nodeId)

    def copyWith(self, millis=None, counter=None, nodeId=None):      # hlc.dart:27-31
        return Hlc(self.millis if millis is None else millis,
                   self.counter if counter is None else counter,
                   self.nodeId if nodeId is None else nodeId)

    apply = copyWith

    @classmethod
    def parse(cls, timestamp: str, idDecoder=None):                  # hlc.dart:39-46
        colon = timestamp.rfind(":")
        if colon < 0:
            raise ValueError(f"RangeError: no ':' in {timestamp!r}")
        counter_dash = timestamp.find("-", colon)
        node_dash = timestamp.find("-", counter_dash + 1) if counter_dash >= 0 else -1
        if counter_dash < 0 or node_dash < 0:
            raise ValueError(f"RangeError: malformed timestamp {timestamp!r}")
        millis = millis_from_iso(timestamp[:counter_dash])
        cs = timestamp[counter_dash + 1:node_dash]
        if not re.fullmatch(r"[+-]?[0-9A-Fa-f]+", cs):
            raise ValueError(f"FormatException: {cs}")
        counter = wrap64(int(cs, 16))
        node = timestamp[node_dash + 1:]
        return cls(millis, counter, idDecoder(node) if idDecoder else node)

    @classmethod
    def send(cls, canonical: "Hlc", millis: int | None = None) -> "Hlc":   # hlc.dart:51-74
        if millis is None:
            millis = now_millis()
        millis_old, counter_old = canonical.millis, canonical.counter
        millis_new = max(millis_old, millis)
        counter_new = counter_old + 1 if millis_old == millis_new else 0
        if wrap64(millis_new - millis) > MAX_DRIFT:
            raise ClockDriftException(millis_new, millis)
        if counter_new > MAX_COUNTER:
            raise OverflowException(counter_new)
        return cls(millis_new, counter_new, canonical.nodeId)

    @classmethod
    def recv(cls, canonical: "Hlc", remote: "Hlc", millis: int | None = None) -> "Hlc":  # :80-97
        if millis is None:
            millis = now_millis()
        if canonical.logicalTime >= remote.logicalTime:
            return canonical
        if canonical.nodeId == remote.nodeId:
            raise DuplicateNodeException(str(canonical.nodeId))
        if wrap64(remote.millis - millis) > MAX_DRIFT:
            raise ClockDriftException(remote.millis, millis)
        return cls.fromLogicalTime(remote.logicalTime, canonical.nodeId)

    def toJson(self) -> str:
        return str(self)

    def __str__(self) -> str:                                        # hlc.dart:101-104
        c = ("-" + format(-self.counter, "X")) if self.counter < 0 else format(self.counter, "X")
        return f"{iso_from_millis(self.millis)}-{c.rjust(4, '0')}-{self.nodeId}"

    def pack(self) -> str:                                           # hlc.dart:110-119
        return (_b36(self.millis).rjust(10, "0")[:10] + _b36(self.counter).rjust(4, "0")[:4]
                + str(self.nodeId))

    @staticmethod
    def unpack(packed: str) -> "Hlc":                                # hlc.dart:122-128
        return Hlc(int(packed[:10], 36), int(packed[10:14], 36), packed[14:])

    @staticmethod
    def randomNodeId() -> str:                                       # hlc.dart:133-141
        r = random.SystemRandom()
        return (_b36(r.randrange(1 << 32)) + _b36(r.randrange(1 << 32))).rjust(10, "0")[:10]

    def compareTo(self, other: "Hlc") -> int:                       # hlc.dart:157-161
        a, b = self.logicalTime, other.logicalTime
        if a != b:
            return -1 if a < b else 1
        return compare_node_ids(self.nodeId, other.nodeId)

    def __eq__(self, other):
        return isinstance(other, Hlc) and self.compareTo(other) == 0

    def __hash__(self):
        return hash(str(self))

    def __lt__(self, other):
        return self.compareTo(other) < 0

    def __le__(self, other):
        return self < other or self == other

    def __gt__(self, other):
        return self.compareTo(other) > 0

    def __ge__(self, other):
        return self > other or self == other

    def __repr__(self):
        return f"Hlc({self})"


def _b36(n: int) -> str:
    if n < 0:
        return "-" + _b36(-n)
    digits = "0123456789abcdefghijklmnopqrstuvwxyz"
    out = ""
    while True:
        n, r = divmod(n, 36)
        out = digits[r] + out
        if n == 0:
            return out
