"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's merge path.

This module is the *checker*, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The shipped path (``crdt_amd``) must never import anything under
``oracle/``.

It restates, in plain Python, the sequential semantics of the Dart package
``crdt`` v4.0.2 (``/root/reference``; ``pubspec.yaml:3``) for the code on the
``MapCrdt`` merge path, object for object:

* ``Hlc``            — ``lib/src/hlc.dart:11-162``
* exceptions         — ``lib/src/hlc.dart:164-189``
* ``Record``         — ``lib/src/record.dart:12-39``
* ``Crdt``/``MapCrdt`` — ``lib/src/crdt.dart:7-170``, ``lib/src/map_crdt.dart:9-53``
* ``CrdtJson``       — ``lib/src/crdt_json.dart:5-38``

Deviations (documented in DESIGN.md):

* The reference reads ``DateTime.now()`` per record (``hlc.dart:53,82``).  Here
  every clock read takes an explicit ``wall`` (ms since epoch), constant for one
  call, as ``Hlc.send``/``Hlc.recv`` already allow (``hlc.dart:51,80``).
* Dart ``int`` is a wrapping signed 64-bit integer; ``_wrap64`` reproduces it.
* ``DateTime.parse`` of a string without a zone designator is read as UTC here
  (Dart would use the host's local zone).  The reference itself only ever emits
  ``...Z`` strings (``hlc.dart:102``).

Parity pinning: this restatement is checked against every known-answer test of
``test/hlc_test.dart`` and the merge / delta / sync groups of
``test/map_crdt_test.dart`` and the ``crdtTests`` suite of
``test/crdt_test.dart`` (transliterated in ``tests/test_oracle_kat.py``).  The
``modified`` stamps and the canonical clock after a merge are not pinned by any
reference test; they rest on the source reading of ``crdt.dart:82,86-87,93``.
"""
from __future__ import annotations

import json
import datetime as _dt
import re

SHIFT = 16                      # hlc.dart:3
MAX_COUNTER = 0xFFFF            # hlc.dart:4
MAX_DRIFT = 60000               # hlc.dart:5

_M64 = (1 << 64) - 1


def _wrap64(x: int) -> int:
    """Dart VM int arithmetic: two's-complement 64-bit wrap."""
    x &= _M64
    return x - (1 << 64) if x >> 63 else x


def _trunc_div(a: int, b: int) -> int:
    """Dart ``~/`` on ints: truncating division."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


# ---------------------------------------------------------------------------
# Dart String.compareTo: UTF-16 code-unit lexicographic order [SDK]
# ---------------------------------------------------------------------------
def _utf16_units(s: str):
    b = s.encode("utf-16-be", "surrogatepass")
    return [int.from_bytes(b[i:i + 2], "big") for i in range(0, len(b), 2)]


def dart_compare(a, b) -> int:
    """``(a as Comparable).compareTo(b)`` for the node-id types the path uses."""
    if isinstance(a, str) and isinstance(b, str):
        ua, ub = _utf16_units(a), _utf16_units(b)
        return (ua > ub) - (ua < ub)
    if isinstance(a, int) and isinstance(b, int) and not isinstance(a, bool):
        return (a > b) - (a < b)
    raise TypeError(f"cannot compare {type(a).__name__} with {type(b).__name__}")


# ---------------------------------------------------------------------------
# DateTime helpers (UTC) — the subset of dart:core the path touches [SDK].
# Written independently of crdt_amd/hlc.py (which uses the civil-from-days arithmetic and a
# regular expression): calendar maths through Python's datetime.date ordinals, shifted by whole
# 400-year Gregorian cycles for years outside 1..9999, and a character scanner for the grammar.
# ---------------------------------------------------------------------------
_EPOCH_ORDINAL = _dt.date(1970, 1, 1).toordinal()
_CYCLE_DAYS = 146097                    # days in 400 Gregorian years (the calendar repeats)
_MAX_ORDINAL = _dt.date.max.toordinal()
_MAX_MS = 8640000000000000              # DateTime's range: +-10^8 days


def _ymd_from_epoch_days(days: int):
    """(year, month, day) of a day count since 1970-01-01, any year."""
    o = days + _EPOCH_ORDINAL
    cycles = 0
    if o < 1:
        cycles = -((1 - o + _CYCLE_DAYS - 1) // _CYCLE_DAYS)
    elif o > _MAX_ORDINAL:
        cycles = (o - _MAX_ORDINAL + _CYCLE_DAYS - 1) // _CYCLE_DAYS
    d = _dt.date.fromordinal(o - cycles * _CYCLE_DAYS)
    return d.year + 400 * cycles, d.month, d.day


def _epoch_days(year: int, month: int, day: int) -> int:
    """Days since 1970-01-01 of year-month-1 plus day - 1 (day may overflow the month, as DateTime
    normalises it); month in 1..12, any year."""
    cycles = 0
    if year < 1:
        cycles = -((1 - year + 399) // 400)
    elif year > 9999:
        cycles = (year - 9999 + 399) // 400
    first = _dt.date(year - 400 * cycles, month, 1).toordinal()
    return first - _EPOCH_ORDINAL + cycles * _CYCLE_DAYS + day - 1


def iso_from_millis(ms: int) -> str:
    """``DateTime.fromMillisecondsSinceEpoch(ms, isUtc: true).toIso8601String()``."""
    if abs(ms) > _MAX_MS:
        raise ValueError(f"RangeError: {ms}")
    days = ms // 86400000
    in_day = ms - days * 86400000
    y, mo, d = _ymd_from_epoch_days(days)
    t = _dt.time(in_day // 3600000, in_day // 60000 % 60, in_day // 1000 % 60, in_day % 1000 * 1000)
    if abs(y) <= 9999:
        year = ("-%04d" % -y) if y < 0 else "%04d" % y
    else:
        year = ("-%06d" % -y) if y < 0 else "+%06d" % y
    return "%s-%02d-%02dT%s.%03dZ" % (year, mo, d, t.strftime("%H:%M:%S"), t.microsecond // 1000)


class _Scan:
    """A cursor over the date string (DateTime.parse's grammar, scanned by hand)."""

    def __init__(self, s: str):
        self.s, self.i = s, 0

    def peek(self, chars: str) -> bool:
        return self.i < len(self.s) and self.s[self.i] in chars

    def take(self, chars: str) -> str:
        if self.peek(chars):
            self.i += 1
            return self.s[self.i - 1]
        return ""

    def digits(self, lo: int, hi: int):
        j = self.i
        while j < len(self.s) and j - self.i < hi and "0" <= self.s[j] <= "9":
            j += 1
        if j - self.i < lo:
            return None
        out = int(self.s[self.i:j])
        self.i = j
        return out

    def run_of_digits(self) -> str:
        j = self.i
        while j < len(self.s) and "0" <= self.s[j] <= "9":
            j += 1
        out = self.s[self.i:j]
        self.i = j
        return out


def millis_from_iso(s: str) -> int:
    """``DateTime.parse(s).millisecondsSinceEpoch`` (zone-less strings read as UTC).  The year takes
    4 to 6 digits: the longest that lets the rest of the string parse (a compact "20010909T..."
    has a 4-digit year)."""
    bad = ValueError(f"FormatException: Invalid date format {s}")
    for ylen in (6, 5, 4):
        try:
            return _millis_from_iso(s, ylen, bad)
        except _NoParse:
            continue
    raise bad


class _NoParse(Exception):
    pass


def _millis_from_iso(s: str, ylen: int, bad: ValueError) -> int:
    c = _Scan(s)
    sign = c.take("+-")
    year = c.digits(ylen, ylen)
    if year is None:
        raise _NoParse
    year = -year if sign == "-" else year
    c.take("-")
    month = c.digits(2, 2)
    c.take("-")
    day = c.digits(2, 2)
    if month is None or day is None:
        raise _NoParse
    hour = minute = second = micros = 0
    zone = None
    if c.take(" T"):
        hour = c.digits(2, 2)
        if hour is None:
            raise _NoParse
        save = c.i
        c.take(":")
        mm = c.digits(2, 2)
        if mm is None:
            c.i = save
        else:
            minute = mm
            save = c.i
            c.take(":")
            ss = c.digits(2, 2)
            if ss is None:
                c.i = save
            else:
                second = ss
                if c.take(".,"):
                    frac = c.run_of_digits()
                    if not frac:
                        raise _NoParse
                    micros = int(frac[:6].ljust(6, "0"))
        save = c.i
        c.take(" ")
        if c.take("zZ"):
            zone = 0
        elif c.peek("+-"):
            zsign = -1 if c.take("+-") == "-" else 1
            zh = c.digits(2, 2)
            if zh is None:
                raise _NoParse
            save2 = c.i
            c.take(":")
            zm = c.digits(2, 2)
            if zm is None:
                c.i = save2
                zm = 0
            zone = zsign * (zh * 60 + zm)
        else:
            c.i = save
    if c.i != len(s):
        raise _NoParse
    year += (month - 1) // 12                 # month overflow, as DateTime normalises it
    month = (month - 1) % 12 + 1
    total_us = ((_epoch_days(year, month, day) * 24 + hour) * 60 + minute) * 60 + second
    total_us = total_us * 1000000 + micros
    if zone:
        total_us -= zone * 60 * 1000000
    ms = _trunc_div(total_us, 1000)
    if abs(ms) > _MAX_MS:
        raise ValueError(f"FormatException: Time out of range {s}")
    return ms


def _parse_hex_int(s: str) -> int:
    """``int.parse(s, radix: 16)``: optional sign then hex digits."""
    if not re.fullmatch(r"[+-]?[0-9A-Fa-f]+", s):
        raise ValueError(f"FormatException: {s}")
    return _wrap64(int(s, 16))


def _radix16_upper(n: int) -> str:
    return ("-" + format(-n, "X")) if n < 0 else format(n, "X")


# ---------------------------------------------------------------------------
# Exceptions — hlc.dart:164-189
# ---------------------------------------------------------------------------
class ClockDriftException(Exception):
    def __init__(self, millis_ts: int, millis_wall: int):
        self.drift = _wrap64(millis_ts - millis_wall)          # hlc.dart:167
        super().__init__(str(self))

    def __str__(self):                                          # hlc.dart:170
        return f"Clock drift of {self.drift} ms exceeds maximum ({MAX_DRIFT})"


class OverflowException(Exception):
    def __init__(self, counter: int):
        self.counter = counter
        super().__init__(str(self))

    def __str__(self):                                          # hlc.dart:179
        return f"Timestamp counter overflow: {self.counter}"


class DuplicateNodeException(Exception):
    def __init__(self, node_id: str):
        self.node_id = node_id
        super().__init__(str(self))

    def __str__(self):                                          # hlc.dart:188
        return f"Duplicate node: {self.node_id}"


# ---------------------------------------------------------------------------
# Hlc — hlc.dart:11-162
# ---------------------------------------------------------------------------
class Hlc:
    __slots__ = ("millis", "counter", "node_id")

    def __init__(self, millis: int, counter: int, node_id):
        # hlc.dart:18-23 (asserts are off in release builds)
        self.millis = millis if millis < 0x0001000000000000 else _trunc_div(millis, 1000)
        self.counter = counter
        self.node_id = node_id

    @property
    def logical_time(self) -> int:                              # hlc.dart:16
        return _wrap64(_wrap64(self.millis << SHIFT) + self.counter)

    @classmethod
    def zero(cls, node_id):                                     # hlc.dart:25
        return cls(0, 0, node_id)

    @classmethod
    def from_logical_time(cls, lt: int, node_id):               # hlc.dart:37
        return cls(lt >> SHIFT, lt & MAX_COUNTER, node_id)

    @classmethod
    def parse(cls, timestamp: str, id_decoder=None):            # hlc.dart:39-46
        colon = timestamp.rfind(":")
        if colon < 0:
            raise ValueError("RangeError: no ':' in timestamp")
        counter_dash = timestamp.find("-", colon)
        if counter_dash < 0:
            raise ValueError("RangeError: no counter dash")
        node_dash = timestamp.find("-", counter_dash + 1)
        if node_dash < 0:
            raise ValueError("RangeError: no node dash")
        millis = millis_from_iso(timestamp[:counter_dash])
        counter = _parse_hex_int(timestamp[counter_dash + 1:node_dash])
        node_id = timestamp[node_dash + 1:]
        return cls(millis, counter, id_decoder(node_id) if id_decoder else node_id)

    @classmethod
    def send(cls, canonical: "Hlc", millis: int) -> "Hlc":      # hlc.dart:51-74
        millis_old = canonical.millis
        counter_old = canonical.counter
        millis_new = max(millis_old, millis)
        counter_new = counter_old + 1 if millis_old == millis_new else 0
        if _wrap64(millis_new - millis) > MAX_DRIFT:
            raise ClockDriftException(millis_new, millis)
        if counter_new > MAX_COUNTER:
            raise OverflowException(counter_new)
        return cls(millis_new, counter_new, canonical.node_id)

    @classmethod
    def recv(cls, canonical: "Hlc", remote: "Hlc", millis: int) -> "Hlc":   # hlc.dart:80-97
        if canonical.logical_time >= remote.logical_time:
            return canonical
        if canonical.node_id == remote.node_id:
            raise DuplicateNodeException(str(canonical.node_id))
        if _wrap64(remote.millis - millis) > MAX_DRIFT:
            raise ClockDriftException(remote.millis, millis)
        return cls.from_logical_time(remote.logical_time, canonical.node_id)

    def compare_to(self, other: "Hlc") -> int:                  # hlc.dart:157-161
        a, b = self.logical_time, other.logical_time
        if a != b:
            return -1 if a < b else 1
        return dart_compare(self.node_id, other.node_id)

    def __eq__(self, other):                                    # hlc.dart:146-147
        return isinstance(other, Hlc) and self.compare_to(other) == 0

    def __hash__(self):
        return hash(str(self))

    def __lt__(self, other):
        return self.compare_to(other) < 0

    def __le__(self, other):
        return self < other or self == other

    def __gt__(self, other):
        return self.compare_to(other) > 0

    def __ge__(self, other):                                    # hlc.dart:155
        return self > other or self == other

    def __str__(self):                                          # hlc.dart:101-104
        c = _radix16_upper(self.counter).rjust(4, "0")
        return f"{iso_from_millis(self.millis)}-{c}-{self.node_id}"

    def to_json(self) -> str:
        return str(self)

    __repr__ = __str__


# ---------------------------------------------------------------------------
# Record — record.dart:12-39
# ---------------------------------------------------------------------------
class Record:
    __slots__ = ("hlc", "value", "modified")

    def __init__(self, hlc: Hlc, value, modified: Hlc):
        self.hlc = hlc
        self.value = value
        self.modified = modified

    @property
    def is_deleted(self) -> bool:                               # record.dart:17
        return self.value is None

    @classmethod
    def from_json(cls, key, m: dict, modified: Hlc, value_decoder=None, node_id_decoder=None):
        hlc = Hlc.parse(m["hlc"], node_id_decoder)             # record.dart:21-26
        v = m.get("value")
        value = v if value_decoder is None or v is None else value_decoder(key, v)
        return cls(hlc, value, modified)

    def to_json(self, key, value_encoder=None) -> dict:         # record.dart:28-31
        return {"hlc": self.hlc.to_json(),
                "value": self.value if value_encoder is None else value_encoder(key, self.value)}

    def __eq__(self, other):                                    # record.dart:33-35 (ignores modified)
        return isinstance(other, Record) and self.hlc == other.hlc and self.value == other.value

    def __repr__(self):
        return f"Record({self.hlc}, {self.value!r}, mod={self.modified})"


# ---------------------------------------------------------------------------
# CrdtJson — crdt_json.dart:5-38
# ---------------------------------------------------------------------------
class CrdtJson:
    @staticmethod
    def encode(record_map: dict, key_encoder=None, value_encoder=None) -> str:
        out = {}
        for k, r in record_map.items():                         # crdt_json.dart:8-17
            out[str(k) if key_encoder is None else key_encoder(k)] = r.to_json(k, value_encoder)
        return json.dumps(out, separators=(",", ":"), ensure_ascii=False)

    @staticmethod
    def decode(js: str, canonical_time: Hlc, wall: int, key_decoder=None,
               value_decoder=None, node_id_decoder=None) -> dict:
        now = Hlc(wall, 0, canonical_time.node_id)              # crdt_json.dart:23 (Hlc.now)
        modified = canonical_time if canonical_time >= now else now   # :24
        out = {}
        for k, v in json.loads(js).items():                     # :25-35
            key = k if key_decoder is None else key_decoder(k)
            out[key] = Record.from_json(k, v, modified, value_decoder, node_id_decoder)
        return out


# ---------------------------------------------------------------------------
# Crdt + MapCrdt — crdt.dart:7-170, map_crdt.dart:9-53
# ---------------------------------------------------------------------------
class MapCrdt:
    """In-memory CRDT; ``wall`` stands in for ``DateTime.now()``."""

    def __init__(self, node_id, seed: dict | None = None):
        self.node_id = node_id
        self._map: dict = {}                                    # map_crdt.dart:10
        self.events: list = []                                  # map_crdt.dart:11 (watch stream)
        self.refresh_canonical_time()                           # crdt.dart:31-33, runs BEFORE the seed
        if seed:
            self._map.update(seed)                              # map_crdt.dart:17

    # --- SPI (map_crdt.dart:20-52) ---
    def contains_key(self, key) -> bool:
        return key in self._map

    def get_record(self, key):
        return self._map.get(key)

    def put_record(self, key, record: Record):
        self._map[key] = record
        self.events.append((key, record.value))

    def put_records(self, records: dict):
        self._map.update(records)                               # map_crdt.dart:34
        for k, r in records.items():
            self.events.append((k, r.value))

    def record_map(self, modified_since: Hlc | None = None) -> dict:   # map_crdt.dart:42-45
        since = modified_since.logical_time if modified_since is not None else 0
        return {k: r for k, r in self._map.items() if not (r.modified.logical_time < since)}

    def purge(self):
        self._map.clear()

    # --- Crdt (crdt.dart) ---
    @property
    def canonical_time(self) -> Hlc:
        return self._canonical_time

    @property
    def map(self) -> dict:                                      # crdt.dart:22-24
        return {k: r.value for k, r in self.record_map().items() if not r.is_deleted}

    @property
    def is_empty(self) -> bool:
        return len(self.map) == 0

    @property
    def length(self) -> int:
        return len(self.map)

    @property
    def keys(self) -> list:
        return list(self.map.keys())

    @property
    def values(self) -> list:
        return list(self.map.values())

    def get(self, key):                                         # crdt.dart:36
        r = self.get_record(key)
        return None if r is None else r.value

    def put(self, key, value, wall: int):                       # crdt.dart:39-43
        self._canonical_time = Hlc.send(self._canonical_time, wall)
        self.put_record(key, Record(self._canonical_time, value, self._canonical_time))

    def put_all(self, values: dict, wall: int):                 # crdt.dart:46-54
        if not values:
            return
        self._canonical_time = Hlc.send(self._canonical_time, wall)
        c = self._canonical_time
        self.put_records({k: Record(c, v, c) for k, v in values.items()})

    def delete(self, key, wall: int):                           # crdt.dart:58
        self.put(key, None, wall)

    def is_deleted(self, key):                                  # crdt.dart:62
        r = self.get_record(key)
        return None if r is None else r.is_deleted

    def clear(self, wall: int, purge: bool = False):            # crdt.dart:67-73
        if purge:
            self.purge()
        else:
            self.put_all({k: None for k in self.map}, wall)

    def merge(self, remote_records: dict, wall: int):           # crdt.dart:77-94
        local_records = self.record_map()                       # :78 full copy
        self.trace = {"phase": "recv", "index": -1, "present": 0}
        to_remove = []
        for idx, key in enumerate(list(remote_records.keys())):  # :80-85 removeWhere [SDK MapMixin]
            value = remote_records[key]
            self.trace["index"] = idx
            self._canonical_time = Hlc.recv(self._canonical_time, value.hlc, wall)
            self.trace["present"] += key in local_records
            lr = local_records.get(key)
            if lr is not None and lr.hlc >= value.hlc:
                to_remove.append(key)
        for key in to_remove:
            del remote_records[key]
        c = self._canonical_time                                # :86-87 one stamp for all winners
        updated = {k: Record(v.hlc, v.value, c) for k, v in remote_records.items()}
        self.put_records(updated)                               # :90
        self.trace["phase"] = "send"
        self._canonical_time = Hlc.send(self._canonical_time, wall)   # :93

    def merge_json(self, js: str, wall: int, key_decoder=None, value_decoder=None):
        m = CrdtJson.decode(js, self._canonical_time, wall,     # crdt.dart:100-109
                            key_decoder=key_decoder, value_decoder=value_decoder)
        self.merge(m, wall)

    def refresh_canonical_time(self):                           # crdt.dart:114-121
        m = self.record_map()
        lt = max((r.hlc.logical_time for r in m.values()), default=0)
        self._canonical_time = Hlc.from_logical_time(lt, self.node_id)

    def to_json(self, modified_since: Hlc | None = None, key_encoder=None, value_encoder=None) -> str:
        return CrdtJson.encode(self.record_map(modified_since), key_encoder, value_encoder)
