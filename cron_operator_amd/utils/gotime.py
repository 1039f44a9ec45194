"""Go ``time`` semantics in Python, as needed by the cron engine and the API types.

The reference schedules through ``robfig/cron/v3`` on Go ``time.Time`` values
(``internal/controller/cron_controller.go:389-437``).  Go wall-clock arithmetic
differs from Python ``datetime`` in the details that matter for cron parity:

* ``time.Date`` normalises out-of-range fields (day 32, month 13, hour -1) and
  resolves a local wall time that falls in a DST gap or overlap with its own
  rule (look the offset up at the wall time read as UTC, then re-check it at the
  resulting instant).  Python's ``fold`` picks a different instant for gaps.
* ``Time.Add`` is absolute (nanoseconds), ``Time.AddDate`` is wall-clock and
  goes through ``time.Date`` normalisation.
* ``Time.Truncate`` works on absolute time since 0001-01-01 UTC, not on the
  local wall clock.
* The zero ``Time`` is 0001-01-01T00:00:00Z; ``IsZero`` compares to it.

``GoTime`` reproduces exactly these rules on top of an integer
``(unix_seconds, nanoseconds, location)`` triple, with the proleptic-Gregorian
day arithmetic done in integers (no ``datetime`` on the hot path).  Time-zone
offsets come from the IANA database, looked up in Go's order (:func:`tzif_bytes`):
``$ZONEINFO``, the system zoneinfo directories, then the ``tzdata`` wheel (Go's
embedded ``time/tzdata``).
"""
from __future__ import annotations

import os
import re
from datetime import datetime
from functools import lru_cache
from typing import List, Optional, Tuple

NANOS = 1_000_000_000
SECOND = NANOS
MINUTE = 60 * SECOND
HOUR = 60 * MINUTE

# Seconds between 0001-01-01T00:00:00Z (Go's zero time) and the Unix epoch.
UNIX_TO_ABS = 62135596800
ZERO_UNIX = -UNIX_TO_ABS


def days_from_civil(y: int, m: int, d: int) -> int:
    """Days since 1970-01-01 of the proleptic Gregorian date (y, m, d).

    ``d`` may be out of range (0, 32, -5 ...) -- it is simply added, which is
    how Go's ``time.Date`` normalises the day field.
    """
    # normalise the month first (m is 1-based)
    y += (m - 1) // 12
    m = (m - 1) % 12 + 1
    yy = y - (1 if m <= 2 else 0)
    era = yy // 400
    yoe = yy - era * 400
    mp = m - 3 if m > 2 else m + 9
    doy = (153 * mp + 2) // 5
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468 + (d - 1)


def civil_from_days(z: int) -> Tuple[int, int, int]:
    """Inverse of :func:`days_from_civil` for in-range dates."""
    z += 719468
    era = z // 146097
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = mp + 3 if mp < 10 else mp - 9
    y = yoe + era * 400 + (1 if m <= 2 else 0)
    return y, m, d


# --------------------------------------------------------------------------- locations


class Location:
    """A Go ``*time.Location``: maps an absolute instant to a UTC offset."""

    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name

    def offset_at(self, unix: int) -> int:  # seconds east of UTC
        raise NotImplementedError

    @property
    def fixed(self) -> Optional[int]:
        """The constant offset, or None if the zone has transitions."""
        return None

    def __repr__(self) -> str:
        return f"Location({self.name!r})"


class FixedZone(Location):
    __slots__ = ("offset",)

    def __init__(self, name: str, offset: int):
        super().__init__(name)
        self.offset = offset

    def offset_at(self, unix: int) -> int:
        return self.offset

    @property
    def fixed(self) -> Optional[int]:
        return self.offset


class ZoneLocation(Location):
    """An IANA zone, resolved through :mod:`zoneinfo`."""

    __slots__ = ("tz", "_cache", "key")

    def __init__(self, name: str, tz, key: Optional[str] = None):
        super().__init__(name)
        self.tz = tz
        self.key = key or name
        self._cache: dict = {}

    def offset_at(self, unix: int) -> int:
        off = self._cache.get(unix)
        if off is not None:
            return off
        try:
            dt = datetime.fromtimestamp(unix, self.tz)
            off = int(dt.utcoffset().total_seconds())
        except (OverflowError, ValueError, OSError):
            # outside datetime's year range: extrapolate from the nearest edge
            edge = 253402214400 if unix > 0 else -62135596800 + 86400
            off = int(datetime.fromtimestamp(edge, self.tz).utcoffset().total_seconds())
        if len(self._cache) > 4096:
            self._cache.clear()
        self._cache[unix] = off
        return off


UTC = FixedZone("UTC", 0)


def _zone_dirs() -> List[str]:
    """System zoneinfo directories: :data:`zoneinfo.TZPATH` (``PYTHONTZPATH`` when set,
    else Go's list, ``/usr/share/zoneinfo`` first)."""
    try:
        import zoneinfo

        return [d for d in zoneinfo.TZPATH if d]
    except ImportError:  # pragma: no cover - py<3.9
        return ["/usr/share/zoneinfo", "/usr/lib/zoneinfo", "/usr/share/lib/zoneinfo", "/etc/zoneinfo"]


def tzif_bytes(name: str) -> bytes:
    """The TZif data of IANA zone ``name`` (or of an absolute file path).

    Search order of Go's ``time.LoadLocation``: ``$ZONEINFO`` (a directory or a
    zip of the zoneinfo tree), the system zoneinfo directories, then the ``tzdata``
    wheel -- the counterpart of Go's embedded ``time/tzdata``.  Both cron engines read
    zones through here, so an image with only the OS ``tzdata`` package (no wheel)
    and one with only the wheel resolve the same names."""
    if name.startswith("/"):
        with open(name, "rb") as fh:
            return fh.read()
    if not name or name.startswith(".") or ".." in name.split("/") or "\\" in name:
        raise ValueError(f"unknown time zone {name}")
    zi = os.environ.get("ZONEINFO")
    if zi:
        try:
            if zi.endswith(".zip"):
                import zipfile

                with zipfile.ZipFile(zi) as zf:
                    return zf.read(name)
            with open(os.path.join(zi, name), "rb") as fh:
                return fh.read()
        except (OSError, KeyError):
            pass
    for d in _zone_dirs():
        try:
            with open(os.path.join(d, name), "rb") as fh:
                data = fh.read()
        except OSError:
            continue
        if data[:4] == b"TZif":
            return data
    try:
        from importlib import resources

        node = resources.files("tzdata").joinpath("zoneinfo", *name.split("/"))
        data = node.read_bytes()
        if data[:4] == b"TZif":
            return data
    except (ImportError, OSError, TypeError, AttributeError):
        pass
    raise ValueError(f"unknown time zone {name}")


def _zoneinfo_from(name: str):
    import io
    from zoneinfo import ZoneInfo

    return ZoneInfo.from_file(io.BytesIO(tzif_bytes(name)), key=name)


@lru_cache(maxsize=256)
def load_location(name: str) -> Location:
    """Go ``time.LoadLocation``: "" and "UTC" are UTC, "Local" is :data:`LOCAL`."""
    if name == "" or name == "UTC":
        return UTC
    if name == "Local":
        return LOCAL
    if name.startswith("/") or ".." in name or "\\" in name:
        raise ValueError(f"unknown time zone {name}")
    try:
        tz = _zoneinfo_from(name)
    except Exception:
        raise ValueError(f"unknown time zone {name}") from None
    return ZoneLocation(name, tz)


def _resolve_local() -> Location:
    """Go's ``time.Local`` initialisation: $TZ, else /etc/localtime, else UTC."""
    tzenv = os.environ.get("TZ")
    if tzenv is not None:
        if tzenv == "" or tzenv in ("UTC", ":UTC"):
            return FixedZone("Local", 0)
        name = tzenv[1:] if tzenv.startswith(":") else tzenv
        try:
            return ZoneLocation("Local", _zoneinfo_from(name), key=name)
        except Exception:
            return FixedZone("Local", 0)
    try:
        from zoneinfo import ZoneInfo

        with open("/etc/localtime", "rb") as fh:
            return ZoneLocation("Local", ZoneInfo.from_file(fh), key="/etc/localtime")
    except Exception:
        return FixedZone("Local", 0)


class _LocalProxy(Location):
    """``time.Local``: a distinguished location the cron engine treats specially."""

    __slots__ = ("_impl",)

    def __init__(self):
        super().__init__("Local")
        self._impl: Optional[Location] = None

    def impl(self) -> Location:
        if self._impl is None:
            self._impl = _resolve_local()
        return self._impl

    def reset(self) -> None:
        """Re-read $TZ (tests change it)."""
        self._impl = None

    def offset_at(self, unix: int) -> int:
        return self.impl().offset_at(unix)

    @property
    def fixed(self) -> Optional[int]:
        return self.impl().fixed


LOCAL = _LocalProxy()


# --------------------------------------------------------------------------- GoTime


class GoTime:
    """An instant plus a location, with Go ``time.Time`` method semantics."""

    __slots__ = ("sec", "nsec", "loc")

    def __init__(self, sec: int, nsec: int = 0, loc: Location = UTC):
        self.sec = sec
        self.nsec = nsec
        self.loc = loc

    # -- constructors
    @staticmethod
    def zero() -> "GoTime":
        return GoTime(ZERO_UNIX, 0, UTC)

    @staticmethod
    def unix(sec: int, nsec: int = 0, loc: Location = LOCAL) -> "GoTime":
        sec += nsec // NANOS
        nsec %= NANOS
        return GoTime(sec, nsec, loc)

    @staticmethod
    def from_unix_nano(ns: int, loc: Location = LOCAL) -> "GoTime":
        return GoTime(ns // NANOS, ns % NANOS, loc)

    @staticmethod
    def date(year: int, month: int, day: int, hour: int = 0, minute: int = 0, sec: int = 0,
             nsec: int = 0, loc: Location = UTC) -> "GoTime":
        """Go ``time.Date`` including field normalisation and DST resolution."""
        sec += nsec // NANOS
        nsec %= NANOS
        wall = days_from_civil(year, month, day) * 86400 + hour * 3600 + minute * 60 + sec
        fixed = loc.fixed
        if fixed is not None:
            return GoTime(wall - fixed, nsec, loc)
        off = loc.offset_at(loc.offset_at(wall) * -1 + wall)
        return GoTime(wall - off, nsec, loc)

    # -- accessors
    def offset(self) -> int:
        fixed = self.loc.fixed
        return fixed if fixed is not None else self.loc.offset_at(self.sec)

    def _wall(self) -> int:
        return self.sec + self.offset()

    def fields(self) -> Tuple[int, int, int, int, int, int]:
        """(year, month, day, hour, minute, second) in the time's location."""
        w = self._wall()
        days, rem = divmod(w, 86400)
        y, m, d = civil_from_days(days)
        return y, m, d, rem // 3600, (rem // 60) % 60, rem % 60

    def year(self) -> int:
        return self.fields()[0]

    def month(self) -> int:
        return self.fields()[1]

    def day(self) -> int:
        return self.fields()[2]

    def hour(self) -> int:
        return (self._wall() % 86400) // 3600

    def minute(self) -> int:
        return (self._wall() % 3600) // 60

    def second(self) -> int:
        return self._wall() % 60

    def nanosecond(self) -> int:
        return self.nsec

    def weekday(self) -> int:
        """0 = Sunday, as Go's ``time.Weekday``."""
        return (self._wall() // 86400 + 4) % 7

    def unix_seconds(self) -> int:
        return self.sec

    def unix_nano(self) -> int:
        return self.sec * NANOS + self.nsec

    def is_zero(self) -> bool:
        return self.sec == ZERO_UNIX and self.nsec == 0

    # -- arithmetic
    def add(self, d_ns: int) -> "GoTime":
        ns = self.nsec + d_ns
        return GoTime(self.sec + ns // NANOS, ns % NANOS, self.loc)

    def add_date(self, years: int, months: int, days: int) -> "GoTime":
        y, m, d, hh, mm, ss = self.fields()
        return GoTime.date(y + years, m + months, d + days, hh, mm, ss, self.nsec, self.loc)

    def truncate(self, d_ns: int) -> "GoTime":
        """Go ``Time.Truncate``: rounds down on absolute time since year 1."""
        if d_ns <= 0:
            return self
        abs_ns = (self.sec + UNIX_TO_ABS) * NANOS + self.nsec
        r = abs_ns % d_ns
        return self.add(-r)

    def in_(self, loc: Location) -> "GoTime":
        return GoTime(self.sec, self.nsec, loc)

    def utc(self) -> "GoTime":
        return GoTime(self.sec, self.nsec, UTC)

    def sub(self, other: "GoTime") -> int:
        """Duration self - other in nanoseconds."""
        return (self.sec - other.sec) * NANOS + (self.nsec - other.nsec)

    # -- comparisons
    def key(self) -> Tuple[int, int]:
        return (self.sec, self.nsec)

    def before(self, o: "GoTime") -> bool:
        return (self.sec, self.nsec) < (o.sec, o.nsec)

    def after(self, o: "GoTime") -> bool:
        return (self.sec, self.nsec) > (o.sec, o.nsec)

    def equal(self, o: "GoTime") -> bool:
        return self.sec == o.sec and self.nsec == o.nsec

    def __eq__(self, o) -> bool:  # instant equality (Go's Equal), location-agnostic
        return isinstance(o, GoTime) and self.sec == o.sec and self.nsec == o.nsec

    def __lt__(self, o: "GoTime") -> bool:
        return (self.sec, self.nsec) < (o.sec, o.nsec)

    def __le__(self, o: "GoTime") -> bool:
        return (self.sec, self.nsec) <= (o.sec, o.nsec)

    def __hash__(self) -> int:
        return hash((self.sec, self.nsec))

    # -- formatting
    def rfc3339(self, nanos: bool = False) -> str:
        off = self.offset()
        if _native_format is not None:
            s = _native_format(self.sec + off, self.nsec if nanos else 0, off)
            if s is not None:
                return s
        y, m, d, hh, mm, ss = self.fields()
        frac = ""
        if nanos and self.nsec:
            frac = "." + f"{self.nsec:09d}".rstrip("0")
        if off == 0:
            tz = "Z"
        else:
            sign = "+" if off > 0 else "-"
            a = abs(off)
            tz = f"{sign}{a // 3600:02d}:{(a // 60) % 60:02d}"
        return f"{y:04d}-{m:02d}-{d:02d}T{hh:02d}:{mm:02d}:{ss:02d}{frac}{tz}"

    def __repr__(self) -> str:
        if self.is_zero():
            return "GoTime(zero)"
        return f"GoTime({self.rfc3339(nanos=True)} {self.loc.name})"


_RFC3339_RE = re.compile(
    r"^(\d{4})-(\d{2})-(\d{2})[Tt](\d{2}):(\d{2}):(\d{2})(\.\d{1,9})?([Zz]|[+-]\d{2}:\d{2})$")


# Native twins of the hot formatting/parsing paths (``_cron_engine.rfc3339_z`` / ``format_rfc3339``),
# installed by ops/cron_native.py when the extension loads; each returns None for anything
# outside the shape it handles and the Python code below decides (tests/test_gotime.py).
_native_parse_z = None
_native_format = None


def install_native(parse_z, fmt) -> None:
    """Use the native timestamp helpers (``None`` restores the pure-Python paths)."""
    global _native_parse_z, _native_format
    _native_parse_z, _native_format = parse_z, fmt
    _parse_cached.cache_clear()
    _format_utc_cached.cache_clear()


def parse_rfc3339(s: str, loc: Location = LOCAL) -> GoTime:
    """Parse like ``time.Parse(time.RFC3339, s)`` then move the result to ``loc``.

    ``metav1.Time.UnmarshalJSON`` calls ``.Local()`` on the parsed value.
    Fractional seconds are accepted (Go accepts them on parse even though the
    layout has none).  Results are cached: the same timestamps are parsed over
    and over (every reconcile re-reads a Cron's history and its children's
    conditions), and GoTime values are immutable.
    """
    return _parse_cached(s, loc)


@lru_cache(maxsize=1 << 16)
def _parse_cached(s: str, loc: Location) -> GoTime:
    # fast path: "YYYY-MM-DDTHH:MM:SSZ" (what metav1.Time always writes)
    if _native_parse_z is not None:
        sec = _native_parse_z(s)
        if sec is not None:
            return GoTime(sec, 0, loc)
    if len(s) == 20 and s[19] == "Z" and s[10] == "T" and s[4] == "-" and s[13] == ":":
        try:
            y, mo, d = int(s[0:4]), int(s[5:7]), int(s[8:10])
            hh, mi, ss = int(s[11:13]), int(s[14:16]), int(s[17:19])
        except ValueError:
            y = -1
        if y >= 0 and 1 <= mo <= 12 and 1 <= d <= 31 and hh < 24 and mi < 60 and ss < 60 and \
                s[7] == "-" and s[16] == ":":
            return GoTime(days_from_civil(y, mo, d) * 86400 + hh * 3600 + mi * 60 + ss, 0, loc)
    return _parse_slow(s, loc)


def _parse_slow(s: str, loc: Location) -> GoTime:
    mt = _RFC3339_RE.match(s)
    if not mt:
        raise ValueError(f'parsing time "{s}" as RFC3339: cannot parse')
    y, mo, d, hh, mi, ss = (int(mt.group(i)) for i in range(1, 7))
    if not (1 <= mo <= 12 and 1 <= d <= 31 and hh < 24 and mi < 60 and ss < 60):
        raise ValueError(f'parsing time "{s}": field out of range')
    frac = mt.group(7)
    nsec = int((frac[1:] + "000000000")[:9]) if frac else 0
    tz = mt.group(8)
    off = 0
    if tz not in ("Z", "z"):
        sign = 1 if tz[0] == "+" else -1
        off = sign * (int(tz[1:3]) * 3600 + int(tz[4:6]) * 60)
    sec = days_from_civil(y, mo, d) * 86400 + hh * 3600 + mi * 60 + ss - off
    return GoTime(sec, nsec, loc)


def format_rfc3339_utc(t: GoTime) -> str:
    """``metav1.Time.MarshalJSON``: UTC, second precision.  Cached by unix second: a
    reconcile re-serialises every history timestamp of its Cron."""
    return _format_utc_cached(t.sec)


@lru_cache(maxsize=1 << 16)
def _format_utc_cached(sec: int) -> str:
    if _native_format is not None:
        s = _native_format(sec, 0, 0)
        if s is not None:
            return s
    days, rem = divmod(sec, 86400)
    y, m, d = civil_from_days(days)
    return f"{y:04d}-{m:02d}-{d:02d}T{rem // 3600:02d}:{(rem // 60) % 60:02d}:{rem % 60:02d}Z"


# --------------------------------------------------------------------------- durations

_UNITS = {
    "ns": 1,
    "us": 1_000,
    "µs": 1_000,  # micro sign
    "μs": 1_000,  # greek mu
    "ms": 1_000_000,
    "s": SECOND,
    "m": MINUTE,
    "h": HOUR,
}

_MAX_DURATION = (1 << 63) - 1


def parse_duration(s: str) -> int:
    """Go ``time.ParseDuration`` -> nanoseconds (int64 range)."""
    orig = s
    if s == "":
        raise ValueError(f'time: invalid duration "{orig}"')
    neg = False
    if s[0] in "+-":
        neg = s[0] == "-"
        s = s[1:]
    if s == "0":
        return 0
    if s == "":
        raise ValueError(f'time: invalid duration "{orig}"')
    total = 0
    while s:
        i = 0
        while i < len(s) and s[i].isdigit() and s[i].isascii():
            i += 1
        whole = s[:i]
        s = s[i:]
        pre = i > 0
        frac = ""
        post = False
        if s.startswith("."):
            s = s[1:]
            j = 0
            while j < len(s) and s[j].isdigit() and s[j].isascii():
                j += 1
            frac = s[:j]
            s = s[j:]
            post = j > 0
        if not pre and not post:
            raise ValueError(f'time: invalid duration "{orig}"')
        j = 0
        while j < len(s) and s[j] != "." and not (s[j].isdigit() and s[j].isascii()):
            j += 1
        if j == 0:
            raise ValueError(f'time: missing unit in duration "{orig}"')
        unit = s[:j]
        s = s[j:]
        if unit not in _UNITS:
            raise ValueError(f'time: unknown unit "{unit}" in duration "{orig}"')
        scale = _UNITS[unit]
        v = int(whole) if whole else 0
        if v > _MAX_DURATION // scale:
            raise ValueError(f'time: invalid duration "{orig}"')
        v *= scale
        if frac:
            # Go accumulates the fraction with float64 precision
            f = int(frac)
            v += int(f * (scale / (10 ** len(frac))))
        total += v
        if total > _MAX_DURATION + (1 if neg else 0):
            raise ValueError(f'time: invalid duration "{orig}"')
    return -total if neg else total



def _frac(v: int, unit: int) -> str:
    whole, rest = divmod(v, unit)
    if not rest:
        return str(whole)
    digits = len(str(unit)) - 1
    return f"{whole}.{rest:0{digits}d}".rstrip("0")


def format_duration(ns: int) -> str:
    """Go ``time.Duration.String()``: ``1.5s``, ``2m3.25s``, ``1h0m0s``, ``250ms``, ``0s``."""
    if ns == 0:
        return "0s"
    sign = "-" if ns < 0 else ""
    u = abs(ns)
    if u < SECOND:
        if u < 1_000:
            return f"{sign}{u}ns"
        if u < 1_000_000:
            return f"{sign}{_frac(u, 1_000)}µs"
        return f"{sign}{_frac(u, 1_000_000)}ms"
    h, rem = divmod(u, HOUR)
    m, rem = divmod(rem, MINUTE)
    out = sign
    if h:
        out += f"{h}h"
    if h or m:
        out += f"{m}m"
    return out + _frac(rem, SECOND) + "s"
