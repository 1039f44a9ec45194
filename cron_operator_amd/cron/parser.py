"""Standard 5-field cron parser with robfig ``ParseStandard`` semantics.

Used by the reconciler at the point where the reference calls
``cronv3.ParseStandard(cron.Spec.Schedule)`` (``internal/controller/cron_controller.go:392``).

Accepted grammar (upstream [ext] behaviour, pinned by tests):

* optional ``CRON_TZ=<zone> `` or ``TZ=<zone> `` prefix (IANA zone name,
  ``Local``, ``UTC``);
* descriptors ``@yearly @annually @monthly @weekly @daily @midnight @hourly``
  and ``@every <go-duration>``;
* otherwise exactly five whitespace-separated fields
  ``minute hour day-of-month month day-of-week``; seconds are fixed at 0;
* each field is a comma list of ``*``/``?``/``N``/``N-M`` with optional ``/step``;
  ``N/step`` means ``N-max/step``; month names ``jan..dec`` and weekday names
  ``sun..sat`` (case-insensitive); day-of-week is 0..6 (7 is rejected);
* ``*``/``?`` sets :data:`STAR_BIT` unless a step > 1 is given.

Error strings mirror the library so user-visible ``unparsable cron`` messages
read the same.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from ..utils.gotime import LOCAL, Location, load_location, parse_duration
from .schedule import STAR_BIT, Schedule, SpecSchedule, every

Bounds = Tuple[int, int, Optional[Dict[str, int]]]

SECONDS: Bounds = (0, 59, None)
MINUTES: Bounds = (0, 59, None)
HOURS: Bounds = (0, 23, None)
DOM: Bounds = (1, 31, None)
MONTHS: Bounds = (1, 12, {
    "jan": 1, "feb": 2, "mar": 3, "apr": 4, "may": 5, "jun": 6,
    "jul": 7, "aug": 8, "sep": 9, "oct": 10, "nov": 11, "dec": 12,
})
DOW: Bounds = (0, 6, {
    "sun": 0, "mon": 1, "tue": 2, "wed": 3, "thu": 4, "fri": 5, "sat": 6,
})


class CronParseError(ValueError):
    pass


def _bits(lo: int, hi: int, step: int) -> int:
    if step == 1:
        return ((1 << (hi + 1)) - 1) & ~((1 << lo) - 1)
    out = 0
    for i in range(lo, hi + 1, step):
        out |= 1 << i
    return out


def all_bits(r: Bounds) -> int:
    return _bits(r[0], r[1], 1) | STAR_BIT


_GO_INT_MAX = 2**63 - 1  # strconv.Atoi on 64-bit Go


def _atoi(expr: str) -> int:
    """Go ``strconv.Atoi``: optional sign, ASCII digits only."""
    s = expr
    body = s[1:] if s[:1] in ("+", "-") else s
    if body == "" or not all("0" <= c <= "9" for c in body):
        raise CronParseError(f'failed to parse int from {expr}: strconv.Atoi: parsing "{expr}": invalid syntax')
    v = int(s)
    if v > _GO_INT_MAX or v < -_GO_INT_MAX - 1:
        raise CronParseError(f'failed to parse int from {expr}: strconv.Atoi: parsing "{expr}": value out of range')
    return v


def _must_parse_int(expr: str) -> int:
    num = _atoi(expr)
    if num < 0:
        raise CronParseError(f"negative number ({num}) not allowed: {expr}")
    return num


def _parse_int_or_name(expr: str, names: Optional[Dict[str, int]]) -> int:
    if names is not None:
        v = names.get(expr.lower())
        if v is not None:
            return v
    return _must_parse_int(expr)


def get_range(expr: str, r: Bounds) -> int:
    lo_b, hi_b, names = r
    range_and_step = expr.split("/")
    low_and_high = range_and_step[0].split("-")
    single_digit = len(low_and_high) == 1
    extra = 0
    if low_and_high[0] in ("*", "?"):
        start, end = lo_b, hi_b
        extra = STAR_BIT
    else:
        start = _parse_int_or_name(low_and_high[0], names)
        if len(low_and_high) == 1:
            end = start
        elif len(low_and_high) == 2:
            end = _parse_int_or_name(low_and_high[1], names)
        else:
            raise CronParseError(f"too many hyphens: {expr}")
    if len(range_and_step) == 1:
        step = 1
    elif len(range_and_step) == 2:
        step = _must_parse_int(range_and_step[1])
        if single_digit:
            end = hi_b
        if step > 1:
            extra = 0
    else:
        raise CronParseError(f"too many slashes: {expr}")
    if start < lo_b:
        raise CronParseError(f"beginning of range ({start}) below minimum ({lo_b}): {expr}")
    if end > hi_b:
        raise CronParseError(f"end of range ({end}) above maximum ({hi_b}): {expr}")
    if start > end:
        raise CronParseError(f"beginning of range ({start}) beyond end of range ({end}): {expr}")
    if step == 0:
        raise CronParseError(f"step of range should be a positive number: {expr}")
    return _bits(start, end, step) | extra


def get_field(field: str, r: Bounds) -> int:
    bits = 0
    for expr in (p for p in field.split(",") if p != ""):
        bits |= get_range(expr, r)
    return bits


def _go_fields(s: str) -> List[str]:
    """``strings.Fields``: split on Unicode whitespace runs."""
    return s.split()


def _parse_descriptor(desc: str, loc: Location) -> Schedule:
    one = lambda r: 1 << r[0]  # noqa: E731
    if desc in ("@yearly", "@annually"):
        return SpecSchedule(one(SECONDS), one(MINUTES), one(HOURS), one(DOM), one(MONTHS), all_bits(DOW), loc)
    if desc == "@monthly":
        return SpecSchedule(one(SECONDS), one(MINUTES), one(HOURS), one(DOM), all_bits(MONTHS), all_bits(DOW), loc)
    if desc == "@weekly":
        return SpecSchedule(one(SECONDS), one(MINUTES), one(HOURS), all_bits(DOM), all_bits(MONTHS), one(DOW), loc)
    if desc in ("@daily", "@midnight"):
        return SpecSchedule(one(SECONDS), one(MINUTES), one(HOURS), all_bits(DOM), all_bits(MONTHS), all_bits(DOW), loc)
    if desc == "@hourly":
        return SpecSchedule(one(SECONDS), one(MINUTES), all_bits(HOURS), all_bits(DOM), all_bits(MONTHS),
                            all_bits(DOW), loc)
    prefix = "@every "
    if desc.startswith(prefix):
        try:
            d = parse_duration(desc[len(prefix):])
        except ValueError as e:
            raise CronParseError(f"failed to parse duration {desc}: {e}") from None
        return every(d)
    raise CronParseError(f"unrecognized descriptor: {desc}")


def parse_standard(spec: str) -> Schedule:
    """``cronv3.ParseStandard`` equivalent.  Raises :class:`CronParseError`."""
    if len(spec) == 0:
        raise CronParseError("empty spec string")
    loc: Location = LOCAL
    if spec.startswith("TZ=") or spec.startswith("CRON_TZ="):
        i = spec.find(" ")
        eq = spec.find("=")
        if i < 0:
            # upstream slices spec[eq+1:-1] and panics; report it as a parse error
            raise CronParseError(f"provided bad location {spec[eq + 1:]}: missing schedule after time zone")
        name = spec[eq + 1:i]
        try:
            loc = load_location(name)
        except ValueError as e:
            raise CronParseError(f"provided bad location {name}: {e}") from None
        spec = spec[i:].strip()
    if spec.startswith("@"):
        return _parse_descriptor(spec, loc)
    fields = _go_fields(spec)
    if len(fields) != 5:
        raise CronParseError(f"expected exactly 5 fields, found {len(fields)}: [{' '.join(fields)}]")
    expanded = ["0"] + fields
    second = get_field(expanded[0], SECONDS)
    minute = get_field(expanded[1], MINUTES)
    hour = get_field(expanded[2], HOURS)
    dom = get_field(expanded[3], DOM)
    month = get_field(expanded[4], MONTHS)
    dow = get_field(expanded[5], DOW)
    return SpecSchedule(second, minute, hour, dom, month, dow, loc)
