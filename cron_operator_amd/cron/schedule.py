"""Cron schedule model and next-fire computation (pure-Python twin of the native engine).

Behavioural contract: ``robfig/cron/v3`` ``ParseStandard`` + ``Schedule.Next`` as
used by the reference at ``internal/controller/cron_controller.go:392,405,409,436``
(upstream library is [ext], not vendored; semantics re-derived and pinned by the
hand-derived vectors and the native-vs-Python differential tests in
``tests/test_cron_engine.py``):

* a :class:`SpecSchedule` is six 64-bit field masks (second is fixed to ``0`` by
  the standard 5-field parser) with bit 63 (:data:`STAR_BIT`) recording that the
  field was written as ``*``/``?``;
* ``next(t)`` returns the first matching second strictly after ``t`` in the
  schedule's location (``t``'s own location when the spec carried no
  ``CRON_TZ=``/``TZ=`` prefix), or the zero time when nothing matches within
  five years;
* day matching ANDs day-of-month and day-of-week when either carries the star
  bit, and ORs them otherwise.

The field walk follows the library's algorithm (month -> day -> hour -> minute ->
second with wrap-around restarts) so DST behaviour matches, but the hour/minute/
second loops jump straight to the next set bit whenever the UTC offset does not
change across the jump, which keeps ``* * * * *`` at O(1) instead of 59 steps.
"""
from __future__ import annotations

from typing import Optional, Tuple

from ..utils.gotime import LOCAL, MINUTE, NANOS, SECOND, GoTime, Location

STAR_BIT = 1 << 63
_LOW63 = STAR_BIT - 1


class Schedule:
    """Anything with ``next(t) -> GoTime``."""

    def next(self, t: GoTime) -> GoTime:  # pragma: no cover - interface
        raise NotImplementedError


def _next_bit(mask: int, start: int, limit: int) -> int:
    """Lowest set bit index ``>= start`` and ``<= limit`` in ``mask``, or -1."""
    m = (mask & _LOW63) >> start
    if m == 0:
        return -1
    b = (m & -m).bit_length() - 1 + start
    return b if b <= limit else -1


class SpecSchedule(Schedule):
    __slots__ = ("second", "minute", "hour", "dom", "month", "dow", "location")

    def __init__(self, second: int, minute: int, hour: int, dom: int, month: int, dow: int,
                 location: Location = LOCAL):
        self.second = second
        self.minute = minute
        self.hour = hour
        self.dom = dom
        self.month = month
        self.dow = dow
        self.location = location

    def masks(self) -> Tuple[int, int, int, int, int, int]:
        return (self.second, self.minute, self.hour, self.dom, self.month, self.dow)

    def __eq__(self, o) -> bool:
        return isinstance(o, SpecSchedule) and self.masks() == o.masks() and \
            self.location is o.location

    def __repr__(self) -> str:
        return (f"SpecSchedule(sec={self.second:#x}, min={self.minute:#x}, hour={self.hour:#x}, "
                f"dom={self.dom:#x}, month={self.month:#x}, dow={self.dow:#x}, loc={self.location.name})")

    def day_matches(self, t: GoTime) -> bool:
        dom_match = (1 << t.day()) & self.dom != 0
        dow_match = (1 << t.weekday()) & self.dow != 0
        if self.dom & STAR_BIT or self.dow & STAR_BIT:
            return dom_match and dow_match
        return dom_match or dow_match

    def next(self, t: GoTime) -> GoTime:
        orig_loc = t.loc
        loc = self.location
        if loc is LOCAL:
            loc = t.loc
        if self.location is not LOCAL:
            t = t.in_(self.location)

        # Start at the earliest possible time (the upcoming second).
        t = t.add(SECOND - t.nsec)
        added = False
        year_limit = t.year() + 5

        while True:  # WRAP
            if t.year() > year_limit:
                return GoTime.zero()

            wrapped = False
            # --- month
            while (1 << t.month()) & self.month == 0:
                if not added:
                    added = True
                    y, m, _d, _h, _mi, _s = t.fields()
                    t = GoTime.date(y, m, 1, 0, 0, 0, 0, loc)
                t = t.add_date(0, 1, 0)
                if t.month() == 1:
                    wrapped = True
                    break
            if wrapped:
                continue

            # --- day
            while not self.day_matches(t):
                if not added:
                    added = True
                    y, m, d, _h, _mi, _s = t.fields()
                    t = GoTime.date(y, m, d, 0, 0, 0, 0, loc)
                t = t.add_date(0, 0, 1)
                h = t.hour()
                if h != 0:
                    if h > 12:
                        t = t.add((24 - h) * 3600 * NANOS)
                    else:
                        t = t.add(-h * 3600 * NANOS)
                if t.day() == 1:
                    wrapped = True
                    break
            if wrapped:
                continue

            # --- hour
            while (1 << t.hour()) & self.hour == 0:
                if not added:
                    added = True
                    y, m, d, h, _mi, _s = t.fields()
                    t = GoTime.date(y, m, d, h, 0, 0, 0, loc)
                cur = t.hour()
                nb = _next_bit(self.hour, cur + 1, 23)
                steps = (nb - cur) if nb >= 0 else (24 - cur)
                cand = t.add(steps * 3600 * NANOS)
                if steps > 1 and cand.offset() != t.offset():
                    cand = t.add(3600 * NANOS)  # offset changes: walk hour by hour
                t = cand
                if t.hour() == 0:
                    wrapped = True
                    break
            if wrapped:
                continue

            # --- minute
            while (1 << t.minute()) & self.minute == 0:
                if not added:
                    added = True
                    t = t.truncate(MINUTE)
                cur = t.minute()
                nb = _next_bit(self.minute, cur + 1, 59)
                steps = (nb - cur) if nb >= 0 else (60 - cur)
                cand = t.add(steps * MINUTE)
                if steps > 1 and cand.offset() != t.offset():
                    cand = t.add(MINUTE)
                t = cand
                if t.minute() == 0:
                    wrapped = True
                    break
            if wrapped:
                continue

            # --- second
            while (1 << t.second()) & self.second == 0:
                if not added:
                    added = True
                    t = t.truncate(SECOND)
                cur = t.second()
                nb = _next_bit(self.second, cur + 1, 59)
                steps = (nb - cur) if nb >= 0 else (60 - cur)
                cand = t.add(steps * SECOND)
                if steps > 1 and cand.offset() != t.offset():
                    cand = t.add(SECOND)
                t = cand
                if t.second() == 0:
                    wrapped = True
                    break
            if wrapped:
                continue

            return t.in_(orig_loc)


class ConstantDelaySchedule(Schedule):
    """``@every <duration>``: fires every ``delay`` after rounding down to the second."""

    __slots__ = ("delay",)

    def __init__(self, delay_ns: int):
        self.delay = delay_ns

    def __eq__(self, o) -> bool:
        return isinstance(o, ConstantDelaySchedule) and o.delay == self.delay

    def __repr__(self) -> str:
        return f"ConstantDelaySchedule({self.delay}ns)"

    def next(self, t: GoTime) -> GoTime:
        return t.add(self.delay - t.nsec)


def every(duration_ns: int) -> ConstantDelaySchedule:
    if duration_ns < SECOND:
        duration_ns = SECOND
    # Go's % truncates toward zero; duration is >= 1s here so it is positive
    return ConstantDelaySchedule(duration_ns - duration_ns % SECOND)


def missed_runs(sched: Schedule, earliest: GoTime, now: GoTime,
                count_limit: Optional[int] = None) -> Tuple[GoTime, int, bool]:
    """HOT LOOP 3 of the reference (``cron_controller.go:408-430``).

    Iterates ``t = Next(earliest); !t.After(now); t = Next(t)``.  Returns
    ``(last_missed, missed_count, unschedulable)``; ``last_missed`` is the zero
    time when nothing was missed.  ``unschedulable`` reports that ``Next``
    returned the zero time inside the loop.
    """
    last = GoTime.zero()
    n = 0
    t = sched.next(earliest)
    while not t.after(now):
        if t.is_zero():
            return GoTime.zero(), n, True
        last = t
        n += 1
        if count_limit is not None and n >= count_limit:
            break
        t = sched.next(t)
    return last, n, False
