"""Cron semantics against an independent oracle.

The golden vectors in ``test_cron_engine.py`` were derived by hand.  This test checks
both engines (Python and native) against a second, deliberately different
implementation of robfig/cron v3's ``ParseStandard`` + ``Next`` semantics, in UTC:

* fields are parsed into plain Python *sets* (no bit masks, no shared parser code);
* ``Next`` is a direct search: walk the days after ``t``, keep the days whose month and
  day match, and take the first matching hour/minute -- no field-by-field carry logic.

The rules encoded here are robfig's documented ones (``parser.go``/``spec.go``): ``*``
and ``?`` set the "star" flag, a step greater than 1 clears it (``*/2`` is not a star),
``a/n`` means ``a-max/n``, month and weekday names are case-insensitive, and the day
matches on *day-of-month AND day-of-week* when either field is a star, otherwise on
*day-of-month OR day-of-week*.  A schedule with no match within five years has no next
time (the engines return the zero time).
"""
from __future__ import annotations

import datetime as dt
from typing import Optional, Set, Tuple

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from cron_operator_amd.cron.engine import NativeEngine, PythonEngine
from cron_operator_amd.utils.gotime import UTC, GoTime

ENGINES = [PythonEngine(), NativeEngine()]
MONTHS = {m: i + 1 for i, m in enumerate("jan feb mar apr may jun jul aug sep oct nov dec".split())}
DOWS = {d: i for i, d in enumerate("sun mon tue wed thu fri sat".split())}
BOUNDS = [(0, 59, {}), (0, 23, {}), (1, 31, {}), (1, 12, MONTHS), (0, 6, DOWS)]


def _num(s: str, names) -> int:
    return names[s.lower()] if s.lower() in names else int(s)


def oracle_field(expr: str, lo: int, hi: int, names) -> Tuple[Set[int], bool]:
    values: Set[int] = set()
    star = False
    for part in expr.split(","):
        rng, _, step_s = part.partition("/")
        step = int(step_s) if step_s else 1
        if rng in ("*", "?"):
            a, b = lo, hi
            part_star = step <= 1
        elif "-" in rng:
            x, y = rng.split("-")
            a, b = _num(x, names), _num(y, names)
            part_star = False
        else:
            a = _num(rng, names)
            b = hi if step_s else a
            part_star = False
        values.update(range(a, b + 1, step))
        star = star or part_star
    return values, star


def oracle_next(spec: str, t: dt.datetime) -> Optional[dt.datetime]:
    """``t`` carries the schedule's zone; the search runs on its wall clock (exact for zones
    without DST transitions)."""
    fields = spec.split()
    (mins, _), (hours, _), (doms, dom_star), (months, _), (dows, dow_star) = (
        oracle_field(f, lo, hi, names) for f, (lo, hi, names) in zip(fields, BOUNDS))
    start = t.replace(second=0, microsecond=0) + dt.timedelta(minutes=1)
    day = start.date()
    while day.year <= start.year + 5:  # robfig: give up past year(t) + 5
        dom_ok, dow_ok = day.day in doms, (day.isoweekday() % 7) in dows
        day_ok = (dom_ok and dow_ok) if (dom_star or dow_star) else (dom_ok or dow_ok)
        if day.month in months and day_ok:
            first = day == start.date()
            for h in sorted(hours):
                if first and h < start.hour:
                    continue
                for m in sorted(mins):
                    if first and h == start.hour and m < start.minute:
                        continue
                    return dt.datetime(day.year, day.month, day.day, h, m, tzinfo=t.tzinfo)
        day += dt.timedelta(days=1)
    return None


def _part(lo: int, hi: int, names=None, star_ok: bool = True):
    nums = st.integers(lo, hi)
    ranges = st.tuples(nums, nums).map(lambda ab: f"{min(ab)}-{max(ab)}")
    steps = st.integers(1, max(1, (hi - lo) // 2))
    opts = [nums.map(str), ranges,
            st.tuples(ranges, steps).map(lambda r: f"{r[0]}/{r[1]}"),
            st.tuples(nums, steps).map(lambda r: f"{r[0]}/{r[1]}")]
    if star_ok:
        opts += [st.just("*"), steps.map(lambda s: f"*/{s}")]
    if names:
        opts.append(st.sampled_from(sorted(names)).map(lambda n: n.upper() if len(n) % 2 else n))
    return st.one_of(*opts)


def _field(lo: int, hi: int, names=None, question: bool = False):
    one = _part(lo, hi, names)
    if question:
        one = st.one_of(one, st.just("?"))
    return st.lists(one, min_size=1, max_size=2).map(",".join)


specs = st.tuples(_field(0, 59), _field(0, 23), _field(1, 31, question=True), _field(1, 12, MONTHS),
                  _field(0, 6, DOWS, question=True)).map(" ".join)


@settings(max_examples=400, deadline=None)
@given(spec=specs, start=st.integers(min_value=1_767_225_600, max_value=1_924_992_000))  # 2026 .. 2031
def test_engines_match_an_independent_oracle(spec, start):
    t = dt.datetime.fromtimestamp(start, dt.timezone.utc)
    want = oracle_next(spec, t)
    for eng in ENGINES:
        got = eng.next(eng.parse(spec), GoTime(start, 0, UTC))
        if want is None:
            assert got.is_zero(), (eng.name, spec, t)
        else:
            assert (got.sec, got.nsec) == (int(want.timestamp()), 0), (eng.name, spec, t, want)


@pytest.mark.parametrize("spec", ["0 0 13 * 5", "0 0 * * 5", "0 0 1 * */2", "0 0 1 * */1", "0 0 ? * 1",
                                  "0 0 29 2 *", "0 0 30 2 *", "5/15 3-23/7 */10 JAN,jul SUN-wed"])
def test_oracle_agrees_on_the_classic_cases(spec):
    start = 1_767_268_800  # 2026-01-01T12:00:00Z
    t = dt.datetime.fromtimestamp(start, dt.timezone.utc)
    want = oracle_next(spec, t)
    for eng in ENGINES:
        got = eng.next(eng.parse(spec), GoTime(start, 0, UTC))
        assert (None if got.is_zero() else got.sec) == (None if want is None else int(want.timestamp())), \
            (eng.name, spec)


# zones without DST transitions in the tested years: the oracle's wall-clock search is exact
FIXED_ZONES = ["Etc/GMT-5", "Etc/GMT+7", "Asia/Kolkata", "Asia/Tokyo", "Asia/Shanghai"]


@settings(max_examples=200, deadline=None)
@given(spec=specs, zone=st.sampled_from(FIXED_ZONES),
       start=st.integers(min_value=1_767_225_600, max_value=1_924_992_000))
def test_cron_tz_schedules_match_the_oracle(spec, zone, start):
    """``CRON_TZ=<zone> <spec>``: the schedule runs on the zone's wall clock."""
    from zoneinfo import ZoneInfo

    t = dt.datetime.fromtimestamp(start, ZoneInfo(zone))
    want = oracle_next(spec, t)
    for eng in ENGINES:
        got = eng.next(eng.parse(f"CRON_TZ={zone} {spec}"), GoTime(start, 0, UTC))
        assert (None if got.is_zero() else got.sec) == (None if want is None else int(want.timestamp())), \
            (eng.name, zone, spec, t)
