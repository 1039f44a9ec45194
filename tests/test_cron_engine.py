"""Cron engine: golden vectors (robfig ParseStandard/Next semantics) on both
backends, plus a native-vs-Python differential property test.

Upstream robfig/cron/v3 is not vendored and Go is not available here, so the
expected values below were derived by hand from the library's documented
algorithm (see cron/schedule.py); "parity unpinned" against a live Go run.
The reference's own vectors are included verbatim:
``60 31 30 2 *`` -> unparsable, ``0 0 30 2 *`` -> unschedulable, ``*/1`` -> (now, now+1m)
(``internal/controller/cron_controller_test.go:162-223``).
"""
from __future__ import annotations

import random

import pytest
from hypothesis import given, settings, strategies as st

from cron_operator_amd.cron.engine import NativeEngine, PythonEngine, ScheduleError
from cron_operator_amd.cron.parser import parse_standard
from cron_operator_amd.utils.gotime import HOUR, MINUTE, SECOND, UTC, GoTime, load_location, parse_rfc3339

ENGINES = [PythonEngine(), NativeEngine()]
IDS = ["python", "native"]


def T(s: str) -> GoTime:
    return parse_rfc3339(s, UTC)


def iso(t: GoTime) -> str:
    return "zero" if t.is_zero() else t.utc().rfc3339()


NEXT_CASES = [
    ("*/1 * * * *", "2026-01-01T12:00:00Z", ["2026-01-01T12:01:00Z", "2026-01-01T12:02:00Z"]),
    ("* * * * *", "2026-01-01T12:00:59Z", ["2026-01-01T12:01:00Z"]),
    ("*/5 * * * *", "2026-01-01T12:03:30Z", ["2026-01-01T12:05:00Z", "2026-01-01T12:10:00Z"]),
    ("0 0 * * *", "2026-01-01T12:00:00Z", ["2026-01-02T00:00:00Z", "2026-01-03T00:00:00Z"]),
    # 2026-01-01 is a Thursday
    ("0 9 * * mon-fri", "2026-01-01T12:00:00Z", ["2026-01-02T09:00:00Z", "2026-01-05T09:00:00Z"]),
    ("0 0 1,15 * *", "2026-01-01T12:00:00Z", ["2026-01-15T00:00:00Z", "2026-02-01T00:00:00Z"]),
    # dom and dow both restricted -> OR
    ("0 0 13 * 5", "2026-01-01T12:00:00Z",
     ["2026-01-02T00:00:00Z", "2026-01-09T00:00:00Z", "2026-01-13T00:00:00Z", "2026-01-16T00:00:00Z"]),
    # dom is * -> AND (Fridays only)
    ("0 0 * * 5", "2026-01-01T12:00:00Z", ["2026-01-02T00:00:00Z", "2026-01-09T00:00:00Z"]),
    # */2 clears the star bit on dow -> OR with dom=1
    ("0 0 1 * */2", "2026-01-01T12:00:00Z",
     ["2026-01-03T00:00:00Z", "2026-01-04T00:00:00Z", "2026-01-06T00:00:00Z"]),
    ("0 0 1 * *", "2026-01-01T12:00:00Z", ["2026-02-01T00:00:00Z"]),
    ("0 0 1 * ?", "2026-01-01T12:00:00Z", ["2026-02-01T00:00:00Z"]),
    ("0 0 * jan,jul sun", "2026-01-01T12:00:00Z", ["2026-01-04T00:00:00Z", "2026-01-11T00:00:00Z"]),
    ("0 0 * JAN-FEB SUN", "2026-01-26T12:00:00Z", ["2026-02-01T00:00:00Z"]),
    ("30 4 1-7 * 1", "2026-01-01T12:00:00Z", ["2026-01-02T04:30:00Z"]),
    ("5/15 * * * *", "2026-01-01T12:00:00Z", ["2026-01-01T12:05:00Z", "2026-01-01T12:20:00Z"]),
    ("10-20/5 * * * *", "2026-01-01T12:12:00Z", ["2026-01-01T12:15:00Z", "2026-01-01T12:20:00Z",
                                                 "2026-01-01T13:10:00Z"]),
    ("0 0 29 2 *", "2026-01-01T12:00:00Z", ["2028-02-29T00:00:00Z", "2032-02-29T00:00:00Z"]),
    ("0 0 30 2 *", "2026-01-01T12:00:00Z", ["zero"]),
    ("0 0 31 4 *", "2026-01-01T12:00:00Z", ["zero"]),
    ("@hourly", "2026-01-01T12:30:00Z", ["2026-01-01T13:00:00Z"]),
    ("@daily", "2026-01-01T12:30:00Z", ["2026-01-02T00:00:00Z"]),
    ("@midnight", "2026-01-01T12:30:00Z", ["2026-01-02T00:00:00Z"]),
    ("@weekly", "2026-01-01T12:30:00Z", ["2026-01-04T00:00:00Z"]),
    ("@monthly", "2026-01-01T12:30:00Z", ["2026-02-01T00:00:00Z"]),
    ("@yearly", "2026-01-01T12:30:00Z", ["2027-01-01T00:00:00Z"]),
    ("@annually", "2026-01-01T12:30:00Z", ["2027-01-01T00:00:00Z"]),
    ("@every 1h30m", "2026-01-01T12:00:00Z", ["2026-01-01T13:30:00Z", "2026-01-01T15:00:00Z"]),
    ("@every 500ms", "2026-01-01T12:00:00Z", ["2026-01-01T12:00:01Z"]),
    ("0\t0  *  * *", "2026-01-01T12:00:00Z", ["2026-01-02T00:00:00Z"]),
    ("CRON_TZ=Asia/Tokyo 0 9 * * *", "2026-01-01T12:00:00Z", ["2026-01-02T00:00:00Z"]),
    ("TZ=UTC 0 9 * * *", "2026-01-01T12:00:00Z", ["2026-01-02T09:00:00Z"]),
    ("CRON_TZ=Asia/Kolkata 0 0 * * *", "2026-01-01T12:00:00Z", ["2026-01-01T18:30:00Z"]),
    # US DST start 2026-03-08: 02:30 does not exist, robfig skips that day
    ("CRON_TZ=America/New_York 30 2 * * *", "2026-03-07T17:00:00Z",
     ["2026-03-09T06:30:00Z", "2026-03-10T06:30:00Z"]),
    # US DST end 2026-11-01: 01:30 happens twice and fires twice
    ("CRON_TZ=America/New_York 30 1 * * *", "2026-10-31T16:00:00Z",
     ["2026-11-01T05:30:00Z", "2026-11-01T06:30:00Z", "2026-11-02T06:30:00Z"]),
    # Southern hemisphere DST (Sydney, starts first Sunday of October 2026: 2026-10-04 02:00 -> 03:00)
    ("CRON_TZ=Australia/Sydney 30 2 * * *", "2026-10-02T12:00:00Z",
     ["2026-10-02T16:30:00Z", "2026-10-04T15:30:00Z"]),
]


@pytest.mark.parametrize("engine", ENGINES, ids=IDS)
@pytest.mark.parametrize("spec,start,expected", NEXT_CASES)
def test_next_golden(engine, spec, start, expected):
    s = engine.parse(spec)
    t = T(start)
    got = []
    for _ in expected:
        t = engine.next(s, t)
        got.append(iso(t))
        if t.is_zero():
            break
    assert got == expected


PARSE_ERRORS = [
    ("", "empty spec string"),
    ("60 31 30 2 *", "end of range (60) above maximum (59): 60"),
    ("* * * *", "expected exactly 5 fields, found 4: [* * * *]"),
    ("* * * * * *", "expected exactly 5 fields, found 6: [* * * * * *]"),
    ("0 0 * * 7", "end of range (7) above maximum (6): 7"),
    ("a * * * *", 'failed to parse int from a: strconv.Atoi: parsing "a": invalid syntax'),
    ("1-2-3 * * * *", "too many hyphens: 1-2-3"),
    ("1/2/3 * * * *", "too many slashes: 1/2/3"),
    ("*/0 * * * *", "step of range should be a positive number: */0"),
    ("5-1 * * * *", "beginning of range (5) beyond end of range (1): 5-1"),
    ("0 0 0 * *", "beginning of range (0) below minimum (1): 0"),
    ("-1 * * * *", 'failed to parse int from : strconv.Atoi: parsing "": invalid syntax'),
    ("@foo", "unrecognized descriptor: @foo"),
    ("@every 1d", 'failed to parse duration @every 1d: time: unknown unit "d" in duration "1d"'),
    ("@every", "unrecognized descriptor: @every"),
    ("CRON_TZ=Mars/Base * * * * *", "provided bad location Mars/Base: unknown time zone Mars/Base"),
    ("0 0 L * *", 'failed to parse int from L: strconv.Atoi: parsing "L": invalid syntax'),
    ("0 0 * foo *", 'failed to parse int from foo: strconv.Atoi: parsing "foo": invalid syntax'),
]


@pytest.mark.parametrize("engine", ENGINES, ids=IDS)
@pytest.mark.parametrize("spec,msg", PARSE_ERRORS)
def test_parse_errors(engine, spec, msg):
    with pytest.raises(ScheduleError) as ei:
        engine.parse(spec)
    assert str(ei.value) == msg


@pytest.mark.parametrize("engine", ENGINES, ids=IDS)
def test_reference_get_next_schedule_vectors(engine):
    # cron_controller_test.go:162-223 -- now = 2026-01-01T12:00:00Z, created 5 minutes earlier
    now = T("2026-01-01T12:00:00Z")
    created = now.add(-5 * MINUTE)
    s = engine.parse("*/1 * * * *")
    last, n, bad = engine.missed(s, created, now)
    assert not bad and n == 5 and last == now
    assert engine.next(s, now).sec == now.add(MINUTE).sec
    s2 = engine.parse("0 0 30 2 *")
    last, n, bad = engine.missed(s2, created, now)
    assert bad and last.is_zero()


@pytest.mark.parametrize("engine", ENGINES, ids=IDS)
def test_missed_counts_long_outage(engine):
    now = T("2026-03-01T00:00:30Z")
    earliest = T("2025-03-01T00:00:00Z")
    s = engine.parse("* * * * *")
    last, n, bad = engine.missed(s, earliest, now)
    assert not bad
    assert n == 365 * 24 * 60  # one year of minutes (2025 is not a leap year)
    assert iso(last) == "2026-03-01T00:00:00Z"
    s = engine.parse("0 9 * * mon-fri")
    last, n, _ = engine.missed(s, T("2026-01-01T00:00:00Z"), T("2026-02-01T00:00:00Z"))
    assert n == 22 and iso(last) == "2026-01-30T09:00:00Z"


def test_missed_fast_path_matches_walk():
    rng = random.Random(5)
    ne, pe = ENGINES[1], ENGINES[0]
    specs = ["* * * * *", "*/7 3-5 * * *", "0 0 1,15 * *", "15 10 * * 1,3", "0 12 13 * 5", "0 0 29 2 *",
             "@hourly", "*/10 * * 2 *", "CRON_TZ=Asia/Tokyo 0 */3 * * *", "0 0 * * 0"]
    for spec in specs:
        for _ in range(3):
            start = T("2025-06-01T00:00:00Z").add(rng.randrange(0, 200 * 24 * 3600) * SECOND)
            end = start.add(rng.randrange(3 * 24 * 3600, 40 * 24 * 3600) * SECOND)
            a = ne.missed(ne.parse(spec), start, end)
            b = pe.missed(pe.parse(spec), start, end)
            assert (iso(a[0]), a[1], a[2]) == (iso(b[0]), b[1], b[2]), spec


# ---------------------------------------------------------------- differential property test

_field = st.sampled_from(["*", "?", "*/2", "*/5", "1", "3", "1-5", "1,3,5", "2-10/3", "0", "10-20", "*/15"])
_dow = st.sampled_from(["*", "?", "0", "1-5", "mon", "sat,sun", "*/2", "1,3", "6"])
_mon = st.sampled_from(["*", "1", "2", "jan-mar", "*/3", "6,12", "11"])
_dom = st.sampled_from(["*", "?", "1", "13", "1-7", "28-31", "*/10", "15,30", "29", "31"])
_zone = st.sampled_from(["", "CRON_TZ=America/New_York ", "CRON_TZ=Europe/Berlin ", "TZ=Asia/Kolkata ",
                         "CRON_TZ=Australia/Lord_Howe ", "CRON_TZ=UTC "])


@settings(max_examples=300, deadline=None)
@given(minute=_field, hour=st.sampled_from(["*", "0", "2", "1-3", "*/6", "23", "9-17"]), dom=_dom, mon=_mon,
       dow=_dow, zone=_zone, start=st.integers(min_value=1_700_000_000, max_value=1_900_000_000),
       nsec=st.sampled_from([0, 1, 999_999_999]))
def test_native_matches_python(minute, hour, dom, mon, dow, zone, start, nsec):
    spec = f"{zone}{minute} {hour} {dom} {mon} {dow}"
    pe, ne = ENGINES
    ps, ns = pe.parse(spec), ne.parse(spec)
    t0 = GoTime(start, nsec, UTC)
    a = b = t0
    for _ in range(3):
        a = pe.next(ps, a)
        b = ne.next(ns, b)
        assert (a.sec, a.nsec) == (b.sec, b.nsec), (spec, iso(t0))
        if a.is_zero():
            break


@settings(max_examples=200, deadline=None)
@given(zone=st.sampled_from(["America/New_York", "Europe/London", "Australia/Sydney", "Asia/Tokyo",
                             "America/Sao_Paulo", "Pacific/Chatham", "Africa/Casablanca", "America/Santiago"]),
       unix=st.integers(min_value=0, max_value=4_102_444_800))
def test_native_zone_offsets_match_zoneinfo(zone, unix):
    from cron_operator_amd.ops import cron_native

    loc = load_location(zone)
    zid = cron_native.zone_id(loc)
    assert cron_native.load().zone_offset(zid, unix) == loc.offset_at(unix)


def test_parse_python_equals_native_masks():
    from cron_operator_amd.ops import cron_native

    mod = cron_native.load()
    for spec in ["*/5 1-3 * jan-jun mon,fri", "0 0 1 * *", "@weekly", "5/15 * ? * *"]:
        p = parse_standard(spec)
        assert mod.parse(spec).masks()[:6] == p.masks(), spec


def test_unicode_whitespace_spec_uses_python_path():
    e = ENGINES[1]
    s = e.parse("0 0 * * *")  # NBSP: strings.Fields splits on it
    assert iso(e.next(s, T("2026-01-01T12:00:00Z"))) == "2026-01-02T00:00:00Z"


def test_every_rounds_to_second():
    e = ENGINES[1]
    s = e.parse("@every 90s")
    t = GoTime(T("2026-01-01T12:00:00Z").sec, 500_000_000, UTC)
    assert iso(e.next(s, t)) == "2026-01-01T12:01:30Z"
    assert e.next(s, t).nsec == 0
    assert e.parse("@every 1h").impl.delay == HOUR


# ---------------------------------------------------------------- zone lookup without the tzdata wheel

_NO_WHEEL_PROBE = r'''
import json, os, sys
sys.modules["tzdata"] = None  # hide the wheel: zones must come from the system directory
import yaml
from cron_operator_amd.cron.engine import NativeEngine, PythonEngine
from cron_operator_amd.utils.gotime import LOCAL, UTC, GoTime, parse_rfc3339
spec = yaml.safe_load(open(sys.argv[1]))["spec"]["schedule"]
specs = [spec, "CRON_TZ=America/New_York 0 9 * * mon-fri", "TZ=Europe/Berlin 30 1 * * *",
         "CRON_TZ=Australia/Lord_Howe */30 * * * *", "0 2 * * *"]
out = {}
for s in specs:
    row = []
    for eng in (PythonEngine(), NativeEngine()):
        sched = eng.parse(s)
        t = parse_rfc3339("2026-03-07T00:00:00Z")
        ts = []
        for _ in range(40):
            t = eng.next(sched, t)
            ts.append((t.sec, t.nsec))
        if s == "0 2 * * *":  # Local: $TZ of this process
            ts.append(eng.next(sched, GoTime(1772841600, 0, LOCAL)).sec)
        row.append(ts)
    out[s] = row
print(json.dumps(out))
'''


@pytest.mark.parametrize("local_tz", ["Asia/Shanghai", "America/Los_Angeles"])
def test_zones_resolve_from_system_dir_without_tzdata_wheel(tmp_path, local_tz):
    """The image may ship only the OS zoneinfo tree (no ``tzdata`` wheel): both engines must
    resolve ``CRON_TZ=``/``TZ=`` specs and a named ``$TZ`` from ``PYTHONTZPATH`` and agree,
    including the flagship example's schedule (robfig ``CRON_TZ=``)."""
    import json
    import os
    import shutil
    import subprocess
    import sys
    from importlib import resources

    src = resources.files("tzdata").joinpath("zoneinfo")
    zdir = tmp_path / "zoneinfo"
    shutil.copytree(str(src), zdir, ignore=shutil.ignore_patterns("__init__.py", "__pycache__"))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    example = os.path.join(root, "examples/mi355x/cron-pytorch-ddp-mi355x.yaml")
    env = dict(os.environ, PYTHONTZPATH=str(zdir), TZ=local_tz, PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", _NO_WHEEL_PROBE, example], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert "CRON_TZ=Asia/Shanghai 30 2 * * *" in out
    for spec, (py, nat) in out.items():
        assert py == nat, spec
    # 02:30 Asia/Shanghai is 18:30 UTC the day before
    first = out["CRON_TZ=Asia/Shanghai 30 2 * * *"][0][0][0]
    assert GoTime(first, 0, UTC).rfc3339() == "2026-03-07T18:30:00Z"


def test_zone_lookup_fails_cleanly_without_any_source(tmp_path):
    """No wheel and no zoneinfo directory: both engines reject the zone the same way."""
    import os
    import subprocess
    import sys

    probe = r'''
import sys
sys.modules["tzdata"] = None
from cron_operator_amd.cron.engine import NativeEngine, PythonEngine, ScheduleError
for eng in (PythonEngine(), NativeEngine()):
    try:
        eng.parse("CRON_TZ=Asia/Shanghai 30 2 * * *")
    except ScheduleError as e:
        print("ERR", type(eng).__name__, e)
    else:
        print("OK", type(eng).__name__)
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONTZPATH=str(tmp_path / "empty"), PYTHONPATH=root)
    env.pop("ZONEINFO", None)
    r = subprocess.run([sys.executable, "-c", probe], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 2 and all(x.startswith("ERR") for x in lines), lines
    assert all("unknown time zone Asia/Shanghai" in x for x in lines), lines
