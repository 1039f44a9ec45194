"""Native RFC 3339 helpers (``_cron_engine.rfc3339_z`` / ``format_rfc3339``) against the
pure-Python paths of utils/gotime.py they replace: same value, or None and the Python code
decides.  CPU only."""
from __future__ import annotations

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from cron_operator_amd.ops import cron_native
from cron_operator_amd.utils import gotime
from cron_operator_amd.utils.gotime import UTC, FixedZone, GoTime, parse_rfc3339

mod = cron_native.load()


@pytest.fixture
def python_only():
    """The pure-Python paths, for the oracle side of a comparison."""
    gotime.install_native(None, None)
    try:
        yield
    finally:
        gotime.install_native(mod.rfc3339_z, mod.format_rfc3339)


def _py_parse(s: str):
    saved = gotime._native_parse_z, gotime._native_format
    gotime._native_parse_z = gotime._native_format = None
    try:
        return gotime._parse_cached.__wrapped__(s, UTC).key()
    except ValueError:
        return "error"
    finally:
        gotime._native_parse_z, gotime._native_format = saved


def _py_format(t: GoTime, nanos: bool) -> str:
    saved = gotime._native_parse_z, gotime._native_format
    gotime._native_parse_z = gotime._native_format = None
    try:
        return t.rfc3339(nanos=nanos)
    finally:
        gotime._native_parse_z, gotime._native_format = saved


def test_installed_when_the_engine_loads():
    assert gotime._native_parse_z is mod.rfc3339_z
    assert gotime._native_format is mod.format_rfc3339


@pytest.mark.parametrize("s,want", [
    ("2026-01-01T00:00:00Z", 1767225600),
    ("1970-01-01T00:00:00Z", 0),
    ("0000-03-01T00:00:00Z", -62162035200),
    ("9999-12-31T23:59:59Z", 253402300799),
    ("2024-02-31T00:00:00Z", 1709337600),  # day 31 of February is added like Go's Date (-> Mar 2)
])
def test_rfc3339_z_values(s, want):
    assert mod.rfc3339_z(s) == want
    assert _py_parse(s) == (want, 0)


@pytest.mark.parametrize("s", [
    "2026-01-01T00:00:00z", "2026-01-01t00:00:00Z", "2026-01-01T00:00:00+00:00", "2026-01-01T00:00:00.5Z",
    "2026-13-01T00:00:00Z", "2026-00-01T00:00:00Z", "2026-01-00T00:00:00Z", "2026-01-32T00:00:00Z",
    "2026-01-01T24:00:00Z", "2026-01-01T00:60:00Z", "2026-01-01T00:00:60Z", "+202-01-01T00:00:00Z",
    " 202-01-01T00:00:00Z", "2026-01-01 00:00:00Z", "٢026-01-01T00:00:00Z", "2026-01-01T00:00:00Zx", "",
])
def test_rfc3339_z_declines_other_shapes(s):
    assert mod.rfc3339_z(s) is None


@settings(max_examples=400, deadline=None)
@given(st.integers(0, 9999), st.integers(0, 13), st.integers(0, 32), st.integers(0, 24), st.integers(0, 60),
       st.integers(0, 60), st.sampled_from(["Z", "z", "+01:00", ".25Z"]))
def test_parse_matches_python(y, mo, d, hh, mi, ss, tail):
    s = f"{y:04d}-{mo:02d}-{d:02d}T{hh:02d}:{mi:02d}:{ss:02d}{tail}"
    got = mod.rfc3339_z(s)
    want = _py_parse(s)
    if got is not None:
        assert (got, 0) == want
    # through the public function (native first, Python for the rest): same as pure Python
    try:
        pub = gotime._parse_cached.__wrapped__(s, UTC).key()
    except ValueError:
        pub = "error"
    assert pub == want


@settings(max_examples=400, deadline=None)
@given(st.text(alphabet="0123456789-:TZz+. ٣", min_size=18, max_size=22))
def test_parse_fuzz_matches_python(s):
    try:
        pub = gotime._parse_cached.__wrapped__(s, UTC).key()
    except ValueError:
        pub = "error"
    assert pub == _py_parse(s)


@settings(max_examples=500, deadline=None)
@given(st.integers(-62135596800 - 86400 * 800, 253402300799 + 86400 * 800), st.integers(0, 999_999_999),
       st.sampled_from([0, 3600, -3600, 19800, -34200, 45 * 60, 14 * 3600, -(12 * 3600 + 59), 99 * 3600 + 3599]),
       st.booleans())
def test_format_matches_python(sec, nsec, off, nanos):
    loc = UTC if off == 0 else FixedZone("X", off)
    t = GoTime(sec, nsec, loc)
    assert t.rfc3339(nanos=nanos) == _py_format(t, nanos)


@pytest.mark.parametrize("sec,nsec,nanos,want", [
    (0, 0, False, "1970-01-01T00:00:00Z"),
    (0, 500_000_000, True, "1970-01-01T00:00:00.5Z"),
    (0, 1, True, "1970-01-01T00:00:00.000000001Z"),
    (1767225600, 120_000_000, False, "2026-01-01T00:00:00Z"),
])
def test_format_values(sec, nsec, nanos, want):
    assert GoTime(sec, nsec, UTC).rfc3339(nanos=nanos) == want


def test_format_outside_years_0_to_9999_falls_back():
    assert mod.format_rfc3339(-62167219200 - 1, 0, 0) is None  # 0000-01-01 minus one second
    t = GoTime(-62167219200 - 86400, 0, UTC)
    assert t.rfc3339() == _py_format(t, False)


def test_format_utc_cached_and_parse_roundtrip():
    for sec in (0, 1767225600, 253402300799, -62167219200):
        s = gotime.format_rfc3339_utc(GoTime(sec, 0, UTC))
        assert parse_rfc3339(s, UTC).sec == sec


def test_python_only_fixture_restores(python_only):
    assert gotime._native_parse_z is None
    assert parse_rfc3339("2026-01-01T00:00:00Z", UTC).sec == 1767225600
