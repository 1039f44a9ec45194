"""The in-repo Prometheus client (``runtime/promlite.py``): values, histogram buckets,
escaping, and a text exposition that a standard Prometheus parser accepts."""
from __future__ import annotations

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from cron_operator_amd.runtime import promlite as pl


def _parse(text: str):
    parser = pytest.importorskip("prometheus_client.parser")
    return {f.name: f for f in parser.text_string_to_metric_families(text)}


@settings(max_examples=100, deadline=None)
@given(values=st.lists(st.floats(min_value=0, max_value=100, allow_nan=False), max_size=50))
def test_histogram_buckets_are_cumulative_le_counts(values):
    reg = pl.Registry()
    bounds = (0.5, 1.0, 5.0, 50.0)
    h = pl.Histogram("h_seconds", "doc", ["a"], buckets=bounds, registry=reg)
    hx = h.labels("x")  # a child appears in the exposition once it is created
    for v in values:
        hx.observe(v)
    fam = _parse(reg.exposition().decode())["h_seconds"]
    got = {s.labels["le"]: s.value for s in fam.samples if s.name == "h_seconds_bucket"}
    for b in bounds:
        assert got[pl._fmt(b)] == sum(1 for v in values if v <= b)
    assert got["+Inf"] == len(values)
    total = [s.value for s in fam.samples if s.name == "h_seconds_sum"]
    assert total and abs(total[0] - sum(values)) < 1e-6


def test_counter_gauge_and_escaping_round_trip():
    reg = pl.Registry()
    c = pl.Counter("reqs_total", "Requests.\nSecond line", ["code", "host"], registry=reg)
    g = pl.Gauge("depth", "Depth", ["name"], registry=reg)
    u = pl.Counter("plain_total", "No labels", registry=reg)
    c.labels("200", 'we"ird\\host\n').inc()
    c.labels(code="200", host='we"ird\\host\n').inc(2)
    g.labels("q").inc(5)
    g.labels("q").dec(2)
    u.inc()
    with pytest.raises(ValueError):
        c.labels("200", "h").inc(-1)
    with pytest.raises(ValueError):
        c.labels("only-one")
    with pytest.raises(ValueError):
        pl.Counter("reqs_total", "dup", registry=reg)
    fams = _parse(reg.exposition().decode())
    (s,) = [s for s in fams["reqs"].samples if s.name == "reqs_total" and s.labels["host"] != "h"]
    assert s.labels == {"code": "200", "host": 'we"ird\\host\n'} and s.value == 3
    assert fams["depth"].samples[0].value == 3
    assert fams["plain"].samples[0].value == 1
    assert 'reqs_total{code="200",host="h"} 0' in reg.exposition().decode()  # sorted label names


def test_operator_registry_exposes_controller_runtime_names():
    from cron_operator_amd.runtime import metrics

    metrics.child(metrics.RECONCILE_TOTAL, "cron", "success").inc()
    fams = _parse(metrics.exposition().decode())
    for name in ("controller_runtime_reconcile", "controller_runtime_reconcile_time_seconds", "workqueue_depth",
                 "rest_client_requests", "process_cpu_seconds", "process_resident_memory_bytes", "python_info"):
        assert name in fams, name


def test_supervisor_merges_shard_expositions():
    """runtime/supervisor.py: one HELP/TYPE per family, every sample labelled by shard,
    histogram series kept under their family; the result parses."""
    from cron_operator_amd.runtime.supervisor import merge_expositions

    a = ("# HELP x_total Things.\n# TYPE x_total counter\nx_total{kind=\"a\"} 1.0\n"
         "# HELP h_seconds Lat.\n# TYPE h_seconds histogram\nh_seconds_bucket{le=\"+Inf\"} 2.0\n"
         "h_seconds_sum 0.5\nh_seconds_count 2.0\n# HELP g Plain.\n# TYPE g gauge\ng 3.0\n")
    b = a.replace("1.0", "4.0")
    out = merge_expositions([("0", a), ("1", b)])
    assert out.count("# TYPE x_total counter") == 1
    assert 'x_total{shard="0",kind="a"} 1.0' in out and 'x_total{shard="1",kind="a"} 4.0' in out
    assert 'g{shard="1"} 3.0' in out and 'h_seconds_sum{shard="0"} 0.5' in out
    fams = _parse(out)
    assert {s.labels["shard"] for s in fams["x"].samples} == {"0", "1"}
    assert len(fams["h_seconds"].samples) == 6


def test_available_cpus_reads_cgroup_quotas(tmp_path):
    """`--shard-processes auto`: the container's CPU quota, rounded up, capped by affinity."""
    import os

    from cron_operator_amd.cmd.main import build_parser
    from cron_operator_amd.runtime.supervisor import available_cpus

    affinity = len(os.sched_getaffinity(0))
    v2 = tmp_path / "v2"
    v2.mkdir()
    (v2 / "cpu.max").write_text("150000 100000\n")
    assert available_cpus(str(v2)) == min(2, affinity)
    (v2 / "cpu.max").write_text("max 100000\n")
    assert available_cpus(str(v2)) == affinity
    v1 = tmp_path / "v1"
    (v1 / "cpu").mkdir(parents=True)
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("100000\n")
    (v1 / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    assert available_cpus(str(v1)) == 1
    (v1 / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")
    assert available_cpus(str(v1)) == affinity
    assert available_cpus(str(tmp_path / "none")) == affinity
    a = build_parser().parse_args(["start", "--shard-processes", "auto"])
    assert a.shard_processes >= 1
    assert build_parser().parse_args(["start", "--shard-processes", "3"]).shard_processes == 3


# ---------------------------------------------------------------- native series vs their Python twins

_native = pytest.mark.skipif(not pl.NATIVE, reason="_promlite not built or disabled")
_num = st.one_of(st.floats(allow_nan=True, allow_infinity=True), st.integers(-10**6, 10**6))


@_native
@settings(max_examples=200, deadline=None)
@given(bounds=st.lists(st.floats(-1e6, 1e6, allow_nan=False), min_size=1, max_size=20).map(lambda b: tuple(sorted(b))),
       values=st.lists(_num, max_size=60))
def test_native_histogram_matches_python_series(bounds, values):
    nat, py = pl._HistogramChild(bounds), pl._PyHistogramChild(bounds)
    for v in values:
        nat.observe(v)
        py.observe(v)
    assert nat.counts == py.counts and nat.count == py.count and nat.bounds == py.bounds
    assert (nat.sum == py.sum) or (nat.sum != nat.sum and py.sum != py.sum)  # NaN sums stay NaN


@_native
@settings(max_examples=200, deadline=None)
@given(ops=st.lists(st.tuples(st.sampled_from(["inc", "dec", "set", "inc1"]), _num), max_size=40))
def test_native_counter_and_gauge_match_python_series(ops):
    pairs = [(pl._CounterChild(), pl._PyCounterChild()), (pl._GaugeChild(), pl._PyGaugeChild())]
    for op, v in ops:
        for nat, py in pairs:
            fn = op[:3]
            if not hasattr(py, fn):
                continue
            outcomes = []
            for s in (nat, py):
                try:
                    getattr(s, fn)() if op == "inc1" else getattr(s, fn)(v)
                    outcomes.append(None)
                except ValueError as e:
                    outcomes.append(str(e))
            assert outcomes[0] == outcomes[1]
            assert (nat.value == py.value) or (nat.value != nat.value and py.value != py.value)
            assert nat.get() == nat.value or nat.value != nat.value


@_native
def test_native_series_render_like_python_series(monkeypatch):
    def expo():
        reg = pl.Registry()
        c = pl.Counter("c_total", "c", ["code"], registry=reg)
        g = pl.Gauge("g", "g", registry=reg)
        h = pl.Histogram("h_seconds", "h", ["verb"], buckets=(0.1, 1.0), registry=reg)
        c.labels("200").inc(3)
        g.set(7)
        g.dec(2.5)
        for v in (0.05, 0.1, 0.5, 3.0):
            h.labels("GET").observe(v)
        return reg.exposition()

    native = expo()
    monkeypatch.setattr(pl, "_CounterChild", pl._PyCounterChild)
    monkeypatch.setattr(pl, "_GaugeChild", pl._PyGaugeChild)
    monkeypatch.setattr(pl, "_HistogramChild", pl._PyHistogramChild)
    assert native == expo()


@_native
def test_native_series_refuse_bad_arguments():
    with pytest.raises(ValueError, match="counters can only increase"):
        pl._CounterChild().inc(-1)
    with pytest.raises(TypeError):
        pl._CounterChild().inc("x")
    with pytest.raises(ValueError):
        pl._HistogramChild((2.0, 1.0))
    assert pl._GaugeChild().set("2.5") is None  # float(value), like the Python series
