"""Client-side QPS starvation is visible, like client-go's.

The reference configures its client with ``--qps 30 --burst 50``
(``/root/reference/cmd/operator/start.go:152-154,218-219``); client-go then logs
``Waited for <d> due to client-side throttling ...`` when a request waits on that
bucket for long [ext, rest/request.go].  At the reference chart's ``qps: 30`` a 1000-Cron
minutely workload would need ~83 QPS (this chart ships 150, ``tests/test_chart_sizing.py``),
so this log is how an under-budgeted operator says it is starved.
"""
from __future__ import annotations

import asyncio
import io
import re
import time

from cron_operator_amd.api.v1alpha1 import CRON_GVR, new_cron
from cron_operator_amd.runtime import client as rc
from cron_operator_amd.runtime import metrics
from cron_operator_amd.testing.env import TestEnv
from cron_operator_amd.utils.logging import get_logger, new_from_options, set_logger

NS = "default"
PT_TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}}
LINE = re.compile(r"Waited for ([0-9.]+(?:ms|s)) due to client-side throttling, not priority and fairness, "
                  r"request: (POST|PATCH|DELETE|GET|PUT):\S*/apis/")


def _slow_waits(verbs=("create", "patch")) -> int:
    """Observations above 1 s in ``rest_client_rate_limiter_duration_seconds``."""
    total = 0
    for v in verbs:
        h = metrics.REST_RATE_LIMIT.labels(v, "in-memory")
        total += sum(h.counts[h.bounds.index(1.0) + 1:])
    return total


async def test_starved_client_logs_throttling_and_stays_bounded():
    """qps=2 and 20 Crons firing together: requests queue on the token bucket for seconds.
    The throttling line appears at Info, the limiter histogram records >1 s waits, and the
    throttled logger keeps the Info volume to one line per 10 s however many requests wait."""
    prev = get_logger()
    buf = io.StringIO()
    set_logger(new_from_options(encoder="console", level="info", stream=buf))
    rc.THROTTLED_LOGGER._last.clear()
    before = _slow_waits()
    env = TestEnv(qps=2, burst=2)
    try:
        setup = env.new_client()  # unthrottled: only the operator's client is starved
        for i in range(20):
            c = new_cron(f"c{i:02d}", NS, "*/1 * * * *", PT_TMPL)
            await setup.create(CRON_GVR, c.to_dict(), NS)
        await env.start_manager()
        t0 = time.monotonic()
        env.clock.advance(60)  # every Cron's tick is due: 20 CREATEs + 20 PATCHes at 2 QPS
        # until several requests have waited > 1 s (each one is a candidate log line)
        while time.monotonic() - t0 < 10 and (LINE.search(buf.getvalue()) is None or
                                              _slow_waits() - before < 3):
            await asyncio.sleep(0.1)
    finally:
        await env.stop()
        set_logger(prev)
    out = buf.getvalue()
    lines = [ln for ln in out.splitlines() if "client-side throttling" in ln]
    assert len(lines) == 1, lines
    m = LINE.search(lines[0])
    assert m is not None, lines[0]
    assert _slow_waits() - before >= 3


def test_throttled_logger_levels_and_intervals():
    """client-go's settings: with V(2) enabled one line per second at V(2), else one Info
    line per 10 s; the first enabled setting decides."""
    now = [100.0]
    tl = rc.ThrottledLogger(clock=lambda: now[0])
    for level, interval in (("info", 10.0), ("2", 1.0)):
        buf = io.StringIO()
        log = new_from_options(encoder="console", level=level, stream=buf)
        tl._last.clear()
        written = 0
        for _ in range(50):  # 50 messages over 5 s
            written += tl.info(log, "Waited for 1.5s due to client-side throttling")
            now[0] += 0.1
        assert written == (1 if interval == 10.0 else 5), (level, written)
        assert buf.getvalue().count("Waited for") == written


def test_v3_logs_every_wait_over_50ms():
    buf = io.StringIO()
    prev = get_logger()
    set_logger(new_from_options(encoder="console", level="3", stream=buf))
    try:
        env = TestEnv()
        rc.THROTTLED_LOGGER._last.clear()
        env.client._log_throttle(0.08, "get", CRON_GVR, NS, "x", "")
    finally:
        set_logger(prev)
    assert buf.getvalue().count("Waited for 80ms due to client-side throttling") == 1
    assert "/apis/apps.kubedl.io/v1alpha1/namespaces/default/crons/x" in buf.getvalue()
