"""Per-reconcile tracing: spans for reconcile -> list -> create/delete -> status patch.

The reference has no tracing (OpenTelemetry/pprof are indirect
deps only); its observability is logs, events and controller-runtime metrics.
SURVEY 5.1 suggests a per-reconcile span carrying the schedule tick, the CREATE
and the status write, because that is exactly what the tick->create latency
metric is made of.  This module provides it without external dependencies:

* :func:`span` -- ``with span("create", kind=...):`` (sync or inside
  coroutines); parent/child links follow ``contextvars``, so concurrent
  reconciles on one event loop get separate traces.
* sinks: an in-memory ring (``Tracer.spans()``), an optional JSON-lines file
  (``--trace-file``), and export as Chrome trace-event JSON
  (``Tracer.chrome_trace()``; open in Perfetto / chrome://tracing), also served
  at ``/debug/traces`` on the probe server.
* sampling per root span (``--trace-sample-rate``); when tracing is off,
  :func:`span` returns a shared no-op object, so instrumented code pays one
  attribute check.
"""
from __future__ import annotations

import contextvars
import json
import os
import random
import threading
import time
from collections import deque
from typing import Any, Deque, Dict, List, Optional

_current: contextvars.ContextVar[Optional["Span"]] = contextvars.ContextVar("cron_operator_span", default=None)


class _NoopSpan:
    __slots__ = ()

    def __enter__(self) -> "_NoopSpan":
        return self

    def __exit__(self, *exc: Any) -> None:
        return None

    def set(self, **attrs: Any) -> None:
        return None

    def event(self, name: str, **attrs: Any) -> None:
        return None


NOOP = _NoopSpan()


class Span:
    __slots__ = ("tracer", "name", "trace_id", "span_id", "parent_id", "start_ns", "end_ns", "attrs", "events",
                 "status", "_token", "sampled")

    def __init__(self, tracer: "Tracer", name: str, parent: Optional["Span"], attrs: Dict[str, Any], sampled: bool):
        self.tracer = tracer
        self.name = name
        self.trace_id = parent.trace_id if parent is not None else tracer._new_id(16)
        self.span_id = tracer._new_id(8)
        self.parent_id = parent.span_id if parent is not None else ""
        self.start_ns = 0
        self.end_ns = 0
        self.attrs = attrs
        self.events: List[Dict[str, Any]] = []
        self.status = "ok"
        self._token: Optional[contextvars.Token] = None
        self.sampled = sampled

    def __enter__(self) -> "Span":
        self.start_ns = time.time_ns()
        self._token = _current.set(self)
        return self

    def __exit__(self, et: Any, ev: Any, tb: Any) -> None:
        self.end_ns = time.time_ns()
        if ev is not None:
            self.status = "error"
            self.attrs["error"] = f"{type(ev).__name__}: {ev}"[:500]
        if self._token is not None:
            _current.reset(self._token)
            self._token = None
        if self.sampled:
            self.tracer._finish(self)

    def set(self, **attrs: Any) -> None:
        self.attrs.update(attrs)

    def event(self, name: str, **attrs: Any) -> None:
        self.events.append({"name": name, "time_ns": time.time_ns(), **attrs})

    def to_dict(self) -> Dict[str, Any]:
        return {"name": self.name, "traceId": self.trace_id, "spanId": self.span_id, "parentSpanId": self.parent_id,
                "startTimeUnixNano": self.start_ns, "endTimeUnixNano": self.end_ns,
                "durationMs": round((self.end_ns - self.start_ns) / 1e6, 4), "status": self.status,
                "attributes": self.attrs, "events": self.events}


class Tracer:
    def __init__(self, enabled: bool = False, capacity: int = 20000, sample_rate: float = 1.0,
                 file: str = "", service: str = "cron-operator"):
        self.enabled = enabled
        self.sample_rate = sample_rate
        self.service = service
        self._ring: Deque[Dict[str, Any]] = deque(maxlen=capacity)
        self._lock = threading.Lock()
        self._rng = random.Random()
        self._fh = open(file, "a", buffering=1) if file else None
        self.finished = 0

    def _new_id(self, nbytes: int) -> str:
        return "%0*x" % (nbytes * 2, self._rng.getrandbits(nbytes * 8))

    def span(self, name: str, /, **attrs: Any):
        if not self.enabled:
            return NOOP
        parent = _current.get()
        if parent is None:
            sampled = self.sample_rate >= 1.0 or self._rng.random() < self.sample_rate
        else:
            sampled = parent.sampled
        return Span(self, name, parent, attrs, sampled)

    def _finish(self, s: Span) -> None:
        d = s.to_dict()
        with self._lock:
            self._ring.append(d)
            self.finished += 1
        if self._fh is not None:
            try:
                self._fh.write(json.dumps(d, default=str) + "\n")
            except (OSError, ValueError):
                pass

    def spans(self) -> List[Dict[str, Any]]:
        with self._lock:
            return list(self._ring)

    def clear(self) -> None:
        with self._lock:
            self._ring.clear()

    def chrome_trace(self) -> Dict[str, Any]:
        """Chrome trace-event format: one complete ("X") event per span, one track per trace."""
        events = []
        tids: Dict[str, int] = {}
        for d in self.spans():
            tid = tids.setdefault(d["traceId"], len(tids) + 1)
            events.append({"name": d["name"], "cat": "cron-operator", "ph": "X",
                           "ts": d["startTimeUnixNano"] / 1000.0,
                           "dur": max(0.0, (d["endTimeUnixNano"] - d["startTimeUnixNano"]) / 1000.0),
                           "pid": os.getpid(), "tid": tid,
                           "args": {**{k: v for k, v in d["attributes"].items()}, "status": d["status"],
                                    "spanId": d["spanId"], "parentSpanId": d["parentSpanId"]}})
            for ev in d["events"]:
                events.append({"name": ev["name"], "ph": "i", "s": "t", "ts": ev["time_ns"] / 1000.0,
                               "pid": os.getpid(), "tid": tid,
                               "args": {k: v for k, v in ev.items() if k not in ("name", "time_ns")}})
        return {"traceEvents": events, "displayTimeUnit": "ms",
                "metadata": {"service": self.service, "spans": len(events)}}

    def close(self) -> None:
        if self._fh is not None:
            self._fh.close()
            self._fh = None


_TRACER = Tracer(enabled=False)


def get_tracer() -> Tracer:
    return _TRACER


def set_tracer(t: Tracer) -> Tracer:
    global _TRACER
    old, _TRACER = _TRACER, t
    return old


def span(name: str, /, **attrs: Any):
    """Start a span on the global tracer (no-op when tracing is disabled)."""
    t = _TRACER
    if not t.enabled:
        return NOOP
    return t.span(name, **attrs)


