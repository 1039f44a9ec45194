"""A small Prometheus client: counters, gauges, histograms, text exposition.

The operator updates about eight series per reconcile (workqueue, reconcile,
REST client, status patches).  With ``prometheus_client`` each update takes a
mutex and runs an observability check, which came to ~6% of an operator shard's
CPU in the benchmark profile.  The operator is one asyncio thread, so a child
series here is a plain object whose ``inc``/``observe`` is an attribute update.

The exposition is the Prometheus text format 0.0.4, written the way the Go
client (``client_golang``, which the reference's controller-runtime uses) writes
it: counters keep their ``_total`` name and there are no ``_created`` samples.
:class:`ProcessCollector` and :class:`PythonCollector` stand in for the Go
client's process and runtime collectors (``process_*``, ``python_*``).
"""
from __future__ import annotations

import gc
import math
import os
import platform
import resource
import threading
from bisect import bisect_left
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

INF = float("inf")
DEFAULT_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.075, 0.1, 0.25, 0.5, 0.75, 1.0, 2.5, 5.0, 7.5, 10.0)


def _escape_label(v: str) -> str:
    return v.replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def _escape_help(v: str) -> str:
    return v.replace("\\", "\\\\").replace("\n", "\\n")


def _fmt(v: float) -> str:
    if v == INF:
        return "+Inf"
    if v == -INF:
        return "-Inf"
    if math.isnan(v):
        return "NaN"
    if v == int(v) and abs(v) < 1e15:
        return str(int(v))
    return repr(float(v))


def _labels(names: Sequence[str], values: Sequence[str], extra: Optional[Tuple[str, str]] = None) -> str:
    """``{a="x",b="y"}`` with label names sorted, as the Go client writes them (``le`` last)."""
    parts = [f'{n}="{_escape_label(v)}"' for n, v in sorted(zip(names, values))]
    if extra is not None:
        parts.append(f'{extra[0]}="{extra[1]}"')
    return "{" + ",".join(parts) + "}" if parts else ""


class Registry:
    def __init__(self) -> None:
        self._collectors: List["Collector"] = []
        self._names: Dict[str, "Collector"] = {}
        self._lock = threading.Lock()

    def register(self, c: "Collector") -> None:
        with self._lock:
            for n in c.names():
                if n in self._names:
                    raise ValueError(f"duplicate metric {n}")
            for n in c.names():
                self._names[n] = c
            self._collectors.append(c)

    def exposition(self) -> bytes:
        out: List[str] = []
        for c in list(self._collectors):
            c.render(out)
        return ("\n".join(out) + "\n").encode()


class Collector:
    def names(self) -> Iterable[str]:
        return ()

    def render(self, out: List[str]) -> None:
        raise NotImplementedError


class _Metric(Collector):
    kind = "untyped"

    def __init__(self, name: str, documentation: str, labelnames: Sequence[str] = (),
                 registry: Optional[Registry] = None):
        self.name = name
        self.documentation = documentation
        self.labelnames = tuple(labelnames)
        self._children: Dict[Tuple[str, ...], object] = {}
        if not self.labelnames:
            self._children[()] = self._new_child()
        if registry is not None:
            registry.register(self)

    def names(self) -> Iterable[str]:
        return (self.name,)

    def _new_child(self):
        raise NotImplementedError

    def labels(self, *values: str, **kw: str):
        if kw:
            values = tuple(kw[n] for n in self.labelnames)
        if len(values) != len(self.labelnames):
            raise ValueError(f"{self.name}: expected labels {self.labelnames}, got {values}")
        key = tuple(str(v) for v in values)
        c = self._children.get(key)
        if c is None:
            c = self._children[key] = self._new_child()
        return c

    def _only(self):
        if self.labelnames:
            raise ValueError(f"{self.name} has labels {self.labelnames}: use .labels()")
        return self._children[()]

    def render(self, out: List[str]) -> None:
        out.append(f"# HELP {self.name} {_escape_help(self.documentation)}")
        out.append(f"# TYPE {self.name} {self.kind}")
        for key, child in sorted(self._children.items()):
            self._render_child(out, key, child)

    def _render_child(self, out: List[str], key: Tuple[str, ...], child) -> None:
        out.append(f"{self.name}{_labels(self.labelnames, key)} {_fmt(child.value)}")


class _PyCounterChild:
    __slots__ = ("value",)

    def __init__(self) -> None:
        self.value = 0.0

    def inc(self, amount: float = 1.0) -> None:
        if amount < 0:
            raise ValueError("counters can only increase")
        self.value += amount

    def get(self) -> float:
        return self.value


class Counter(_Metric):
    kind = "counter"

    def _new_child(self):
        return _CounterChild()

    def inc(self, amount: float = 1.0) -> None:
        self._only().inc(amount)


class _PyGaugeChild:
    __slots__ = ("value",)

    def __init__(self) -> None:
        self.value = 0.0

    def inc(self, amount: float = 1.0) -> None:
        self.value += amount

    def dec(self, amount: float = 1.0) -> None:
        self.value -= amount

    def set(self, value: float) -> None:
        self.value = float(value)

    def get(self) -> float:
        return self.value


class Gauge(_Metric):
    kind = "gauge"

    def _new_child(self):
        return _GaugeChild()

    def inc(self, amount: float = 1.0) -> None:
        self._only().inc(amount)

    def dec(self, amount: float = 1.0) -> None:
        self._only().dec(amount)

    def set(self, value: float) -> None:
        self._only().set(value)


class _PyHistogramChild:
    __slots__ = ("bounds", "counts", "sum", "count")

    def __init__(self, bounds: Tuple[float, ...]) -> None:
        self.bounds = bounds
        self.counts = [0] * (len(bounds) + 1)  # last slot: above every finite bound
        self.sum = 0.0
        self.count = 0

    def observe(self, v: float) -> None:
        self.counts[bisect_left(self.bounds, v)] += 1  # le semantics: v <= bound
        self.sum += v
        self.count += 1


def _series_classes():
    """The series classes: ``_promlite``'s (``ops/csrc/promlite.cpp``: one C call per update) or
    the Python ones above, which are their oracle (``CRON_OPERATOR_NATIVE_METRICS=python``)."""
    want = os.environ.get("CRON_OPERATOR_NATIVE_METRICS", "auto").lower()
    if want != "python":
        try:
            from ..ops import build as _build

            if _build.needs_build("_promlite"):
                _build.build_extension("_promlite")
            from ..ops import _promlite  # type: ignore[attr-defined]

            return _promlite.Counter, _promlite.Gauge, _promlite.Histogram
        except Exception:  # noqa: BLE001 - the Python series remain
            if want == "native":
                raise
    return _PyCounterChild, _PyGaugeChild, _PyHistogramChild


_CounterChild, _GaugeChild, _HistogramChild = _series_classes()
NATIVE = _CounterChild is not _PyCounterChild


class Histogram(_Metric):
    kind = "histogram"

    def __init__(self, name: str, documentation: str, labelnames: Sequence[str] = (),
                 buckets: Sequence[float] = DEFAULT_BUCKETS, registry: Optional[Registry] = None):
        bounds = tuple(sorted(float(b) for b in buckets if float(b) != INF))
        if not bounds:
            raise ValueError("histogram needs at least one finite bucket")
        self.bounds = bounds
        super().__init__(name, documentation, labelnames, registry)

    def _new_child(self):
        return _HistogramChild(self.bounds)

    def observe(self, v: float) -> None:
        self._only().observe(v)

    def _render_child(self, out: List[str], key: Tuple[str, ...], child: _HistogramChild) -> None:
        acc = 0
        for b, n in zip(self.bounds, child.counts):
            acc += n
            out.append(f"{self.name}_bucket{_labels(self.labelnames, key, ('le', _fmt(b)))} {acc}")
        out.append(f"{self.name}_bucket{_labels(self.labelnames, key, ('le', '+Inf'))} {child.count}")
        out.append(f"{self.name}_sum{_labels(self.labelnames, key)} {_fmt(child.sum)}")
        out.append(f"{self.name}_count{_labels(self.labelnames, key)} {child.count}")


class ObservedGauge(Collector):
    """Series read from live objects at scrape time (no per-event update cost): each
    :meth:`observe` binds a label set to ``fn(obj)`` for an object held weakly, so a
    controller or client that goes away drops its series.  ``kind`` is ``gauge`` or
    ``counter``."""

    def __init__(self, name: str, documentation: str, labelnames: Sequence[str] = (), kind: str = "gauge",
                 registry: Optional[Registry] = None):
        self.name = name
        self.documentation = documentation
        self.labelnames = tuple(labelnames)
        self.kind = kind
        self._bound: Dict[Tuple[str, ...], Tuple[Any, Any]] = {}
        if registry is not None:
            registry.register(self)

    def names(self) -> Iterable[str]:
        return (self.name,)

    def observe(self, labels: Sequence[str], obj: Any, fn: Any) -> None:
        import weakref

        self._bound[tuple(str(v) for v in labels)] = (weakref.ref(obj), fn)

    def value(self, *labels: str) -> Optional[float]:
        hit = self._bound.get(tuple(labels))
        obj = hit[0]() if hit is not None else None
        return None if obj is None else float(hit[1](obj))  # type: ignore[index]

    def render(self, out: List[str]) -> None:
        out.append(f"# HELP {self.name} {_escape_help(self.documentation)}")
        out.append(f"# TYPE {self.name} {self.kind}")
        for key, (ref, fn) in sorted(self._bound.items()):
            obj = ref()
            if obj is None:
                continue
            out.append(f"{self.name}{_labels(self.labelnames, key)} {_fmt(float(fn(obj)))}")


class ProcessCollector(Collector):
    """``process_*`` series from ``/proc/self`` (the Go client's process collector)."""

    def __init__(self, registry: Optional[Registry] = None):
        try:
            self._ticks = os.sysconf("SC_CLK_TCK")
            self._page = os.sysconf("SC_PAGESIZE")
            with open("/proc/stat") as fh:
                self._btime = next(float(ln.split()[1]) for ln in fh if ln.startswith("btime"))
            self.ok = True
        except (OSError, ValueError, StopIteration):
            self.ok = False
        if registry is not None:
            registry.register(self)

    def names(self) -> Iterable[str]:
        return ("process_cpu_seconds_total", "process_resident_memory_bytes", "process_virtual_memory_bytes",
                "process_start_time_seconds", "process_open_fds", "process_max_fds")

    def render(self, out: List[str]) -> None:
        if not self.ok:
            return
        try:
            with open("/proc/self/stat") as fh:
                f = fh.read().rsplit(")", 1)[1].split()
            fds = len(os.listdir("/proc/self/fd"))
        except OSError:
            return
        vals = [
            ("process_cpu_seconds_total", "counter", "Total user and system CPU time spent in seconds.",
             (int(f[11]) + int(f[12])) / self._ticks),
            ("process_resident_memory_bytes", "gauge", "Resident memory size in bytes.", int(f[21]) * self._page),
            ("process_virtual_memory_bytes", "gauge", "Virtual memory size in bytes.", int(f[20])),
            ("process_start_time_seconds", "gauge", "Start time of the process since unix epoch in seconds.",
             self._btime + int(f[19]) / self._ticks),
            ("process_open_fds", "gauge", "Number of open file descriptors.", fds),
            ("process_max_fds", "gauge", "Maximum number of open file descriptors.",
             resource.getrlimit(resource.RLIMIT_NOFILE)[0]),
        ]
        for name, kind, doc, v in vals:
            out.append(f"# HELP {name} {doc}")
            out.append(f"# TYPE {name} {kind}")
            out.append(f"{name} {_fmt(float(v))}")


class PythonCollector(Collector):
    """``python_info`` and ``python_gc_*`` (the Go client's runtime collector counterpart)."""

    def __init__(self, registry: Optional[Registry] = None):
        if registry is not None:
            registry.register(self)

    def names(self) -> Iterable[str]:
        return ("python_info", "python_gc_objects_collected_total", "python_gc_objects_uncollectable_total",
                "python_gc_collections_total")

    def render(self, out: List[str]) -> None:
        major, minor, patch = platform.python_version_tuple()
        out.append("# HELP python_info Python platform information")
        out.append("# TYPE python_info gauge")
        out.append(f'python_info{{implementation="{platform.python_implementation()}",major="{major}",'
                   f'minor="{minor}",patchlevel="{patch}",version="{platform.python_version()}"}} 1')
        stats = gc.get_stats()
        for name, key, doc in (("python_gc_objects_collected_total", "collected", "Objects collected during gc"),
                               ("python_gc_objects_uncollectable_total", "uncollectable",
                                "Uncollectable objects found during GC"),
                               ("python_gc_collections_total", "collections",
                                "Number of times this generation was collected")):
            out.append(f"# HELP {name} {doc}")
            out.append(f"# TYPE {name} counter")
            for gen, st in enumerate(stats):
                out.append(f'{name}{{generation="{gen}"}} {st.get(key, 0)}')
