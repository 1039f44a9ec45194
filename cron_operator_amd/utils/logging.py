"""Structured logr/zap-style logging.

Mirrors what the reference gets from controller-runtime's zap integration
(``cmd/operator/start.go:244-265``): ``--zap-devel``, ``--zap-encoder``
(``json``/``console``), ``--zap-log-level`` (``debug``/``info``/``error``/
``panic`` or an integer verbosity), ``--zap-stacktrace-level`` and
``--zap-time-encoding``; capital level names, ISO8601 timestamps and short
``file:line`` callers.  The API is logr's: ``info``/``error``/``v(n)``/
``with_values``/``with_name``; the per-reconcile logger carries
``controller=cron`` and ``Cron={name,namespace}`` like ``logConstructor``
(``internal/controller/util.go:27-41``).

Level checks happen before any formatting so disabled lines cost one compare.
"""
from __future__ import annotations

import json
import sys
import threading
import time
import traceback
from typing import Any, Dict, IO, Optional, Tuple

# zap levels: debug=-1, info=0, warn=1, error=2, dpanic=3, panic=4, fatal=5; V(n) == -n
_LEVEL_NAMES = {"debug": -1, "info": 0, "warn": 1, "error": 2, "dpanic": 3, "panic": 4, "fatal": 5}


def parse_level(s: str) -> int:
    s = str(s).strip().lower()
    if s in _LEVEL_NAMES:
        return _LEVEL_NAMES[s]
    try:
        n = int(s)
    except ValueError:
        raise ValueError(f'invalid log level "{s}"') from None
    if n <= 0:
        raise ValueError(f'invalid log level "{s}"')
    return -n


def level_name(lvl: int) -> str:
    for k, v in _LEVEL_NAMES.items():
        if v == lvl:
            return k.upper()
    return f"LEVEL({lvl})"


class ObjectRef:
    """``klog.KRef``: renders ``{"name","namespace"}`` in JSON, ``ns/name`` in text."""

    __slots__ = ("namespace", "name")

    def __init__(self, namespace: str, name: str):
        self.namespace = namespace
        self.name = name

    def to_json(self) -> Any:
        if self.namespace:
            return {"name": self.name, "namespace": self.namespace}
        return {"name": self.name}

    def __str__(self) -> str:
        return f"{self.namespace}/{self.name}" if self.namespace else self.name


def _jsonable(v: Any) -> Any:
    if isinstance(v, ObjectRef):
        return v.to_json()
    if isinstance(v, BaseException):
        return str(v)
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    if isinstance(v, (list, tuple)) and not hasattr(v, "_fields"):  # named tuples (GVK, keys) log as str()
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    return str(v)


class Sink:
    """Thread-safe line writer + encoder configuration."""

    def __init__(self, stream: Optional[IO[str]] = None, encoder: str = "json", level: int = 0,
                 stacktrace_level: int = 2, time_encoding: str = "iso8601", development: bool = False):
        self.stream = stream if stream is not None else sys.stderr
        self.encoder = encoder
        self.level = level
        self.stacktrace_level = stacktrace_level
        self.time_encoding = time_encoding
        self.development = development
        self._mu = threading.Lock()
        self.lines_written = 0

    def enabled(self, lvl: int) -> bool:
        return lvl >= self.level

    def _ts(self, now: float) -> Any:
        te = self.time_encoding
        if te == "epoch":
            return now
        if te == "millis":
            return now * 1000.0
        if te == "nano":
            return int(now * 1e9)
        lt = time.gmtime(now)
        base = time.strftime("%Y-%m-%dT%H:%M:%S", lt)
        if te == "rfc3339":
            return base + "Z"
        if te == "rfc3339nano":
            return f"{base}.{int((now % 1) * 1e9):09d}".rstrip("0").rstrip(".") + "Z"
        # iso8601 (zap's ISO8601TimeEncoder: millisecond precision, numeric offset)
        return f"{base}.{int((now % 1) * 1000):03d}Z"

    def write(self, lvl: int, logger: str, caller: str, msg: str, kv: Dict[str, Any],
              err: Optional[BaseException] = None) -> None:
        now = time.time()
        stack = None
        if lvl >= self.stacktrace_level:
            stack = "".join(traceback.format_stack(limit=12)[:-3])
        if self.encoder == "console":
            parts = [str(self._ts(now)), level_name(lvl)]
            if logger:
                parts.append(logger)
            parts.append(caller)
            parts.append(msg)
            fields = dict(kv)
            if err is not None:
                fields["error"] = str(err)
            if fields:
                parts.append(json.dumps({k: _jsonable(v) for k, v in fields.items()}, separators=(",", ":"),
                                        default=str))
            line = "\t".join(parts)
            if stack:
                line += "\n" + stack.rstrip()
        else:
            rec: Dict[str, Any] = {"level": level_name(lvl).lower() if lvl >= -1 else str(lvl),
                                   "ts": self._ts(now)}
            if logger:
                rec["logger"] = logger
            rec["caller"] = caller
            rec["msg"] = msg
            for k, v in kv.items():
                rec[k] = _jsonable(v)
            if err is not None:
                rec["error"] = str(err)
            if stack:
                rec["stacktrace"] = stack
            line = json.dumps(rec, separators=(",", ":"), default=str)
        with self._mu:
            self.stream.write(line + "\n")
            self.lines_written += 1

    def flush(self) -> None:
        try:
            self.stream.flush()
        except Exception:
            pass


def _caller(depth: int = 2) -> str:
    """``file:line`` of the log call (frame 0 is this function, 1 is Logger.info/error)."""
    f = sys._getframe(depth)
    fn = f.f_code.co_filename
    parts = fn.replace("\\", "/").split("/")
    short = "/".join(parts[-2:]) if len(parts) >= 2 else fn
    return f"{short}:{f.f_lineno}"


class Logger:
    """logr.Logger equivalent."""

    __slots__ = ("_sink", "_name", "_kv", "_v")

    def __init__(self, sink: "Sink", name: str = "", kv: Optional[Dict[str, Any]] = None, v: int = 0):
        self._sink = sink
        self._name = name
        self._kv = kv or {}
        self._v = v

    @property
    def sink(self) -> Sink:
        return self._sink

    def enabled(self) -> bool:
        return self._sink.enabled(-self._v)

    def v(self, level: int) -> "Logger":
        return Logger(self._sink, self._name, self._kv, self._v + level)

    def with_values(self, **kv: Any) -> "Logger":
        d = dict(self._kv)
        d.update(kv)
        return Logger(self._sink, self._name, d, self._v)

    def with_kv(self, pairs: Tuple[Tuple[str, Any], ...]) -> "Logger":
        d = dict(self._kv)
        d.update(pairs)
        return Logger(self._sink, self._name, d, self._v)

    def with_name(self, name: str) -> "Logger":
        return Logger(self._sink, f"{self._name}.{name}" if self._name else name, self._kv, self._v)

    def info(self, msg: str, **kv: Any) -> None:
        lvl = -self._v
        if lvl < self._sink.level:
            return
        if kv:
            d = dict(self._kv)
            d.update(kv)
        else:
            d = self._kv
        self._sink.write(lvl, self._name, _caller(), msg, d)

    def error(self, err: Optional[BaseException], msg: str, **kv: Any) -> None:
        if 2 < self._sink.level:
            return
        d = dict(self._kv)
        d.update(kv)
        self._sink.write(2, self._name, _caller(), msg, d, err)


_root_lock = threading.Lock()
_root = Logger(Sink(encoder="console", level=0))


def set_logger(logger: Logger) -> None:
    global _root
    with _root_lock:
        _root = logger


def get_logger(name: str = "") -> Logger:
    return _root.with_name(name) if name else _root



def new_from_options(encoder: Optional[str] = None, level: Optional[str] = None, devel: bool = False,
                     stacktrace_level: Optional[str] = None, time_encoding: Optional[str] = None,
                     stream: Optional[IO[str]] = None) -> Logger:
    """``logzap.New(UseFlagOptions(opts), ...)`` as configured in ``setupLog``."""
    if devel:
        enc, lvl, st = "console", -1, 1  # development: console, debug, stacktraces from warn
    else:
        enc, lvl, st = "json", 0, 2
    if encoder:
        if encoder not in ("json", "console"):
            raise ValueError(f'invalid encoder value "{encoder}"')
        enc = encoder
    if level is not None:
        lvl = parse_level(level)
    if stacktrace_level is not None:
        st = parse_level(stacktrace_level)
    te = time_encoding or "iso8601"
    if te not in ("epoch", "millis", "nano", "iso8601", "rfc3339", "rfc3339nano"):
        raise ValueError(f'invalid time-encoding value "{te}"')
    return Logger(Sink(stream=stream, encoder=enc, level=lvl, stacktrace_level=st, time_encoding=te,
                       development=devel))


def log_constructor(base: Logger, kind: str):
    """``logConstructor`` (``internal/controller/util.go:27-41``)."""
    name = kind.lower()
    base_logger = base.with_values(controller=name)

    def construct(req=None) -> Logger:
        if req is not None:
            return base_logger.with_kv(((kind, ObjectRef(req.namespace, req.name)),))
        return base_logger

    return construct
