"""Schedule engine facade used by the reconciler.

Two interchangeable backends with identical semantics:

* ``native`` -- ``ops/csrc/cron_engine.cpp`` (default when built): parse, next,
  and the missed-run scan with whole-day counting;
* ``python`` -- :mod:`.parser` / :mod:`.schedule` (reference twin, used for
  differential tests and as the fallback on a box without a C++ compiler).

Selection: ``$CRON_OPERATOR_ENGINE`` = ``native`` | ``python`` | ``auto``
(default ``auto``: native if it builds/imports, python otherwise with a
warning).  ``native`` fails loudly if the extension cannot be loaded.

Parsed schedules are cached by spec string (a Cron's spec rarely changes and
the reference re-parses it on every reconcile, ``cron_controller.go:392``).
"""
from __future__ import annotations

import logging
import os
import threading
from collections import OrderedDict
from typing import Any, Optional, Tuple

from ..utils.gotime import GoTime
from . import parser as pyparser
from .schedule import missed_runs as py_missed_runs

log = logging.getLogger(__name__)


class ScheduleError(ValueError):
    """Parse failure; ``str()`` is the robfig message."""


class _Parsed:
    __slots__ = ("spec", "impl")

    def __init__(self, spec: str, impl: Any):
        self.spec = spec
        self.impl = impl


class CronEngine:
    name = "base"

    def __init__(self, cache_size: int = 8192):
        self._cache: "OrderedDict[str, Any]" = OrderedDict()
        self._cache_size = cache_size
        self._mu = threading.Lock()

    # -- parse with LRU cache (errors are cached too: a bad spec stays bad)
    def parse(self, spec: str) -> _Parsed:
        hit = self._cache.get(spec)  # a single dict read is atomic: the hot path takes no lock
        if hit.__class__ is _Parsed:
            return hit  # (recency is only refreshed on the locked path: eviction is roughly LRU)
        with self._mu:
            hit = self._cache.get(spec)
            if hit is not None:
                self._cache.move_to_end(spec)
        if hit is None:
            try:
                hit = _Parsed(spec, self._parse(spec))
            except ValueError as e:
                hit = ScheduleError(str(e))
            with self._mu:
                self._cache[spec] = hit
                if len(self._cache) > self._cache_size:
                    self._cache.popitem(last=False)
        if isinstance(hit, ScheduleError):
            raise hit
        return hit

    def _parse(self, spec: str) -> Any:
        raise NotImplementedError

    def next(self, sched: _Parsed, t: GoTime) -> GoTime:
        raise NotImplementedError

    def missed(self, sched: _Parsed, earliest: GoTime, now: GoTime) -> Tuple[GoTime, int, bool]:
        """(last_missed, count, unschedulable) over ``(earliest, now]``."""
        raise NotImplementedError


class PythonEngine(CronEngine):
    name = "python"

    def _parse(self, spec: str) -> Any:
        return pyparser.parse_standard(spec)

    def next(self, sched: _Parsed, t: GoTime) -> GoTime:
        return sched.impl.next(t)

    def missed(self, sched: _Parsed, earliest: GoTime, now: GoTime) -> Tuple[GoTime, int, bool]:
        last, n, bad = py_missed_runs(sched.impl, earliest, now.in_(earliest.loc))
        if not last.is_zero():
            last = last.in_(earliest.loc)
        return last, n, bad


class NativeEngine(CronEngine):
    name = "native"

    def __init__(self, cache_size: int = 8192):
        super().__init__(cache_size)
        from ..ops import cron_native

        self._native = cron_native
        self._mod = cron_native.load()
        self._zero = self._mod.ZERO_UNIX

    def _parse(self, spec: str) -> Any:
        if any(c.isspace() and not c.isascii() for c in spec):
            # strings.Fields splits on Unicode spaces too; keep the exotic path in Python
            return pyparser.parse_standard(spec)
        return self._mod.parse(spec)

    def next(self, sched: _Parsed, t: GoTime) -> GoTime:
        impl = sched.impl
        if not isinstance(impl, self._mod.Schedule):
            return impl.next(t)
        sec, nsec = impl.next(t.sec, t.nsec, self._native.zone_id(t.loc))
        if sec == self._zero and nsec == 0:
            return GoTime.zero()
        return GoTime(sec, nsec, t.loc)

    def missed(self, sched: _Parsed, earliest: GoTime, now: GoTime) -> Tuple[GoTime, int, bool]:
        impl = sched.impl
        if not isinstance(impl, self._mod.Schedule):
            return PythonEngine.missed(self, sched, earliest, now)  # type: ignore[arg-type]
        ls, ln, n, bad = impl.missed(earliest.sec, earliest.nsec, now.sec, now.nsec,
                                     self._native.zone_id(earliest.loc))
        if ls == self._zero and ln == 0:
            return GoTime.zero(), n, bad
        return GoTime(ls, ln, earliest.loc), n, bad


_default: Optional[CronEngine] = None
_default_mu = threading.Lock()


def make_engine(kind: Optional[str] = None) -> CronEngine:
    kind = (kind or os.environ.get("CRON_OPERATOR_ENGINE", "auto")).lower()
    if kind == "python":
        return PythonEngine()
    if kind == "native":
        return NativeEngine()
    try:
        return NativeEngine()
    except Exception as e:  # noqa: BLE001
        log.warning("native cron engine unavailable (%s); using the Python engine", e)
        return PythonEngine()


def default_engine() -> CronEngine:
    global _default
    if _default is None:
        with _default_mu:
            if _default is None:
                _default = make_engine()
    return _default
