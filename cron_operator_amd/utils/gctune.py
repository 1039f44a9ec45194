"""Garbage-collector tuning for a long-lived cache-heavy process.

The operator keeps every watched object in informer caches (1000 Crons plus 11000
PyTorchJobs in the headline bench).  CPython's cyclic GC re-scans all of them on
every generation-2 collection even though JSON trees are acyclic and are freed
by reference counting; measured in the bench, that was ~1.7 s of pauses per run
(8 full collections).  Two standard remedies, applied at startup/sync points:

* :func:`freeze` -- collect once, then move everything that survived into the
  permanent generation (``gc.freeze``), so later collections skip the synced
  cache (objects replaced later are still freed by refcounting);
* :func:`tune` -- a larger generation-0 threshold, so short-lived reconcile
  garbage is collected in fewer, cheaper passes.

Disabled with ``CRON_OPERATOR_GC_TUNING=0``; ``CRON_OPERATOR_GC_THRESHOLDS=g0,g1,g2`` replaces
the thresholds.
"""
from __future__ import annotations

import gc
import os

_ENABLED = os.environ.get("CRON_OPERATOR_GC_TUNING", "1") not in ("0", "false", "no")
DEFAULT_THRESHOLDS = (50_000, 20, 100)


def _thresholds_from_env():
    raw = os.environ.get("CRON_OPERATOR_GC_THRESHOLDS", "")
    try:
        t = tuple(int(x) for x in raw.split(","))
    except ValueError:
        return None
    return t if len(t) == 3 and all(x >= 0 for x in t) else None


def enabled() -> bool:
    return _ENABLED


def tune(thresholds=DEFAULT_THRESHOLDS) -> None:
    if _ENABLED:
        gc.set_threshold(*(_thresholds_from_env() or thresholds))


def freeze() -> None:
    """Collect, then exempt every surviving object from future collections."""
    if _ENABLED:
        gc.collect()
        gc.freeze()


class GcStats:
    """Collections per generation and time spent in the cyclic GC while installed
    (``gc.callbacks``), to tell GC pauses apart from real work in a benchmark."""

    def __init__(self) -> None:
        import time

        self._now = time.perf_counter
        self.collections = [0, 0, 0]
        self.gen_seconds = [0.0, 0.0, 0.0]
        self.seconds = 0.0
        self._t0 = 0.0
        self._on = False

    def _cb(self, phase: str, info) -> None:
        if phase == "start":
            self._t0 = self._now()
        else:
            dt = self._now() - self._t0
            gen = info.get("generation", 0)
            self.seconds += dt
            self.gen_seconds[gen] += dt
            self.collections[gen] += 1

    def start(self) -> "GcStats":
        if not self._on:
            gc.callbacks.append(self._cb)
            self._on = True
        return self

    def stop(self) -> "GcStats":
        if self._on:
            gc.callbacks.remove(self._cb)
            self._on = False
        return self

    def to_dict(self):
        return {"collections": list(self.collections), "ms": round(self.seconds * 1000, 2),
                "ms_by_generation": [round(x * 1000, 2) for x in self.gen_seconds]}
