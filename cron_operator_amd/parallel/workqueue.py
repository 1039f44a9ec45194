"""Rate-limited, delaying, priority work queue with per-key serialisation.

This is the concurrency core the reference inherits from controller-runtime
([ext] client-go ``workqueue``): up to ``--max-concurrent-reconciles`` workers
(``cmd/operator/start.go:215``) pull keys, and the queue guarantees one key is
never processed by two workers at once (SURVEY 2.3 "controller parallelism",
5.2).  Semantics:

* **dedupe** -- adding a key that is already queued is a no-op (its priority is
  raised if the new add is more urgent);
* **serialisation** -- a key added while a worker holds it is parked ("dirty")
  and re-queued when the worker calls :meth:`done`;
* **delays** -- :meth:`add_after` keeps only the earliest pending deadline per key
  and is driven by the injected :class:`~cron_operator_amd.utils.clock.Clock`
  (one timer for the whole queue, not one per key);
* **rate limiting** -- :meth:`add_rate_limited` asks the limiter for a backoff
  (default: per-item exponential 5ms->1000s max'd with a 10qps/100 bucket);
* **priority** -- larger numbers are served first (FIFO within a priority).  The
  controller enqueues due schedule requeues above event-driven work so a tick
  across many Crons is not starved by the watch events it triggers.

Metrics follow the ``workqueue_*`` names.
"""
from __future__ import annotations

import asyncio
import heapq
import itertools
import os
import time
from collections import deque
from typing import Deque, Dict, Hashable, List, Optional, Set, Tuple

from ..runtime import metrics
from ..runtime.ratelimit import RateLimiter, default_controller_rate_limiter
from ..utils.clock import Clock, RealClock, TimerHandle
from ..utils.gotime import NANOS


class ShutDown(Exception):
    pass


_EMPTY = object()  # get(): nothing queued


def _new_core(depth, adds, latency, work):
    """A ``_workqueue.Core`` (``ops/csrc/workqueue.cpp``), or None without the extension or with
    ``CRON_OPERATOR_NATIVE_QUEUE=python``."""
    want = os.environ.get("CRON_OPERATOR_NATIVE_QUEUE", "auto").lower()
    if want == "python":
        return None
    try:
        from ..ops import build as _build

        if _build.needs_build("_workqueue"):
            _build.build_extension("_workqueue")
        from ..ops import _workqueue  # type: ignore[attr-defined]
    except Exception:  # noqa: BLE001 - the Python core remains
        if want == "native":
            raise
        return None
    return _workqueue.Core(depth, adds, latency, work, _EMPTY)


class WorkQueue:
    def __init__(self, name: str = "", clock: Optional[Clock] = None, rate_limiter: Optional[RateLimiter] = None,
                 controller: str = "", native: Optional[bool] = None):
        self.name = name
        self.clock = clock or RealClock()
        self.rate_limiter = rate_limiter or default_controller_rate_limiter()
        self._heap: List[Tuple[int, int, Hashable]] = []
        self._queued: Dict[Hashable, Tuple[int, int]] = {}   # key -> (neg priority, seq) of its live entry
        self._seq = itertools.count()
        self._dirty: Dict[Hashable, int] = {}                 # key -> best requested priority while processing
        self._processing: Set[Hashable] = set()
        self._added_at: Dict[Hashable, float] = {}
        self._started_at: Dict[Hashable, float] = {}
        self._waiters: Deque[asyncio.Future] = deque()
        # delaying
        self._wait_heap: List[Tuple[int, int, Hashable]] = []
        self._wait_when: Dict[Hashable, Tuple[int, int]] = {}  # key -> (when_ns, priority)
        self._timer: Optional[TimerHandle] = None
        self._timer_when: Optional[int] = None
        self._shutdown = False
        lbl = (name, controller or name)
        self._m_depth = metrics.WQ_DEPTH.labels(*lbl)
        self._m_adds = metrics.WQ_ADDS.labels(*lbl)
        self._m_latency = metrics.WQ_LATENCY.labels(*lbl)
        self._m_work = metrics.WQ_WORK.labels(*lbl)
        self._m_retries = metrics.WQ_RETRIES.labels(*lbl)
        self._m_unfinished = metrics.WQ_UNFINISHED.labels(*lbl)
        self._m_longest = metrics.WQ_LONGEST.labels(*lbl)
        self._adds = 0
        self._gets = 0
        # the queueing core (dedupe, parking, priorities, metering) in C++ when built; the
        # Python methods below are its fallback and oracle (CRON_OPERATOR_NATIVE_QUEUE=python)
        self._core = _new_core(self._m_depth, self._m_adds, self._m_latency, self._m_work) \
            if native is not False else None
        if self._core is not None:
            self.add = self._core.add  # type: ignore[method-assign]
            self.done = self._core.done  # type: ignore[method-assign]

    @property
    def adds(self) -> int:
        return self._core.adds if self._core is not None else self._adds

    @property
    def gets(self) -> int:
        return self._core.gets if self._core is not None else self._gets

    # ------------------------------------------------------------------ core queue
    def __len__(self) -> int:
        return len(self._core) if self._core is not None else len(self._queued)

    def _push(self, item: Hashable, priority: int) -> None:
        entry = (-priority, next(self._seq))
        self._queued[item] = entry
        heapq.heappush(self._heap, (entry[0], entry[1], item))
        self._added_at.setdefault(item, time.perf_counter())
        self._m_depth.set(len(self._queued))
        while self._waiters:
            fut = self._waiters.popleft()
            if not fut.done():
                fut.set_result(None)
                break

    def add(self, item: Hashable, priority: int = 0) -> None:
        if self._shutdown:
            return
        cur = self._queued.get(item)
        if cur is not None:
            if -cur[0] < priority:  # raise priority: push a fresher entry, old one goes stale
                self._push(item, priority)
            return  # already dirty: client-go neither queues nor counts it again
        if item in self._processing:
            prev = self._dirty.get(item)
            if prev is None:
                self._adds += 1
                self._m_adds.inc()
            self._dirty[item] = priority if prev is None else max(prev, priority)
            return
        self._adds += 1
        self._m_adds.inc()
        self._push(item, priority)

    async def get(self) -> Hashable:
        """Next key (waits).  Raises :class:`ShutDown` once shut down and drained."""
        core = self._core
        pop = core.pop if core is not None else self._pop
        while True:
            item = pop()
            if item is not _EMPTY:
                return item
            if self._shutdown:
                raise ShutDown()
            fut = asyncio.get_running_loop().create_future()
            if core is not None:
                core.add_waiter(fut)
            else:
                self._waiters.append(fut)
            try:
                await fut
            except asyncio.CancelledError:
                if core is not None:
                    core.remove_waiter(fut)
                elif fut in self._waiters:
                    self._waiters.remove(fut)
                raise

    def _pop(self) -> Hashable:
        """The most urgent queued key, now processing; ``_EMPTY`` when nothing is queued."""
        while self._heap:
            negp, seq, item = heapq.heappop(self._heap)
            live = self._queued.get(item)
            if live is None or live != (negp, seq):
                continue  # stale entry
            del self._queued[item]
            self._processing.add(item)
            now = time.perf_counter()
            t_add = self._added_at.pop(item, now)
            self._m_latency.observe(now - t_add)
            self._started_at[item] = now
            self._m_depth.set(len(self._queued))
            self._gets += 1
            return item
        return _EMPTY

    def done(self, item: Hashable) -> None:
        self._processing.discard(item)
        t0 = self._started_at.pop(item, None)
        if t0 is not None:
            self._m_work.observe(time.perf_counter() - t0)
        prio = self._dirty.pop(item, None)
        if prio is not None:
            self._push(item, prio)

    def shutdown(self) -> None:
        self._shutdown = True
        if self._timer is not None:
            self._timer.cancel()
        if self._core is not None:
            self._core.shutdown()
        while self._waiters:
            fut = self._waiters.popleft()
            if not fut.done():
                fut.set_result(None)

    @property
    def shutting_down(self) -> bool:
        return self._shutdown

    def processing(self) -> int:
        return self._core.processing() if self._core is not None else len(self._processing)

    def idle(self) -> bool:
        """Nothing queued, parked or in flight (delayed items do not count)."""
        if self._core is not None:
            return self._core.idle()
        return not self._queued and not self._processing and not self._dirty

    def update_unfinished_metrics(self) -> None:
        now = time.perf_counter()
        started = self._core.started() if self._core is not None else self._started_at.values()
        ages = [now - t for t in started]
        self._m_unfinished.set(sum(ages))
        self._m_longest.set(max(ages) if ages else 0.0)

    # ------------------------------------------------------------------ delaying
    def add_after(self, item: Hashable, delay_s: float, priority: int = 0) -> None:
        if self._shutdown:
            return
        if delay_s <= 0:
            self.add(item, priority)
            return
        when = self.clock.now_ns() + int(delay_s * NANOS)
        self.add_at(item, when, priority)

    def add_at(self, item: Hashable, when_ns: int, priority: int = 0) -> None:
        if self._shutdown:
            return
        if when_ns <= self.clock.now_ns():
            self.add(item, priority)
            return
        cur = self._wait_when.get(item)
        if cur is not None and cur[0] <= when_ns:
            return
        self._wait_when[item] = (when_ns, priority)
        heapq.heappush(self._wait_heap, (when_ns, next(self._seq), item))
        self._arm()

    def _arm(self) -> None:
        while self._wait_heap:
            when, _, item = self._wait_heap[0]
            cur = self._wait_when.get(item)
            if cur is None or cur[0] != when:
                heapq.heappop(self._wait_heap)
                continue
            break
        if not self._wait_heap:
            return
        when = self._wait_heap[0][0]
        if self._timer is not None and self._timer_when is not None and self._timer_when <= when:
            return
        if self._timer is not None:
            self._timer.cancel()
        self._timer_when = when
        self._timer = self.clock.call_at(when, self._fire)

    def _fire(self) -> None:
        self._timer = None
        self._timer_when = None
        now = self.clock.now_ns()
        while self._wait_heap and self._wait_heap[0][0] <= now:
            when, _, item = heapq.heappop(self._wait_heap)
            cur = self._wait_when.get(item)
            if cur is None or cur[0] != when:
                continue
            del self._wait_when[item]
            self.add(item, cur[1])
        self._arm()

    def waiting(self) -> int:
        return len(self._wait_when)


    # ------------------------------------------------------------------ rate limiting
    def add_rate_limited(self, item: Hashable, priority: int = 0) -> None:
        self._m_retries.inc()
        self.add_after(item, self.rate_limiter.when(item), priority)

    def forget(self, item: Hashable) -> None:
        self.rate_limiter.forget(item)

    def num_requeues(self, item: Hashable) -> int:
        return self.rate_limiter.num_requeues(item)
