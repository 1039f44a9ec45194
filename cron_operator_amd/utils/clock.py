"""Injectable clocks.

The reference reads wall time directly (``time.Now()`` at
``internal/controller/cron_controller.go:160``) and relies on controller-runtime
timers for ``RequeueAfter``; its tests can only steer time through
``getNextSchedule(ctx, cron, now)`` (``cron_controller_test.go:164``).  Every
time-dependent piece of this framework (reconciler, workqueue delays, leader
election, fake apiserver timestamps, fake training-operator) takes a
:class:`Clock` instead, so tests and the benchmark can run minutes of schedule
time in milliseconds.

``call_at`` is the only timer primitive; it is driven by the asyncio loop for
:class:`RealClock` and by :meth:`FakeClock.advance` / :meth:`FakeClock.set` for
:class:`FakeClock`.
"""
from __future__ import annotations

import asyncio
import heapq
import itertools
import time
from typing import Callable, List, Optional, Tuple

from .gotime import LOCAL, NANOS, GoTime, Location


class TimerHandle:
    __slots__ = ("when", "cb", "cancelled", "_h")

    def __init__(self, when: int, cb: Callable[[], None]):
        self.when = when
        self.cb = cb
        self.cancelled = False
        self._h = None

    def cancel(self) -> None:
        self.cancelled = True
        if self._h is not None:
            self._h.cancel()


class Clock:
    """Abstract clock: nanoseconds since the Unix epoch."""

    def now_ns(self) -> int:
        raise NotImplementedError

    def now(self, loc: Location = LOCAL) -> GoTime:
        return GoTime.from_unix_nano(self.now_ns(), loc)

    def monotonic(self) -> float:
        """Seconds, for measuring durations (wall-clock even for FakeClock)."""
        return time.perf_counter()

    def call_at(self, when_ns: int, cb: Callable[[], None]) -> TimerHandle:
        raise NotImplementedError

    def call_later(self, delay_ns: int, cb: Callable[[], None]) -> TimerHandle:
        return self.call_at(self.now_ns() + max(0, delay_ns), cb)

    async def sleep(self, seconds: float) -> None:
        if seconds <= 0:
            await asyncio.sleep(0)
            return
        fut = asyncio.get_running_loop().create_future()

        def _wake() -> None:
            if not fut.done():
                fut.set_result(None)

        h = self.call_later(int(seconds * NANOS), _wake)
        try:
            await fut
        finally:
            h.cancel()


class RealClock(Clock):
    def now_ns(self) -> int:
        return time.time_ns()

    def call_at(self, when_ns: int, cb: Callable[[], None]) -> TimerHandle:
        h = TimerHandle(when_ns, cb)
        loop = asyncio.get_running_loop()
        delay = max(0.0, (when_ns - time.time_ns()) / NANOS)

        def _fire() -> None:
            if not h.cancelled:
                cb()

        h._h = loop.call_later(delay, _fire)
        return h

    async def sleep(self, seconds: float) -> None:
        await asyncio.sleep(max(0.0, seconds))


class FakeClock(Clock):
    """Manually advanced clock.  Timers fire synchronously inside :meth:`advance`."""

    def __init__(self, start_ns: Optional[int] = None):
        self._now = time.time_ns() if start_ns is None else start_ns
        self._heap: List[Tuple[int, int, TimerHandle]] = []
        self._seq = itertools.count()

    def now_ns(self) -> int:
        return self._now

    def call_at(self, when_ns: int, cb: Callable[[], None]) -> TimerHandle:
        h = TimerHandle(when_ns, cb)
        heapq.heappush(self._heap, (when_ns, next(self._seq), h))
        return h

    def pending(self) -> int:
        return sum(1 for _, _, h in self._heap if not h.cancelled)


    def set(self, t_ns: int) -> int:
        """Move time to ``t_ns`` (never backwards) and fire due timers in order."""
        fired = 0
        target = max(t_ns, self._now)
        while self._heap and self._heap[0][0] <= target:
            when, _, h = heapq.heappop(self._heap)
            if h.cancelled:
                continue
            self._now = max(self._now, when)
            h.cb()
            fired += 1
        self._now = target
        return fired

    def advance(self, seconds: float) -> int:
        return self.set(self._now + int(seconds * NANOS))

    def step(self, ns: int) -> int:
        return self.set(self._now + ns)

    async def sleep(self, seconds: float) -> None:
        # virtual sleep: resolves when someone advances the clock far enough
        await Clock.sleep(self, seconds)


_default_clock: Clock = RealClock()


