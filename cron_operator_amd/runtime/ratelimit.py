"""Rate limiters: the client-side token bucket and the workqueue limiters.

* :class:`TokenBucket` -- ``flowcontrol.NewTokenBucketRateLimiter(qps, burst)``
  that client-go puts in front of every API request; the reference configures
  it with ``--qps 30 --burst 50`` (``cmd/operator/start.go:152-154,218-219``).
  A negative qps disables throttling (client-go semantics).

  Unlike client-go's bucket (one FIFO of sleepers), a request waiting for a token
  carries a **priority**: when the bucket is backed up, tokens go to
  :data:`PRIORITY_HIGH` waiters first (a tick's CREATE, the lease renewal), then
  :data:`PRIORITY_NORMAL` (reads, informer LIST/WATCH), then :data:`PRIORITY_LOW`
  (writes a reconcile can defer: status PATCHes, history-GC DELETEs, events) -- FIFO
  within a class.  Under throttling a tick's jobs are then created at the full QPS
  instead of sharing it with the bookkeeping writes around them, so schedule->create
  latency is bounded by *creates* per QPS, not by all requests per QPS.  A low waiter
  older than ``max_defer`` seconds is served before everything else, so deferrable
  writes are delayed, never starved.  With no backlog a request takes a token at
  once, whatever its priority, exactly as before -- except that with ``low_reserve``
  a low request leaves that many tokens in the bucket: the operator's client keeps its
  whole burst for the next tick's CREATEs (``--tick-burst-reserve``), and status
  PATCHes / GC DELETEs run at the refill rate instead of draining it just before a tick.
* :class:`ItemExponentialFailureRateLimiter`, :class:`BucketRateLimiter`,
  :class:`MaxOfRateLimiter` -- the workqueue's default controller limiter
  (per-item exponential backoff 5ms..1000s, max'd with an overall 10 qps /
  100 burst bucket) [ext] client-go ``DefaultTypedControllerRateLimiter``.

All of these run on real (monotonic) time, even when schedule time is a
FakeClock: they model request pacing, not schedule semantics.
"""
from __future__ import annotations

import asyncio
import threading
import time
from collections import deque
from typing import Deque, Dict, Hashable, List, Optional, Tuple

PRIORITY_LOW = 0
PRIORITY_NORMAL = 1
PRIORITY_HIGH = 2


class _PriorityWaiters:
    """Three FIFO classes of waiting futures; :meth:`_next` serves the most urgent class, or a
    low waiter older than ``max_defer`` seconds before anything else (delayed, never starved)."""

    def __init__(self, max_defer: float):
        self.max_defer = max_defer
        # waiters per priority class (index = priority): (future, enqueue monotonic time)
        self._waiters: Tuple[Deque[Tuple["asyncio.Future[None]", float]], ...] = (deque(), deque(), deque())
        self._n_waiting = 0
        self.granted_by_priority = [0, 0, 0]
        self.aged_grants = 0  # low-priority grants promoted by max_defer

    @property
    def waiting(self) -> int:
        """Requests queued right now."""
        return self._n_waiting

    def waiting_at(self, priority: int) -> int:
        """Requests of one priority class queued right now (cancelled ones may still count
        until the next grant passes them)."""
        return len(self._waiters[priority])

    def _enqueue(self, priority: int, now: float) -> "asyncio.Future[None]":
        fut = asyncio.get_running_loop().create_future()
        self._waiters[priority].append((fut, now))
        self._n_waiting += 1
        return fut

    def _discard(self, priority: int, fut: "asyncio.Future[None]") -> None:
        q = self._waiters[priority]
        for i, (f, _) in enumerate(q):
            if f is fut:
                del q[i]
                self._n_waiting -= 1
                return

    def _next(self, low_ok: bool = True) -> Optional[Tuple["asyncio.Future[None]", int]]:
        """Pop the waiter to serve: an over-aged low waiter, else the most urgent class
        (``low_ok`` False: a low waiter that is not over-aged is not served now)."""
        low = self._waiters[PRIORITY_LOW]
        if low and time.monotonic() - low[0][1] > self.max_defer:
            self.aged_grants += 1
            self._n_waiting -= 1
            return low.popleft()[0], PRIORITY_LOW
        for p in (PRIORITY_HIGH, PRIORITY_NORMAL, PRIORITY_LOW):
            q = self._waiters[p]
            if q:
                if p == PRIORITY_LOW and not low_ok:
                    return None
                self._n_waiting -= 1
                return q.popleft()[0], p
        return None


class TokenBucket(_PriorityWaiters):
    """``low_reserve``: tokens a :data:`PRIORITY_LOW` request may not spend -- it takes one only
    while at least ``1 + low_reserve`` are left (an over-aged one excepted).  Deferrable writes
    then run at the refill rate without draining the burst, and the next schedule tick finds the
    bucket full for its CREATEs (``-1``: the whole burst, ``burst - 1``)."""

    def __init__(self, qps: float, burst: int, max_defer: float = 20.0, low_reserve: int = 0):
        super().__init__(max_defer)
        self.qps = float(qps)
        self.burst = max(1, int(burst))
        self.low_reserve = self.burst - 1 if low_reserve < 0 else min(int(low_reserve), self.burst - 1)
        self._tokens = float(self.burst)
        self._last = time.monotonic()
        self._lock = threading.Lock()
        self.total_wait = 0.0
        self.max_wait_by_priority = [0.0, 0.0, 0.0]  # the longest wait per priority class (s)
        self.accepted = 0
        self._timer: Optional[asyncio.TimerHandle] = None

    @property
    def unlimited(self) -> bool:
        return self.qps < 0

    def _reserve(self) -> float:
        """Take one token, returning how long the caller must wait for it."""
        with self._lock:
            now = time.monotonic()
            self._tokens = min(float(self.burst), self._tokens + (now - self._last) * self.qps)
            self._last = now
            self._tokens -= 1.0
            self.accepted += 1
            if self._tokens >= 0:
                return 0.0
            return -self._tokens / self.qps

    def try_accept(self) -> bool:
        with self._lock:
            now = time.monotonic()
            self._tokens = min(float(self.burst), self._tokens + (now - self._last) * self.qps)
            self._last = now
            if self._tokens >= 1.0:
                self._tokens -= 1.0
                self.accepted += 1
                return True
            return False

    def _refill(self, now: float) -> None:
        self._tokens = min(float(self.burst), self._tokens + (now - self._last) * self.qps)
        self._last = now

    async def wait(self, priority: int = PRIORITY_NORMAL) -> float:
        """Take one token, waiting for it if the bucket is empty; returns the wait in seconds."""
        if self.unlimited:
            return 0.0
        if self.qps == 0:
            raise ValueError("qps 0 would block forever")
        now = time.monotonic()
        w = self._waiters
        if priority == PRIORITY_LOW:
            fast, need = not self._n_waiting, 1.0 + self.low_reserve
        else:  # only waiters of its own class or a more urgent one go first (held low ones do not)
            fast = not w[PRIORITY_HIGH] and (priority == PRIORITY_HIGH or not w[PRIORITY_NORMAL])
            need = 1.0
        if fast:
            with self._lock:
                self._refill(now)
                if self._tokens >= need:
                    self._tokens -= 1.0
                    self.accepted += 1
                    self.granted_by_priority[priority] += 1
                    return 0.0
        loop = asyncio.get_running_loop()
        fut = self._enqueue(priority, now)
        if priority != PRIORITY_LOW and self._timer is not None:
            # the armed grant may be timed for held low waiters (the reserve refilled): re-time it
            self._timer.cancel()
            self._timer = None
        self._arm(loop)
        try:
            await fut
        except asyncio.CancelledError:
            if not fut.done() or fut.cancelled():
                self._discard(priority, fut)
            else:  # granted and cancelled in the same turn: hand the token back
                with self._lock:
                    self._tokens += 1.0
                    self.accepted -= 1
                self._arm(loop)
            raise
        d = time.monotonic() - now
        self.total_wait += d
        if d > self.max_wait_by_priority[priority]:
            self.max_wait_by_priority[priority] = d
        return d

    def _arm(self, loop: asyncio.AbstractEventLoop) -> None:
        """Schedule the next grant for when a token is due (one timer for all waiters)."""
        if self._timer is not None or not self._n_waiting:
            return
        with self._lock:
            now = time.monotonic()
            self._refill(now)
            w = self._waiters
            need = 1.0
            if not w[PRIORITY_HIGH] and not w[PRIORITY_NORMAL]:
                need += self.low_reserve  # only low waiters: due when the reserve is refilled ...
            delay = max(0.0, (need - self._tokens) / self.qps)
            low = w[PRIORITY_LOW]
            if need > 1.0 and low:
                # ... or when the oldest of them is over-aged (it may spend the reserve then)
                aged_at = max(0.0, low[0][1] + self.max_defer - now) + 1e-4
                delay = min(delay, max(aged_at, (1.0 - self._tokens) / self.qps))
        self._timer = loop.call_later(delay, self._grant, loop)

    def _grant(self, loop: asyncio.AbstractEventLoop) -> None:
        self._timer = None
        with self._lock:
            self._refill(time.monotonic())
            while self._tokens >= 1.0 and self._n_waiting:
                nxt = self._next(self._tokens >= 1.0 + self.low_reserve)
                if nxt is None:
                    break
                fut, p = nxt
                if fut.done():  # cancelled while queued
                    continue
                self._tokens -= 1.0
                self.accepted += 1
                self.granted_by_priority[p] += 1
                fut.set_result(None)
        self._arm(loop)

    def when(self) -> float:
        """Non-blocking reservation (seconds until the token is due)."""
        if self.unlimited:
            return 0.0
        return self._reserve()


class InflightGate(_PriorityWaiters):
    """At most ``limit`` requests in flight; the rest wait in priority order (the client's
    cap on concurrent API requests -- deferred reconcile tails can have many writes ready at
    once, and an HTTP/1.1 pool would otherwise open one connection per request)."""

    def __init__(self, limit: int, max_defer: float = 20.0):
        super().__init__(max_defer)
        self.limit = max(1, int(limit))
        self.inflight = 0
        self.peak = 0

    async def acquire(self, priority: int = PRIORITY_NORMAL) -> None:
        if self.inflight < self.limit and not self._n_waiting:
            self.inflight += 1
            self.granted_by_priority[priority] += 1
            if self.inflight > self.peak:
                self.peak = self.inflight
            return
        fut = self._enqueue(priority, time.monotonic())
        try:
            await fut
        except asyncio.CancelledError:
            if fut.done() and not fut.cancelled():
                self.release()  # granted and cancelled in the same turn: pass the slot on
            else:
                self._discard(priority, fut)
            raise

    def release(self) -> None:
        self.inflight -= 1
        while self._n_waiting and self.inflight < self.limit:
            nxt = self._next()
            if nxt is None:
                break
            fut, p = nxt
            if fut.done():  # cancelled while queued
                continue
            self.inflight += 1
            self.granted_by_priority[p] += 1
            if self.inflight > self.peak:
                self.peak = self.inflight
            fut.set_result(None)


def make_client_limiter(qps: float, burst: int, max_defer: float = 20.0,
                        low_reserve: int = 0) -> Optional[TokenBucket]:
    """client-go: qps==0 -> default 5/10; qps<0 -> no limiter."""
    if qps == 0:
        qps, burst = 5.0, 10
    if qps < 0:
        return None
    return TokenBucket(qps, burst, max_defer, low_reserve)


# --------------------------------------------------------------------------- workqueue limiters


class RateLimiter:
    def when(self, item: Hashable) -> float:
        raise NotImplementedError

    def forget(self, item: Hashable) -> None:
        raise NotImplementedError

    def num_requeues(self, item: Hashable) -> int:
        raise NotImplementedError


class ItemExponentialFailureRateLimiter(RateLimiter):
    def __init__(self, base_delay: float = 0.005, max_delay: float = 1000.0):
        self.base = base_delay
        self.max = max_delay
        self._failures: Dict[Hashable, int] = {}

    def when(self, item: Hashable) -> float:
        exp = self._failures.get(item, 0)
        self._failures[item] = exp + 1
        if exp > 62:
            return self.max
        return min(self.base * (2 ** exp), self.max)

    def forget(self, item: Hashable) -> None:
        self._failures.pop(item, None)

    def num_requeues(self, item: Hashable) -> int:
        return self._failures.get(item, 0)


class BucketRateLimiter(RateLimiter):
    def __init__(self, qps: float = 10.0, burst: int = 100):
        self.bucket = TokenBucket(qps, burst)

    def when(self, item: Hashable) -> float:
        return self.bucket.when()

    def forget(self, item: Hashable) -> None:
        pass

    def num_requeues(self, item: Hashable) -> int:
        return 0


class MaxOfRateLimiter(RateLimiter):
    def __init__(self, *limiters: RateLimiter):
        self.limiters: List[RateLimiter] = list(limiters)

    def when(self, item: Hashable) -> float:
        return max(lim.when(item) for lim in self.limiters)

    def forget(self, item: Hashable) -> None:
        for lim in self.limiters:
            lim.forget(item)

    def num_requeues(self, item: Hashable) -> int:
        return max(lim.num_requeues(item) for lim in self.limiters)


def default_controller_rate_limiter() -> RateLimiter:
    return MaxOfRateLimiter(ItemExponentialFailureRateLimiter(0.005, 1000.0), BucketRateLimiter(10.0, 100))
