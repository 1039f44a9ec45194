"""Rate limiters: the client-side token bucket and the workqueue limiters.

* :class:`TokenBucket` -- ``flowcontrol.NewTokenBucketRateLimiter(qps, burst)``
  that client-go puts in front of every API request; the reference configures
  it with ``--qps 30 --burst 50`` (``cmd/operator/start.go:152-154,218-219``).
  A negative qps disables throttling (client-go semantics).
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
from typing import Dict, Hashable, List, Optional


class TokenBucket:
    def __init__(self, qps: float, burst: int):
        self.qps = float(qps)
        self.burst = max(1, int(burst))
        self._tokens = float(self.burst)
        self._last = time.monotonic()
        self._lock = threading.Lock()
        self.total_wait = 0.0
        self.accepted = 0

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

    async def wait(self) -> float:
        if self.unlimited:
            return 0.0
        if self.qps == 0:
            raise ValueError("qps 0 would block forever")
        d = self._reserve()
        if d > 0:
            self.total_wait += d
            await asyncio.sleep(d)
        return d

    def when(self) -> float:
        """Non-blocking reservation (seconds until the token is due)."""
        if self.unlimited:
            return 0.0
        return self._reserve()


def make_client_limiter(qps: float, burst: int) -> Optional[TokenBucket]:
    """client-go: qps==0 -> default 5/10; qps<0 -> no limiter."""
    if qps == 0:
        qps, burst = 5.0, 10
    if qps < 0:
        return None
    return TokenBucket(qps, burst)


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
