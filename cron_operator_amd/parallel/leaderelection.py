"""Lease-based leader election (``coordination.k8s.io/v1`` Lease).

The reference enables leader election with ID ``619a52b8.kubedl.io``
(``cmd/operator/start.go:160-162``; on by default in the chart,
``charts/cron-operator/values.yaml:57-59``), using controller-runtime's defaults
[ext]: lease duration 15s, renew deadline 10s, retry period 2s, no release on
cancel.  Only the leader runs informers and workers; losing the lease ends the
process (controller-runtime exits with "leader election lost").

The algorithm is client-go's ``tryAcquireOrRenew``: create the Lease if absent;
take it over when ``leaseDurationSeconds`` have passed *on the local clock* since
the record was last seen to change (bumping ``leaseTransitions`` and
``acquireTime``); renew by updating ``renewTime`` with optimistic concurrency,
each renewal window bounded by ``renewDeadline``.  All timing goes through the
injected clock so fail-over, clock skew and hung requests are testable in
virtual time.
"""
from __future__ import annotations

import asyncio
import os
import random
import socket
import uuid
from typing import Any, Awaitable, Callable, Dict, Optional

from ..api import errors
from ..api.meta import GroupVersionResource
from ..runtime import metrics
from ..runtime.ratelimit import PRIORITY_HIGH
from ..utils import aio, jsonutil
from ..utils.clock import Clock, RealClock
from ..utils.gotime import NANOS, UTC, GoTime, parse_rfc3339
from ..utils.logging import get_logger

LEASES = GroupVersionResource("coordination.k8s.io", "v1", "leases")
JITTER_FACTOR = 1.2  # client-go leaderelection.JitterFactor


def default_identity() -> str:
    return f"{socket.gethostname()}_{uuid.uuid4()}"


def _micro(t_ns: int) -> str:
    g = GoTime(t_ns // NANOS, t_ns % NANOS, UTC)
    base = g.rfc3339()[:-1]
    return f"{base}.{(t_ns % NANOS) // 1000:06d}Z"


def _parse_micro(s: Optional[str]) -> Optional[int]:
    if not s:
        return None
    t = parse_rfc3339(s)
    return t.sec * NANOS + t.nsec


def in_cluster_namespace() -> str:
    """Namespace for the lease: $POD_NAMESPACE, the SA namespace file, else "default"."""
    ns = os.environ.get("POD_NAMESPACE")
    if ns:
        return ns
    try:
        with open("/var/run/secrets/kubernetes.io/serviceaccount/namespace") as fh:
            return fh.read().strip() or "default"
    except OSError:
        return "default"


class LeaderElector:
    """client-go's ``LeaderElector`` semantics on a Lease lock.

    * **Expiry is judged from local observation**, never from the holder's clock:
      ``observed_time`` is this process's clock reading when it last saw the lease
      record *change*; another holder's lease counts as valid until
      ``observed_time + leaseDurationSeconds``.  A follower whose clock runs ahead
      therefore cannot steal a lease that is still being renewed.
    * **Every renewal window is bounded by ``renew_deadline``** (client-go wraps it in
      ``context.WithTimeout(RenewDeadline)``): attempts inside the window, including
      an in-flight GET/PUT, are cancelled when it closes, and the elector steps down.
    * The leader renews optimistically with its cached lease object (one PUT), and
      falls back to GET + PUT when that fails.
    """

    def __init__(self, client, name: str, namespace: str, identity: Optional[str] = None,
                 clock: Optional[Clock] = None, lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, release_on_cancel: bool = False):
        if lease_duration <= renew_deadline:
            raise ValueError("leaseDuration must be greater than renewDeadline")
        if renew_deadline <= retry_period * JITTER_FACTOR:
            raise ValueError("renewDeadline must be greater than retryPeriod*JitterFactor")
        self.client = client
        self.name = name
        self.namespace = namespace
        self.identity = identity or default_identity()
        self.clock = clock or RealClock()
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.release_on_cancel = release_on_cancel
        self.is_leader = False
        self.elected = asyncio.Event()
        self.lost = asyncio.Event()
        self.observed_holder: Optional[str] = None
        # the last lease record seen (spec), the local time it was seen to change, and the
        # lease object it came from (carries the resourceVersion for optimistic renewals)
        self.observed_spec: Optional[Dict[str, Any]] = None
        self.observed_time_ns = 0
        self._lease: Optional[Dict[str, Any]] = None
        # the longest successful renewal window so far (injected clock, seconds): a renewal that
        # waits behind other traffic shows here long before it reaches renew_deadline
        self.max_renew_s = 0.0
        self._m = metrics.LEADER_STATUS.labels(name)
        self.log = get_logger("leaderelection").with_values(lease=f"{namespace}/{name}", identity=self.identity)

    # ------------------------------------------------------------------ observed record
    def _observe(self, spec: Dict[str, Any], lease: Optional[Dict[str, Any]]) -> None:
        self.observed_spec = dict(spec)
        self.observed_time_ns = self.clock.now_ns()
        self.observed_holder = spec.get("holderIdentity") or ""
        self._lease = lease

    def holds_lease(self) -> bool:
        """``IsLeader``: the last observed record names this identity."""
        return self.observed_spec is not None and self.observed_spec.get("holderIdentity") == self.identity

    def _lease_valid(self, now_ns: int) -> bool:
        if self.observed_spec is None:
            return False
        dur = int(self.observed_spec.get("leaseDurationSeconds") or self.lease_duration)
        return self.observed_time_ns + dur * NANOS > now_ns

    def _record(self, now_ns: int, acquire: Optional[str], transitions: int) -> Dict[str, Any]:
        return {"holderIdentity": self.identity, "leaseDurationSeconds": int(self.lease_duration),
                "acquireTime": acquire or _micro(now_ns), "renewTime": _micro(now_ns),
                "leaseTransitions": transitions}

    async def _put(self, lease: Dict[str, Any], spec: Dict[str, Any]) -> bool:
        body = dict(lease)
        body["spec"] = spec
        try:
            updated = await self.client.update(LEASES, body, priority=PRIORITY_HIGH)
        except errors.ApiError as e:
            self.log.v(1).info("lease update failed", error=str(e))
            return False
        self._observe(spec, updated if isinstance(updated, dict) else body)
        return True

    # ------------------------------------------------------------------ tryAcquireOrRenew
    async def try_acquire_or_renew(self) -> bool:
        now = self.clock.now_ns()
        # 1. fast path: the leader renews its cached lease object with one PUT
        if self.holds_lease() and self._lease_valid(now) and self._lease is not None:
            old = self.observed_spec or {}
            if await self._put(self._lease, self._record(now, old.get("acquireTime"),
                                                         int(old.get("leaseTransitions") or 0))):
                return True
            self.log.v(1).info("optimistic lease renewal failed, falling back to GET")
        # 2. read (or create) the lease
        try:
            lease = await self.client.get(LEASES, self.namespace, self.name, priority=PRIORITY_HIGH)
        except errors.ApiError as e:
            if not errors.is_not_found(e):
                self.log.error(e, "error retrieving resource lock")
                return False
            spec = self._record(now, None, 0)
            body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                    "metadata": {"name": self.name, "namespace": self.namespace}, "spec": spec}
            try:
                created = await self.client.create(LEASES, body, self.namespace, priority=PRIORITY_HIGH)
            except errors.ApiError as ce:
                self.log.v(1).info("lease create lost the race", error=str(ce))
                return False
            self._observe(spec, created if isinstance(created, dict) else body)
            return True
        spec = lease.get("spec") or {}
        # 3. a changed record restarts the local expiry clock
        if self.observed_spec is None or not jsonutil.json_equal(spec, self.observed_spec):
            self._observe(spec, lease)
        else:
            self._lease = lease
        if (spec.get("holderIdentity") or "") and self._lease_valid(now) and not self.holds_lease():
            return False
        # 4. take over or renew
        if self.holds_lease():
            new_spec = self._record(now, spec.get("acquireTime"), int(spec.get("leaseTransitions") or 0))
        else:
            new_spec = self._record(now, None, int(spec.get("leaseTransitions") or 0) + 1)
        return await self._put(lease, new_spec)

    async def _try_until(self, deadline_ns: int) -> bool:
        """One ``tryAcquireOrRenew`` cancelled at ``deadline_ns`` on the injected clock."""
        if self.clock.now_ns() >= deadline_ns:
            return False
        loop = asyncio.get_running_loop()
        task = loop.create_task(self.try_acquire_or_renew())
        expired = loop.create_future()

        def _expire() -> None:
            if not expired.done():
                expired.set_result(None)

        timer = self.clock.call_at(deadline_ns, _expire)
        try:
            await asyncio.wait({task, expired}, return_when=asyncio.FIRST_COMPLETED)
        finally:
            timer.cancel()
        if task.done():
            return bool(task.result()) if not task.cancelled() and task.exception() is None else False
        await aio.cancel_and_wait(task)
        return False

    def _jitter(self, d: float) -> float:
        return d * (1.0 + JITTER_FACTOR * random.random())

    async def acquire(self) -> None:
        """``acquire``: retry every ``retryPeriod`` (jittered by 1.2) until elected."""
        self.log.info("attempting to acquire leader lease")
        while True:
            if await self._try_until(self.clock.now_ns() + int(self.renew_deadline * NANOS)):
                self.is_leader = True
                self._m.set(1)
                self.elected.set()
                self.log.info("successfully acquired lease")
                return
            await self.clock.sleep(self._jitter(self.retry_period))

    async def renew_once(self) -> bool:
        """One renewal window: try now, then every ``retryPeriod``, all of it (in-flight
        requests included) bounded by ``renewDeadline``."""
        t0 = self.clock.now_ns()
        deadline = t0 + int(self.renew_deadline * NANOS)
        while True:
            if await self._try_until(deadline):
                took = (self.clock.now_ns() - t0) / NANOS
                if took > self.max_renew_s:
                    self.max_renew_s = took
                if took > self.retry_period:
                    self.log.info("slow lease renewal", seconds=round(took, 3),
                                  renewDeadline=self.renew_deadline)
                return True
            if self.clock.now_ns() >= deadline:
                return False
            await self._sleep_until(min(deadline, self.clock.now_ns() + int(self.retry_period * NANOS)))
            if self.clock.now_ns() >= deadline:
                return False

    async def _sleep_until(self, when_ns: int) -> None:
        await self.clock.sleep(max(0, when_ns - self.clock.now_ns()) / NANOS)

    async def renew_loop(self) -> None:
        """Renew every ``retryPeriod`` until a renewal window closes without success."""
        while True:
            if not await self.renew_once():
                self.is_leader = False
                self._m.set(0)
                self.lost.set()
                self.log.info("failed to renew lease", reason="renew deadline exceeded")
                return
            await self.clock.sleep(self.retry_period)

    async def release(self) -> None:
        if not self.is_leader:
            return
        try:
            lease = await self.client.get(LEASES, self.namespace, self.name, priority=PRIORITY_HIGH)
            spec = lease.get("spec") or {}
            if spec.get("holderIdentity") != self.identity:
                return
            now = self.clock.now_ns()
            spec.update({"holderIdentity": "", "leaseDurationSeconds": 1, "renewTime": _micro(now),
                         "acquireTime": _micro(now)})
            await self.client.update(LEASES, lease, priority=PRIORITY_HIGH)
        except errors.ApiError as e:
            self.log.error(e, "failed to release lease")
        self.is_leader = False
        self._m.set(0)

    async def run(self, on_started: Callable[[], Awaitable[None]], on_stopped: Callable[[], None]) -> None:
        """Campaign, then lead: ``on_started`` runs *concurrently* with the renewals (client-go
        starts ``OnStartedLeading`` in its own goroutine), so a slow cache sync cannot let
        the lease lapse; losing the lease cancels it."""
        started: Optional[asyncio.Task] = None
        try:
            await self.acquire()
            started = asyncio.get_running_loop().create_task(on_started())
            renew = asyncio.get_running_loop().create_task(self.renew_loop())
            try:
                done, _ = await asyncio.wait({started, renew}, return_when=asyncio.FIRST_COMPLETED)
                if started in done and started.exception() is not None:
                    raise started.exception()  # type: ignore[misc]
                await renew
            finally:
                # wait for an in-flight renewal PUT to end before release() writes the lease
                await aio.cancel_and_wait(renew)
            on_stopped()
        except asyncio.CancelledError:
            if self.release_on_cancel:
                await self.release()
            raise
        finally:
            if started is not None and not started.done():
                await aio.cancel_and_wait(started)
