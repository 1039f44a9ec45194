"""Lease-based leader election (``coordination.k8s.io/v1`` Lease).

The reference enables leader election with ID ``619a52b8.kubedl.io``
(``cmd/operator/start.go:160-162``; on by default in the chart,
``charts/cron-operator/values.yaml:57-59``), using controller-runtime's defaults
[ext]: lease duration 15s, renew deadline 10s, retry period 2s, no release on
cancel.  Only the leader runs informers and workers; losing the lease ends the
process (controller-runtime exits with "leader election lost").

The algorithm is client-go's ``tryAcquireOrRenew``: create the Lease if absent;
take it over when the holder's ``renewTime + leaseDurationSeconds`` has passed
(bumping ``leaseTransitions`` and ``acquireTime``); renew by updating
``renewTime`` with optimistic concurrency.  All timing goes through the
injected clock so fail-over is testable in virtual time.
"""
from __future__ import annotations

import asyncio
import os
import random
import socket
import uuid
from typing import Awaitable, Callable, Optional

from ..api import errors
from ..api.meta import GroupVersionResource
from ..runtime import metrics
from ..utils.clock import Clock, RealClock
from ..utils.gotime import NANOS, UTC, GoTime, parse_rfc3339
from ..utils.logging import get_logger

LEASES = GroupVersionResource("coordination.k8s.io", "v1", "leases")


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
    def __init__(self, client, name: str, namespace: str, identity: Optional[str] = None,
                 clock: Optional[Clock] = None, lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, release_on_cancel: bool = False):
        if lease_duration <= renew_deadline:
            raise ValueError("leaseDuration must be greater than renewDeadline")
        if renew_deadline <= retry_period * 1.2:
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
        self._m = metrics.LEADER_STATUS.labels(name)
        self.log = get_logger("leaderelection").with_values(lease=f"{namespace}/{name}", identity=self.identity)

    async def try_acquire_or_renew(self) -> bool:
        now = self.clock.now_ns()
        try:
            lease = await self.client.get(LEASES, self.namespace, self.name)
        except errors.ApiError as e:
            if not errors.is_not_found(e):
                self.log.error(e, "error retrieving resource lock")
                return False
            body = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                    "metadata": {"name": self.name, "namespace": self.namespace},
                    "spec": {"holderIdentity": self.identity, "leaseDurationSeconds": int(self.lease_duration),
                             "acquireTime": _micro(now), "renewTime": _micro(now), "leaseTransitions": 0}}
            try:
                await self.client.create(LEASES, body, self.namespace)
            except errors.ApiError as ce:
                self.log.v(1).info("lease create lost the race", error=str(ce))
                return False
            self.observed_holder = self.identity
            return True
        spec = lease.get("spec") or {}
        holder = spec.get("holderIdentity") or ""
        self.observed_holder = holder
        renew = _parse_micro(spec.get("renewTime")) or 0
        dur = int(spec.get("leaseDurationSeconds") or self.lease_duration)
        if holder and holder != self.identity and renew + dur * NANOS > now:
            return False
        new_spec = dict(spec)
        if holder != self.identity:
            new_spec["acquireTime"] = _micro(now)
            new_spec["leaseTransitions"] = int(spec.get("leaseTransitions") or 0) + (1 if holder else 0)
        new_spec["holderIdentity"] = self.identity
        new_spec["leaseDurationSeconds"] = int(self.lease_duration)
        new_spec["renewTime"] = _micro(now)
        lease["spec"] = new_spec
        try:
            await self.client.update(LEASES, lease)
        except errors.ApiError as e:
            self.log.v(1).info("lease update failed", error=str(e))
            return False
        self.observed_holder = self.identity
        return True

    def _jitter(self, d: float) -> float:
        return d * (1.0 + 0.2 * random.random())

    async def acquire(self) -> None:
        self.log.info("attempting to acquire leader lease")
        while True:
            if await self.try_acquire_or_renew():
                self.is_leader = True
                self._m.set(1)
                self.elected.set()
                self.log.info("successfully acquired lease")
                return
            await self.clock.sleep(self._jitter(self.retry_period))

    async def renew_loop(self) -> None:
        """Renew until a renewal cannot be completed within ``renew_deadline``."""
        while True:
            await self.clock.sleep(self.retry_period)
            start = self.clock.now_ns()
            ok = False
            while self.clock.now_ns() - start < self.renew_deadline * NANOS:
                if await self.try_acquire_or_renew():
                    ok = True
                    break
                await self.clock.sleep(self.retry_period)
            if not ok:
                self.is_leader = False
                self._m.set(0)
                self.lost.set()
                self.log.info("failed to renew lease", reason="renew deadline exceeded")
                return

    async def release(self) -> None:
        if not self.is_leader:
            return
        try:
            lease = await self.client.get(LEASES, self.namespace, self.name)
            spec = lease.get("spec") or {}
            if spec.get("holderIdentity") != self.identity:
                return
            now = self.clock.now_ns()
            spec.update({"holderIdentity": "", "leaseDurationSeconds": 1, "renewTime": _micro(now),
                         "acquireTime": _micro(now)})
            await self.client.update(LEASES, lease)
        except errors.ApiError as e:
            self.log.error(e, "failed to release lease")
        self.is_leader = False
        self._m.set(0)

    async def run(self, on_started: Callable[[], Awaitable[None]], on_stopped: Callable[[], None]) -> None:
        try:
            await self.acquire()
            await on_started()
            await self.renew_loop()
            on_stopped()
        except asyncio.CancelledError:
            if self.release_on_cancel:
                await self.release()
            raise
