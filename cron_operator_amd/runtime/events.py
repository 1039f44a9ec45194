"""Event recorder: broadcaster, correlation (count aggregation) and spam filter.

The reference emits four Event reasons through ``mgr.GetEventRecorderFor("cron")``
(``cmd/operator/start.go:187``): ``Deadline`` (Normal),
``FailedCreate`` (Warning), ``OverridePolicy`` (Normal) and
``TooManyMissedTimes`` (Warning).  client-go's recorder [ext] writes core/v1
Events asynchronously, folds repeats of the same (object, type, reason,
message) into one Event whose ``count``/``lastTimestamp`` are PATCHed, and
drops bursts from a single object with a token bucket (25 burst, 1 per 5
minutes).  This module does the same; recording never blocks a reconcile.

The reference's unit tests pass ``recorder=nil`` and would panic on any event
path; :class:`FakeRecorder` records into a list instead.
"""
from __future__ import annotations

import asyncio
import time
from collections import OrderedDict
from typing import Any, Dict, List, Optional, Tuple

from ..api import errors
from ..api.meta import GroupVersionResource
from ..utils import aio
from ..utils.clock import Clock, RealClock
from ..utils.gotime import GoTime, UTC
from ..utils.logging import get_logger
from .client import Client
from .ratelimit import PRIORITY_LOW, TokenBucket

EVENTS_GVR = GroupVersionResource("", "v1", "events")

Normal = "Normal"
Warning = "Warning"


def _involved(obj: Dict[str, Any]) -> Dict[str, Any]:
    m = obj.get("metadata") or {}
    ref = {"kind": obj.get("kind", ""), "namespace": m.get("namespace", ""), "name": m.get("name", ""),
           "uid": m.get("uid", ""), "apiVersion": obj.get("apiVersion", ""),
           "resourceVersion": m.get("resourceVersion", "")}
    return {k: v for k, v in ref.items() if v}


class EventRecorder:
    """``record.EventRecorder``: ``event`` / ``eventf``."""

    def event(self, obj: Dict[str, Any], etype: str, reason: str, message: str) -> None:
        raise NotImplementedError

    def eventf(self, obj: Dict[str, Any], etype: str, reason: str, fmt: str, *args: Any) -> None:
        self.event(obj, etype, reason, fmt % args if args else fmt)


class FakeRecorder(EventRecorder):
    """In-memory recorder for tests (``record.FakeRecorder``)."""

    def __init__(self):
        self.events: List[Tuple[str, str, str, str]] = []  # (key, type, reason, message)

    def event(self, obj: Dict[str, Any], etype: str, reason: str, message: str) -> None:
        m = obj.get("metadata") or {}
        self.events.append((f"{m.get('namespace', '')}/{m.get('name', '')}", etype, reason, message))

    def reasons(self) -> List[str]:
        return [e[2] for e in self.events]


class Broadcaster:
    """Queues events and writes them to the API with correlation."""

    def __init__(self, client: Client, clock: Optional[Clock] = None, queue_size: int = 1000,
                 spam_burst: int = 25, spam_qps: float = 1.0 / 300.0, cache_size: int = 4096):
        self.client = client
        self.clock = clock or RealClock()
        self._q: "asyncio.Queue[Tuple[str, Dict[str, Any], str, str, str]]" = asyncio.Queue(queue_size)
        self._task: Optional[asyncio.Task] = None
        self._seen: "OrderedDict[Tuple, Tuple[str, str, int]]" = OrderedDict()  # key -> (ns, name, count)
        self._spam: "OrderedDict[Tuple, TokenBucket]" = OrderedDict()
        self._spam_burst = spam_burst
        self._spam_qps = spam_qps
        self._cache_size = cache_size
        self.dropped = 0
        self.written = 0
        self.log = get_logger("events")

    def recorder_for(self, component: str) -> "Recorder":
        return Recorder(self, component)

    def enqueue(self, component: str, obj: Dict[str, Any], etype: str, reason: str, message: str) -> None:
        try:
            self._q.put_nowait((component, obj, etype, reason, message))
        except asyncio.QueueFull:
            self.dropped += 1

    def start(self) -> None:
        if self._task is None:
            self._task = asyncio.get_running_loop().create_task(self._run(), name="event-broadcaster")

    async def stop(self, drain: bool = True) -> None:
        if drain:
            await self.flush(timeout=2.0)
        if self._task is not None:
            task, self._task = self._task, None
            await aio.cancel_and_wait(task)

    async def flush(self, timeout: float = 5.0) -> None:
        deadline = time.monotonic() + timeout
        while not self._q.empty() and time.monotonic() < deadline:
            await asyncio.sleep(0.005)
        if self._task is not None:
            await asyncio.sleep(0)

    def _ts(self) -> str:
        return GoTime(self.clock.now_ns() // 1_000_000_000, 0, UTC).rfc3339()

    async def _run(self) -> None:
        while True:
            item = await self._q.get()
            try:
                await self._write(*item)
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001 - events are best effort
                self.log.v(2).info("unable to write event", error=str(e))

    def _spam_ok(self, key: Tuple) -> bool:
        b = self._spam.get(key)
        if b is None:
            b = TokenBucket(self._spam_qps, self._spam_burst)
            self._spam[key] = b
            if len(self._spam) > self._cache_size:
                self._spam.popitem(last=False)
        return b.try_accept()

    async def _write(self, component: str, obj: Dict[str, Any], etype: str, reason: str, message: str) -> None:
        inv = _involved(obj)
        ns = inv.get("namespace") or "default"
        src_key = (component, inv.get("kind"), ns, inv.get("name"), inv.get("uid"))
        if not self._spam_ok(src_key):
            self.dropped += 1
            return
        key = src_key + (etype, reason, message)
        now = self._ts()
        seen = self._seen.get(key)
        if seen is not None:
            ens, ename, count = seen
            try:
                await self.client.patch(EVENTS_GVR, ens, ename, {"count": count + 1, "lastTimestamp": now},
                                        priority=PRIORITY_LOW)
                self._seen[key] = (ens, ename, count + 1)
                self._seen.move_to_end(key)
                self.written += 1
                return
            except errors.ApiError as e:
                if not errors.is_not_found(e):
                    raise
                del self._seen[key]
        name = f"{inv.get('name', 'unknown')}.{time.time_ns():x}"
        ev = {"apiVersion": "v1", "kind": "Event",
              "metadata": {"name": name, "namespace": ns},
              "involvedObject": inv, "reason": reason, "message": message, "type": etype,
              "source": {"component": component}, "firstTimestamp": now, "lastTimestamp": now, "count": 1,
              "reportingComponent": component, "reportingInstance": ""}
        await self.client.create(EVENTS_GVR, ev, ns, priority=PRIORITY_LOW)  # yields to a tick's CREATEs
        self.written += 1
        self._seen[key] = (ns, name, 1)
        if len(self._seen) > self._cache_size:
            self._seen.popitem(last=False)


class Recorder(EventRecorder):
    def __init__(self, broadcaster: Broadcaster, component: str):
        self.broadcaster = broadcaster
        self.component = component

    def event(self, obj: Dict[str, Any], etype: str, reason: str, message: str) -> None:
        if etype not in (Normal, Warning):
            raise ValueError(f"unsupported event type: {etype!r}")
        self.broadcaster.enqueue(self.component, obj, etype, reason, message)
