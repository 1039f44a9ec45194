"""Controller: watches -> work queue -> N reconcile workers.

Equivalent of ``ctrl.NewControllerManagedBy(mgr).For(&Cron{}).Owns(...)``
(``internal/controller/cron_controller.go:70-77``) plus the controller-runtime
worker loop it drives [ext]:

* ``for_(gvk)`` enqueues the object's own key on add/update/delete;
* ``owns(gvk)`` maps a child event to its *controller* owner of the For kind;
* ``watches(gvk, map_fn)`` is the generic map-function source;
* predicates filter events before they reach the queue;
* result handling matches controller-runtime: error -> rate-limited requeue
  (``result=error``), ``requeue_after`` -> forget + delayed add
  (``requeue_after``), ``requeue`` -> rate-limited (``requeue``), else forget
  (``success``); panics are recovered and counted;
* ``controller_runtime_*`` and ``workqueue_*`` metrics, per-request loggers from
  a log constructor (``internal/controller/util.go:27-41``) with a
  ``reconcileID``.

**Deferred tails.**  A reconcile may hand back its last writes instead of waiting for
them: ``Result.tail`` is a future that finishes those writes and resolves to the final
:class:`Result` (or raises the reconcile's error).  The worker is then free to take the
next key at once, while the key itself stays *processing* in the queue until the tail
has finished -- the queue parks any new add of that key ("dirty") exactly as it does
during the reconcile proper, so per-key serialisation and the no-duplicate guarantee
are unchanged.  The reference's deferred status patch (``cron_controller.go:107-120``)
runs on the worker goroutine after the CREATE (``:229-238``): under apiserver latency a
fire then holds a worker for two sequential write round trips; with a tail it holds it
for one.  ``max_tails`` bounds the tails in flight (past it a worker awaits its own
tail inline, which is the plain behaviour).
"""
from __future__ import annotations

import asyncio
import time
import traceback
import uuid
from dataclasses import dataclass
from functools import lru_cache
from typing import Any, Awaitable, Callable, Dict, List, Optional, Tuple

from ..api.meta import GroupVersionKind, NamespacedName, controller_ref
from ..parallel.workqueue import ShutDown, WorkQueue
from ..utils import aio
from ..utils.clock import Clock
from ..utils.logging import Logger, get_logger, log_constructor
from . import metrics, tracing
from .informer import EventHandler, Informer

Request = NamespacedName

PRIORITY_EVENT = 0
PRIORITY_SCHEDULE = 10


@dataclass
class Result:
    requeue: bool = False
    requeue_after: float = 0.0  # seconds
    requeue_after_ns: int = 0   # exact form (schedule requeues land on the tick)
    # a future finishing the reconcile's last writes; resolves to the final Result (see module doc)
    tail: Optional["asyncio.Future[Result]"] = None

    def after_ns(self) -> int:
        return self.requeue_after_ns or int(self.requeue_after * 1e9)

    def is_zero(self) -> bool:
        return not self.requeue and self.after_ns() == 0


class TerminalError(Exception):
    """An error that should not be retried (``reconcile.TerminalError``)."""


class Reconciler:
    async def reconcile(self, req: Request, log: Logger) -> Result:
        raise NotImplementedError


Predicate = Callable[[str, Optional[Dict[str, Any]], Dict[str, Any]], bool]  # (event, old, new) -> keep?


def generation_changed(event: str, old: Optional[Dict[str, Any]], new: Dict[str, Any]) -> bool:
    if event != "update" or old is None:
        return True
    return (old.get("metadata") or {}).get("generation") != (new.get("metadata") or {}).get("generation")


def _key(obj: Dict[str, Any]) -> Request:
    m = obj.get("metadata") or {}
    return Request(m.get("namespace", ""), m.get("name", ""))



@lru_cache(maxsize=1 << 17)
def shard_of(namespace: str, name: str, count: int) -> int:
    """Stable shard of an object key: FNV-1a (32-bit) of ``namespace/name`` modulo ``count``.
    Python's ``hash()`` is salted per process, so it cannot be used across replicas.  Memoised:
    every watch event of every Cron and child is routed through it."""
    h = 0x811C9DC5
    for b in f"{namespace}/{name}".encode():
        h = ((h ^ b) * 0x01000193) & 0xFFFFFFFF
    return h % count if count > 1 else 0

class Controller:
    def __init__(self, name: str, reconciler: Reconciler, clock: Clock, max_concurrent_reconciles: int = 1,
                 logger: Optional[Logger] = None, recover_panic: bool = True, queue: Optional[WorkQueue] = None,
                 max_tails: int = 0):
        self.name = name
        self.reconciler = reconciler
        self.shard: Tuple[int, int] = (0, 1)
        self.clock = clock
        self.max_concurrent = max(1, max_concurrent_reconciles)
        base = logger or get_logger()
        self.log = base.with_values(controller=name)
        self._log_ctor = log_constructor(base, "Cron") if name == "cron" else None
        self._loggers: Dict[Request, Logger] = {}
        self.recover_panic = recover_panic
        self.queue = queue or WorkQueue(name, clock, controller=name)
        self._sources: List[Tuple[Informer, EventHandler]] = []
        self._workers: List[asyncio.Task] = []
        self.active = 0
        # deferred tails in flight (key stays processing until each one finishes); 0 -> default bound
        self.max_tails = max_tails if max_tails > 0 else max(1024, 100 * self.max_concurrent)
        self._tails: Dict["asyncio.Future[Result]", Tuple[Request, Logger, float]] = {}
        self.tails_started = 0
        self.reconciles = 0
        self.errors = 0
        self.started = False
        self.result_counts: Dict[str, int] = {}
        self.on_result: Optional[Callable[[Request, Optional[Result], Optional[BaseException]], None]] = None
        self._m_active = metrics.ACTIVE_WORKERS.labels(name)  # a gauge child: ``.value`` is its sample
        self._m_total: Dict[str, Any] = {}
        self._m_time = metrics.RECONCILE_TIME.labels(name)
        metrics.MAX_CONCURRENT.labels(name).set(self.max_concurrent)
        self.for_kind: Optional[GroupVersionKind] = None

    def set_log_constructor(self, ctor: Callable[[Optional[Request]], Logger]) -> None:
        self._log_ctor = ctor
        self._loggers.clear()

    # ------------------------------------------------------------------ sources
    def set_shard(self, index: int, count: int) -> None:
        """Only reconcile keys of shard ``index`` out of ``count`` (see :func:`shard_of`)."""
        if count < 1 or not 0 <= index < count:
            raise ValueError(f"invalid shard {index}/{count}")
        self.shard = (index, count)

    def _handler(self, mapper: Callable[[Dict[str, Any]], List[Request]],
                 predicates: List[Predicate]) -> EventHandler:
        q = self.queue
        if self.shard[1] > 1:  # horizontal sharding: drop keys owned by other shards
            inner = mapper
            index, count = self.shard

            def mapper(obj: Dict[str, Any]) -> List[Request]:  # type: ignore[no-redef]
                return [r for r in inner(obj) if shard_of(r.namespace, r.name, count) == index]

        ok: Predicate
        if len(predicates) == 1:
            ok = predicates[0]  # the common case: no generator per event
        else:
            def ok(event: str, old: Optional[Dict[str, Any]], new: Dict[str, Any]) -> bool:
                for p in predicates:
                    if not p(event, old, new):
                        return False
                return True

        def on_add(obj: Dict[str, Any]) -> None:
            if ok("create", None, obj):
                for r in mapper(obj):
                    q.add(r, PRIORITY_EVENT)

        def on_update(old: Dict[str, Any], new: Dict[str, Any]) -> None:
            if ok("update", old, new):
                reqs = mapper(new)
                for r in reqs:
                    q.add(r, PRIORITY_EVENT)
                # an owner change moves the child: also wake the previous owner
                prev = mapper(old)
                if prev != reqs:
                    for r in prev:
                        q.add(r, PRIORITY_EVENT)

        def on_delete(obj: Dict[str, Any]) -> None:
            if ok("delete", None, obj):
                for r in mapper(obj):
                    q.add(r, PRIORITY_EVENT)

        return EventHandler(on_add, on_update, on_delete)

    def watch_for(self, informer: Informer, gvk: GroupVersionKind,
                  predicates: Optional[List[Predicate]] = None) -> None:
        """``For(&Cron{})``: enqueue the object itself."""
        self.for_kind = gvk
        h = self._handler(lambda o: [_key(o)], list(predicates or []))
        self._sources.append((informer, h))
        informer.add_handler(h)

    def watch_owned(self, informer: Informer, owner: GroupVersionKind,
                    predicates: Optional[List[Predicate]] = None) -> None:
        """``Owns(&Child{})``: enqueue the child's controller owner of kind ``owner``."""

        def mapper(obj: Dict[str, Any]) -> List[Request]:
            ref = controller_ref(obj)
            if ref is None or ref.get("kind") != owner.kind:
                return []
            if (ref.get("apiVersion", "").split("/")[0]) != owner.group:
                return []
            return [Request((obj.get("metadata") or {}).get("namespace", ""), ref.get("name", ""))]

        h = self._handler(mapper, list(predicates or []))
        self._sources.append((informer, h))
        informer.add_handler(h)

    def watch_map(self, informer: Informer, fn: Callable[[Dict[str, Any]], List[Request]],
                  predicates: Optional[List[Predicate]] = None) -> None:
        h = self._handler(fn, list(predicates or []))
        self._sources.append((informer, h))
        informer.add_handler(h)

    # ------------------------------------------------------------------ workers
    def _logger_for(self, req: Request) -> Logger:
        base = self._loggers.get(req)
        if base is None:
            base = self._log_ctor(req) if self._log_ctor else self.log.with_values(
                **{"namespace": req.namespace, "name": req.name})
            if len(self._loggers) >= 1 << 16:
                self._loggers.clear()
            self._loggers[req] = base  # loggers are immutable: one per key is reused
        if base.sink.level > 0:  # info disabled: skip the per-request ID
            return base
        return base.with_values(reconcileID=str(uuid.uuid4()))

    def _count(self, label: str) -> None:
        self.result_counts[label] = self.result_counts.get(label, 0) + 1
        c = self._m_total.get(label)
        if c is None:
            c = self._m_total[label] = metrics.RECONCILE_TOTAL.labels(self.name, label)
        c.inc()

    def in_flight(self) -> int:
        """Reconciles running on a worker plus deferred tails still writing."""
        return self.active + len(self._tails)

    async def process_one(self, req: Request) -> bool:
        """Reconcile ``req``.  False: the reconcile left a deferred tail, which calls
        ``queue.done(req)`` itself when it finishes; True: the caller calls it."""
        log = self._logger_for(req)
        self.active += 1
        self._m_active.value = float(self.active)
        t0 = time.perf_counter()
        result: Optional[Result] = None
        err: Optional[BaseException] = None
        try:
            if tracing.get_tracer().enabled:
                with tracing.span("reconcile", controller=self.name, namespace=req.namespace, name=req.name) as sp:
                    result = await self.reconciler.reconcile(req, log)
                    if result is None:
                        result = Result()
                    sp.set(requeue_after_ms=result.after_ns() / 1e6, deferred_tail=result.tail is not None)
            else:
                result = await self.reconciler.reconcile(req, log)
                if result is None:
                    result = Result()
            tail = result.tail
            if tail is not None and len(self._tails) >= self.max_tails:
                result = await tail  # too many tails in flight: finish this one on the worker
                tail = None
        except asyncio.CancelledError:
            raise
        except Exception as e:  # noqa: BLE001 - recover like RecoverPanic
            err = e
            tail = None
            if not self.recover_panic:
                raise
        finally:
            self.active -= 1
            self._m_active.value = float(self.active)
        if tail is not None:
            self._tails[tail] = (req, log, t0)
            self.tails_started += 1
            tail.add_done_callback(self._tail_done)
            return False
        self._finish(req, log, t0, result, err)
        return True

    def _tail_done(self, tail: "asyncio.Future[Result]") -> None:
        """A deferred tail finished: handle its result and release its key."""
        entry = self._tails.pop(tail, None)
        if entry is None:
            return
        req, log, t0 = entry
        try:
            if tail.cancelled():  # shutdown / leader loss: the key is simply released
                return
            err = tail.exception()
            result = None if err is not None else (tail.result() or Result())
            try:
                self._finish(req, log, t0, result, err)
            except Exception as e:  # noqa: BLE001 - a done callback must not raise into the loop
                log.error(e, "Failed to handle a deferred reconcile result")
        finally:
            self.queue.done(req)

    def _finish(self, req: Request, log: Logger, t0: float, result: Optional[Result],
                err: Optional[BaseException]) -> None:
        """Result handling after a reconcile (and its tail) finished."""
        q = self.queue
        self._m_time.observe(time.perf_counter() - t0)
        self.reconciles += 1
        if err is not None:
            self.errors += 1
            if isinstance(err, TerminalError):
                metrics.TERMINAL_ERRORS.labels(self.name).inc()
            else:
                q.add_rate_limited(req, PRIORITY_EVENT)
            metrics.RECONCILE_ERRORS.labels(self.name).inc()
            self._count("error")
            if not isinstance(err, Exception) or type(err).__name__ in ("AttributeError", "TypeError", "KeyError"):
                metrics.RECONCILE_PANICS.labels(self.name).inc()
                log.error(err, "Observed a panic", stacktrace="".join(traceback.format_exception(err))[-2000:])
            else:
                log.error(err, "Reconciler error")
        elif result.after_ns() > 0:  # type: ignore[union-attr]
            q.forget(req)
            q.add_at(req, self.clock.now_ns() + result.after_ns(), PRIORITY_SCHEDULE)  # type: ignore[union-attr]
            self._count("requeue_after")
        elif result.requeue:  # type: ignore[union-attr]
            q.add_rate_limited(req, PRIORITY_EVENT)
            self._count("requeue")
        else:
            q.forget(req)
            self._count("success")
        if self.on_result is not None:
            self.on_result(req, result, err)

    async def _worker(self) -> None:
        q = self.queue
        while True:
            try:
                req = await q.get()
            except ShutDown:
                return
            release = True
            try:
                release = await self.process_one(req)
            finally:
                if release:
                    q.done(req)

    def start(self) -> None:
        if self.started:
            return
        self.started = True
        loop = asyncio.get_running_loop()
        for i in range(self.max_concurrent):
            self._workers.append(loop.create_task(self._worker(), name=f"{self.name}-worker-{i}"))
        self._workers.append(loop.create_task(self._unfinished_loop(), name=f"{self.name}-metrics"))

    async def _unfinished_loop(self, interval: float = 0.5) -> None:
        """workqueue_unfinished_work_seconds / ..._longest_running_processor_seconds, refreshed
        every 500 ms like client-go's ``updateUnfinishedWorkLoop``."""
        while True:
            await asyncio.sleep(interval)
            self.queue.update_unfinished_metrics()

    async def stop(self) -> None:
        self.queue.shutdown()
        workers, self._workers = self._workers, []
        # deferred tails are cancelled with the workers (controller-runtime cancels the context
        # of every in-flight reconcile); their done callbacks release the keys
        await aio.cancel_and_wait(*workers, *list(self._tails))
        self.started = False

    async def wait_idle(self, settle: float = 0.0, timeout: float = 60.0) -> bool:
        """Wait until the queue has nothing queued or in flight (delayed items excluded)."""
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if self.queue.idle():
                if settle <= 0:
                    return True
                await asyncio.sleep(settle)
                if self.queue.idle():
                    return True
            await asyncio.sleep(0.001)
        return False


ReconcileFunc = Callable[[Request, Logger], Awaitable[Result]]
