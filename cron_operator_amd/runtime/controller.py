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

**Released worker slots.**  ``--max-concurrent-reconciles`` bounds the reconciles that are
*deciding* (reading caches, computing status).  A reconcile about to do nothing but API writes
may call :func:`release_worker`: its worker slot goes to the next queued key at once, while
the reconcile finishes its writes on the same task.  The key stays *processing* in the queue
until that reconcile returns -- the queue parks any new add of the key ("dirty") exactly as
before -- so per-key serialisation and the no-duplicate guarantee are unchanged.  The
reference's deferred status patch (``cron_controller.go:107-120``) runs on the worker after
the CREATE (``:229-238``): under apiserver latency a fire holds a worker for two sequential
write round trips; with a released slot it holds it for none.  ``max_released`` bounds the
reconciles writing after a release (with that many writing, new keys wait for a worker as
usual).  Workers are long-lived tasks started on demand: ``max_concurrent`` at start, and one
more only when a release finds no parked worker to take its slot -- a controller whose
reconciler never releases (``--compat-mode reference``) runs exactly ``max_concurrent``, and
one that does keeps as many spares as releases ever overlapped.  A release costs two counter
updates, not a task.

The bound is deliberately not the client's in-flight cap: under a backed-up QPS bucket the
released reconciles' writes wait *in the bucket*, where a tick's CREATEs overtake status
PATCHes (``runtime/ratelimit.py``); capping writers at the in-flight cap would move that
wait back into the work queue, where it is FIFO.
"""
from __future__ import annotations

import asyncio
import contextvars
import time
import traceback
import uuid
from dataclasses import dataclass
from functools import lru_cache
from collections import deque
from typing import Any, Awaitable, Callable, Deque, Dict, List, Optional, Tuple

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
    # absolute form (clock ns): the requeue lands here however long the reconcile took to return
    # -- a schedule requeue computed before a reconcile's deferred writes (which may wait on a
    # throttled client for seconds) would otherwise land that much after the tick
    requeue_at_ns: int = 0

    def after_ns(self) -> int:
        return self.requeue_after_ns or int(self.requeue_after * 1e9)

    def is_zero(self) -> bool:
        return not self.requeue and self.after_ns() == 0


class _Slot:
    """One worker's claim on a ``--max-concurrent-reconciles`` slot for one reconcile."""

    __slots__ = ("ctrl", "held")

    def __init__(self, ctrl: "Controller"):
        self.ctrl = ctrl
        self.held = True

    def release(self) -> bool:
        if not self.held:
            return False
        self.held = False
        self.ctrl._on_release()
        self.ctrl._slot_release()
        return True


_SLOT: "contextvars.ContextVar[Optional[_Slot]]" = contextvars.ContextVar("cron_operator_worker_slot",
                                                                            default=None)


def release_worker() -> bool:
    """Give this reconcile's worker slot to the next queued key; the caller keeps running (its
    key stays processing until it returns).  False outside a controller worker, or when the
    slot was already released."""
    slot = _SLOT.get()
    return slot is not None and slot.release()


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
                 max_released: int = 0):
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
        # reconciles still writing after release_worker() (their keys stay processing); 0 -> default
        self.max_released = max_released if max_released > 0 else max(1024, 100 * self.max_concurrent)
        self.released = 0        # writing after a release, right now
        self.releases = 0        # release_worker() calls, total
        self._free_slots = self.max_concurrent
        self._slot_waiters: Deque[asyncio.Future] = deque()
        self._spawned = 0  # worker tasks started (max_concurrent at start, more on demand)
        metrics.RECONCILES_WRITING.observe((name,), self, lambda c: c.released)
        metrics.WORKER_RELEASES.observe((name,), self, lambda c: c.releases)
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
        """Reconciles holding a worker slot plus released ones still writing."""
        return self.active + self.released

    # ------------------------------------------------------------------ worker slots
    async def _slot_acquire(self) -> None:
        if self._free_slots > 0 and not self._slot_waiters:
            self._free_slots -= 1
            return
        fut = asyncio.get_running_loop().create_future()
        self._slot_waiters.append(fut)
        try:
            await fut
        except asyncio.CancelledError:
            if fut.done() and not fut.cancelled():
                self._slot_release()  # granted and cancelled in the same turn: pass it on
            elif fut in self._slot_waiters:
                self._slot_waiters.remove(fut)
            raise

    def _slot_release(self) -> None:
        # LIFO: the worker that parked last takes the slot -- a handful of hot worker tasks
        # cycle while the spares (max_released of them) stay parked and cold
        while self._slot_waiters:
            fut = self._slot_waiters.pop()
            if not fut.done():
                fut.set_result(None)  # the slot moves to this waiter
                return
        self._free_slots += 1

    def _on_release(self) -> None:
        self.active -= 1
        self.released += 1
        self.releases += 1
        self._m_active.value = float(self.active)
        if not self._slot_waiters and self.started and self._spawned < self.max_concurrent + self.max_released:
            # no parked worker to take the slot about to be freed: start one (spare workers
            # exist only as many as releases ever overlapped, up to max_released)
            self._spawn_worker()

    def _spawn_worker(self) -> None:
        self._workers.append(asyncio.get_running_loop().create_task(
            self._worker(), name=f"{self.name}-worker-{self._spawned}"))
        self._spawned += 1

    async def process_one(self, req: Request) -> None:
        log = self._logger_for(req)
        self.active += 1
        self._m_active.value = float(self.active)
        slot = _SLOT.get()
        t0 = time.perf_counter()
        result: Optional[Result] = None
        err: Optional[BaseException] = None
        try:
            if tracing.get_tracer().enabled:
                with tracing.span("reconcile", controller=self.name, namespace=req.namespace, name=req.name) as sp:
                    result = await self.reconciler.reconcile(req, log)
                    if result is None:
                        result = Result()
                    sp.set(requeue_after_ms=result.after_ns() / 1e6,
                           released_worker=slot is not None and not slot.held)
            else:
                result = await self.reconciler.reconcile(req, log)
                if result is None:
                    result = Result()
        except asyncio.CancelledError:
            raise
        except Exception as e:  # noqa: BLE001 - recover like RecoverPanic
            err = e
            if not self.recover_panic:
                raise
        finally:
            if slot is not None and not slot.held:
                self.released -= 1
            else:
                self.active -= 1
                self._m_active.value = float(self.active)
        self._finish(req, log, t0, result, err)

    def _finish(self, req: Request, log: Logger, t0: float, result: Optional[Result],
                err: Optional[BaseException]) -> None:
        """Result handling after a reconcile finished."""
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
            at = result.requeue_at_ns or self.clock.now_ns() + result.after_ns()  # type: ignore[union-attr]
            q.add_at(req, at, PRIORITY_SCHEDULE)
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
        """Take a slot, then a key; reconcile it (the reconcile may hand its slot on early with
        :func:`release_worker`); release the key and the slot."""
        q = self.queue
        slot = _Slot(self)  # one per worker task, in the task's own context
        slot.held = False
        _SLOT.set(slot)
        while True:
            if self._free_slots > 0 and not self._slot_waiters:  # _slot_acquire's fast path, inline
                self._free_slots -= 1
            else:
                await self._slot_acquire()
            slot.held = True
            try:
                req = await q.get()
            except ShutDown:
                slot.held = False
                self._slot_release()
                return
            except BaseException:  # cancellation: the slot goes back
                slot.held = False
                self._slot_release()
                raise
            try:
                await self.process_one(req)
            finally:
                q.done(req)
                if slot.held:
                    slot.held = False
                    self._slot_release()

    def start(self) -> None:
        if self.started:
            return
        self.started = True
        loop = asyncio.get_running_loop()
        # max_concurrent workers decide at any time; up to max_released more are started on
        # demand, when a release finds no parked worker to hand its slot to (_on_release)
        self._spawned = 0
        for _ in range(self.max_concurrent):
            self._spawn_worker()
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
        # controller-runtime cancels the context of every in-flight reconcile, released or not
        await aio.cancel_and_wait(*workers)
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
