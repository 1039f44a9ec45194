"""List-watch informers, indexers and the shared cache.

controller-runtime serves the reference's ``client.Get(Cron)`` from an
informer cache and watches PyTorchJob/TFJob through ``Owns()``
(``internal/controller/cron_controller.go:70-77,96``).  Its *unstructured* child
LIST, however, bypasses the cache and hits the apiserver on every reconcile
(SURVEY C15).  Here every watched kind -- including children of any GVK -- is
served from an informer, and children are indexed by the
``kubedl.io/cron-name`` label so the per-reconcile child lookup is a dict hit.

:class:`Informer` implements the reflector loop: paged LIST, then WATCH from
the list's resourceVersion; a closed watch resumes from the last seen version;
410 Expired triggers a relist whose diff is replayed as add/update/delete
events.  Objects in the store are read-only snapshots.

Watch liveness: every WATCH carries a random ``timeoutSeconds`` in [300, 600)
as client-go's reflector sends, and a watchdog drops a stream that delivered
nothing -- no event, no BOOKMARK -- for ``watch_idle_timeout`` seconds (a
half-open connection after a silent network drop); the reflector then resumes
from the last resourceVersion, relisting on 410.  The HTTP transport also enables
TCP keepalive on its connections.

Periodic resync (controller-runtime's ``SyncPeriod``, default 10 h with up to
10% jitter): every object in the store is re-delivered to the handlers as an
update whose old and new object are the same, so every Cron is reconciled at
least that often even if no event arrives (a safety net against missed events).
"""
from __future__ import annotations

import asyncio
import random
from functools import partial
from typing import Any, Callable, Dict, Iterable, List, Optional, Set, Tuple

from ..api import errors
from ..api.meta import GroupVersionKind, GroupVersionResource
from ..utils import aio, jsonutil
from ..utils.clock import Clock, TimerHandle
from ..utils.gotime import NANOS
from ..utils.logging import get_logger
from .client import Client

IndexFunc = Callable[[Dict[str, Any]], List[str]]

NAMESPACE_INDEX = "namespace"

# client-go reflector: each WATCH carries timeoutSeconds in [5 min, 10 min)
MIN_WATCH_TIMEOUT = 300.0
# no event and no BOOKMARK for this long (apiservers send a bookmark about once a
# minute to watches that allow them): the connection is presumed dead
WATCH_IDLE_TIMEOUT = 150.0
WATCH_TIMEOUT_GRACE = 30


def obj_key(obj: Dict[str, Any]) -> str:
    m = obj.get("metadata") or {}
    ns = m.get("namespace", "")
    return f"{ns}/{m.get('name', '')}" if ns else m.get("name", "")


def namespace_index(obj: Dict[str, Any]) -> List[str]:
    return [(obj.get("metadata") or {}).get("namespace", "")]


def label_index(label: str) -> IndexFunc:
    """Index by ``namespace/<label value>`` (objects without the label are not indexed)."""

    def fn(obj: Dict[str, Any]) -> List[str]:
        m = obj.get("metadata") or {}
        v = (m.get("labels") or {}).get(label)
        return [] if v is None else [f"{m.get('namespace', '')}/{v}"]

    fn.label = label  # type: ignore[attr-defined]  # lets the native bookkeeping index it too
    return fn



class EventHandler:
    """add/update/delete callbacks (``cache.ResourceEventHandlerFuncs``)."""

    def __init__(self, on_add: Optional[Callable[[Dict[str, Any]], None]] = None,
                 on_update: Optional[Callable[[Dict[str, Any], Dict[str, Any]], None]] = None,
                 on_delete: Optional[Callable[[Dict[str, Any]], None]] = None):
        self.on_add = on_add
        self.on_update = on_update
        self.on_delete = on_delete


Transform = Callable[[Dict[str, Any]], Dict[str, Any]]


def strip_managed_fields(obj: Dict[str, Any]) -> Dict[str, Any]:
    """``cache.TransformStripManagedFields``: server-side-apply bookkeeping no controller reads."""
    m = obj.get("metadata")
    if type(m) is dict and "managedFields" in m:
        del m["managedFields"]
    return obj


class Informer:
    """A reflector + indexed store (``cache.SharedIndexInformer``).

    ``transform`` (client-go ``SetTransform``) rewrites every object before it is
    stored or handed to handlers -- e.g. dropping fields no consumer reads to keep
    a large cache small.  Objects reaching it were decoded for this informer alone,
    so it may modify them in place.  ``keep`` then decides what is stored at all: a
    filter the apiserver cannot apply (one shard's hash share of a fleet).
    """

    def __init__(self, client: Client, target: Any, namespace: str = "", label_selector: Optional[str] = None,
                 field_selector: Optional[str] = None, indexers: Optional[Dict[str, IndexFunc]] = None,
                 page_size: int = 500, name: str = "", resync_period: float = 0.0,
                 clock: Optional[Clock] = None, transform: Optional[Transform] = None,
                 min_watch_timeout: float = MIN_WATCH_TIMEOUT, watch_idle_timeout: float = WATCH_IDLE_TIMEOUT,
                 decoder: Any = None, list_decoder: Any = None,
                 keep: Optional[Callable[[Dict[str, Any]], bool]] = None):
        self.client = client
        # ``keep`` (after ``transform``): objects it rejects are not stored -- an object that
        # stops passing it leaves the store as a deletion.  A filter the apiserver cannot apply
        # (a hash of name and labels: one shard's share of an unassigned fleet), applied as each
        # LIST page and watch event arrives, so the rest is never held
        self.keep = keep
        # watch-event decoder for byte transports (a jsonutil.Codec): it may skip subtrees no
        # consumer reads and reuse memoised ones; None decodes plainly.  ``list_decoder`` does
        # the same for LIST pages (paths under ``items/*``): the initial LIST then shares what
        # later watch events share (a child's labels and owner references with its siblings')
        self.decoder = decoder
        self.list_decoder = list_decoder
        self._watch_kw: Dict[str, Any] = {"decoder": decoder} if decoder is not None else {}
        # watch liveness: every WATCH asks the server to end it after a random
        # [min, 2*min) seconds (client-go reflector), and a watch silent for
        # ``watch_idle_timeout`` seconds -- no event and no bookmark -- is dropped and
        # re-established from the last resourceVersion (a half-open connection)
        self.min_watch_timeout = min_watch_timeout
        self.watch_idle_timeout = watch_idle_timeout
        self.idle_timeouts = 0
        self._last_item = 0.0
        self._idle_limit = 0.0
        self._watchdog: Optional[asyncio.TimerHandle] = None
        self.transform = transform
        self._pretransformed = False  # _replace() of a LIST whose pages were transformed already
        # ``derive`` (set with :meth:`set_derive`): a per-object memo computed once per stored
        # object version -- readers that only need facts derived from an object (a child's
        # classification) take them from ``derived`` instead of re-reading the object
        self.derive: Optional[Callable[[Dict[str, Any]], Any]] = None
        self.derived: Dict[str, Any] = {}
        self._prederived: Dict[int, Any] = {}  # id(LIST item) -> derived right after its transform
        self.resync_period = resync_period
        self.clock = clock
        self._resync_timer: Optional[TimerHandle] = None
        self.resyncs = 0
        self.target = target
        self.namespace = namespace
        self.label_selector = label_selector
        self.field_selector = field_selector
        self.page_size = page_size
        self.name = name or str(target)
        self.store: Dict[str, Dict[str, Any]] = {}
        self.indexers: Dict[str, IndexFunc] = {NAMESPACE_INDEX: namespace_index}
        self.indexers.update(indexers or {})
        self.indices: Dict[str, Dict[str, Set[str]]] = {n: {} for n in self.indexers}
        self._native_spec()
        self.handlers: List[EventHandler] = []
        self.synced = asyncio.Event()
        # the outcome of the most recent LIST: ``list_error`` is its error (None after a
        # success) and ``_attempted`` is set after every attempt, so a reader waiting for
        # the first sync learns of a failing LIST instead of waiting without bound
        self.list_error: Optional[BaseException] = None
        self.list_failures = 0
        self._attempted = asyncio.Event()
        self.last_rv = ""
        self._task: Optional[asyncio.Task] = None
        self._watch = None
        self._stopped = False
        self.relists = 0
        self.events = 0
        self.log = get_logger("informer").with_values(resource=self.name)

    # ------------------------------------------------------------------ indexing
    def add_indexer(self, name: str, fn: IndexFunc) -> None:
        if name in self.indexers:
            return
        self.indexers[name] = fn
        idx: Dict[str, Set[str]] = {}
        for k, obj in self.store.items():
            for v in fn(obj):
                idx.setdefault(v, set()).add(k)
        self.indices[name] = idx
        self._native_spec()

    def _native_spec(self) -> None:
        """Use the native event bookkeeping (``_fastjson.store_apply``: key, store, derived
        memo, indexes) when every indexer is one it knows -- the namespace index or a label
        index; any other index function keeps the Python path."""
        spec = []
        for name, fn in self.indexers.items():
            if fn is namespace_index:
                spec.append((name, None))
            elif isinstance(getattr(fn, "label", None), str):
                spec.append((name, fn.label))  # type: ignore[attr-defined]
            else:
                self._napply, self._nspec = None, ()
                return
        self._napply = jsonutil.store_apply
        self._nspec = tuple(spec)

    def _index(self, key: str, obj: Optional[Dict[str, Any]], old: Optional[Dict[str, Any]]) -> None:
        for name, fn in self.indexers.items():
            idx = self.indices[name]
            if old is not None and obj is not None:
                if fn is namespace_index:
                    continue  # the store key carries the namespace: an update cannot move it
                ov = fn(old)
                nv = fn(obj)
                if ov == nv:
                    continue  # an update that keeps its index values: the key is filed already
                for v in ov:
                    s = idx.get(v)
                    if s is not None:
                        s.discard(key)
                        if not s:
                            del idx[v]
                for v in nv:
                    idx.setdefault(v, set()).add(key)
                continue
            if old is not None:
                for v in fn(old):
                    s = idx.get(v)
                    if s is not None:
                        s.discard(key)
                        if not s:
                            del idx[v]
            if obj is not None:
                for v in fn(obj):
                    idx.setdefault(v, set()).add(key)

    # ------------------------------------------------------------------ reads
    def get(self, namespace: str, name: str, copy: bool = True) -> Optional[Dict[str, Any]]:
        obj = self.store.get(f"{namespace}/{name}" if namespace else name)
        if obj is None:
            return None
        return jsonutil.deepcopy(obj) if copy else obj

    def list(self, namespace: Optional[str] = None, copy: bool = True) -> List[Dict[str, Any]]:
        if namespace:
            keys: Iterable[str] = self.indices[NAMESPACE_INDEX].get(namespace, ())
            objs = [self.store[k] for k in keys]
        else:
            objs = list(self.store.values())
        return [jsonutil.deepcopy(o) for o in objs] if copy else objs

    def set_derive(self, fn: Callable[[Dict[str, Any]], Any]) -> None:
        """Install the per-object memo function and compute it for what is stored already."""
        self.derive = fn
        self.derived = {k: fn(o) for k, o in self.store.items()}

    def derived_by_index(self, index: str, value: str) -> List[Any]:
        """``derive(obj)`` of every object under ``value`` of ``index``."""
        return jsonutil.pick(self.derived, self.indices.get(index, {}).get(value, ()))

    def by_index(self, index: str, value: str, copy: bool = True) -> List[Dict[str, Any]]:
        keys = self.indices.get(index, {}).get(value, ())
        objs = [self.store[k] for k in keys]
        return [jsonutil.deepcopy(o) for o in objs] if copy else objs

    def add_handler(self, h: EventHandler) -> None:
        self.handlers.append(h)
        # late registration: replay the current state as adds (client-go behaviour)
        if h.on_add is not None:
            for obj in list(self.store.values()):
                h.on_add(obj)

    # ------------------------------------------------------------------ store mutation + dispatch
    def _apply(self, etype: str, obj: Dict[str, Any]) -> None:
        if self.transform is not None and not self._pretransformed:
            obj = self.transform(obj)
        self.events += 1
        if self.keep is not None and etype != "DELETED" and not self.keep(obj):
            etype = "DELETED"
        na = self._napply
        if na is not None:
            # key, store write/delete, derived-memo drop and index upkeep in one native call
            r = na(self.store, self.derived, self.indices, self._nspec, etype == "DELETED", obj)
            if r is not None:
                key, old = r
                if etype == "DELETED":
                    if old is not None:
                        for h in self.handlers:
                            if h.on_delete:
                                h.on_delete(obj)
                    return
                if self.derive is not None:
                    pre = self._prederived.pop(id(obj), None) if self._prederived else None
                    self.derived[key] = pre if pre is not None else self.derive(obj)
                if old is None:
                    for h in self.handlers:
                        if h.on_add:
                            h.on_add(obj)
                else:
                    for h in self.handlers:
                        if h.on_update:
                            h.on_update(old, obj)
                return
        key = obj_key(obj)
        old = self.store.get(key)
        if etype == "DELETED":
            if old is None:
                return
            del self.store[key]
            if self.derive is not None:
                self.derived.pop(key, None)
            self._index(key, None, old)
            for h in self.handlers:
                if h.on_delete:
                    h.on_delete(obj)
            return
        self.store[key] = obj
        if self.derive is not None:
            pre = self._prederived.pop(id(obj), None) if self._prederived else None
            self.derived[key] = pre if pre is not None else self.derive(obj)
        self._index(key, obj, old)
        if old is None:
            for h in self.handlers:
                if h.on_add:
                    h.on_add(obj)
        else:
            for h in self.handlers:
                if h.on_update:
                    h.on_update(old, obj)

    def resync(self) -> None:
        """Re-deliver every stored object as an update with ``old is new``."""
        self.resyncs += 1
        for obj in list(self.store.values()):
            for h in self.handlers:
                if h.on_update:
                    h.on_update(obj, obj)

    def _arm_resync(self) -> None:
        if self.resync_period <= 0 or self.clock is None or self._stopped:
            return
        delay = self.resync_period * (1.0 + 0.1 * random.random())
        self._resync_timer = self.clock.call_later(int(delay * NANOS), self._on_resync)

    def _on_resync(self) -> None:
        self._resync_timer = None
        if self._stopped:
            return
        self.resync()
        self._arm_resync()

    def _replace(self, items: List[Dict[str, Any]]) -> None:
        seen = set()
        for obj in items:
            key = obj_key(obj)
            seen.add(key)
            old = self.store.get(key)
            if old is not None and (old.get("metadata") or {}).get("resourceVersion") == \
                    (obj.get("metadata") or {}).get("resourceVersion"):
                continue
            self._apply("ADDED" if old is None else "MODIFIED", obj)  # _apply transforms
        for key in [k for k in self.store if k not in seen]:
            self._apply("DELETED", self.store[key])

    # ------------------------------------------------------------------ reflector
    def _transform_derive(self, tf: Transform, obj: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        """A LIST item transformed and derived at once, as a watch event is: a transform may hand
        the derive function what only the untransformed object had (``compact_child``).  None for
        an item ``keep`` rejects (never derived)."""
        out = tf(obj)
        if self.keep is not None and not self.keep(out):
            return None
        self._prederived[id(out)] = self.derive(out)  # type: ignore[misc]
        return out

    async def _list_pages(self) -> Dict[str, Any]:
        """Paged LIST (client-go pager) whose items are transformed page by page, as each page
        arrives: a large initial LIST then never holds every untrimmed object at once (the
        process's peak memory, which it keeps as RSS, would be set by that moment)."""
        out: Optional[Dict[str, Any]] = None
        cont: Optional[str] = None
        tf = self.transform
        while True:
            page = await self.client.list(self.target, self.namespace, self.label_selector,
                                          limit=self.page_size, continue_=cont, decoder=self.list_decoder)
            keep = self.keep
            if tf is not None and self.derive is not None:
                page["items"] = [o for o in map(partial(self._transform_derive, tf), page.get("items") or [])
                                 if o is not None]
            elif tf is not None:
                page["items"] = [tf(o) for o in page.get("items") or []] if keep is None else \
                    [o for o in map(tf, page.get("items") or []) if keep(o)]
            elif keep is not None:
                page["items"] = [o for o in page.get("items") or [] if keep(o)]
            if out is None:
                out = page
            else:
                out["items"].extend(page.get("items") or [])
                out["metadata"]["resourceVersion"] = (page.get("metadata") or {}).get("resourceVersion")
            cont = (page.get("metadata") or {}).get("continue")
            if not cont:
                break
        assert out is not None
        (out.get("metadata") or {}).pop("continue", None)
        return out

    async def _list(self) -> None:
        try:
            lst = await self._list_pages() if not self.field_selector else \
                await self.client.list(self.target, self.namespace, self.label_selector, self.field_selector)
        except asyncio.CancelledError:
            raise
        except Exception as e:
            self.list_error = e
            self.list_failures += 1
            self._attempted.set()
            raise
        self.list_error = None
        self.list_failures = 0
        self._attempted.set()
        self.relists += 1
        # the paged LIST transformed its items already (a field-selector LIST did not)
        self._pretransformed = self.transform is not None and not self.field_selector
        try:
            self._replace(lst.get("items") or [])
        finally:
            self._pretransformed = False
            self._prederived.clear()  # items _replace skipped (unchanged) were derived for nothing
        self.last_rv = (lst.get("metadata") or {}).get("resourceVersion", "")
        if not self.synced.is_set():
            self.synced.set()

    async def wait_synced(self, timeout: Optional[float] = None) -> None:
        """Wait for the first successful LIST.  Raises the LIST's error as soon as an attempt
        fails (403 Forbidden, 404, 5xx, a transport error) -- client-go's reflector only logs
        it and retries, but a caller that needs the data now (a reconcile) must not hold its
        worker while the informer backs off -- and :class:`asyncio.TimeoutError` after
        ``timeout`` seconds without an outcome."""
        loop = asyncio.get_running_loop()
        deadline = None if timeout is None else loop.time() + timeout
        while not self.synced.is_set():
            if self.list_error is not None:
                raise self.list_error
            self._attempted.clear()
            if deadline is None:
                await self._attempted.wait()
                continue
            left = deadline - loop.time()
            if left <= 0:
                raise asyncio.TimeoutError(f"informer {self.name} has not synced after {timeout}s")
            try:
                await asyncio.wait_for(self._attempted.wait(), left)
            except asyncio.TimeoutError:
                raise asyncio.TimeoutError(f"informer {self.name} has not synced after {timeout}s") from None

    async def run(self) -> None:
        backoff = 0.1
        need_list = True
        while not self._stopped:
            try:
                if need_list:
                    await self._list()
                    need_list = False
                timeout_s = int(self.min_watch_timeout * (1.0 + random.random())) \
                    if self.min_watch_timeout > 0 else None
                self._watch = await self.client.watch(self.target, self.namespace, self.last_rv,
                                                      self.label_selector, self.field_selector,
                                                      timeout_seconds=timeout_s, **self._watch_kw)
                self._arm_watchdog(timeout_s)
                loop = asyncio.get_running_loop()
                w = self._watch
                try:
                    take = getattr(w, "take_ready", None)
                    if take is not None:
                        # batched: every event that arrived is applied per wake-up
                        while True:
                            batch = take()
                            if not batch:
                                if not await w.wait_ready():
                                    break
                                continue
                            self._last_item = loop.time()
                            self._on_batch(batch)
                    else:
                        async for etype, obj in w:
                            self._last_item = loop.time()
                            self._on_item(etype, obj)
                except BaseException:
                    # an ERROR event, a failing handler or a cancel ends this watch: close it, or its
                    # connection stays registered with the loop and keeps buffering events nobody
                    # takes (the next attempt resumes from last_rv on a new one)
                    w.stop()
                    raise
                finally:
                    self._disarm_watchdog()
                backoff = 0.1
            except asyncio.CancelledError:
                raise
            except errors.ApiError as e:
                if errors.is_gone(e):
                    need_list = True
                    self.log.v(1).info("watch expired, relisting")
                    continue
                self.log.error(e, "failed to list" if need_list else "watch failed")
                if e.code == 404:
                    need_list = True
                await asyncio.sleep(backoff * (1 + random.random()))
                backoff = min(backoff * 2, 30.0)
            except Exception as e:  # noqa: BLE001 - transport errors: retry with backoff
                if self._stopped:
                    break
                self.log.error(e, "list/watch failed")
                need_list = need_list or not self.last_rv
                await asyncio.sleep(backoff * (1 + random.random()))
                backoff = min(backoff * 2, 30.0)

    def _on_batch(self, batch: List[Tuple[str, Dict[str, Any]]]) -> None:
        """Every event of one wake-up, in order (:meth:`_on_item` without a call per event)."""
        apply = self._apply
        for etype, obj in batch:
            if etype == "ERROR":
                raise errors.ApiError.from_status(int(obj.get("code") or 500), obj)
            rv = (obj.get("metadata") or {}).get("resourceVersion")
            if etype != "BOOKMARK":
                apply(etype, obj)
            if rv:
                self.last_rv = rv

    def _on_item(self, etype: str, obj: Dict[str, Any]) -> None:
        """One watch event: apply it (BOOKMARKs only move the resume point); ERROR raises."""
        if etype == "ERROR":
            raise errors.ApiError.from_status(int(obj.get("code") or 500), obj)
        rv = (obj.get("metadata") or {}).get("resourceVersion")
        if etype != "BOOKMARK":
            self._apply(etype, obj)
        if rv:
            self.last_rv = rv

    # ------------------------------------------------------------------ watch liveness
    def _arm_watchdog(self, timeout_s: Optional[int]) -> None:
        idle = self.watch_idle_timeout
        if timeout_s:
            # the server should have ended the watch by then: a grace period past it is dead
            idle = min(idle, timeout_s + WATCH_TIMEOUT_GRACE) if idle > 0 else timeout_s + WATCH_TIMEOUT_GRACE
        if idle <= 0:
            return
        loop = asyncio.get_running_loop()
        self._idle_limit = idle
        self._last_item = loop.time()
        self._watchdog = loop.call_later(idle, self._check_idle)

    def _disarm_watchdog(self) -> None:
        if self._watchdog is not None:
            self._watchdog.cancel()
            self._watchdog = None

    def _check_idle(self) -> None:
        self._watchdog = None
        w = self._watch
        if w is None or self._stopped:
            return
        loop = asyncio.get_running_loop()
        quiet = loop.time() - self._last_item
        if quiet < self._idle_limit:
            self._watchdog = loop.call_later(self._idle_limit - quiet, self._check_idle)
            return
        self.idle_timeouts += 1
        self.log.info("watch silent, re-establishing it", seconds=round(quiet, 1))
        try:
            w.stop()
        except Exception:  # noqa: BLE001 - the stream is being dropped anyway
            pass

    def start(self) -> asyncio.Task:
        if self._task is None:
            self._task = asyncio.get_running_loop().create_task(self.run(), name=f"informer:{self.name}")
            self._arm_resync()
        return self._task

    async def stop(self) -> None:
        self._stopped = True
        self._disarm_watchdog()
        if self._resync_timer is not None:
            self._resync_timer.cancel()
            self._resync_timer = None
        if self._watch is not None:
            try:
                self._watch.stop()
            except Exception:
                pass
        if self._task is not None:
            await aio.cancel_and_wait(self._task)


class Cache:
    """Shared informers keyed by (resource, namespace, selector) -- ``cache.Cache``."""

    def __init__(self, client: Client, namespace: str = "", resync_period: float = 0.0,
                 clock: Optional[Clock] = None, min_watch_timeout: float = MIN_WATCH_TIMEOUT,
                 watch_idle_timeout: float = WATCH_IDLE_TIMEOUT):
        self.client = client
        self.min_watch_timeout = min_watch_timeout
        self.watch_idle_timeout = watch_idle_timeout
        self.namespace = namespace
        self.resync_period = resync_period
        self.clock = clock
        self._informers: Dict[Tuple[Any, str, Optional[str]], Informer] = {}
        self._started = False

    async def _resolve(self, target: Any) -> GroupVersionResource:
        if isinstance(target, GroupVersionKind):
            return (await self.client.mapper.resource_for(target))[0]
        return target

    async def get_informer(self, target: Any, label_selector: Optional[str] = None,
                           indexers: Optional[Dict[str, IndexFunc]] = None,
                           transform: Optional[Transform] = None, decoder: Any = None,
                           list_decoder: Any = None,
                           keep: Optional[Callable[[Dict[str, Any]], bool]] = None) -> Informer:
        """The shared informer for ``(target, namespace, selector)``.  ``transform`` and
        ``decoder`` (and ``keep``) apply when this call creates it (like ``cache.Options.ByObject[...].Transform``)."""
        gvr = await self._resolve(target)
        key = (gvr, self.namespace, label_selector)
        inf = self._informers.get(key)
        if inf is None:
            inf = Informer(self.client, gvr, self.namespace, label_selector, indexers=indexers,
                           name=f"{gvr.resource}.{gvr.group}" if gvr.group else gvr.resource,
                           resync_period=self.resync_period, clock=self.clock, transform=transform,
                           min_watch_timeout=self.min_watch_timeout, watch_idle_timeout=self.watch_idle_timeout,
                           decoder=decoder, list_decoder=list_decoder, keep=keep)
            self._informers[key] = inf
            if self._started:
                inf.start()
        else:
            for n, fn in (indexers or {}).items():
                inf.add_indexer(n, fn)
        return inf

    def informers(self) -> List[Informer]:
        return list(self._informers.values())

    def start(self) -> None:
        self._started = True
        for inf in self._informers.values():
            inf.start()

    async def wait_for_sync(self, timeout: Optional[float] = None) -> bool:
        waits = [inf.synced.wait() for inf in self._informers.values()]
        if not waits:
            return True
        try:
            await asyncio.wait_for(asyncio.gather(*waits), timeout)
            return True
        except asyncio.TimeoutError:
            return False

    async def stop(self) -> None:
        for inf in list(self._informers.values()):
            await inf.stop()
