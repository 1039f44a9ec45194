"""Label-routed horizontal sharding (``--shard-routing=labels``).

The reference runs one leader-elected replica; this operator can split
its Crons across ``--shard-count`` replicas.  Two routings exist:

``hash`` (:func:`cron_operator_amd.runtime.controller.shard_of`)
    every shard watches *all* Crons and children, stores only its own share
    (:func:`hash_keep`, an informer ``keep`` filter), and its event handler drops
    the keys of other shards.  Nothing is written to user objects, but N shards
    decode N times the watch traffic.
``labels`` (default; this module)
    every Cron and child carries ``kubedl.io/shard=<index>-of-<count>`` and shard
    *i*'s informers select on its own value, so the apiserver sends each event to
    one shard only.  Total operator work stays O(events) as shards are added.

Assignment is done by the shards themselves.  Each one also watches the objects
whose shard label is missing or belongs to another shard count
(``kubedl.io/shard notin (0-of-n, ..., n-1-of-n)``), which is an empty watch in
steady state, and labels the ones whose Cron hashes (``shard_of``, FNV-1a of
``namespace/name``) to itself.  The labelled object leaves that watch and enters
the shard's main informers: the apiserver turns a label change into DELETED /
ADDED per watch selector.  Children created by the reconciler carry the label
from the start; children of a Cron that moved (after a change of shard count) are
relabelled the same way, keyed by their ``kubedl.io/cron-name`` label.

A change of ``--shard-count`` needs every shard restarted with the new count, as
with hash routing; objects are then relabelled in the background.

**Assignment order.**  A Cron is labelled only after its own unassigned children are
labelled *and* this shard's child informers hold them: were the Cron to join the
shard's Cron informer first, its reconcile would list no running child -- under
``Forbid`` it would start a second job beside the running one, under ``Replace`` it
would miss the job it must delete, and ``status.active``/``history`` would drop
entries.  This matters on the first start with label routing (a fresh install or an
upgrade from hash routing, where every object is unlabelled) and after a change of
shard count.  The wait for the informers is bounded (``observe_timeout``); a child
deleted meanwhile never shows up there and only costs that bound.  A child whose label
PATCH keeps failing (403, a webhook's 422) is given up after ``max_child_attempts``:
its Cron is then assigned without it instead of being parked for good.
"""
from __future__ import annotations

import asyncio
from typing import Any, Callable, Dict, List, Optional, Set, Tuple

from ..api import errors
from ..api.meta import GroupVersionKind
from ..api.v1alpha1.groupversion import LABEL_CRON_NAME, LABEL_PREFIX_KUBEDL
from ..runtime.client import Client
from ..runtime.controller import shard_of
from ..runtime.informer import Cache, EventHandler, Informer
from ..utils import aio
from ..utils.logging import Logger, get_logger

LABEL_SHARD = LABEL_PREFIX_KUBEDL + "/shard"
ROUTINGS = ("hash", "labels")


def shard_label_value(index: int, count: int) -> str:
    return f"{index}-of-{count}"


def shard_selector(index: int, count: int) -> str:
    """Selector of the Crons shard ``index`` owns."""
    return f"{LABEL_SHARD}={shard_label_value(index, count)}"


def child_selector(index: int, count: int) -> str:
    """Selector of the children shard ``index`` owns."""
    return f"{LABEL_CRON_NAME},{shard_selector(index, count)}"


def hash_keep(index: int, count: int, child: bool) -> Callable[[Dict[str, Any]], bool]:
    """Informer ``keep`` filter of hash routing: the Crons (children: the jobs of the Crons) that
    hash to shard ``index``.  A child without a cron-name label is kept, as without sharding."""
    def keep(obj: Dict[str, Any]) -> bool:
        m = obj.get("metadata") or {}
        if child:
            cron = (m.get("labels") or {}).get(LABEL_CRON_NAME)
            if cron is None:
                return True
        else:
            cron = m.get("name", "")
        return shard_of(m.get("namespace", ""), cron, count) == index
    return keep


def unassigned_selector(count: int) -> str:
    """Objects without a valid label for ``count`` shards (``notin`` also matches a missing label)."""
    return f"{LABEL_SHARD} notin ({','.join(shard_label_value(i, count) for i in range(count))})"


_KEPT_METADATA = ("name", "namespace", "uid", "resourceVersion", "labels")


def persistent_failure(e: errors.ApiError) -> bool:
    """A refusal that retrying will not change: a 4xx other than 404 (gone: nothing to label),
    409 (a racing write: retry), 429 (throttled: retry).  5xx and transport errors are transient."""
    return 400 <= e.code < 500 and e.code not in (404, 409, 429)


def metadata_only(obj: Dict[str, Any]) -> Dict[str, Any]:
    """Informer transform for the unassigned watches: assignment reads only names and labels.
    Before the first assignment (a fresh install, or a new shard count) those watches hold
    the whole fleet, so every shard process would otherwise cache every Cron and job in
    full once -- and keep that peak as its resident size."""
    m = obj.get("metadata") or {}
    return {"apiVersion": obj.get("apiVersion"), "kind": obj.get("kind"),
            "metadata": {k: m[k] for k in _KEPT_METADATA if k in m}}


_DROPPED = (("spec",), ("status",), ("metadata", "managedFields"), ("metadata", "annotations"))
_CODECS: List[Any] = []


def _metadata_codecs() -> Tuple[Any, Any]:
    """(watch event, LIST page) codecs of the unassigned watches: an object's spec, status,
    managed fields and annotations are never built.  On a first start with label routing
    every shard LISTs the whole unlabelled fleet through these watches; decoding it whole,
    page by page, set each shard process's peak (and so its resident size) by the fleet."""
    if not _CODECS:
        from ..utils import jsonutil

        _CODECS.extend((jsonutil.Codec(skip=[("object",) + p for p in _DROPPED]),
                        jsonutil.Codec(skip=[("items", "*") + p for p in _DROPPED])))
    return _CODECS[0], _CODECS[1]


class ShardAssigner:
    """Labels this shard's unassigned Crons and children (a leader-only runnable)."""

    def __init__(self, client: Client, index: int, count: int, workers: int = 4,
                 retry_delay: float = 1.0, logger: Optional[Logger] = None, observe_timeout: float = 10.0,
                 max_child_attempts: int = 5):
        if count < 1 or not 0 <= index < count:
            raise ValueError(f"invalid shard {index}/{count}")
        self.client = client
        self.index = index
        self.count = count
        self.value = shard_label_value(index, count)
        self.workers = max(1, workers)
        self.retry_delay = retry_delay
        self.log = logger or get_logger("shard-assigner")
        self.informers: Dict[GroupVersionKind, Informer] = {}
        self._queue: "asyncio.Queue[Tuple[GroupVersionKind, str, str]]" = asyncio.Queue()
        self._queued: Set[Tuple[GroupVersionKind, str, str]] = set()
        self.labelled = 0
        self.errors = 0
        self._bg: Set[asyncio.Task] = set()
        self.observe_timeout = observe_timeout
        # a child whose label PATCH keeps failing (403 on a kind without patch rights, 422 from
        # an admission webhook) is given up after this many attempts, so its Cron is not parked
        # for good; a later event on the child offers it again
        self.max_child_attempts = max(1, max_child_attempts)
        self._attempts: Dict[Tuple[GroupVersionKind, str, str], int] = {}
        # failures of any kind per key (retry backoff), persistent or not
        self._failures: Dict[Tuple[GroupVersionKind, str, str], int] = {}
        self.abandoned = 0
        self._child_kinds: Set[GroupVersionKind] = set()
        # (namespace, cron) -> child keys queued for labelling / labelled but maybe not observed yet
        self._children_left: Dict[Tuple[str, str], Set[Tuple[GroupVersionKind, str, str]]] = {}
        self._children_done: Dict[Tuple[str, str], List[Tuple[GroupVersionKind, str, str]]] = {}
        # Crons parked until their children are labelled: (namespace, cron) -> the Cron's key
        self._parked: Dict[Tuple[str, str], Tuple[GroupVersionKind, str, str]] = {}
        self._child_owner: Dict[Tuple[GroupVersionKind, str, str], Tuple[str, str]] = {}
        self._cron_gvk: Optional[GroupVersionKind] = None
        # does this shard's child informer hold the (labelled) child?  set by setup_with_manager
        self.observed: Optional[Callable[[GroupVersionKind, str, str], bool]] = None

    def watch_soon(self, cache: Cache, gvk: GroupVersionKind, child: bool) -> asyncio.Task:
        """:meth:`watch` as a task the assigner holds on to (the loop keeps only weak
        references to tasks, so an unheld one can be collected before it finishes)."""
        task = asyncio.get_running_loop().create_task(self.watch(cache, gvk, child))
        self._bg.add(task)
        task.add_done_callback(self._bg.discard)
        return task

    async def watch(self, cache: Cache, gvk: GroupVersionKind, child: bool) -> Informer:
        """Watch ``gvk``'s unassigned objects (children: only those with a cron-name label)."""
        inf = self.informers.get(gvk)
        if inf is not None:
            return inf
        sel = f"{LABEL_CRON_NAME},{unassigned_selector(self.count)}" if child else unassigned_selector(self.count)
        event, page = _metadata_codecs()
        # only this shard's share is stored: the other shards' objects are dropped as they arrive
        # (on a first start every shard LISTs the whole unassigned fleet)
        inf = await cache.get_informer(gvk, label_selector=sel, transform=metadata_only, decoder=event,
                                       list_decoder=page, keep=lambda o: self.owns(o, child))
        self.informers[gvk] = inf
        if child:
            self._child_kinds.add(gvk)
        else:
            self._cron_gvk = gvk
        inf.add_handler(EventHandler(on_add=lambda o: self._offer(gvk, o, child),
                                     on_update=lambda _old, o: self._offer(gvk, o, child)))
        for o in list(inf.store.values()):
            self._offer(gvk, o, child)
        return inf

    def owns(self, obj: Dict[str, Any], child: bool) -> bool:
        m = obj.get("metadata") or {}
        cron = (m.get("labels") or {}).get(LABEL_CRON_NAME, "") if child else m.get("name", "")
        return shard_of(m.get("namespace", ""), cron, self.count) == self.index

    def _offer(self, gvk: GroupVersionKind, obj: Dict[str, Any], child: bool) -> None:
        if not self.owns(obj, child):
            return
        m = obj.get("metadata") or {}
        ns = m.get("namespace", "")
        key = (gvk, ns, m.get("name", ""))
        if key not in self._queued:
            self._queued.add(key)
            if child:
                ck = (ns, (m.get("labels") or {}).get(LABEL_CRON_NAME, ""))
                self._children_left.setdefault(ck, set()).add(key)
                self._child_owner[key] = ck
            self._queue.put_nowait(key)

    def pending(self) -> int:
        return len(self._queued)

    async def run(self) -> None:
        # every unassigned child must be known before any Cron is labelled (assignment order)
        await asyncio.gather(*(inf.synced.wait() for inf in list(self.informers.values())))
        tasks: List[asyncio.Task] = [asyncio.get_running_loop().create_task(self._worker())
                                     for _ in range(self.workers)]
        try:
            await asyncio.gather(*tasks)
        finally:
            # awaited, not only cancelled: no label PATCH may land after shutdown
            await aio.cancel_and_wait(*tasks)

    def _child_finished(self, key: Tuple[GroupVersionKind, str, str], labelled: bool) -> None:
        """A child key left the queue (labelled, or gone): release its Cron when it was the last."""
        ck = self._child_owner.pop(key, None)
        left = self._children_left.get(ck) if ck is not None else None
        if left is None:
            return
        left.discard(key)
        cron_key = (self._cron_gvk, ck[0], ck[1]) if ck is not None else None  # type: ignore[index]
        if labelled and cron_key in self._queued:
            # the Cron waits for its labelling: it waits for these children to be observed too
            # (an already-assigned Cron, or an orphan child's missing Cron, has nothing to wait for)
            self._children_done.setdefault(ck, []).append(key)  # type: ignore[arg-type]
        if not left:
            del self._children_left[ck]  # type: ignore[arg-type]
            cron_key = self._parked.pop(ck, None)  # type: ignore[arg-type]
            if cron_key is not None:
                self._queue.put_nowait(cron_key)

    async def _children_observed(self, ns: str, cron: str) -> None:
        """Wait (bounded) until this shard's child informers hold the Cron's relabelled children."""
        done = self._children_done.pop((ns, cron), None)
        if not done or self.observed is None:
            return
        loop = asyncio.get_running_loop()
        deadline = loop.time() + self.observe_timeout
        while not all(self.observed(g, n, nm) for g, n, nm in done):
            if loop.time() >= deadline:
                self.log.info("Relabelled children not observed in time; assigning the Cron anyway",
                              namespace=ns, cron=cron)
                return
            await asyncio.sleep(0.02)

    async def _worker(self) -> None:
        patch = {"metadata": {"labels": {LABEL_SHARD: self.value}}}
        while True:
            key = await self._queue.get()
            gvk, ns, name = key
            child = gvk in self._child_kinds
            if not child:
                if self._children_left.get((ns, name)):
                    self._parked[(ns, name)] = key  # re-queued by the last child's _child_finished
                    continue
                await self._children_observed(ns, name)
            try:
                await self.client.patch(gvk, ns, name, patch, "merge", discard_response=True)
                self.labelled += 1
            except errors.ApiError as e:
                if not errors.is_not_found(e):
                    self.errors += 1
                    self.log.error(e, "Failed to assign shard", kind=gvk.kind, namespace=ns, name=name)
                    await asyncio.sleep(self._backoff(key))
                    inf = self.informers.get(gvk)
                    # only a persistent refusal counts toward giving a child up (403, a webhook's
                    # 422): throttling (429), conflicts and server errors are retried for as long
                    # as they last -- a child given up on is invisible to its shard's informer
                    if inf is not None and inf.get(ns, name, copy=False) is not None \
                            and not (child and persistent_failure(e) and self._give_up(key)):
                        self._queue.put_nowait(key)  # still unassigned: retry
                        continue
                if child:
                    self._child_finished(key, False)
                self._forget(key)
                continue
            except Exception as e:  # noqa: BLE001 - transport errors: retry, never give up
                self.errors += 1
                self.log.error(e, "Failed to assign shard", kind=gvk.kind, namespace=ns, name=name)
                await asyncio.sleep(self._backoff(key))
                self._queue.put_nowait(key)
                continue
            if child:
                self._child_finished(key, True)
            self._forget(key)

    def _backoff(self, key: Tuple[GroupVersionKind, str, str]) -> float:
        """Seconds to wait before retrying ``key``'s label PATCH: ``retry_delay`` doubled per
        failure of that key, capped at 32x (a long apiserver outage is not hammered)."""
        n = self._failures.get(key, 0)
        self._failures[key] = n + 1
        return self.retry_delay * (1 << min(n, 5))

    def _forget(self, key: Tuple[GroupVersionKind, str, str]) -> None:
        self._attempts.pop(key, None)
        self._failures.pop(key, None)
        self._queued.discard(key)

    def _give_up(self, key: Tuple[GroupVersionKind, str, str]) -> bool:
        """Count a persistently refused label PATCH of child ``key``; True once it reached
        ``max_child_attempts`` (the caller then releases the child's Cron, which is assigned
        without it)."""
        n = self._attempts.get(key, 0) + 1
        if n < self.max_child_attempts:
            self._attempts[key] = n
            return False
        self.abandoned += 1
        gvk, ns, name = key
        self.log.info("Giving up labelling a child; its Cron is assigned without it", kind=gvk.kind,
                      namespace=ns, name=name, attempts=n)
        return True
