"""In-process fake Kubernetes API server -- the framework's envtest.

The reference's integration tier runs a real kube-apiserver + etcd with no
controllers (``internal/controller/suite_test.go:53-124``).  Neither binary
exists here, so this module provides the same contract in-process:

* CRUD on any registered resource, namespaced or cluster-scoped; LIST with label
  and field selectors and limit/continue paging; a global etcd-like
  ``resourceVersion`` counter;
* WATCH with resume-from-resourceVersion out of a bounded event window (410
  Expired beyond it), synthetic ADDED events for ``rv=""/"0"``, and filtered
  watches that turn "stops matching" into DELETED like the watch cache;
* ``/status`` subresource semantics (main-resource writes ignore status, status
  writes ignore everything else), ``generation`` bumps on spec changes, and
  no-op writes that do not bump ``resourceVersion`` or emit events;
* JSON merge patch, JSON patch, optimistic concurrency (409 Conflict),
  AlreadyExists/NotFound, ``generateName``, finalizers + ``deletionTimestamp``;
* CRD installation through the API with structural-schema pruning, defaulting
  and validation (:mod:`.schema`);
* optional ownerReference garbage collection (background / foreground /
  orphan) -- envtest has none, so it is opt-in;
* fault injection and per-verb latency (:class:`FaultInjector`), and request
  accounting for the benchmark's API-request model;
* an injectable :class:`~cron_operator_amd.utils.clock.Clock` for timestamps.

Transports: :mod:`.http` serves it over the real Kubernetes REST paths;
:class:`cron_operator_amd.runtime.client.InMemoryTransport` calls it directly.
The core is synchronous and must be driven from one thread (one asyncio loop).
"""
from __future__ import annotations

import asyncio
import base64
import random
import string
import uuid
from collections import defaultdict, deque
from dataclasses import dataclass, field
from typing import Any, Callable, Deque, Dict, Iterable, List, Optional, Set, Tuple

from ..api import errors
from ..api.meta import GroupVersionResource
from ..api.selectors import compile_selectors
from ..utils import jsonutil
from ..utils.clock import Clock, RealClock
from ..utils.gotime import GoTime, UTC
from . import schema as sch
from .registry import ResourceInfo, builtin_resources, resources_from_crd

_NAME_CHARS = "bcdfghjklmnpqrstvwxz2456789"
_DNS1123_SUB = set(string.ascii_lowercase + string.digits + "-.")


def _ts(clock: Clock) -> str:
    return GoTime(clock.now_ns() // 1_000_000_000, 0, UTC).rfc3339()


# --------------------------------------------------------------------------- faults


@dataclass
class Fault:
    verb: str = "*"            # get list create update patch delete watch, or *
    resource: str = "*"        # plural resource name or *
    subresource: Optional[str] = None  # None = any
    code: int = 500
    reason: str = "InternalError"
    message: str = "injected fault"
    times: int = -1            # -1 = unlimited
    probability: float = 1.0
    name: Optional[str] = None
    # True: the verb is applied and *then* the error is returned -- a lost response
    # (timeout after commit), the case deterministic job names exist for
    after: bool = False
    retry_after: Optional[int] = None  # seconds: sent as Retry-After (APF-style 429 throttling)

    def matches(self, verb: str, resource: str, sub: Optional[str], name: Optional[str]) -> bool:
        if self.times == 0:
            return False
        if self.verb != "*" and self.verb != verb:
            return False
        if self.resource != "*" and self.resource != resource:
            return False
        if self.subresource is not None and self.subresource != (sub or ""):
            return False
        if self.name is not None and self.name != name:
            return False
        return True


class FaultInjector:
    """Per-verb error injection and latency (the reference has none), and watch lag.

    ``watch_lag[resource] = (min_s, max_s)`` (``"*"``: every resource) delays each event of a
    watch stream by a random ``min_s..max_s`` drawn per event from that stream's own generator:
    the Cron stream and the job streams fall behind independently, as a real apiserver's watch
    cache and a busy client's informers do.  A stream stays in order (an event never overtakes
    the one before it), and its end waits for what it still carries."""

    def __init__(self, seed: int = 0):
        self.faults: List[Fault] = []
        self.latency: Dict[str, float] = {}  # verb -> seconds ("*" default)
        self.watch_lag: Dict[str, Tuple[float, float]] = {}  # resource -> (min s, max s)
        self._rng = random.Random(seed)

    def lag_for(self, resource: str) -> Optional[Tuple[float, float]]:
        return self.watch_lag.get(resource) or self.watch_lag.get("*")

    def lag_rng(self) -> random.Random:
        """A generator of one watch stream's delays (seeded from this injector's)."""
        return random.Random(self._rng.random())

    def add(self, **kw: Any) -> Fault:
        f = Fault(**kw)
        self.faults.append(f)
        return f

    def clear(self) -> None:
        self.faults.clear()
        self.latency.clear()
        self.watch_lag.clear()

    def check(self, verb: str, resource: str, sub: Optional[str] = None, name: Optional[str] = None,
              after: bool = False) -> None:
        for f in self.faults:
            if f.after == after and f.matches(verb, resource, sub, name) and self._rng.random() < f.probability:
                if f.times > 0:
                    f.times -= 1
                raise errors.ApiError(f.code, f.reason, f.message, retry_after=f.retry_after)

    def delay_for(self, verb: str) -> float:
        return self.latency.get(verb, self.latency.get("*", 0.0))


# --------------------------------------------------------------------------- watch


class Watcher:
    """One WATCH stream.  Events are ``(type, object)``; ``None`` ends the stream."""

    def __init__(self, server: "APIServer", info: ResourceInfo, namespace: Optional[str],
                 pred: Callable[[Dict[str, Any]], bool], bookmarks: bool, copy_events: bool = True):
        self.copy_events = copy_events  # False: consumer serialises immediately (HTTP), stored objects are immutable
        self.server = server
        self.info = info
        self.namespace = namespace or None
        self.pred = pred
        self._match = getattr(pred, "_fn", pred)
        # label routing key of the selector (Selector.pinned): lets _emit skip watchers by index
        self.pinned: Optional[Tuple[str, str]] = getattr(pred, "pinned", None)
        # the selector reads only labels (+ the namespace above): an update that keeps both
        # cannot move the object in or out of scope
        self.labels_only = getattr(pred, "field_selector", None) == ""
        self.bookmarks = bookmarks
        self.queue: "asyncio.Queue[Optional[Tuple[str, Dict[str, Any]]]]" = asyncio.Queue()
        # set by a consumer that takes events synchronously (the HTTP front end): events go
        # straight to it instead of through the queue; ``None`` ends the stream
        self.sink: Optional[Callable[[Optional[Tuple[str, Dict[str, Any]]]], None]] = None
        self.closed = False
        # a stalled stream stays open but delivers nothing more -- no events, no bookmarks,
        # no end -- like a connection whose peer vanished without a FIN (fault injection)
        self.stalled = False
        self.sent = 0
        # watch lag (FaultInjector.watch_lag): events scheduled for later delivery, in order
        self.lagged = 0               # scheduled, not delivered yet
        self._lag_at = 0.0            # delivery time of the last scheduled event
        self._lag_rng: Optional[random.Random] = None
        self._lag_q: Deque[Tuple[float, Optional[Tuple[str, Dict[str, Any]]]]] = deque()
        self._lag_timer: Optional[asyncio.TimerHandle] = None

    def _in_scope(self, obj: Dict[str, Any]) -> bool:
        if self.namespace is not None and (obj.get("metadata") or {}).get("namespace") != self.namespace:
            return False
        return self._match(obj)

    def offer(self, etype: str, obj: Dict[str, Any], old: Optional[Dict[str, Any]]) -> None:
        if self.closed:
            return
        now_in = self._in_scope(obj)
        self.offer_scoped(etype, obj, old, now_in,
                          self._in_scope(old) if etype == "MODIFIED" and old is not None else False)

    def offer_scoped(self, etype: str, obj: Dict[str, Any], old: Optional[Dict[str, Any]], now_in: bool,
                     was_in: bool) -> None:
        """:meth:`offer` with the selector already evaluated on ``obj`` and ``old``."""
        if self.closed:
            return
        if etype == "MODIFIED" and old is not None:
            if was_in and not now_in:
                self._put("DELETED", obj)
            elif now_in and not was_in:
                self._put("ADDED", obj)
            elif now_in:
                self._put("MODIFIED", obj)
            return
        if now_in:
            self._put(etype, obj)

    def _put(self, etype: str, obj: Dict[str, Any]) -> None:
        if self.stalled:
            return
        self.sent += 1
        self._send((etype, jsonutil.deepcopy(obj) if self.copy_events else obj))

    def _send(self, ev: Optional[Tuple[str, Dict[str, Any]]]) -> None:
        """Deliver now, or -- under watch lag -- after this stream's next delay, never before an
        event already scheduled (a lagging stream is late, not reordered): one FIFO per stream,
        drained by one timer at its head (asyncio's timer heap does not keep equal deadlines in
        order)."""
        lag = self.server.faults.lag_for(self.info.resource) if self.server.faults.watch_lag else None
        if lag is None and not self.lagged:
            self._deliver(ev)
            return
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:
            self._deliver(ev)
            return
        if self._lag_rng is None:
            self._lag_rng = self.server.faults.lag_rng()
        lo, hi = lag if lag is not None else (0.0, 0.0)
        at = max(loop.time() + self._lag_rng.uniform(lo, hi), self._lag_at)
        self._lag_at = at
        self._lag_q.append((at, ev))
        self.lagged += 1
        if self._lag_timer is None:
            self._lag_timer = loop.call_at(at, self._drain_lagged)

    def _drain_lagged(self) -> None:
        self._lag_timer = None
        loop = asyncio.get_running_loop()
        now = loop.time()
        q = self._lag_q
        while q and q[0][0] <= now:
            _, ev = q.popleft()
            self.lagged -= 1
            if self.stalled and ev is not None:
                continue
            self._deliver(ev)
        if q:
            self._lag_timer = loop.call_at(q[0][0], self._drain_lagged)

    def _deliver(self, ev: Optional[Tuple[str, Dict[str, Any]]]) -> None:
        if self.sink is not None:
            self.sink(ev)
        else:
            self.queue.put_nowait(ev)

    def bookmark(self, rv: int) -> None:
        if self.bookmarks and not self.closed and not self.stalled:
            self._send(("BOOKMARK", {"kind": self.info.kind, "apiVersion": self.info.api_version,
                                     "metadata": {"resourceVersion": str(rv)}}))

    def stop(self) -> None:
        if not self.closed:
            self.closed = True
            self.server._remove_watcher(self)
            self._send(None)  # after what the stream still carries

    def __aiter__(self):
        return self

    async def __anext__(self) -> Tuple[str, Dict[str, Any]]:
        if self.closed and self.queue.empty() and not self.lagged:
            raise StopAsyncIteration
        ev = await self.queue.get()
        if ev is None:
            raise StopAsyncIteration
        return ev


# --------------------------------------------------------------------------- server


@dataclass
class RequestStats:
    by_verb: Dict[str, int] = field(default_factory=lambda: defaultdict(int))
    by_resource_verb: Dict[Tuple[str, str], int] = field(default_factory=lambda: defaultdict(int))
    total: int = 0

    def record(self, verb: str, resource: str) -> None:
        self.by_verb[verb] += 1
        self.by_resource_verb[(resource, verb)] += 1
        self.total += 1

    def snapshot(self) -> Dict[str, Any]:
        return {"total": self.total, "by_verb": dict(self.by_verb),
                "by_resource_verb": {f"{r}:{v}": n for (r, v), n in self.by_resource_verb.items()}}


class APIServer:
    def __init__(self, clock: Optional[Clock] = None, gc: bool = False, watch_window: int = 200_000,
                 auto_create_namespaces: bool = False, tokens: Optional[Dict[str, Dict[str, Any]]] = None,
                 authorization: str = "AlwaysAllow"):
        self.clock = clock or RealClock()
        self.gc_enabled = gc
        self.auto_create_namespaces = auto_create_namespaces
        self.faults = FaultInjector()
        self.stats = RequestStats()
        # bearer token -> user info ({"username", "groups"}); None disables authn in HTTP mode
        self.tokens = tokens
        self.authorizer: Optional[Callable[[Dict[str, Any], Dict[str, Any]], bool]] = None
        # "RBAC": HTTP requests are authorized against stored (Cluster)Roles/Bindings
        self.rbac = None
        if authorization == "RBAC":
            from .rbac import RBACAuthorizer

            self.rbac = RBACAuthorizer(self)
            self.authorizer = self.rbac
        elif authorization != "AlwaysAllow":
            raise ValueError(f"unknown authorization mode {authorization!r}")
        self._rv = 0
        self._resources: Dict[Tuple[str, str, str], ResourceInfo] = {}
        self._by_kind: Dict[Tuple[str, str, str], ResourceInfo] = {}
        # (group, resource) -> namespace -> name -> stored object (never mutated in place)
        self._data: Dict[Tuple[str, str], Dict[str, Dict[str, Dict[str, Any]]]] = defaultdict(dict)
        # (group, resource) -> label key -> value -> namespace -> names: the label index a LIST
        # that pins key=value reads instead of scanning the namespace (_label_index)
        self._label_idx: Dict[Tuple[str, str], Dict[str, Dict[str, Dict[str, Set[str]]]]] = {}
        self._watchers: Dict[Tuple[str, str], List[Watcher]] = defaultdict(list)
        # per resource: (selector groups to always check, {label key: {value: groups pinned to it}})
        self._watch_plan: Dict[Tuple[str, str], Any] = {}
        self._log: Dict[Tuple[str, str], Deque[Tuple[int, str, Dict[str, Any], Optional[Dict[str, Any]]]]] = {}
        self._log_floor: Dict[Tuple[str, str], int] = defaultdict(int)
        self._watch_window = watch_window
        self._owners: Dict[str, Set[Tuple[str, str, str, str]]] = defaultdict(set)  # owner uid -> dependents
        self._gc_pending: List[Tuple[str, str]] = []
        self.create_hooks: List[Callable[[ResourceInfo, Dict[str, Any]], None]] = []
        self._compiled_schemas: Dict[Tuple[str, str, str, int], Tuple[Any, Any]] = {}
        # verbs return deep copies unless a caller that serialises immediately opts out
        self.copy_responses = True
        # verbs copy their input bodies unless the caller hands over private, never-reused
        # objects (the HTTP front end: every body is freshly decoded for the request)
        self.copy_inputs = True
        self._rng = random.Random(7)
        for ri in builtin_resources():
            self.register(ri)
        for ns in ("default", "kube-system", "kube-public", "kube-node-lease"):
            self._put_raw(self._resources[("", "v1", "namespaces")], "", self._new_namespace(ns))

    # ------------------------------------------------------------------ registry
    def register(self, ri: ResourceInfo) -> None:
        self._resources[(ri.group, ri.version, ri.resource)] = ri
        self._by_kind[(ri.group, ri.version, ri.kind)] = ri

    def resources(self) -> List[ResourceInfo]:
        return list(self._resources.values())

    def resource(self, gvr: GroupVersionResource) -> ResourceInfo:
        ri = self._resources.get((gvr.group, gvr.version, gvr.resource))
        if ri is None:
            raise errors.ApiError(404, "NotFound", f"the server could not find the requested resource "
                                                   f"({gvr.resource}.{gvr.group})" if gvr.group else
                                  f"the server could not find the requested resource ({gvr.resource})")
        return ri


    def install_crd(self, crd: Dict[str, Any]) -> Dict[str, Any]:
        """Create (or replace) a CRD object and register its resources."""
        ri = self._resources[("apiextensions.k8s.io", "v1", "customresourcedefinitions")]
        name = (crd.get("metadata") or {}).get("name", "")
        existing = self._get_raw(ri, "", name)
        if existing is None:
            return self.create(ri.gvr, "", crd)
        body = jsonutil.deepcopy(crd)
        body.setdefault("metadata", {})["resourceVersion"] = existing["metadata"]["resourceVersion"]
        return self.update(ri.gvr, "", name, body)

    def _on_crd_written(self, crd: Dict[str, Any]) -> None:
        for r in resources_from_crd(crd):
            self.register(r)
        # mark Established like the real apiextensions controller
        st = crd.setdefault("status", {})
        st["conditions"] = [{"type": "NamesAccepted", "status": "True", "reason": "NoConflicts"},
                            {"type": "Established", "status": "True", "reason": "InitialNamesAccepted"}]
        st["acceptedNames"] = dict((crd.get("spec") or {}).get("names") or {})

    # ------------------------------------------------------------------ helpers
    def current_rv(self) -> int:
        return self._rv

    def _next_rv(self) -> int:
        self._rv += 1
        return self._rv

    def _bucket(self, ri: ResourceInfo) -> Dict[str, Dict[str, Dict[str, Any]]]:
        return self._data[(ri.group, ri.resource)]

    def _get_raw(self, ri: ResourceInfo, ns: str, name: str) -> Optional[Dict[str, Any]]:
        return self._bucket(ri).get(ns if ri.namespaced else "", {}).get(name)

    def _put_raw(self, ri: ResourceInfo, ns: str, obj: Dict[str, Any]) -> None:
        ns = ns if ri.namespaced else ""
        objs = self._bucket(ri).setdefault(ns, {})
        name = obj["metadata"]["name"]
        old = objs.get(name)
        objs[name] = obj
        idx = self._label_idx.get((ri.group, ri.resource))
        if idx:
            self._reindex(idx, ns, name, old, obj)

    @staticmethod
    def _reindex(idx: Dict[str, Dict[str, Dict[str, Set[str]]]], ns: str, name: str,
                 old: Optional[Dict[str, Any]], new: Optional[Dict[str, Any]]) -> None:
        """Move ``ns/name`` between the label-index sets of every indexed key whose value changed."""
        ol = ((old.get("metadata") or {}).get("labels") or {}) if old is not None else None
        nl = ((new.get("metadata") or {}).get("labels") or {}) if new is not None else None
        if ol is not None and nl is not None and (ol is nl or ol == nl):
            return
        for key, by_val in idx.items():
            ov = ol.get(key) if ol is not None else None
            nv = nl.get(key) if nl is not None else None
            if ov == nv and ol is not None and nl is not None:
                continue
            if ov is not None:
                s = by_val.get(ov, {}).get(ns)
                if s is not None:
                    s.discard(name)
            if nv is not None:
                by_val.setdefault(nv, {}).setdefault(ns, set()).add(name)

    def _label_index(self, ri: ResourceInfo, key: str) -> Dict[str, Dict[str, Set[str]]]:
        """``value -> namespace -> names`` of the objects labelled ``key`` (built on first use by
        a LIST that pins ``key=value``, then kept up to date by every write)."""
        idx = self._label_idx.setdefault((ri.group, ri.resource), {})
        by_val = idx.get(key)
        if by_val is None:
            by_val = idx[key] = {}
            for ns, objs in self._bucket(ri).items():
                for name, obj in objs.items():
                    v = ((obj.get("metadata") or {}).get("labels") or {}).get(key)
                    if v is not None:
                        by_val.setdefault(v, {}).setdefault(ns, set()).add(name)
        return by_val

    def _new_namespace(self, name: str) -> Dict[str, Any]:
        return {"apiVersion": "v1", "kind": "Namespace",
                "metadata": {"name": name, "uid": str(uuid.uuid4()), "resourceVersion": str(self._next_rv()),
                             "creationTimestamp": _ts(self.clock)},
                "spec": {"finalizers": ["kubernetes"]}, "status": {"phase": "Active"}}

    def _check_namespace(self, ri: ResourceInfo, ns: str) -> None:
        if not ri.namespaced:
            return
        if not ns:
            raise errors.bad_request("an empty namespace may not be set during creation")
        nsri = self._resources[("", "v1", "namespaces")]
        if self._get_raw(nsri, "", ns) is None:
            if self.auto_create_namespaces:
                self._put_raw(nsri, "", self._new_namespace(ns))
                return
            raise errors.not_found("namespaces", "", ns)

    def _emit(self, ri: ResourceInfo, etype: str, obj: Dict[str, Any], old: Optional[Dict[str, Any]],
              rv: int) -> None:
        key = (ri.group, ri.resource)
        log = self._log.get(key)
        if log is None:
            log = self._log[key] = deque()
        log.append((rv, etype, obj, old))
        if len(log) > self._watch_window:
            dropped = log.popleft()
            self._log_floor[key] = dropped[0]
        ws = self._watchers.get(key)
        if not ws:
            return
        plan = self._watch_plan.get(key)
        if plan is None:
            plan = self._watch_plan[key] = self._plan(ws)
        plain, pinned = plan
        groups = plain
        modified = etype == "MODIFIED" and old is not None
        if pinned:
            # watchers whose selector pins a label value only see objects carrying it (before or after)
            groups = list(plain)
            labels = (obj.get("metadata") or {}).get("labels") or {}
            old_labels = ((old.get("metadata") or {}).get("labels") or {}) if modified else None
            for lk, by_value in pinned.items():
                v = labels.get(lk)
                hit = by_value.get(v)
                if hit:
                    groups.extend(hit)
                if old_labels is not None:
                    ov = old_labels.get(lk)
                    if ov != v:
                        hit = by_value.get(ov)
                        if hit:
                            groups.extend(hit)
        same_scope = False
        if modified:
            om = old.get("metadata") or {}  # type: ignore[union-attr]
            nm = obj.get("metadata") or {}
            ol, nl = om.get("labels"), nm.get("labels")
            same_scope = (ol is nl or ol == nl) and om.get("namespace") == nm.get("namespace")
        # one selector evaluation per (namespace, selector) group per event
        for first, members in groups:
            now_in = first._in_scope(obj)
            if not modified:
                was_in = False
            elif same_scope and first.labels_only:
                was_in = now_in
            else:
                was_in = first._in_scope(old)  # type: ignore[arg-type]
            if now_in or was_in:
                for w in members:
                    w.offer_scoped(etype, obj, old, now_in, was_in)

    @staticmethod
    def _plan(ws: List[Watcher]) -> Tuple[List[Tuple[Watcher, List[Watcher]]],
                                         Dict[str, Dict[str, List[Tuple[Watcher, List[Watcher]]]]]]:
        """Watchers grouped by (namespace, selector); groups with a pinned label value indexed
        by it.  A group is ``(representative, members)``."""
        by_sel: Dict[Tuple[Optional[str], Any], List[Watcher]] = {}
        for w in ws:
            by_sel.setdefault((w.namespace, w.pred), []).append(w)
        plain: List[Tuple[Watcher, List[Watcher]]] = []
        pinned: Dict[str, Dict[str, List[Tuple[Watcher, List[Watcher]]]]] = {}
        for members in by_sel.values():
            first = members[0]
            if first.pinned is None:
                plain.append((first, members))
            else:
                pinned.setdefault(first.pinned[0], {}).setdefault(first.pinned[1], []).append((first, members))
        return plain, pinned

    def _remove_watcher(self, w: Watcher) -> None:
        key = (w.info.group, w.info.resource)
        lst = self._watchers.get(key)
        if lst and w in lst:
            lst.remove(w)
            self._watch_plan.pop(key, None)

    def _index_owners(self, ri: ResourceInfo, obj: Optional[Dict[str, Any]], old: Optional[Dict[str, Any]]) -> None:
        if old is not None and obj is not None:
            om, nm = old.get("metadata") or {}, obj.get("metadata") or {}
            oo, no = om.get("ownerReferences"), nm.get("ownerReferences")
            if (oo is no or oo == no) and om.get("name") == nm.get("name"):
                return  # an update that keeps its owners (status writes): nothing to re-file
        if old is not None:
            m = old.get("metadata") or {}
            ref = (ri.group, ri.resource, m.get("namespace", ""), m.get("name", ""))
            for o in m.get("ownerReferences") or []:
                s = self._owners.get(o.get("uid", ""))
                if s is not None:
                    s.discard(ref)
        if obj is not None:
            m = obj.get("metadata") or {}
            ref = (ri.group, ri.resource, m.get("namespace", ""), m.get("name", ""))
            for o in m.get("ownerReferences") or []:
                self._owners[o.get("uid", "")].add(ref)

    def _out(self, obj: Dict[str, Any]) -> Dict[str, Any]:
        """Response object: a private copy, or the stored (immutable) object itself when the
        caller serialises it straight away (HTTP front end)."""
        return jsonutil.deepcopy(obj) if self.copy_responses else obj

    def _compiled(self, ri: ResourceInfo) -> Tuple[sch.CompiledSchema, Optional[sch.CompiledSchema]]:
        key = (ri.group, ri.version, ri.resource, id(ri.schema))
        hit = self._compiled_schemas.get(key)
        if hit is None:
            st = ((ri.schema or {}).get("properties") or {}).get("status")
            hit = (sch.CompiledSchema(ri.schema or {}, root=True),
                   sch.CompiledSchema(st, root=False) if isinstance(st, dict) else None)
            self._compiled_schemas[key] = hit
        return hit

    def _admit(self, ri: ResourceInfo, obj: Dict[str, Any], name: str) -> None:
        if ri.schema is not None:
            if self._compiled(ri)[0](obj):
                return
            errs = sch.validate(obj, ri.schema)
            if errs:
                raise errors.invalid(ri.kind, ri.group, name, errs)

    def _admit_status(self, ri: ResourceInfo, obj: Dict[str, Any], name: str,
                      old_status: Any = None) -> None:
        """Status-subresource writes only change ``status``: admit just that subtree (and of it,
        only the fields not shared by identity with the already-admitted old status)."""
        st_schema = ((ri.schema or {}).get("properties") or {}).get("status")
        if st_schema is None:
            return
        st = obj["status"]
        fast = self._compiled(ri)[1]
        if fast is not None and (fast.check_changed(st, old_status) if old_status is not None else fast(st)):
            return
        errs = sch.validate(st, st_schema, "status")
        if errs:
            raise errors.invalid(ri.kind, ri.group, name, errs)

    def _validate_name(self, ri: ResourceInfo, name: str) -> None:
        if not name:
            raise errors.invalid(ri.kind, ri.group, name, [{"field": "metadata.name", "reason": "FieldValueRequired",
                                                           "message": "Required value: name or generateName is "
                                                                      "required"}])
        bad = (len(name) > 253 or any(c not in _DNS1123_SUB for c in name) or not name[0].isalnum()
               or not name[-1].isalnum())
        if bad and ri.kind not in ("Event",):
            raise errors.invalid(ri.kind, ri.group, name, [{
                "field": "metadata.name", "reason": "FieldValueInvalid",
                "message": f'Invalid value: "{name}": a lowercase RFC 1123 subdomain must consist of lower case '
                           f"alphanumeric characters, '-' or '.', and must start and end with an alphanumeric "
                           f"character"}])

    # ------------------------------------------------------------------ verbs
    def get(self, gvr: GroupVersionResource, namespace: str, name: str) -> Dict[str, Any]:
        ri = self.resource(gvr)
        self.stats.record("get", ri.resource)
        obj = self._get_raw(ri, namespace, name)
        if obj is None:
            raise errors.not_found(ri.resource, ri.group, name)
        return self._out(obj)

    def list(self, gvr: GroupVersionResource, namespace: Optional[str] = None, label_selector: Optional[str] = None,
             field_selector: Optional[str] = None, limit: int = 0, continue_: Optional[str] = None,
             copy: bool = True) -> Dict[str, Any]:
        ri = self.resource(gvr)
        self.stats.record("list", ri.resource)
        pred = compile_selectors(label_selector, field_selector)
        bucket = self._bucket(ri)
        if ri.namespaced and namespace:
            spaces = [namespace]
        else:
            spaces = sorted(bucket.keys())
        start_after = None
        list_rv = self._rv
        if continue_:
            try:
                tok = jsonutil.loads(base64.urlsafe_b64decode(continue_.encode()).decode())
                start_after = tok["k"]
                list_rv = int(tok["rv"])
            except Exception:
                raise errors.bad_request("invalid continue token") from None
        items: List[Dict[str, Any]] = []
        more = None
        pin = pred.pinned
        by_ns = self._label_index(ri, pin[0]).get(pin[1], {}) if pin is not None else None
        for ns in spaces:
            objs = bucket.get(ns) or {}
            names = objs.keys() if by_ns is None else by_ns.get(ns, ())
            # index hits in key order, as etcd returns a range (and as paging needs)
            for name in sorted(names) if (limit or continue_ or by_ns is not None) else names:
                if start_after is not None and f"{ns}/{name}" <= start_after:
                    continue
                obj = objs[name]
                if not pred(obj):
                    continue
                if limit and len(items) >= limit:
                    more = f"{ns}/{name}"
                    break
                items.append(jsonutil.deepcopy(obj) if (copy and self.copy_responses) else obj)
            if more:
                break
        meta: Dict[str, Any] = {"resourceVersion": str(list_rv)}
        if more is not None:
            last = items[-1]["metadata"]
            tok = {"k": f"{last.get('namespace', '')}/{last['name']}", "rv": list_rv}
            meta["continue"] = base64.urlsafe_b64encode(jsonutil.dumpb(tok)).decode()
            meta["remainingItemCount"] = 0
        return {"apiVersion": ri.api_version, "kind": ri.list_kind, "metadata": meta, "items": items}

    def create(self, gvr: GroupVersionResource, namespace: str, obj: Dict[str, Any],
               dry_run: bool = False) -> Dict[str, Any]:
        ri = self.resource(gvr)
        self.stats.record("create", ri.resource)
        body = jsonutil.deepcopy(obj) if self.copy_inputs else obj
        m = body.get("metadata")
        if not isinstance(m, dict):
            m = body["metadata"] = {}
        if ri.namespaced:
            bns = m.get("namespace", "")
            if bns and namespace and bns != namespace:
                raise errors.bad_request("the namespace of the provided object does not match the namespace "
                                         "sent on the request")
            namespace = namespace or bns
            m["namespace"] = namespace
        else:
            m.pop("namespace", None)
            namespace = ""
        if ri.virtual:
            return self._review(ri, body)
        body["apiVersion"] = ri.api_version
        body["kind"] = ri.kind
        name = m.get("name", "")
        if not name and m.get("generateName"):
            for _ in range(16):
                cand = m["generateName"] + "".join(self._rng.choice(_NAME_CHARS) for _ in range(5))
                if self._get_raw(ri, namespace, cand) is None:
                    name = cand
                    break
            m["name"] = name
        self._validate_name(ri, name)
        self._check_namespace(ri, namespace)
        if self._get_raw(ri, namespace, name) is not None:
            raise errors.already_exists(ri.resource, ri.group, name)
        if ri.status_subresource and ri.is_crd:
            body.pop("status", None)
        self._admit(ri, body, name)
        for k in ("resourceVersion", "deletionTimestamp", "deletionGracePeriodSeconds", "selfLink"):
            m.pop(k, None)
        m["uid"] = str(uuid.uuid4())
        m["creationTimestamp"] = _ts(self.clock)
        m["generation"] = 1
        for hook in self.create_hooks:
            hook(ri, body)
        if dry_run:
            return body
        rv = self._next_rv()
        m["resourceVersion"] = str(rv)
        if ri.kind == "CustomResourceDefinition":
            self._on_crd_written(body)
        self._put_raw(ri, namespace, body)
        self._index_owners(ri, body, None)
        self._emit(ri, "ADDED", body, None, rv)
        return self._out(body)

    def _review(self, ri: ResourceInfo, body: Dict[str, Any]) -> Dict[str, Any]:
        body["apiVersion"] = ri.api_version
        body["kind"] = ri.kind
        spec = body.get("spec") or {}
        if ri.kind == "TokenReview":
            user = (self.tokens or {}).get(spec.get("token", ""))
            body["status"] = {"authenticated": user is not None, "user": user or {}}
        elif ri.kind == "SubjectAccessReview":
            allowed = True
            if self.authorizer is not None:
                allowed = bool(self.authorizer({"user": spec.get("user"), "groups": spec.get("groups")}, spec))
            body["status"] = {"allowed": allowed}
        return body

    def _finish_write(self, ri: ResourceInfo, ns: str, name: str, old: Dict[str, Any],
                      new: Dict[str, Any]) -> Dict[str, Any]:
        """Store ``new`` unless it equals ``old`` (no-op writes keep the RV, emit nothing)."""
        nm = new["metadata"]
        nm["resourceVersion"] = old["metadata"]["resourceVersion"]
        if jsonutil.json_equal(old, new):
            return self._out(old)
        # finalizers drained on a terminating object -> delete it now
        if nm.get("deletionTimestamp") and not nm.get("finalizers"):
            return self._remove(ri, ns, name, old)
        rv = self._next_rv()
        nm["resourceVersion"] = str(rv)
        if ri.kind == "CustomResourceDefinition":
            self._on_crd_written(new)
        self._put_raw(ri, ns, new)
        self._index_owners(ri, new, old)
        self._emit(ri, "MODIFIED", new, old, rv)
        return self._out(new)

    def _prepare_update(self, ri: ResourceInfo, old: Dict[str, Any], body: Dict[str, Any],
                        subresource: Optional[str]) -> Dict[str, Any]:
        om = old["metadata"]
        if subresource == "status":
            new = dict(old)  # shallow: only "status" is replaced, the rest is shared immutable storage
            new["metadata"] = dict(old["metadata"])
            if "status" in body:
                new["status"] = body["status"]
            else:
                new.pop("status", None)
            if ri.schema is not None and new.get("status") is not None:
                self._admit_status(ri, new, om["name"], old.get("status"))
            return new
        if subresource not in (None, ""):
            raise errors.ApiError(404, "NotFound", f"the server could not find the requested resource "
                                                   f"({subresource})")
        new = body
        new["apiVersion"] = ri.api_version
        new["kind"] = ri.kind
        nm = new.setdefault("metadata", {})
        # immutable / server-owned metadata
        for k in ("uid", "creationTimestamp", "namespace", "name", "generation", "deletionTimestamp",
                  "deletionGracePeriodSeconds"):
            if k in om:
                nm[k] = om[k]
            else:
                nm.pop(k, None)
        if ri.status_subresource:
            if "status" in old:
                new["status"] = old["status"]
            else:
                new.pop("status", None)
        self._admit(ri, new, om["name"])
        spec_changed = any(not jsonutil.json_equal(old.get(k), new.get(k))
                           for k in set(old) | set(new) if k not in ("metadata", "status", "apiVersion", "kind"))
        if spec_changed:
            nm["generation"] = int(om.get("generation", 1)) + 1
        return new

    def update(self, gvr: GroupVersionResource, namespace: str, name: str, obj: Dict[str, Any],
               subresource: Optional[str] = None) -> Dict[str, Any]:
        ri = self.resource(gvr)
        self.stats.record("update", ri.resource)
        ns = namespace if ri.namespaced else ""
        old = self._get_raw(ri, ns, name)
        body = jsonutil.deepcopy(obj) if self.copy_inputs else obj
        bm = body.get("metadata") or {}
        if bm.get("name") and bm["name"] != name:
            raise errors.bad_request("the name of the object does not match the name on the URL")
        if old is None:
            raise errors.not_found(ri.resource, ri.group, name)
        rv = bm.get("resourceVersion", "")
        if rv and rv != old["metadata"]["resourceVersion"]:
            raise errors.conflict(ri.resource, ri.group, name, "the object has been modified; please apply your "
                                                              "changes to the latest version and try again")
        new = self._prepare_update(ri, old, body, subresource)
        return self._finish_write(ri, ns, name, old, new)

    def patch(self, gvr: GroupVersionResource, namespace: str, name: str, patch: Any,
              patch_type: str = "merge", subresource: Optional[str] = None) -> Dict[str, Any]:
        ri = self.resource(gvr)
        self.stats.record("patch", ri.resource)
        ns = namespace if ri.namespaced else ""
        old = self._get_raw(ri, ns, name)
        if old is None:
            raise errors.not_found(ri.resource, ri.group, name)
        if patch_type in ("merge", "strategic"):
            if patch_type == "strategic" and ri.is_crd:
                raise errors.ApiError(415, "UnsupportedMediaType", "the body of the request was in an unknown "
                                                                   "format - accepted media types include: "
                                                                   "application/json-patch+json, "
                                                                   "application/merge-patch+json")
            if not isinstance(patch, dict):
                raise errors.bad_request("merge patch must be a JSON object")
            # stored objects are never mutated in place, so a status merge shares untouched subtrees
            # (the status path copies metadata and admits only the status); a main-resource patch
            # may be pruned/defaulted in place, so it gets a private tree
            share = not self.copy_inputs and subresource == "status"
            merged = jsonutil.apply_merge_patch(old, patch, share=share)
            if share:
                merged["metadata"] = dict(merged.get("metadata") or {})
        elif patch_type == "json":
            try:
                merged = jsonutil.apply_json_patch(old, patch)
            except (KeyError, IndexError, ValueError, TypeError) as e:
                raise errors.ApiError(422, "Invalid", f"the server rejected our request due to an error in our "
                                                      f"request: {e}") from None
        else:
            raise errors.ApiError(415, "UnsupportedMediaType", f"unsupported patch type {patch_type}")
        pm = (patch.get("metadata") or {}) if isinstance(patch, dict) else {}
        prv = pm.get("resourceVersion")
        if prv and prv != old["metadata"]["resourceVersion"]:
            raise errors.conflict(ri.resource, ri.group, name, "the object has been modified; please apply your "
                                                              "changes to the latest version and try again")
        merged.setdefault("metadata", {})["resourceVersion"] = old["metadata"]["resourceVersion"]
        new = self._prepare_update(ri, old, merged, subresource)
        return self._finish_write(ri, ns, name, old, new)

    def delete(self, gvr: GroupVersionResource, namespace: str, name: str,
               propagation_policy: Optional[str] = None,
               preconditions: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
        ri = self.resource(gvr)
        self.stats.record("delete", ri.resource)
        ns = namespace if ri.namespaced else ""
        old = self._get_raw(ri, ns, name)
        if old is None:
            raise errors.not_found(ri.resource, ri.group, name)
        om = old["metadata"]
        if preconditions:
            if preconditions.get("uid") and preconditions["uid"] != om.get("uid"):
                raise errors.conflict(ri.resource, ri.group, name,
                                      f"Precondition failed: UID in precondition: {preconditions['uid']}, "
                                      f"UID in object meta: {om.get('uid')}")
            if preconditions.get("resourceVersion") and preconditions["resourceVersion"] != om.get("resourceVersion"):
                raise errors.conflict(ri.resource, ri.group, name, "Precondition failed: ResourceVersion mismatch")
        finalizers = list(om.get("finalizers") or [])
        policy = propagation_policy or "Background"
        if policy == "Foreground" and self.gc_enabled and self._owners.get(om.get("uid", "")):
            finalizers.append("foregroundDeletion")
        if policy == "Orphan" and self.gc_enabled:
            self._orphan_dependents(om.get("uid", ""))
        if finalizers:
            if om.get("deletionTimestamp"):
                return self._out(old)
            new = jsonutil.deepcopy(old)
            new["metadata"]["deletionTimestamp"] = _ts(self.clock)
            new["metadata"]["deletionGracePeriodSeconds"] = 0
            new["metadata"]["finalizers"] = finalizers
            rv = self._next_rv()
            new["metadata"]["resourceVersion"] = str(rv)
            self._put_raw(ri, ns, new)
            self._emit(ri, "MODIFIED", new, old, rv)
            if "foregroundDeletion" in finalizers:
                self._schedule_gc(ri, new)
            return self._out(new)
        return self._remove(ri, ns, name, old)

    def _remove(self, ri: ResourceInfo, ns: str, name: str, old: Dict[str, Any]) -> Dict[str, Any]:
        self._bucket(ri).get(ns, {}).pop(name, None)
        idx = self._label_idx.get((ri.group, ri.resource))
        if idx:
            self._reindex(idx, ns if ri.namespaced else "", name, old, None)
        rv = self._next_rv()
        # stored objects are immutable: the tombstone shares everything but its metadata
        gone_obj = dict(old)
        gone_obj["metadata"] = dict(old["metadata"])
        gone_obj["metadata"]["resourceVersion"] = str(rv)
        self._index_owners(ri, None, old)
        self._emit(ri, "DELETED", gone_obj, None, rv)
        if self.gc_enabled:
            self._schedule_gc(ri, old)
        return self._out(gone_obj)

    def delete_collection(self, gvr: GroupVersionResource, namespace: Optional[str],
                          label_selector: Optional[str] = None) -> int:
        lst = self.list(gvr, namespace, label_selector, copy=False)
        n = 0
        for item in lst["items"]:
            m = item["metadata"]
            try:
                self.delete(gvr, m.get("namespace", ""), m["name"])
                n += 1
            except errors.ApiError:
                pass
        return n

    # ------------------------------------------------------------------ garbage collection
    def _schedule_gc(self, ri: ResourceInfo, owner: Dict[str, Any]) -> None:
        uid = (owner.get("metadata") or {}).get("uid", "")
        if not uid:
            return
        self._gc_pending.append((uid, (owner.get("metadata") or {}).get("name", "")))
        try:
            loop = asyncio.get_running_loop()
            loop.call_soon(self.run_gc)
        except RuntimeError:
            self.run_gc()

    def run_gc(self) -> int:
        """Process pending owner deletions; returns the number of dependents deleted."""
        n = 0
        while self._gc_pending:
            uid, _ = self._gc_pending.pop(0)
            for (g, r, ns, name) in list(self._owners.get(uid, ())):
                ri = next((x for x in self._resources.values() if x.group == g and x.resource == r), None)
                if ri is None:
                    continue
                dep = self._get_raw(ri, ns, name)
                if dep is None:
                    continue
                refs = (dep.get("metadata") or {}).get("ownerReferences") or []
                # only collect when no other live owner remains
                others = [o for o in refs if o.get("uid") != uid and self._owner_alive(o, ns)]
                if others:
                    continue
                try:
                    self.delete(ri.gvr, ns, name, propagation_policy="Background")
                    n += 1
                except errors.ApiError:
                    pass
            self._owners.pop(uid, None)
            self._finish_foreground(uid)
        return n

    def _owner_alive(self, ref: Dict[str, Any], ns: str) -> bool:
        for ri in self._resources.values():
            if ri.kind == ref.get("kind") and ri.api_version == ref.get("apiVersion"):
                o = self._get_raw(ri, ns, ref.get("name", ""))
                return o is not None and o["metadata"].get("uid") == ref.get("uid")
        return False

    def _finish_foreground(self, uid: str) -> None:
        for (g, r), spaces in self._data.items():
            for ns, objs in spaces.items():
                for name, obj in list(objs.items()):
                    m = obj["metadata"]
                    if m.get("uid") == uid and "foregroundDeletion" in (m.get("finalizers") or []):
                        ri = next(x for x in self._resources.values() if x.group == g and x.resource == r)
                        new = jsonutil.deepcopy(obj)
                        new["metadata"]["finalizers"] = [f for f in m["finalizers"] if f != "foregroundDeletion"]
                        self._finish_write(ri, ns, name, obj, new)
                        return

    def _orphan_dependents(self, uid: str) -> None:
        for (g, r, ns, name) in list(self._owners.get(uid, ())):
            ri = next((x for x in self._resources.values() if x.group == g and x.resource == r), None)
            if ri is None:
                continue
            dep = self._get_raw(ri, ns, name)
            if dep is None:
                continue
            new = jsonutil.deepcopy(dep)
            new["metadata"]["ownerReferences"] = [o for o in new["metadata"].get("ownerReferences") or []
                                                  if o.get("uid") != uid]
            if not new["metadata"]["ownerReferences"]:
                del new["metadata"]["ownerReferences"]
            self._finish_write(ri, ns, name, dep, new)
        self._owners.pop(uid, None)

    # ------------------------------------------------------------------ watch
    def watch(self, gvr: GroupVersionResource, namespace: Optional[str] = None, resource_version: str = "",
              label_selector: Optional[str] = None, field_selector: Optional[str] = None,
              allow_bookmarks: bool = False, send_initial_events: Optional[bool] = None,
              copy_events: bool = True) -> Watcher:
        ri = self.resource(gvr)
        self.stats.record("watch", ri.resource)
        pred = compile_selectors(label_selector, field_selector)
        w = Watcher(self, ri, namespace if ri.namespaced else None, pred, allow_bookmarks, copy_events)
        key = (ri.group, ri.resource)
        if resource_version in ("", "0") or send_initial_events:
            for ns, objs in self._bucket(ri).items():
                if w.namespace is not None and ns != w.namespace:
                    continue
                for obj in objs.values():
                    if pred(obj):
                        w._put("ADDED", obj)
        else:
            try:
                since = int(resource_version)
            except ValueError:
                raise errors.bad_request(f"invalid resourceVersion {resource_version!r}") from None
            floor = self._log_floor.get(key, 0)
            if since < floor:
                raise errors.gone(f"too old resource version: {since} ({floor + 1})")
            for (rv, etype, obj, old) in self._log.get(key, ()):
                if rv > since:
                    w.offer(etype, obj, old)
        self._watchers[key].append(w)
        self._watch_plan.pop(key, None)
        return w

    def send_bookmarks(self) -> None:
        for lst in self._watchers.values():
            for w in lst:
                w.bookmark(self._rv)

    def stall_watches(self, resource: Optional[str] = None) -> int:
        """Silently stall the open watches (of one plural resource, or all): they deliver
        nothing more and are never ended by the server.  Returns how many were stalled."""
        n = 0
        for (_, res), lst in self._watchers.items():
            if resource is None or res == resource:
                for w in lst:
                    if not w.stalled:
                        w.stalled = True
                        n += 1
        return n

    def close_all_watches(self) -> None:
        for lst in list(self._watchers.values()):
            for w in list(lst):
                w.stop()

    # ------------------------------------------------------------------ conveniences
    def create_namespace(self, name: str) -> Dict[str, Any]:
        ri = self._resources[("", "v1", "namespaces")]
        if self._get_raw(ri, "", name) is not None:
            return jsonutil.deepcopy(self._get_raw(ri, "", name))
        return self.create(ri.gvr, "", {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": name}})

    def objects(self, gvr: GroupVersionResource, namespace: Optional[str] = None) -> Iterable[Dict[str, Any]]:
        """Read-only view of stored objects (no copies; do not mutate)."""
        ri = self.resource(gvr)
        for ns, objs in self._bucket(ri).items():
            if namespace is None or ns == namespace:
                yield from objs.values()

    def count(self, gvr: GroupVersionResource, namespace: Optional[str] = None) -> int:
        ri = self.resource(gvr)
        if namespace is not None:
            return len(self._bucket(ri).get(namespace, {}))
        return sum(len(v) for v in self._bucket(ri).values())
