"""CronReconciler -- the controller logic (reference layer L4).

Reference: ``internal/controller/cron_controller.go:48-437``.  The reconcile
algorithm and its observable behaviour are
reproduced step by step; each step below cites the reference lines.

Where this implementation deliberately differs from the reference, the
difference is a :class:`ReconcilerOptions` switch and
``ReconcilerOptions.reference()`` restores the reference behaviour exactly
(the benchmark's "reference mode" uses it):

=========================  =====================================  =======================================
option                     default here                           reference
=========================  =====================================  =======================================
``list_mode``              ``cache``: children from a label-      ``live``: LIST on every reconcile
                           indexed informer (+ expectations)      (``cron_controller.go:241-266``)
``finished_time``          ``completion``: the job's own           ``now``: ``metav1.Now()`` on every
                           completion time, else first seen       reconcile (Appendix B #3)
``skip_noop_patch``        no PATCH when the merge patch is empty  PATCH sent whenever DeepEqual differs
``own_write_filter``       our own status writes do not requeue   every Cron update requeues (B22)
``workload``               Pod/batch Job/MPIJob adapters on        kubeflow conditions only (B5, App. B #6-7)
``dynamic_watches``        watch whatever kind templates use      PyTorchJob + TFJob only (B22)
``dedupe_ran_tick``        a tick whose job already exists is     the tick runs again when the status
                           recorded, not run again                 write after its CREATE was lost
``overlap_gc_deletes``     history-GC DELETEs run concurrently    each DELETE awaited in turn, before
                           with the rest of the reconcile          the CREATE and the status PATCH
``slim_child_cache``       cached children keep metadata, kind    typed informers cache whole objects
                           and status (``spec`` is never read);    (``Owns(&PyTorchJob{})``)
                           cached Crons drop ``managedFields``
``wire_codecs``            watch events decoded by plan: child     every event decoded whole
                           ``spec`` skipped, Cron ``spec`` and
                           status history entries reused by bytes
``defer_status_write``     once only API writes are left (the      the worker waits for the deferred
                           CREATE, the status PATCH, GC DELETEs)   status patch (``:107-120``) after
                           the reconcile releases its worker       the CREATE (``:229-238``)
                           slot; the key stays processing
``request_priorities``     tick CREATEs (and Replace DELETEs) go   one FIFO token bucket for every
                           first on a backed-up QPS bucket;        request
                           status PATCHes / GC DELETEs / events
                           yield to them
``active_ref_resource_``   ``first``: an active ref keeps the      ``live``: rebuilt with the child's
``version``                resourceVersion the child entered       current resourceVersion on every
                           ``status.active`` with (Kubernetes      reconcile (``:284-304``), so every
                           CronJob semantics)                      training-operator status write costs
                                                                   the Cron a status PATCH
``skip_unchanged_child_``  a child update that changes nothing a   every owned-child event requeues
``updates``                reconcile reads (Created / replica      the Cron (B22)
                           counts / Running writes) is dropped
=========================  =====================================  =======================================

``defer_status_write`` (under a controller worker, ``runtime/controller.py`` ``release_worker``,
and while the client's in-flight cap is not the bottleneck -- ``Client.gate_saturated``): a
fire reconcile otherwise holds its worker slot for two sequential write round trips -- the
CREATE, then the status PATCH that records ``lastScheduleTime``.  Once the fire is decided,
the reconcile hands its slot to the next queued Cron and finishes its writes on its own; its
key stays processing in the work queue until it returns, so a requeue of the key meanwhile
is parked and never starts a second reconcile of it.  Under apiserver latency a tick's
CREATEs then go out at the client's in-flight cap instead of at workers / (two round trips).

``overlap_gc_deletes``: a GC DELETE's outcome feeds nothing else in the
reconcile -- the reference only logs its error and drops the child from
``status.history`` either way (``cron_controller.go:324-333``) -- so the
DELETEs are started as they are decided and awaited together with the status
PATCH at the end.  Under apiserver latency a reconcile then costs one round
trip less per GC'd child; the reconcile still returns only after every DELETE
finished, so per-key serialisation is unchanged.

``wire_codecs`` (:class:`WireCodecs`): the Cron's status write is encoded through
a memo that remembers the bytes of every history entry it writes, and the Cron
informer decodes its watch events through the same memo -- so the echo of our own
write arrives holding the reconciler's own (read-only) entry dicts.  The own-write
check and the next merge patch then compare those entries by identity, and the
bulk of each Cron event (its spec and history) is never rebuilt.  Byte-identical
spans are reused only, so the decoded objects are exactly what a plain decode gives.

``dedupe_ran_tick``: the reference advances ``lastScheduleTime`` only in the
deferred status patch after a successful CREATE (B20).  If that patch fails, or
the CREATE's response is lost after the object was stored, the next reconcile
sees the same missed tick again: under ``Replace`` it deletes the job it just
created and creates it anew, and under ``Forbid`` it waits for the job to finish
and then runs the tick a second time under a new name.  Job names are
``<cron>-<unix(Next(tick))>`` (B18), so the job a tick produced is recognisable
(an ``@every`` job is named ``Next(now)`` at its CREATE: a later-named job created at
or after the tick counts); when it already exists the tick is recorded as run instead
(``tests/test_chaos.py`` drives exactly these faults).

Time comes from the injected clock (the reference calls ``time.Now()``,
``cron_controller.go:160``), which makes every path deterministic in tests.
"""
from __future__ import annotations

import asyncio
import dataclasses
import functools
import json
import operator
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..api import errors
from ..api.meta import (
    GroupVersionKind,
    creation_timestamp,
    set_controller_reference,
    time_from_json,
)
from ..api.v1alpha1 import (
    CRON_GVK,
    CRON_GVR,
    LABEL_CRON_NAME,
    ConcurrentPolicyForbid,
    ConcurrentPolicyReplace,
    Cron,
    CronHistory,
    CronStatus,
    ObjectReference,
    TypedLocalObjectReference,
)
from ..cron.engine import CronEngine, ScheduleError, default_engine
from ..models import kubeflow as kf
from ..models.workload import _summary as workload_summary
from ..models.workload import (
    Classification,
    WorkloadError,
    WorkloadPolicy,
    classify,
    get_default_job_name,
    get_workload_gvk,
    new_empty_workload,
)
from ..runtime import metrics, tracing
from ..runtime.client import Client
from ..runtime.controller import Reconciler, Request, Result, release_worker
from ..runtime.events import Normal, Warning, EventRecorder
from ..runtime.ratelimit import PRIORITY_HIGH, PRIORITY_LOW, PRIORITY_NORMAL
from ..runtime.informer import Cache, Informer
from ..utils import aio, gctune, jsonutil
from ..utils.clock import Clock, RealClock
from ..utils.gotime import LOCAL, NANOS, GoTime
from ..utils.logging import Logger, ObjectRef

CHILD_INDEX = "cron-name"
_SORT_KEY = operator.attrgetter("sort_key")  # _ChildInfo -> creation-time sort key
MAX_INT = 2**63 - 1


def go_quote(s: str) -> str:
    """Go's ``%q`` for the strings we format (JSON escaping is a close match)."""
    return json.dumps(s, ensure_ascii=False)


class _ChildInfo:
    """Everything a reconcile derives from one child object.  Objects are immutable per
    resourceVersion, so with ``classification_cache`` this is computed once per child
    version instead of on every reconcile of its Cron (the 10 history children of a
    Cron were re-parsed ~2x per tick otherwise)."""

    __slots__ = ("rv", "cls", "finished", "sort_key", "gvk", "active_ref", "history_entry", "obj", "name", "uid",
                 "err")

    def __init__(self, rv: str, cls: Optional[Classification], sort_key: Any, gvk: Optional[GroupVersionKind]):
        self.rv = rv
        self.cls = cls
        self.finished = cls is not None and cls.finished
        self.sort_key = sort_key  # None: not computed (the caller sorts by the object's creation time)
        self.gvk = gvk
        self.active_ref: Optional[ObjectReference] = None
        self.history_entry: Optional[CronHistory] = None
        self.obj: Optional[Dict[str, Any]] = None
        self.name = ""
        self.uid = ""
        self.err: Optional[Exception] = None  # a status that cannot be decoded (kf.ConversionError)


def child_info(w: Dict[str, Any], gvk: GroupVersionKind, policy: WorkloadPolicy) -> _ChildInfo:
    """Everything a reconcile needs from child ``w`` (a cached object of the template's kind).

    Runs inside the child informer's event handling (``Informer.derive``), so it never
    raises: an object it cannot read becomes a per-child error (``info.err``) that only
    its own Cron's reconcile reports, instead of stalling the informer on that event."""
    m = w.get("metadata")
    if type(m) is not dict:
        m = {}
    err: Optional[Exception] = None
    cls: Optional[Classification] = None
    sort_key: Any = (0, 0)
    try:
        hit = _CLS_MEMO[0]
        if hit is not None and hit[0] is w:
            cls = hit[1]  # classified by the informer transform a moment ago (compact_child)
            _CLS_MEMO[0] = None
        else:
            cls = classify(w, gvk, policy)
        sort_key = _sort_key(m.get("creationTimestamp"))
    except Exception as e:  # noqa: BLE001 - kf.ConversionError, or a malformed object
        err = e
        cls = None  # never "finished" with an error: it would reach history and fail there
        sort_key = (0, 0)
    info = _ChildInfo(m.get("resourceVersion", ""), cls, sort_key, GroupVersionKind.from_object(w))
    info.obj = w
    info.name = m.get("name", "")
    info.uid = m.get("uid", "")
    info.err = err
    return info


def _sort_key(ts: Any) -> Tuple[int, int]:
    """History order of a child created at ``ts`` (its ``creationTimestamp``): one shared tuple
    per timestamp -- the children a tick creates share their creation second."""
    k = _SORT_KEYS.get(ts) if ts.__class__ is str else None
    if k is None:
        t = time_from_json(ts) if ts else None
        k = t.key() if t is not None else GoTime.zero().key()  # as creation_timestamp() reads it
        if ts.__class__ is str:
            if len(_SORT_KEYS) >= 4096:
                _SORT_KEYS.clear()
            _SORT_KEYS[ts] = k
    return k


_SORT_KEYS: Dict[str, Tuple[int, int]] = {}


def _template_fixed_name(wl: Any) -> bool:
    """Does the workload template set ``metadata.name`` (every run then reuses that name)?"""
    if isinstance(wl, (bytes, str)):
        try:
            wl = jsonutil.loads(wl)
        except ValueError:
            return False
    m = wl.get("metadata") if isinstance(wl, dict) else None
    return isinstance(m, dict) and bool(m.get("name"))


def _gv_str(gvk: GroupVersionKind) -> str:
    """``group/version`` of ``gvk``, one shared string per kind (every history entry holds it)."""
    s = _GV_STR.get(gvk)
    if s is None:
        s = _GV_STR[gvk] = str(gvk.group_version())
    return s


_GV_STR: Dict[GroupVersionKind, str] = {}


# A child as the status sync sees it: its object (``obj``), classification (``cls``/``finished``)
# and, with the classification cache, the memo record shared across reconciles
Child = _ChildInfo


def slim_child(obj: Dict[str, Any]) -> Dict[str, Any]:
    """Informer transform for children: a reconcile reads their metadata, kind and status
    (classification, history, GC, Replace) and never their ``spec`` -- the bulk of a
    PyTorchJob/TFJob -- so the cache keeps everything else (``ReconcilerOptions.slim_child_cache``)."""
    obj.pop("spec", None)
    m = obj.get("metadata")
    if type(m) is dict and "managedFields" in m:
        del m["managedFields"]
    return obj


# the child metadata read anywhere: its key, version, creation (history order) and deletion, the
# cron-name label (index) and the controller owner (event mapping)
CHILD_METADATA = ("name", "namespace", "uid", "resourceVersion", "creationTimestamp", "deletionTimestamp",
                  "labels", "ownerReferences")
# the metadata keys a child commonly carries besides those (skipped at decode when compacting)
CHILD_METADATA_DROPPED = ("generation", "annotations", "finalizers", "generateName", "selfLink",
                          "deletionGracePeriodSeconds")
_COND_KEEP = ("type", "status", "lastTransitionTime")
_TERMINAL_TYPES = frozenset(("Succeeded", "Failed", "Complete"))
_STATUS_KEEP = ("completionTime", "phase", "launcherStatus")


def compact_status(st: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    """The part of a child's ``status`` that :func:`~cron_operator_amd.models.workload.classify`
    reads: the terminal conditions (``Succeeded``/``Failed``/``Complete`` that are ``True``) and
    the last condition, each as type / status / lastTransitionTime; ``completionTime``; a Pod's
    ``phase``; an MPIJob v1alpha1's ``launcherStatus``.  Messages, reasons, ``replicaStatuses``
    and start times -- most of a finished job's status -- are never read.  None: not a shape
    this trims (the caller keeps the status as it is)."""
    out: Dict[str, Any] = {}
    conds = st.get("conditions")
    if conds is not None:
        if type(conds) is not list:
            return None
        keep = []
        last = len(conds) - 1
        for i, c in enumerate(conds):
            if type(c) is not dict:
                return None
            if i == last or (c.get("status") == "True" and c.get("type") in _TERMINAL_TYPES):
                keep.append({k: c[k] for k in _COND_KEEP if k in c})
        out["conditions"] = keep
    for k in _STATUS_KEEP:
        if k in st:
            out[k] = st[k]
    return out


def compact_child(gvk: GroupVersionKind, policy: WorkloadPolicy) -> Callable[[Dict[str, Any]], Dict[str, Any]]:
    """Informer transform for the children of kind ``gvk``: :func:`slim_child`, and the status
    trimmed to what classifies it (:func:`compact_status`) -- kept whole when the trim would
    change the classification or the status does not convert (the reconcile then reports it).
    ``ReconcilerOptions.compact_child_status``: about 60% of a cached finished job is status a
    reconcile never reads (a 10,000-Cron fleet caches 110,000 jobs)."""
    summary = workload_summary
    stubs: Dict[str, Any] = {}  # terminal status type -> the shared stub (False: none fits)

    def transform(obj: Dict[str, Any]) -> Dict[str, Any]:
        slim_child(obj)
        m = obj.get("metadata")
        if type(m) is dict and len(m) > 7:
            # only the metadata a reconcile (and the informer, the event predicates, expectations)
            # reads: annotations -- kubectl's last-applied-configuration holds a whole manifest --
            # finalizers, generation and the like are dropped
            obj["metadata"] = {k: m[k] for k in CHILD_METADATA if k in m}
        st = obj.get("status")
        if type(st) is not dict or not st:
            return obj
        try:
            full = classify(obj, gvk, policy)
        except Exception:  # noqa: BLE001 - an unreadable status stays whole for the reconcile to report
            return obj
        _CLS_MEMO[0] = (obj, full)  # child_info() of this object reuses it
        if full.finished:
            stub = stubs.get(full.status)
            if stub is None:
                stub = stubs[full.status] = finished_stub(gvk, policy, full.status)
            if stub:
                obj["status"] = stub
                return obj
        small = compact_status(st)
        if small is None:
            return obj
        sm = summary(st)
        if sm is not None:
            # an exactly-typed kubeflow status: the trim keeps every True terminal condition and
            # the last one, so the summary (finished, last type, completion / terminal times) is
            # the same by construction -- checked natively, not by a second classification
            sm2 = summary(small)
            ok = sm2 is not None and (sm2[0], sm2[1], sm2[3], sm2[4]) == (sm[0], sm[1], sm[3], sm[4])
            obj["status"] = small
        else:
            obj["status"] = small
            try:
                same = classify(obj, gvk, policy)
                ok = (same.finished, same.status, same.finished_at) == (full.finished, full.status,
                                                                         full.finished_at)
            except Exception:  # noqa: BLE001
                ok = False
        if not ok:
            obj["status"] = st
        return obj
    return transform


def finished_stub(gvk: GroupVersionKind, policy: WorkloadPolicy, status: str) -> Any:
    """A read-only status that every finished child of kind ``gvk`` whose history status is
    ``status`` may share in the cache: it classifies as finished with that status (checked
    here; False when no candidate does).  Its completion time is not in it -- the child's memo
    (:func:`child_info`) takes the classification of the full status from the transform, and a
    history entry keeps the time it recorded.  A finished job then costs the cache no status
    of its own: the 100,000 finished jobs of a 10,000-Cron fleet share a handful."""
    for cand in ({"conditions": [{"type": status, "status": "True"}]}, {"phase": status},
                 {"launcherStatus": status}):
        try:
            c = classify({"status": cand}, gvk, policy)
        except Exception:  # noqa: BLE001
            continue
        if c.finished and c.status == status:
            return cand
    return False


# (object, its Classification) of the child compact_child() transformed last: the informer derives
# the child's memo (child_info) right after transforming it, so the classification is reused
_CLS_MEMO: List[Any] = [None]


class JoinedError(Exception):
    """``errors.Join`` of a reconcile error and a status-patch error."""

    def __init__(self, *errs: BaseException):
        self.errors = [e for e in errs if e is not None]
        super().__init__("\n".join(str(e) for e in self.errors))


@dataclass
class ReconcilerOptions:
    list_mode: str = "cache"                 # "cache" | "live"
    finished_time: str = "completion"        # "completion" | "now"
    skip_noop_patch: bool = True
    own_write_filter: bool = True
    dynamic_watches: bool = True
    # status.active[].resourceVersion: "first" -- the version the child had when it became active
    # (as Kubernetes' CronJob controller records it); "live" -- its current version, rebuilt on
    # every reconcile (cron_controller.go:284-304: each status write of the training-operator then
    # costs the Cron a status PATCH); "omit" -- left empty
    active_ref_resource_version: str = "first"
    # a child update that changes nothing a reconcile reads (classification, completion time,
    # labels, owner, deletion) does not requeue the Cron -- the training-operator's Created /
    # replicaStatuses / Running writes -- unless active refs track the live resourceVersion
    skip_unchanged_child_updates: bool = True
    expectations: bool = True
    expectation_ttl: float = 300.0           # seconds on the injected clock
    fold_created_into_active: bool = True    # add the just-created child to status.active right away
    skip_expected_events: bool = True        # child add/delete events we caused do not requeue the Cron
    classification_cache: bool = True
    dedupe_ran_tick: bool = True
    overlap_gc_deletes: bool = True
    slim_child_cache: bool = True
    # (with slim_child_cache and classification_cache) cached children keep only the status
    # fields their classification reads (compact_child)
    compact_child_status: bool = True
    wire_codecs: bool = True
    defer_status_write: bool = True
    request_priorities: bool = True
    # a Cron that cannot run (unparsable schedule, template without a kind) gets a Warning event
    # (InvalidSchedule / InvalidTemplate) for `kubectl describe`; the reference only logs it
    explain_errors: bool = True
    # cache mode: how long a reconcile waits for a new child informer's first LIST before
    # it falls back to a live LIST; a LIST that *fails* (403, 404, 5xx) is returned as the
    # reconcile's error at once, like the reference's live LIST (cron_controller.go:129-133)
    child_sync_timeout: float = 5.0
    workload: WorkloadPolicy = field(default_factory=WorkloadPolicy)
    static_owned_kinds: Tuple[GroupVersionKind, ...] = (
        GroupVersionKind("kubeflow.org", "v1", "PyTorchJob"),
        GroupVersionKind("kubeflow.org", "v1", "TFJob"),
    )

    def compact_metadata(self) -> bool:
        """Children are cached through :func:`compact_child` (metadata whitelist included)."""
        return self.slim_child_cache and self.compact_child_status and self.classification_cache

    @staticmethod
    def reference() -> "ReconcilerOptions":
        return ReconcilerOptions(list_mode="live", finished_time="now", skip_noop_patch=False,
                                 active_ref_resource_version="live", skip_unchanged_child_updates=False,
                                 own_write_filter=False, dynamic_watches=False, expectations=False,
                                 fold_created_into_active=False, skip_expected_events=False,
                                 classification_cache=False, dedupe_ran_tick=False,
                                 overlap_gc_deletes=False, slim_child_cache=False, compact_child_status=False,
                                 wire_codecs=False,
                                 defer_status_write=False, request_priorities=False, explain_errors=False,
                                 workload=WorkloadPolicy.reference())


class WireCodecs:
    """Plan-driven JSON codecs for the objects this controller exchanges (``_fastjson.Codec``;
    the Python twin ignores memo paths).  One memo is shared: the status-write encoder
    remembers each history entry it writes, the Cron event decoder hands those objects
    back when the watch echoes the same bytes.  ``slim`` also skips what the caches drop
    anyway: a child's ``spec`` and every ``managedFields``.  ``shard=(index, count)`` (hash-routed
    sharding, where every shard watches the whole fleet): the Cron and child decoders build only
    the metadata of another shard's objects (route paths), which the informers' keep filter
    then drops."""

    def __init__(self, slim: bool = True, memo_slots: int = 1 << 14, memo_max_slots: int = 1 << 19,
                 compact_metadata: bool = False, shard: Optional[Tuple[int, int]] = None):
        # grows with the fleet: ~12 values per Cron (its history entries, a labels map and an owner
        # reference) stay remembered up to ~40,000 Crons per process
        self.memo = jsonutil.Memo(memo_slots, memo_max_slots)
        mf = ("metadata", "managedFields")
        child_skip = [("spec",), mf] if slim else []
        if compact_metadata:
            # what compact_child() drops from a child's metadata anyway, never built: the cached
            # child then keeps its decoded metadata dict instead of a filtered copy per event
            child_skip += [("metadata", k) for k in CHILD_METADATA_DROPPED]
        child_memo = [("metadata", "labels"), ("metadata", "ownerReferences")]
        # a Cron's template.workload -- a whole job manifest the reconciler only copies into each
        # new job -- is kept as its JSON text (slim): ~0.6 KB instead of ~6 KB of dicts per Cron
        # when templates differ, decoded afresh per fire instead of deep-copied
        tw = ("spec", "template", "workload")

        def routed(at: Tuple[str, ...], label: Optional[str]) -> Dict[str, Any]:
            return {} if shard is None else {"route_paths": [at], "route": (shard[0], shard[1], label)}

        self.cron_event = jsonutil.Codec(skip=[("object",) + mf] if slim else [],
                                         memo_paths=[("object", "spec"), ("object", "status", "history", "*")],
                                         memo=self.memo, raw_paths=[("object",) + tw] if slim else [],
                                         **routed(("object",), None))
        self.child_event = jsonutil.Codec(skip=[("object",) + p for p in child_skip],
                                          memo_paths=[("object",) + p for p in child_memo], memo=self.memo,
                                          **routed(("object",), LABEL_CRON_NAME))
        self.child_object = jsonutil.Codec(skip=child_skip, memo_paths=child_memo, memo=self.memo)
        # LIST pages: the same plans under items/* (the initial LIST of 110,000 jobs shares labels
        # and owner references as the watch events do, and never builds a spec)
        self.child_list = jsonutil.Codec(skip=[("items", "*") + p for p in child_skip],
                                         memo_paths=[("items", "*") + p for p in child_memo], memo=self.memo,
                                         **routed(("items", "*"), LABEL_CRON_NAME))
        # (a LIST's history entries are not remembered: the reconciler's own entries replace them
        # at its first status write, and only those are forgotten when they rotate out)
        self.cron_list = jsonutil.Codec(skip=[("items", "*") + mf] if slim else [],
                                        memo_paths=[("items", "*", "spec")], memo=self.memo,
                                        raw_paths=[("items", "*") + tw] if slim else [],
                                        **routed(("items", "*"), None))
        self.status_patch = jsonutil.Codec(memo_paths=[("status", "history", "*")], memo=self.memo)


class Expectations:
    """Children we created/deleted that the informer has not observed yet.

    Keyed by ``namespace/cron``.  Entries are dropped when the informer catches
    up (``observe_*``) or after ``ttl`` seconds on the injected clock (like
    client-go's ``ControllerExpectations``, whose TTL runs on ``clock.Clock``), so a
    watch event that never arrives is outlived in virtual time as well.
    """

    def __init__(self, ttl: float, clock: Optional[Clock] = None):
        self.ttl = ttl
        self.clock = clock or RealClock()
        self.created: Dict[str, Dict[str, Tuple[int, Dict[str, Any]]]] = {}  # key -> {uid: (expiry ns, obj)}
        self.deleted: Dict[str, Dict[str, int]] = {}
        self.pending: Dict[str, Dict[str, int]] = {}  # key -> {name: expiry} for in-flight CREATEs

    def _deadline(self) -> int:
        return self.clock.now_ns() + int(self.ttl * NANOS)

    def expect_pending(self, key: str, name: str) -> None:
        self.pending.setdefault(key, {})[name] = self._deadline()

    def drop_pending(self, key: str, name: str) -> None:
        d = self.pending.get(key)
        if d is not None and d.pop(name, None) is not None and not d:
            del self.pending[key]

    def expect_create(self, key: str, obj: Dict[str, Any]) -> None:
        self.drop_pending(key, (obj.get("metadata") or {}).get("name", ""))
        uid = (obj.get("metadata") or {}).get("uid", "")
        if uid:
            self.created.setdefault(key, {})[uid] = (self._deadline(), obj)

    def expect_delete(self, key: str, uid: str) -> None:
        if uid:
            self.deleted.setdefault(key, {})[uid] = self._deadline()

    def observe_add(self, key: str, uid: str) -> None:
        d = self.created.get(key)
        if d is not None and d.pop(uid, None) is not None and not d:
            del self.created[key]

    def observe_delete(self, key: str, uid: str) -> None:
        self.observe_add(key, uid)
        d = self.deleted.get(key)
        if d is not None and d.pop(uid, None) is not None and not d:
            del self.deleted[key]

    def forget(self, key: str) -> None:
        self.created.pop(key, None)
        self.deleted.pop(key, None)
        self.pending.pop(key, None)

    def matches_created(self, key: str, obj: Dict[str, Any]) -> bool:
        """Is ``obj`` exactly the object our CREATE returned (same uid and resourceVersion)?"""
        m = obj.get("metadata") or {}
        p = self.pending.get(key)
        if p and m.get("name", "") in p:
            return True  # the watch event overtook our CREATE response
        d = self.created.get(key)
        if not d:
            return False
        hit = d.get(m.get("uid", ""))
        return hit is not None and (hit[1].get("metadata") or {}).get("resourceVersion") == m.get("resourceVersion")

    def matches_deleted(self, key: str, obj: Dict[str, Any]) -> bool:
        d = self.deleted.get(key)
        return bool(d) and (obj.get("metadata") or {}).get("uid", "") in d

    def adjust(self, key: str, children: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
        cr = self.created.get(key)
        dl = self.deleted.get(key)
        if not cr and not dl:
            return children
        now = self.clock.now_ns()
        if dl:
            for uid in [u for u, exp in dl.items() if exp < now]:
                del dl[uid]
            children = [c for c in children if (c.get("metadata") or {}).get("uid") not in dl]
        if cr:
            for uid in [u for u, (exp, _) in cr.items() if exp < now]:
                del cr[uid]
            present = {(c.get("metadata") or {}).get("uid") for c in children}
            extra = [o for u, (_, o) in cr.items() if u not in present and not (dl and u in dl)]
            if extra:
                children = children + extra
        return children


class CronReconciler(Reconciler):
    def __init__(self, client: Client, cache: Optional[Cache], recorder: EventRecorder,
                 clock: Optional[Clock] = None, engine: Optional[CronEngine] = None,
                 options: Optional[ReconcilerOptions] = None, cron_informer: Optional[Informer] = None,
                 codecs: Optional[WireCodecs] = None):
        self.client = client
        self.cache = cache
        self.recorder = recorder
        self.clock = clock or RealClock()
        self.engine = engine or default_engine()
        self.opts = options or ReconcilerOptions()
        self.cron_informer = cron_informer
        # setup_with_manager passes the instance its Cron informer decodes with (one shared memo)
        self.codecs: Optional[WireCodecs] = codecs if codecs is not None or not self.opts.wire_codecs else \
            WireCodecs(self.opts.slim_child_cache, compact_metadata=self.opts.compact_metadata())
        self.expect = Expectations(self.opts.expectation_ttl, self.clock)
        prio = self.opts.request_priorities
        self._p_create = PRIORITY_HIGH if prio else PRIORITY_NORMAL    # a tick's CREATE, Replace DELETEs
        self._p_deferrable = PRIORITY_LOW if prio else PRIORITY_NORMAL  # status PATCH, history-GC DELETEs
        self.child_informers: Dict[GroupVersionKind, Informer] = {}
        self.on_child_informer: Optional[Callable[[GroupVersionKind, Informer], None]] = None
        # the child informers' selector, and labels stamped on every child (label-routed sharding)
        self.child_selector = LABEL_CRON_NAME
        self.child_labels: Dict[str, str] = {}
        # hash-routed sharding: the child informers store only this shard's Crons' jobs
        self.child_keep: Optional[Callable[[Dict[str, Any]], bool]] = None
        self.shard_assigner: Any = None  # controller.sharding.ShardAssigner with label routing
        # key -> resourceVersion of the Cron object produced by our last status write
        self.own_writes: Dict[str, Tuple[Any, Dict[str, Any]]] = {}  # key -> (generation, status we wrote)
        self.stats = {"creates": 0, "deletes": 0, "patches": 0, "noop_patches_skipped": 0, "lists": 0}
        # child uid -> derived data for one resourceVersion (objects are immutable per resourceVersion)
        self._class_cache: Dict[str, _ChildInfo] = {}
        # key -> (status dict we last wrote, its parsed form): the next reconcile of that Cron
        # usually reads exactly that status back, so it skips re-parsing every history entry
        self._parsed_status: Dict[str, Tuple[Dict[str, Any], CronStatus]] = {}
        # key -> (resourceVersion, status dict) of the Cron version is_own_write() proved to hold
        # exactly that status: the next reconcile then trusts its memo without comparing again
        self._own_rv: Dict[str, Tuple[str, Dict[str, Any]]] = {}
        # key -> (spec dict of the cached Cron, its parsed CronSpec): the Cron informer's codec hands
        # back the same spec object while the spec bytes do not change, so it is parsed once
        self._spec_memo: Dict[str, Tuple[Dict[str, Any], Any]] = {}
        # metric children the hot path updates (label sets fixed)
        self._m_patch_ok = metrics.child(metrics.STATUS_PATCHES, "ok")
        self._m_patch_skipped = metrics.child(metrics.STATUS_PATCHES, "skipped")
        self._m_sched_lat = metrics.child(metrics.SCHEDULE_LATENCY, "cron")
        # key -> (template workload dict, policy, its GVK): checked once per template object
        self._gvk_memo: Dict[str, Tuple[Any, WorkloadPolicy, GroupVersionKind, bool]] = {}
        # tick bookkeeping for latency: key -> (tick unix ns, wall perf_counter when it became due)
        self.latency_observer: Optional[Callable[[str, GoTime, Dict[str, Any]], None]] = None

    def forget_cron(self, key: str) -> None:
        """Drop the per-Cron memos of a Cron that is gone (``namespace/name``)."""
        self._parsed_status.pop(key, None)
        self._spec_memo.pop(key, None)
        self._gvk_memo.pop(key, None)
        self.own_writes.pop(key, None)
        self._own_rv.pop(key, None)
        self.expect.forget(key)

    def forget_child(self, uid: str) -> None:
        """Drop the per-child memo of a deleted child."""
        self._class_cache.pop(uid, None)

    # ------------------------------------------------------------------ entry point
    async def reconcile(self, req: Request, log: Logger) -> Result:
        """``Reconcile`` (``cron_controller.go:90-239``)."""
        log.info("Start reconciling Cron")
        try:
            # B1: cache read; NotFound -> no-op (cron_controller.go:95-104)
            inf = self.cron_informer
            old_obj = inf.get(req.namespace, req.name, copy=False) if inf is not None else \
                await self._get_cron(req)
            if old_obj is None:
                log.info("Skip reconciling Cron for it may have been deleted")
                self.forget_cron(f"{req.namespace}/{req.name}")
                return Result()
            parsed = None
            spec = None
            key = f"{req.namespace}/{req.name}"
            if self.opts.classification_cache:
                memo = self._parsed_status.get(key)
                if memo is not None:
                    ov = self._own_rv.get(key)
                    if (ov is not None and ov[1] is memo[0]
                            and ov[0] == (old_obj.get("metadata") or {}).get("resourceVersion")) \
                            or jsonutil.json_equal(old_obj.get("status") or {}, memo[0]):
                        parsed = memo[1].snapshot()
                sd = old_obj.get("spec")
                sm = self._spec_memo.get(key)
                if sm is not None and sm[0] is sd:
                    spec = sm[1]
            cron = Cron.from_dict(old_obj, status=parsed, spec=spec)
            if spec is None and self.opts.classification_cache and type(old_obj.get("spec")) is dict:
                self._spec_memo[key] = (old_obj["spec"], cron.spec)
            old_status = cron.status.snapshot()

            result = Result()
            err: Optional[BaseException] = None
            gc: Optional[List["asyncio.Future[None]"]] = [] if self.opts.overlap_gc_deletes else None
            # with a controller worker: hand the worker slot on before the API writes -- before a
            # tick's CREATE unless the in-flight cap is the bottleneck right now (the CREATE then
            # runs on this worker), and always before the deferrable writes: they may wait for
            # the tick's token reserve, which no decision on this worker should wait behind
            release = self.opts.defer_status_write and not self.client.gate_saturated()
            try:
                try:
                    result = await self._sync(cron, log, gc, release)
                except Exception as e:  # noqa: BLE001 - joined with the patch error below
                    err = e
                changed = not old_status.semantic_equal(cron.status)
                if self.opts.defer_status_write and (gc or changed):
                    release_worker()  # only writes are left: another Cron may use the slot
                # B2: deferred status patch when status changed semantically (cron_controller.go:107-120)
                if changed:
                    try:
                        await self._patch_status(old_obj, cron, log, key)  # overlaps the running GC DELETEs
                    except Exception as pe:  # noqa: BLE001
                        perr = RuntimeError(f"failed to patch Cron status: {pe}")
                        perr.__cause__ = pe
                        err = JoinedError(err, perr) if err is not None else perr
                    if err is not None:
                        result = Result()
                if gc:
                    await self._await_gc(gc)
            except asyncio.CancelledError:
                # the reconcile itself is cancelled (shutdown, leader loss): stop its DELETEs
                # too instead of waiting up to a request timeout for each
                if gc:
                    aio.cancel_all(gc)
                raise
            if err is not None:
                raise err
            return result
        finally:
            log.info("Finish reconciling Cron")

    async def _get_cron(self, req: Request) -> Optional[Dict[str, Any]]:
        if self.cron_informer is not None:
            return self.cron_informer.get(req.namespace, req.name, copy=False)
        try:
            return await self.client.get(CRON_GVR, req.namespace, req.name)
        except errors.ApiError as e:
            if errors.is_not_found(e):
                return None
            raise

    @staticmethod
    async def _await_gc(gc: List["asyncio.Future[None]"]) -> None:
        """Wait for every overlapped GC DELETE; each logs its own API error (B7), anything
        else it raised is dropped like ``gather(return_exceptions=True)`` would.  A
        cancellation of the reconcile propagates (``asyncio.wait`` neither cancels the
        DELETEs nor mistakes their outcome for the caller's)."""
        await aio.wait_all(gc)

    async def _patch_status(self, old_obj: Dict[str, Any], cron: Cron, log: Logger, key: str = "") -> None:
        new_status = cron.status.to_dict(shared=True)
        old_status = old_obj.get("status") or {}
        codecs = self.codecs
        # share: the patch is only serialised, so it may hold new_status's (read-only) entries
        patch = jsonutil.create_merge_patch({"status": old_status}, {"status": new_status} if new_status else {},
                                            codecs is not None)
        m = old_obj.get("metadata") or {}
        if not key:
            key = f"{m.get('namespace', '')}/{m.get('name', '')}"
        if self.opts.classification_cache:
            self._parsed_status[key] = (new_status, cron.status.snapshot())
        if not patch and self.opts.skip_noop_patch:
            self.stats["noop_patches_skipped"] += 1
            self._m_patch_skipped.inc()
            return
        if self.opts.own_write_filter:
            # recorded before the call: the watch event can overtake the PATCH response
            self.own_writes[key] = (m.get("generation"), new_status)
        body: Any = codecs.status_patch.dumpb(patch) if codecs is not None else patch
        try:
            if tracing.get_tracer().enabled:
                with tracing.span("patch_status", bytes=len(body) if body.__class__ is bytes else
                                  len(jsonutil.dumps(patch))):
                    await self.client.patch(CRON_GVR, m.get("namespace", ""), m.get("name", ""), body, "merge",
                                            "status", discard_response=True, priority=self._p_deferrable)
            else:
                await self.client.patch(CRON_GVR, m.get("namespace", ""), m.get("name", ""), body, "merge",
                                        "status", discard_response=True, priority=self._p_deferrable)
        except Exception:
            self.own_writes.pop(key, None)
            raise
        self.stats["patches"] += 1
        self._m_patch_ok.inc()

    def is_own_write(self, old: Optional[Dict[str, Any]], new: Dict[str, Any]) -> bool:
        """Predicate helper: is this Cron update exactly our last status write?

        True when the new object's status equals the status we sent and nothing
        a reconcile reads besides status changed (same generation, so same spec,
        and no deletion started).  Such an event would only recompute what we
        just wrote.
        """
        if old is new:  # periodic resync: always reconcile
            return False
        m = new.get("metadata") or {}
        key = f"{m.get('namespace', '')}/{m.get('name', '')}"
        hit = self.own_writes.get(key)
        if hit is None:
            return False
        gen, status = hit
        if m.get("generation") != gen or m.get("deletionTimestamp"):
            return False
        if old is not None and (old.get("metadata") or {}).get("deletionTimestamp") != m.get("deletionTimestamp"):
            return False
        if not jsonutil.json_equal(new.get("status") or {}, status):
            return False
        if status and new.get("status") is not status:
            # the cached object keeps the status dict we wrote (equal, just compared) instead of
            # its decoded copy: active refs and lists held once per Cron, not twice
            new["status"] = status
        self._own_rv[key] = (m.get("resourceVersion", ""), status)
        return True

    # ------------------------------------------------------------------ the algorithm
    async def _sync(self, cron: Cron, log: Logger, gc: Optional[List["asyncio.Future[None]"]] = None,
                    release: bool = False) -> Result:
        """B3-B20.  ``release``: hand the controller worker slot on once a fire is decided (only
        API writes are left: B16-B20, then the status PATCH)."""
        policy = self.opts.workload
        # spans (and the attributes they would carry) only when tracing is on
        traced = tracing.get_tracer().enabled
        # B3 (cron_controller.go:122-126)
        wl = cron.spec.template.workload
        gm = self._gvk_memo
        ck = f"{cron.namespace}/{cron.name}"
        hit = gm.get(ck) if wl.__class__ is dict or wl.__class__ is bytes else None
        if hit is not None and hit[0] is wl and hit[1] is policy:
            gvk = hit[2]  # the same (read-only) template object as last time: same checks, same GVK
        else:
            try:
                gvk = get_workload_gvk(wl, policy)
            except WorkloadError as e:
                log.error(e, "Failed to get workload GVK")
                if self.opts.explain_errors:
                    self.recorder.event(cron.to_dict(), Warning, "InvalidTemplate", str(e))
                return Result()
            if wl.__class__ is dict or wl.__class__ is bytes:
                gm[ck] = (wl, policy, gvk, _template_fixed_name(wl))

        # B4 (cron_controller.go:129-133)
        infos: Optional[List[_ChildInfo]] = None
        workloads: List[Dict[str, Any]] = []
        try:
            with (tracing.span("list_children", kind=gvk.kind, mode=self.opts.list_mode) if traced
                  else tracing.NOOP) as sp:
                if self.opts.classification_cache and self.opts.list_mode != "live" and self.cache is not None:
                    inf = self.child_informers.get(gvk)
                    if inf is not None and inf.derive is not None and inf.synced.is_set():
                        if log.enabled():
                            log.v(1).info(f"Listing {gvk.kind}")
                        infos = self._child_infos(inf, cron, gvk)  # the steady state: no await
                    else:
                        infos = await self.list_child_infos(cron, gvk, log)
                if infos is None:
                    workloads = await self.list_workloads(cron, gvk, log, force_live=self.cache is not None
                                                          and self.opts.list_mode != "live"
                                                          and self.opts.classification_cache)
                if traced:
                    sp.set(count=len(workloads) if infos is None else len(infos))
        except Exception as e:
            log.error(e, f"Failed to list {gvk.kind}")
            raise

        # B5 (cron_controller.go:136-152)
        active: List[Child] = []
        terminated: List[Child] = []
        if infos is not None:
            # children classified once per version, at informer-event time (Informer.derive);
            # sorted here once (C-level key) so both partitions come out ordered (B6/B7)
            if len(infos) > 1:
                infos.sort(key=_SORT_KEY)
            presorted = True
            # a child whose status cannot be read (info.err) is never finished
            terminated = [i for i in infos if i.finished]
            if len(terminated) < len(infos):
                active = [i for i in infos if not i.finished and i.err is None]
                for info in infos:
                    if info.err is not None:
                        log.error(info.err, f"Failed to get {gvk.kind} status")
        else:
            presorted = False
        cache = self._class_cache if self.opts.classification_cache else None
        for w in workloads:
            m = w.get("metadata") or {}
            try:
                if cache is not None:
                    uid, rv = m.get("uid", ""), m.get("resourceVersion", "")
                    info = cache.get(uid)
                    if info is None or info.rv != rv:
                        info = _ChildInfo(rv, classify(w, gvk, policy), creation_timestamp(w).key(),
                                          GroupVersionKind.from_object(w))
                        if len(cache) > 500_000:
                            cache.clear()
                        cache[uid] = info
                else:
                    info = _ChildInfo("", classify(w, gvk, policy), None, None)
            except kf.ConversionError as e:
                log.error(e, f"Failed to get {gvk.kind} status")
                continue
            info.obj = w  # this reconcile's copy (a live LIST returns new objects every time)
            info.name = m.get("name", "")
            info.uid = m.get("uid", "")
            (terminated if info.finished else active).append(info)
        chatty = log.enabled()  # info logging on: skip building messages nobody writes otherwise
        if chatty:
            log.info(f"{gvk.kind} count", active=len(active), terminated=len(terminated))

        # B6/B7/B8 (cron_controller.go:155-158)
        with (tracing.span("sync_status", active=len(active), terminated=len(terminated)) if traced
              else tracing.NOOP):
            if gc is not None:  # DELETEs are only started: nothing to await here
                if chatty:
                    log.v(1).info("Syncing Cron status")
                self.sync_active_list(cron, gvk, active, log, presorted)
                self._sync_history(cron, terminated, log, gc, presorted)
            else:
                await self.sync_status(cron, gvk, active, terminated, log, gc)

        now = self.clock.now(LOCAL)

        # B9 (cron_controller.go:163-166)
        if cron.deletion_timestamp is not None:
            log.info("Cron has been deleted", deletionTimestamp=cron.metadata.get("deletionTimestamp"))
            return Result()
        # B10 (cron_controller.go:169-173)
        if cron.spec.suspend:
            log.info("Cron has been suspended")
            return Result()
        # B11 (cron_controller.go:176-180)
        if cron.spec.deadline is not None and now.after(cron.spec.deadline):
            log.info("Cron has reached deadline and will not trigger scheduling anymore")
            self.recorder.event(cron.to_dict(), Normal, "Deadline", "cron has reach deadline and stop scheduling")
            return Result()

        # B12/B21 (cron_controller.go:184-190, 389-437)
        try:
            missed_run, next_run = self.get_next_schedule(cron, now, log)
        except ScheduleError as e:
            log.error(e, "Failed to figure out CronJob schedule")
            if self.opts.explain_errors:
                self.recorder.event(cron.to_dict(), Warning, "InvalidSchedule", str(e))
            return Result()

        # B13 (cron_controller.go:192)
        # the tick as an absolute time too: the deferred writes may keep this reconcile running
        # past `now` (controller-runtime adds RequeueAfter when Reconcile returns, B13)
        scheduled = Result(requeue_after_ns=next_run.sub(now), requeue_at_ns=next_run.unix_nano())
        if log.enabled():
            log = log.with_values(now=now.rfc3339(nanos=True), **{"next run": next_run.rfc3339()})

        # B14 (cron_controller.go:196-199)
        if missed_run.is_zero():
            log.v(1).info("No upcoming schedules, wait until next")
            return scheduled
        if log.enabled():
            log = log.with_values(**{"current run": missed_run.rfc3339()})

        if self.opts.dedupe_ran_tick and self._tick_already_ran(cron, missed_run, active, terminated):
            log.info(f"{gvk.kind} for this run already exists; recording it as scheduled")
            cron.status.last_schedule_time = now
            return scheduled

        # B15 (cron_controller.go:204-207)
        if cron.spec.concurrency_policy == ConcurrentPolicyForbid and active:
            log.v(1).info(f"Skip creating new {gvk.kind} due to concurrency policy forbid", active=len(active))
            return scheduled

        if release:
            release_worker()
        return await self._fire(cron, gvk, active, missed_run, next_run, now, log, scheduled)

    async def _fire(self, cron: Cron, gvk: GroupVersionKind, active: List[Child], missed_run: GoTime,
                    next_run: GoTime, now: GoTime, log: Logger, scheduled: Result) -> Result:
        """B16-B20 (``cron_controller.go:210-238``): Replace, build the job, CREATE it, and
        advance ``lastScheduleTime``."""
        traced = tracing.get_tracer().enabled
        chatty = log.enabled()
        # B16 (cron_controller.go:210-220)
        if cron.spec.concurrency_policy == ConcurrentPolicyReplace:
            for info in active:
                m = info.obj.get("metadata") or {}  # type: ignore[union-attr]
                ref = ObjectRef(m.get("namespace", ""), m.get("name", ""))
                log.info(f"Deleting active {gvk.kind}", **{gvk.kind: ref})
                uid = m.get("uid", "")
                if self.opts.expectations:  # before the call: the watch event may beat the response
                    self.expect.expect_delete(self._ckey(cron), uid)
                try:
                    await self.client.delete(gvk, m.get("namespace", ""), m.get("name", ""),
                                             propagation_policy="Background", discard_response=True,
                                             priority=self._p_create)
                    self.stats["deletes"] += 1
                    metrics.child(metrics.WORKLOADS_DELETED, gvk.kind, "replace").inc()
                except errors.ApiError as e:
                    if not errors.is_not_found(e):
                        if self.opts.expectations:
                            self.expect.observe_delete(self._ckey(cron), uid)
                        log.error(e, f"Failed to delete active {gvk.kind}", **{gvk.kind: ref})
                        raise
                if self.opts.fold_created_into_active:
                    cron.status.active = [a for a in cron.status.active if a.uid != uid]

        # B18 (cron_controller.go:222-225, 349-387)
        try:
            workload = self.new_workload_from_template(cron, next_run)
        except Exception as e:
            raise RuntimeError(f"unable to initialize {gvk.kind} from cron template: {e}") from e

        # B19 (cron_controller.go:227-236)
        wm = workload["metadata"]
        ref = ObjectRef(wm.get("namespace", ""), wm.get("name", ""))
        if chatty:
            log.info(f"Creating {gvk.kind}", **{gvk.kind: ref})
        if self.opts.expectations:
            self.expect.expect_pending(self._ckey(cron), wm.get("name", ""))
        try:
            with (tracing.span("create_workload", kind=gvk.kind, name=wm.get("name", ""),
                               tick=missed_run.rfc3339()) if traced else tracing.NOOP) as sp:
                created = await self.client.create(gvk, workload, wm.get("namespace", ""),
                                                   decoder=self.codecs.child_object if self.codecs else None,
                                                   priority=self._p_create)
                if traced:
                    sp.set(tick_to_create_ms=(self.clock.now_ns() - missed_run.unix_nano()) / 1e6)
            self.stats["creates"] += 1
            metrics.child(metrics.WORKLOADS_CREATED, gvk.kind).inc()
            if self.opts.expectations:
                if self._observed_already(gvk, created):
                    # the watch event overtook the CREATE response: nothing left to expect
                    self.expect.drop_pending(self._ckey(cron), wm.get("name", ""))
                else:
                    self.expect.expect_create(self._ckey(cron), created)
            if self.opts.fold_created_into_active:
                cm = created.get("metadata") or {}
                cgvk = GroupVersionKind.from_object(created)
                cron.status.active.append(ObjectReference(
                    api_version=cgvk.api_version, kind=cgvk.kind, name=cm.get("name", ""),
                    namespace=cm.get("namespace", ""), uid=cm.get("uid", ""),
                    resource_version=cm.get("resourceVersion", "")
                    if self.opts.active_ref_resource_version != "omit" else ""))
            if self.latency_observer is not None:
                self.latency_observer(self._ckey(cron), missed_run, created)
            self._m_sched_lat.observe(
                max(0.0, (self.clock.now_ns() - missed_run.unix_nano()) / 1e9))
        except BaseException as e:  # API or transport error, or cancellation
            if self.opts.expectations and not isinstance(e, asyncio.CancelledError):
                # an API or transport error: nothing is in flight.  A cancelled CREATE (shutdown,
                # leader loss) may already be stored: its pending mark stays until the informer
                # sees the job or the TTL passes
                self.expect.drop_pending(self._ckey(cron), wm.get("name", ""))
            if isinstance(e, errors.ApiError) and errors.is_already_exists(e):
                log.info(f"{gvk.kind} already exists", **{gvk.kind: ref})
                if self.opts.expectations:
                    # the job is stored (an earlier CREATE whose response was lost): its ADDED
                    # event may have been dropped as ours while this CREATE was in flight, so no
                    # event is left to fold it into status.active -- reconcile once more
                    scheduled = Result(requeue=True)
            else:
                if isinstance(e, Exception):
                    self.recorder.eventf(cron.to_dict(), Warning, "FailedCreate", "Error creating %s: %s",
                                         gvk.kind, e)
                raise
        # B20 (cron_controller.go:237)
        cron.status.last_schedule_time = now
        return scheduled

    def _observed_already(self, gvk: GroupVersionKind, created: Dict[str, Any]) -> bool:
        """Does the child informer already hold the object our CREATE returned (same uid)?"""
        inf = self.child_informers.get(gvk)
        if inf is None:
            return False
        m = created.get("metadata") or {}
        cached = inf.get(m.get("namespace", ""), m.get("name", ""), copy=False)
        return cached is not None and (cached.get("metadata") or {}).get("uid") == m.get("uid")

    def _tick_already_ran(self, cron: Cron, missed_run: GoTime, active: List[Child],
                          terminated: List[Child]) -> bool:
        """Does a child named for ``missed_run``'s run exist?  Only for generated names: a
        template with a fixed ``metadata.name`` reuses one name for every run."""
        wl = cron.spec.template.workload
        hit = self._gvk_memo.get(f"{cron.namespace}/{cron.name}")
        fixed = hit[3] if hit is not None and hit[0] is wl else _template_fixed_name(wl)
        if fixed:
            return False
        try:
            ran = self.engine.next(self.engine.parse(cron.spec.schedule), missed_run)
        except ScheduleError:
            return False
        ran_name = get_default_job_name(cron.name, ran)
        prefix = cron.name + "-"
        for lst in (active, terminated):
            for info in lst:
                if info.name == ran_name:
                    return True
                # the name is Next(now) at the CREATE: for a cron spec that is Next(tick), but an
                # `@every` job is named for the moment it was created.  A later-named job created
                # at or after the tick ran it (or a later tick)
                suffix = info.name[len(prefix):] if info.name.startswith(prefix) else ""
                if suffix.isdigit() and int(suffix) > ran.sec:
                    key = info.sort_key
                    if key is None:
                        key = _sort_key(((info.obj or {}).get("metadata") or {}).get("creationTimestamp"))
                    if key[0] >= missed_run.sec:
                        return True
        return False

    # ------------------------------------------------------------------ children
    @staticmethod
    def _ckey(cron: Cron) -> str:
        return f"{cron.namespace}/{cron.name}"

    def child_transform(self, gvk: GroupVersionKind) -> Optional[Callable[[Dict[str, Any]], Dict[str, Any]]]:
        """The informer transform of ``gvk``'s children under these options."""
        o = self.opts
        if not o.slim_child_cache:
            return None
        if o.compact_metadata():
            return compact_child(gvk, o.workload)
        return slim_child

    async def child_informer(self, gvk: GroupVersionKind) -> Informer:
        inf = self.child_informers.get(gvk)
        if inf is None:
            assert self.cache is not None
            from ..runtime.informer import label_index

            inf = await self.cache.get_informer(gvk, label_selector=self.child_selector,
                                                indexers={CHILD_INDEX: label_index(LABEL_CRON_NAME)},
                                                transform=self.child_transform(gvk),
                                                decoder=self.codecs.child_event if self.codecs else None,
                                                list_decoder=self.codecs.child_list if self.codecs else None,
                                                keep=self.child_keep)
            self.child_informers[gvk] = inf
            self.ensure_derive(inf, gvk)
            inf.start()
            if self.on_child_informer is not None:
                self.on_child_informer(gvk, inf)
        return inf

    async def _synced_child_informer(self, gvk: GroupVersionKind) -> Optional[Informer]:
        """The synced child informer of ``gvk``; ``None`` when its first LIST is still running
        after ``child_sync_timeout`` (the caller then LISTs live).  A failed LIST raises: the
        worker is freed and the Cron retried with backoff instead of waiting on an informer
        that cannot sync (e.g. a kind the operator may not list)."""
        inf = await self.child_informer(gvk)
        if not inf.synced.is_set():
            try:
                await inf.wait_synced(self.opts.child_sync_timeout)
            except asyncio.TimeoutError:
                return None
            gctune.freeze()  # a newly synced child cache: long-lived, keep it out of GC scans
        return inf

    async def list_child_infos(self, cron: Cron, gvk: GroupVersionKind, log: Logger) -> Optional[List[_ChildInfo]]:
        """Cache mode: the Cron's children as :class:`_ChildInfo` memos kept by the child
        informer (``Informer.derive``), adjusted by expectations; ``None`` when the informer
        has not synced within ``child_sync_timeout`` (the caller LISTs live)."""
        log.v(1).info(f"Listing {gvk.kind}")
        inf = await self._synced_child_informer(gvk)
        if inf is None:
            return None
        self.ensure_derive(inf, gvk)
        return self._child_infos(inf, cron, gvk)

    def ensure_derive(self, inf: Informer, gvk: GroupVersionKind) -> None:
        """Install the child memo (:func:`child_info`) on ``gvk``'s informer.  Done when the
        informer is created, so each object is derived right after its transform -- which
        hands over the classification of the full status (:func:`compact_child`)."""
        if inf.derive is None and self.opts.classification_cache:
            policy = self.opts.workload
            inf.set_derive(lambda o, g=gvk: child_info(o, g, policy))

    def _child_infos(self, inf: Informer, cron: Cron, gvk: GroupVersionKind) -> List[_ChildInfo]:
        """The Cron's children from the synced informer's memos, adjusted by expectations."""
        self.stats["lists"] += 1
        key = f"{cron.namespace}/{cron.name}"
        infos = inf.derived_by_index(CHILD_INDEX, key)
        if self.opts.expectations and (key in self.expect.created or key in self.expect.deleted):
            objs = [i.obj for i in infos]
            adj = self.expect.adjust(key, objs)  # type: ignore[arg-type]
            if adj is not objs:
                by_id = {id(i.obj): i for i in infos}
                infos = [by_id.get(id(o)) or self._extra_info(o, gvk) for o in adj]
        return infos

    def _extra_info(self, w: Dict[str, Any], gvk: GroupVersionKind) -> _ChildInfo:
        """The memo of a child the informer has not delivered yet (our CREATE's response)."""
        m = w.get("metadata") or {}
        uid, rv = m.get("uid", ""), m.get("resourceVersion", "")
        info = self._class_cache.get(uid)
        if info is None or info.rv != rv or info.obj is not w:
            info = child_info(w, gvk, self.opts.workload)
            self._class_cache[uid] = info
        return info

    async def list_workloads(self, cron: Cron, gvk: GroupVersionKind, log: Logger,
                             force_live: bool = False) -> List[Dict[str, Any]]:
        """``listWorkloads`` (``cron_controller.go:241-266``): children of the template GVK in
        the Cron's namespace labelled ``kubedl.io/cron-name=<name>``."""
        log.v(1).info(f"Listing {gvk.kind}")
        self.stats["lists"] += 1
        inf = None
        if self.opts.list_mode != "live" and self.cache is not None and not force_live:
            inf = await self._synced_child_informer(gvk)
        if inf is None:
            lst = await self.client.list(gvk, cron.namespace, label_selector=f"{LABEL_CRON_NAME}={cron.name}")
            items = lst.get("items") or []
            for it in items:
                # list items may omit apiVersion/kind (built-in kinds); the reference reads them off the GVK
                it.setdefault("apiVersion", gvk.api_version)
                it.setdefault("kind", gvk.kind)
            return items
        children = inf.by_index(CHILD_INDEX, f"{cron.namespace}/{cron.name}", copy=False)
        if self.opts.expectations:
            children = self.expect.adjust(self._ckey(cron), children)
        return children

    # ------------------------------------------------------------------ status
    async def sync_status(self, cron: Cron, gvk: GroupVersionKind, active: List[Child],
                          terminated: List[Child], log: Logger,
                          gc: Optional[List["asyncio.Future[None]"]] = None) -> None:
        """``syncStatus`` (``cron_controller.go:268-282``)."""
        log.v(1).info("Syncing Cron status")
        self.sync_active_list(cron, gvk, active, log)
        await self.sync_cron_history(cron, gvk, terminated, log, gc)

    @staticmethod
    def _sort(items: List[Child]) -> None:
        """``sortByCreationTimestamp`` (``cron_util.go:116-129``): stable, oldest first."""
        if all(x.sort_key is not None for x in items):
            items.sort(key=_SORT_KEY)
        else:
            items.sort(key=lambda x: creation_timestamp(x.obj).key())  # type: ignore[arg-type]

    def sync_active_list(self, cron: Cron, gvk: GroupVersionKind, active: List[Child],
                         log: Logger, presorted: bool = False) -> None:
        """``syncActiveList`` (``cron_controller.go:284-304``)."""
        if log.enabled():
            log.v(1).info("Syncing active list")
        if not presorted:
            self._sort(active)
        refs = []
        rv_mode = self.opts.active_ref_resource_version
        with_rv = rv_mode != "omit"
        # "first": a child already listed keeps the reference it entered status.active with
        prev = {r.uid: r for r in cron.status.active if r.uid} if rv_mode == "first" and cron.status.active \
            else None
        for info in active:
            ref = prev.get(info.uid) if prev else None
            if ref is not None:
                refs.append(ref)
                continue
            ref = info.active_ref
            if ref is None:
                w = info.obj
                m = w.get("metadata") or {}  # type: ignore[union-attr]
                wgvk = GroupVersionKind.from_object(w)  # type: ignore[arg-type]
                ref = info.active_ref = ObjectReference(
                    api_version=wgvk.api_version, kind=wgvk.kind, name=m.get("name", ""),
                    namespace=m.get("namespace", ""), uid=m.get("uid", ""),
                    resource_version=m.get("resourceVersion", "") if with_rv else "")
            refs.append(ref)
        cron.status.active = refs

    async def sync_cron_history(self, cron: Cron, gvk: GroupVersionKind,
                                terminated: List[Child], log: Logger,
                                gc: Optional[List["asyncio.Future[None]"]] = None) -> None:
        """``syncCronHistory`` incl. history-limit GC (``cron_controller.go:306-346``).

        With ``gc`` (a list) the DELETEs are started and appended there instead of
        awaited one by one (``ReconcilerOptions.overlap_gc_deletes``)."""
        for op in self._sync_history(cron, terminated, log, gc):
            await op()

    def _sync_history(self, cron: Cron, terminated: List[Child], log: Logger,
                      gc: Optional[List["asyncio.Future[None]"]], presorted: bool = False) -> List[Any]:
        """The body of :meth:`sync_cron_history`.  GC DELETEs go to ``gc`` as started tasks,
        or (``gc`` is None) are returned as coroutine functions for the caller to await in order."""
        chatty = log.enabled()
        if chatty:
            log.v(1).info("Syncing Cron history")
        ops: List[Any] = []
        if not presorted:
            self._sort(terminated)
        limit = cron.spec.history_limit if cron.spec.history_limit is not None else MAX_INT
        cut = len(terminated) - limit  # the oldest `cut` children are beyond the history limit
        if cut > 0:
            memo = self.codecs.memo if self.codecs is not None else None
            for info in terminated[:cut]:
                he = info.history_entry
                if memo is not None and he is not None and he._json is not None:
                    # its status-history entry leaves for good: the codecs' memo need not keep it
                    # (else dead entries fill the table -- ~1 KiB per fire -- until collisions evict them)
                    memo.forget(he._json)
                w = info.obj
                m = w.get("metadata") or {}  # type: ignore[union-attr]
                wgvk = GroupVersionKind.from_object(w)
                ref = ObjectRef(m.get("namespace", ""), m.get("name", ""))
                if chatty:
                    log.info(f"Deleting terminated {wgvk.kind}", **{wgvk.kind: ref})
                args = (cron, wgvk, m.get("namespace", ""), m.get("name", ""), m.get("uid", ""), ref, log)
                if gc is None:
                    # the coroutine is created only when it is awaited: nothing is left un-awaited
                    # if an earlier DELETE ends the reconcile
                    ops.append(functools.partial(self._gc_delete, *args))
                else:
                    gc.append(asyncio.ensure_future(self._gc_delete(*args)))
            terminated = terminated[cut:]
        if self.opts.finished_time != "now":
            # the steady state: every kept child's entry was built for its current version
            history: List[CronHistory] = [info.history_entry or self._history_entry(cron, info, None)
                                          for info in terminated]
        else:
            now = self.clock.now(LOCAL)
            history = [self._history_entry(cron, info, now) for info in terminated]
        cron.status.history = history
        return ops

    def _history_entry(self, cron: Cron, info: _ChildInfo, now: Optional[GoTime]) -> CronHistory:
        """The ``status.history`` entry of terminated child ``info`` (``cron_controller.go:336-343``).
        ``now``: ``finished_time="now"`` (the reference stamps every entry with the reconcile's
        time).  An entry fully determined by the child's version is remembered in ``info``."""
        w: Dict[str, Any] = info.obj  # type: ignore[assignment]
        c: Classification = info.cls  # type: ignore[assignment]
        m = w.get("metadata") or {}
        wgvk = GroupVersionKind.from_object(w)
        entry = CronHistory(uid=m.get("uid", ""),
                            object=TypedLocalObjectReference(api_group=_gv_str(wgvk),
                                                             kind=wgvk.kind, name=m.get("name", "")),
                            status=c.status, created=creation_timestamp(w))
        if c.finished:
            if now is not None:
                entry.finished = now
            elif c.finished_at is not None:
                entry.finished = c.finished_at
                info.history_entry = entry  # fully determined by this child version
            else:
                # only a child without a completion time needs the previous entries (the last
                # entry with its uid, as a uid -> entry map of them would hold)
                prev = next((h for h in reversed(cron.status.history) if h.uid and h.uid == entry.uid), None)
                if prev is not None and prev.finished is not None:
                    entry.finished = prev.finished
                else:
                    # first observation: second precision so it survives the JSON round trip
                    t = self.clock.now(LOCAL)
                    entry.finished = GoTime(t.sec, 0, t.loc)
        return entry

    async def _gc_delete(self, cron: Cron, gvk: GroupVersionKind, namespace: str, name: str, uid: str,
                         ref: ObjectRef, log: Logger) -> None:
        """One history-limit DELETE (Background); errors are only logged (``cron_controller.go:324-333``)."""
        if self.opts.expectations:  # before the call: the watch event may beat the response
            self.expect.expect_delete(self._ckey(cron), uid)
        try:
            await self.client.delete(gvk, namespace, name, propagation_policy="Background", discard_response=True,
                                     priority=self._p_deferrable)
            self.stats["deletes"] += 1
            metrics.child(metrics.WORKLOADS_DELETED, gvk.kind, "history").inc()
        except asyncio.CancelledError:
            # the DELETE may or may not have reached the apiserver: let the informer decide
            if self.opts.expectations:
                self.expect.observe_delete(self._ckey(cron), uid)
            raise
        except Exception as e:  # noqa: BLE001 - any Delete error is only logged (:324-333)
            if not (isinstance(e, errors.ApiError) and errors.is_not_found(e)):
                if self.opts.expectations:
                    self.expect.observe_delete(self._ckey(cron), uid)
                log.error(e, f"Failed to delete terminated {gvk.kind}", **{gvk.kind: ref})

    # ------------------------------------------------------------------ workload creation
    def new_workload_from_template(self, cron: Cron, schedule_time: GoTime) -> Dict[str, Any]:
        """``newWorkloadFromTemplate`` (``cron_controller.go:348-387``)."""
        w = new_empty_workload(cron.spec.template.workload, self.opts.workload)
        m = w.get("metadata")
        if not isinstance(m, dict):
            m = w["metadata"] = {}
        # generateName is forbidden: a retried create must hit AlreadyExists (:355-362)
        if m.get("generateName"):
            m["generateName"] = ""
            del m["generateName"]
        if not m.get("name"):
            m["name"] = get_default_job_name(cron.name, schedule_time)
        else:
            self.recorder.event(cron.to_dict(), Normal, "OverridePolicy",
                                "metadata.name has been specified in workload template, override cron concurrency "
                                "policy as Forbidden")
            # replaced, not mutated: the parsed spec may be the memo shared across reconciles
            cron.spec = dataclasses.replace(cron.spec, concurrency_policy=ConcurrentPolicyForbid)
        m["namespace"] = cron.namespace
        labels = m.get("labels")
        if not isinstance(labels, dict):
            labels = m["labels"] = {}
        labels[LABEL_CRON_NAME] = cron.name
        if self.child_labels:
            labels.update(self.child_labels)
        set_controller_reference({"metadata": cron.metadata}, CRON_GVK, w)
        return w

    # ------------------------------------------------------------------ schedule
    def get_next_schedule(self, cron: Cron, now: GoTime, log: Optional[Logger] = None) -> Tuple[GoTime, GoTime]:
        """``getNextSchedule`` (``cron_controller.go:389-437``) -> (last missed, next)."""
        spec = cron.spec.schedule
        try:
            sched = self.engine.parse(spec)
        except ScheduleError as e:
            raise ScheduleError(f"unparsable cron {go_quote(spec)}: {e}") from None
        earliest = cron.status.last_schedule_time
        if earliest is None:
            earliest = cron.creation_timestamp
        if earliest.after(now):
            return GoTime.zero(), self.engine.next(sched, now)
        last, missed, bad = self.engine.missed(sched, earliest, now)
        if bad:
            raise ScheduleError(f"unschedulable cron {go_quote(spec)}: no matching time within five years")
        if missed > 1:
            metrics.MISSED_TICKS.inc(missed - 1)
        if missed > 100:
            self.recorder.eventf(cron.to_dict(), Warning, "TooManyMissedTimes",
                                 "too many missed start times: %d. Check clock skew", missed)
            if log is not None:
                log.info("Too many missed times", **{"missed times": missed})
        return last, self.engine.next(sched, now)
