"""``apps.kubedl.io/v1alpha1`` API types: Cron, CronSpec, CronStatus, CronHistory.

Field names, optionality and JSON omission rules follow the reference schema
(``api/v1alpha1/cron_types.go:40-182``) so objects written by either operator
read identically:

* ``Cron`` -- ``metadata``/``status`` are ``omitzero`` (dropped when empty), ``spec``
  always present (``cron_types.go:40-55``);
* ``CronSpec`` -- ``schedule``/``template`` required; ``concurrencyPolicy``
  ``omitempty`` (CRD default ``Allow``); ``suspend``/``deadline``/``historyLimit`` are
  pointers, i.e. present whenever set, including ``false``/``0``
  (``cron_types.go:71-108``);
* ``CronTemplateSpec`` -- inline TypeMeta + opaque ``workload`` (any JSON object,
  ``PreserveUnknownFields``; ``cron_types.go:110-119``);
* ``CronStatus`` -- ``active`` (ObjectReference list), ``history`` (CronHistory
  list), ``lastScheduleTime``; both lists are atomic and omitted when empty
  (``cron_types.go:141-158``);
* ``CronHistory`` -- ``uid``, ``object`` (TypedLocalObjectReference whose
  ``apiGroup`` carries group/version for back-compat), ``status`` (job condition
  type, required), ``created``, ``finished`` (``cron_types.go:160-182``).

``semantic_equal`` reproduces ``apiequality.Semantic.DeepEqual`` as used on the
status at ``cron_controller.go:108``: times compare as instants at full
precision and an empty list equals a missing one.

``deepcopy()`` methods stand in for the generated ``zz_generated.deepcopy.go``.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Union

from ...utils import jsonutil
from ...utils.gotime import GoTime
from ..meta import GroupVersionKind, time_from_json, time_to_json
from .groupversion import CRON_GVK

# ConcurrencyPolicy (cron_types.go:121-139)
ConcurrentPolicyAllow = "Allow"
ConcurrentPolicyForbid = "Forbid"
ConcurrentPolicyReplace = "Replace"
CONCURRENCY_POLICIES = (ConcurrentPolicyAllow, ConcurrentPolicyForbid, ConcurrentPolicyReplace)

# kubeflow JobConditionType values used in history.status
JobCreated = "Created"
JobRunning = "Running"
JobRestarting = "Restarting"
JobSucceeded = "Succeeded"
JobSuspended = "Suspended"
JobFailed = "Failed"


def _t_eq(a: Optional[GoTime], b: Optional[GoTime]) -> bool:
    if a is None or b is None:
        return a is None and b is None
    return a.sec == b.sec and a.nsec == b.nsec


@dataclass(slots=True)
class ObjectReference:
    kind: str = ""
    namespace: str = ""
    name: str = ""
    uid: str = ""
    api_version: str = ""
    resource_version: str = ""
    field_path: str = ""

    def to_dict(self) -> Dict[str, Any]:
        d: Dict[str, Any] = {}
        if self.kind:
            d["kind"] = self.kind
        if self.namespace:
            d["namespace"] = self.namespace
        if self.name:
            d["name"] = self.name
        if self.uid:
            d["uid"] = self.uid
        if self.api_version:
            d["apiVersion"] = self.api_version
        if self.resource_version:
            d["resourceVersion"] = self.resource_version
        if self.field_path:
            d["fieldPath"] = self.field_path
        return d

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "ObjectReference":
        return ObjectReference(kind=d.get("kind", ""), namespace=d.get("namespace", ""), name=d.get("name", ""),
                               uid=d.get("uid", ""), api_version=d.get("apiVersion", ""),
                               resource_version=d.get("resourceVersion", ""), field_path=d.get("fieldPath", ""))


@dataclass(slots=True)
class TypedLocalObjectReference:
    kind: str = ""
    name: str = ""
    api_group: Optional[str] = None

    def to_dict(self) -> Dict[str, Any]:
        d: Dict[str, Any] = {}
        if self.api_group is not None:
            d["apiGroup"] = self.api_group
        d["kind"] = self.kind
        d["name"] = self.name
        return d

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "TypedLocalObjectReference":
        return TypedLocalObjectReference(kind=d.get("kind", ""), name=d.get("name", ""), api_group=d.get("apiGroup"))


@dataclass(slots=True)
class CronHistory:
    object: TypedLocalObjectReference = field(default_factory=TypedLocalObjectReference)
    status: str = ""
    uid: str = ""
    created: Optional[GoTime] = None
    finished: Optional[GoTime] = None
    # to_dict(shared=True) result: entries are complete before they are first serialised and
    # never mutated after (the reconciler reuses one entry per child version across reconciles)
    _json: Optional[Dict[str, Any]] = field(default=None, init=False, repr=False, compare=False)

    def to_dict(self, shared: bool = False) -> Dict[str, Any]:
        """JSON form; ``shared=True`` returns one cached dict per entry (read-only for callers)."""
        if shared and self._json is not None:
            return self._json
        # keys in sorted order, as a real apiserver serves a custom resource back (encoding/json
        # of unstructured content): the watch echo of a status write is then byte-identical to
        # what the wire codec remembered for this entry, and decodes to this very dict
        d: Dict[str, Any] = {}
        if self.created is not None:
            d["created"] = time_to_json(self.created)
        if self.finished is not None:
            d["finished"] = time_to_json(self.finished)
        d["object"] = self.object.to_dict()
        d["status"] = self.status
        if self.uid:
            d["uid"] = self.uid
        if shared:
            self._json = d
        return d

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "CronHistory":
        return CronHistory(object=TypedLocalObjectReference.from_dict(d.get("object") or {}),
                           status=d.get("status", ""), uid=d.get("uid", ""),
                           created=time_from_json(d.get("created")), finished=time_from_json(d.get("finished")))

    def semantic_equal(self, o: "CronHistory") -> bool:
        return (self.uid == o.uid and self.object == o.object and self.status == o.status
                and _t_eq(self.created, o.created) and _t_eq(self.finished, o.finished))


@dataclass(slots=True)
class CronStatus:
    active: List[ObjectReference] = field(default_factory=list)
    history: List[CronHistory] = field(default_factory=list)
    last_schedule_time: Optional[GoTime] = None

    def is_zero(self) -> bool:
        return not self.active and not self.history and self.last_schedule_time is None

    def to_dict(self, shared: bool = False) -> Dict[str, Any]:
        """JSON form; ``shared=True`` reuses each history entry's cached dict (the result is then
        read-only: the reconciler's status write only compares and serialises it)."""
        d: Dict[str, Any] = {}
        if self.active:
            d["active"] = [a.to_dict() for a in self.active]
        if self.history:
            # shared: an entry's cached JSON (never empty) without a call per entry
            d["history"] = [h._json or h.to_dict(True) for h in self.history] if shared else \
                [h.to_dict() for h in self.history]
        if self.last_schedule_time is not None:
            d["lastScheduleTime"] = time_to_json(self.last_schedule_time)
        return d

    @staticmethod
    def from_dict(d: Optional[Dict[str, Any]]) -> "CronStatus":
        d = d or {}
        return CronStatus(active=[ObjectReference.from_dict(a) for a in d.get("active") or []],
                          history=[CronHistory.from_dict(h) for h in d.get("history") or []],
                          last_schedule_time=time_from_json(d.get("lastScheduleTime")))

    def deepcopy(self) -> "CronStatus":
        return CronStatus(active=[dataclasses.replace(a) for a in self.active],
                          history=[CronHistory(object=dataclasses.replace(h.object), status=h.status,
                                               uid=h.uid, created=h.created, finished=h.finished)
                                   for h in self.history],
                          last_schedule_time=self.last_schedule_time)

    def snapshot(self) -> "CronStatus":
        """A copy sharing the (never mutated) entries: the reconciler only ever replaces
        ``active``/``history`` lists and their elements, so a list-level copy is enough to
        compare before/after (the deep copy rebuilt every history entry per reconcile)."""
        return CronStatus(active=list(self.active), history=list(self.history),
                          last_schedule_time=self.last_schedule_time)

    def semantic_equal(self, o: "CronStatus") -> bool:
        if len(self.active) != len(o.active) or len(self.history) != len(o.history):
            return False
        if not _t_eq(self.last_schedule_time, o.last_schedule_time):
            return False
        # a snapshot shares its entries: the same object is equal without a field compare
        if any(a is not b and a != b for a, b in zip(self.active, o.active)):
            return False
        return all(a is b or a.semantic_equal(b) for a, b in zip(self.history, o.history))


# The workload template is kept as parsed JSON (dict) when it came from the API,
# or as raw bytes/str when constructed from a RawExtension in tests.
Workload = Union[Dict[str, Any], bytes, str, None]


@dataclass
class CronTemplateSpec:
    workload: Workload = None
    api_version: str = ""
    kind: str = ""

    def to_dict(self) -> Dict[str, Any]:
        d: Dict[str, Any] = {}
        if self.api_version:
            d["apiVersion"] = self.api_version
        if self.kind:
            d["kind"] = self.kind
        if self.workload is not None:
            w = self.workload
            if isinstance(w, (bytes, str)):
                w = jsonutil.loads(w)
            d["workload"] = w
        return d

    @staticmethod
    def from_dict(d: Optional[Dict[str, Any]]) -> "CronTemplateSpec":
        d = d or {}
        return CronTemplateSpec(workload=d.get("workload"), api_version=d.get("apiVersion", ""),
                                kind=d.get("kind", ""))


@dataclass
class CronSpec:
    schedule: str = ""
    template: CronTemplateSpec = field(default_factory=CronTemplateSpec)
    concurrency_policy: str = ""
    suspend: Optional[bool] = None
    deadline: Optional[GoTime] = None
    history_limit: Optional[int] = None

    def to_dict(self) -> Dict[str, Any]:
        d: Dict[str, Any] = {"schedule": self.schedule, "template": self.template.to_dict()}
        if self.concurrency_policy:
            d["concurrencyPolicy"] = self.concurrency_policy
        if self.suspend is not None:
            d["suspend"] = self.suspend
        if self.deadline is not None:
            d["deadline"] = time_to_json(self.deadline)
        if self.history_limit is not None:
            d["historyLimit"] = self.history_limit
        return d

    @staticmethod
    def from_dict(d: Optional[Dict[str, Any]]) -> "CronSpec":
        d = d or {}
        return CronSpec(schedule=d.get("schedule", ""), template=CronTemplateSpec.from_dict(d.get("template")),
                        concurrency_policy=d.get("concurrencyPolicy", ""), suspend=d.get("suspend"),
                        deadline=time_from_json(d.get("deadline")), history_limit=d.get("historyLimit"))


@dataclass
class Cron:
    """A Cron object.  ``metadata`` stays an ObjectMeta JSON tree."""

    metadata: Dict[str, Any] = field(default_factory=dict)
    spec: CronSpec = field(default_factory=CronSpec)
    status: CronStatus = field(default_factory=CronStatus)
    api_version: str = CRON_GVK.api_version
    kind: str = CRON_GVK.kind

    # -- metadata accessors
    @property
    def name(self) -> str:
        return self.metadata.get("name", "")

    @property
    def namespace(self) -> str:
        return self.metadata.get("namespace", "")

    @property
    def uid(self) -> str:
        return self.metadata.get("uid", "")

    @property
    def resource_version(self) -> str:
        return self.metadata.get("resourceVersion", "")

    @property
    def creation_timestamp(self) -> GoTime:
        t = time_from_json(self.metadata.get("creationTimestamp"))
        return t if t is not None else GoTime.zero()

    @property
    def deletion_timestamp(self) -> Optional[GoTime]:
        return time_from_json(self.metadata.get("deletionTimestamp"))

    def gvk(self) -> GroupVersionKind:
        return CRON_GVK

    def to_dict(self) -> Dict[str, Any]:
        d: Dict[str, Any] = {"apiVersion": self.api_version, "kind": self.kind}
        if self.metadata:
            d["metadata"] = jsonutil.deepcopy(self.metadata)
        d["spec"] = self.spec.to_dict()
        if not self.status.is_zero():
            d["status"] = self.status.to_dict()
        return d

    @staticmethod
    def from_dict(d: Dict[str, Any], status: Optional[CronStatus] = None, spec: Optional[CronSpec] = None) -> "Cron":
        """``status`` / ``spec``: already parsed equivalents of ``d["status"]`` / ``d["spec"]`` (the
        caller vouches for them; a shared ``spec`` is never mutated -- it is replaced)."""
        return Cron(metadata=jsonutil.deepcopy(d.get("metadata") or {}),
                    spec=spec if spec is not None else CronSpec.from_dict(d.get("spec")),
                    status=status if status is not None else CronStatus.from_dict(d.get("status")),
                    api_version=d.get("apiVersion") or CRON_GVK.api_version, kind=d.get("kind") or CRON_GVK.kind)

    def deepcopy(self) -> "Cron":
        return Cron.from_dict(self.to_dict()) if not isinstance(self.spec.template.workload, (bytes, str)) else Cron(
            metadata=jsonutil.deepcopy(self.metadata),
            spec=CronSpec(schedule=self.spec.schedule,
                          template=CronTemplateSpec(self.spec.template.workload, self.spec.template.api_version,
                                                    self.spec.template.kind),
                          concurrency_policy=self.spec.concurrency_policy, suspend=self.spec.suspend,
                          deadline=self.spec.deadline, history_limit=self.spec.history_limit),
            status=self.status.deepcopy(), api_version=self.api_version, kind=self.kind)


def new_cron(name: str, namespace: str, schedule: str, workload: Workload, **spec_kw: Any) -> Cron:
    """Convenience constructor used by tests, examples and the bench."""
    return Cron(metadata={"name": name, "namespace": namespace},
                spec=CronSpec(schedule=schedule, template=CronTemplateSpec(workload=workload), **spec_kw))
