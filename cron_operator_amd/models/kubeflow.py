"""Kubeflow training-operator job status model (``kubeflow.org/v1`` JobStatus).

The reference converts a workload's unstructured ``.status`` into
``kubeflowv1.JobStatus`` (``internal/controller/cron_util.go:90-114``) and asks
``kubeflowutil.IsSucceeded``/``IsFailed`` whether it is terminal
(``cron_controller.go:146``, ``cron_util.go:73-88``).  Both come from the
training-operator module ([ext] ``go.mod:7``), which is not vendored; the shape
below is taken from the fake CRD schemas the reference tests load
(``test/crds/kubeflow.org_pytorchjobs.yaml:4739-4828``).

:func:`job_status_from_unstructured` is strict in the same places the
apimachinery converter is (wrong JSON types raise :class:`ConversionError`, so
the reconciler skips that workload) and lenient where it is lenient
(missing or non-object ``status`` -> empty status; unknown fields ignored, e.g.
MPIJob v1alpha1 ``launcherStatus``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

from ..utils.gotime import GoTime, parse_rfc3339

JobCreated = "Created"
JobRunning = "Running"
JobRestarting = "Restarting"
JobSucceeded = "Succeeded"
JobSuspended = "Suspended"
JobFailed = "Failed"

ConditionTrue = "True"
ConditionFalse = "False"
ConditionUnknown = "Unknown"


class ConversionError(ValueError):
    pass


@dataclass
class JobCondition:
    type: str = ""
    status: str = ""
    reason: str = ""
    message: str = ""
    last_update_time: Optional[GoTime] = None
    last_transition_time: Optional[GoTime] = None


@dataclass
class ReplicaStatus:
    active: int = 0
    succeeded: int = 0
    failed: int = 0
    selector: str = ""
    label_selector: Optional[Dict[str, Any]] = None


@dataclass
class JobStatus:
    conditions: List[JobCondition] = field(default_factory=list)
    replica_statuses: Dict[str, ReplicaStatus] = field(default_factory=dict)
    start_time: Optional[GoTime] = None
    completion_time: Optional[GoTime] = None
    last_reconcile_time: Optional[GoTime] = None


def _str(v: Any, path: str) -> str:
    if v is None:
        return ""
    if not isinstance(v, str):
        raise ConversionError(f"{path}: expected string, got {type(v).__name__}")
    return v


def _int(v: Any, path: str) -> int:
    if v is None:
        return 0
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise ConversionError(f"{path}: expected integer, got {type(v).__name__}")
    if isinstance(v, float) and not v.is_integer():
        raise ConversionError(f"{path}: expected integer, got fractional number")
    return int(v)


def _time(v: Any, path: str) -> Optional[GoTime]:
    if v is None:
        return None
    if not isinstance(v, str):
        raise ConversionError(f"{path}: expected RFC3339 string, got {type(v).__name__}")
    if v == "":
        return None
    try:
        return parse_rfc3339(v)
    except ValueError as e:
        raise ConversionError(f"{path}: {e}") from None


def job_status_from_unstructured(status: Dict[str, Any]) -> JobStatus:
    """The converted status; a status of well-typed JSON (what decoded objects almost always
    are) takes the fast path, anything else the strict one, which raises the precise error."""
    js = _fast_job_status(status)
    return js if js is not None else _strict_job_status(status)


_TIME_FIELDS = ("startTime", "completionTime", "lastReconcileTime")


def _fast_time(v: Any) -> Any:
    """A parsed time, None for absent/empty, or ``_BAD`` when the strict path must decide."""
    if v is None or v == "":
        return None
    if v.__class__ is not str:
        return _BAD
    try:
        return parse_rfc3339(v)
    except ValueError:
        return _BAD


_BAD = object()


def _fast_job_status(status: Dict[str, Any]) -> Optional[JobStatus]:
    """:func:`_strict_job_status` for exactly-typed input without building error paths;
    None when any field needs the strict path (wrong type, unparsable time, float counts)."""
    js = JobStatus()
    conds = status.get("conditions")
    if conds is not None:
        if conds.__class__ is not list:
            return None
        out = js.conditions
        for c in conds:
            if c.__class__ is not dict:
                return None
            t, st, r, m = c.get("type"), c.get("status"), c.get("reason"), c.get("message")
            if (t is not None and t.__class__ is not str) or (st is not None and st.__class__ is not str) or \
                    (r is not None and r.__class__ is not str) or (m is not None and m.__class__ is not str):
                return None
            lu, lt = _fast_time(c.get("lastUpdateTime")), _fast_time(c.get("lastTransitionTime"))
            if lu is _BAD or lt is _BAD:
                return None
            out.append(JobCondition(t or "", st or "", r or "", m or "", lu, lt))
    rs = status.get("replicaStatuses")
    if rs is not None:
        if rs.__class__ is not dict:
            return None
        for k, v in rs.items():
            if v is None:
                continue
            if v.__class__ is not dict:
                return None
            a, su, f, sel, ls = v.get("active"), v.get("succeeded"), v.get("failed"), v.get("selector"), \
                v.get("labelSelector")
            if (a is not None and a.__class__ is not int) or (su is not None and su.__class__ is not int) or \
                    (f is not None and f.__class__ is not int) or (sel is not None and sel.__class__ is not str) or \
                    (ls is not None and ls.__class__ is not dict):
                return None
            js.replica_statuses[k] = ReplicaStatus(a or 0, su or 0, f or 0, sel or "", ls)
    times = [_fast_time(status.get(f)) for f in _TIME_FIELDS]
    if times[0] is _BAD or times[1] is _BAD or times[2] is _BAD:
        return None
    js.start_time, js.completion_time, js.last_reconcile_time = times
    return js


def _strict_job_status(status: Dict[str, Any]) -> JobStatus:
    js = JobStatus()
    conds = status.get("conditions")
    if conds is not None:
        if not isinstance(conds, list):
            raise ConversionError("conditions: expected array")
        for i, c in enumerate(conds):
            if not isinstance(c, dict):
                raise ConversionError(f"conditions[{i}]: expected object")
            p = f"conditions[{i}]"
            js.conditions.append(JobCondition(
                type=_str(c.get("type"), p + ".type"), status=_str(c.get("status"), p + ".status"),
                reason=_str(c.get("reason"), p + ".reason"), message=_str(c.get("message"), p + ".message"),
                last_update_time=_time(c.get("lastUpdateTime"), p + ".lastUpdateTime"),
                last_transition_time=_time(c.get("lastTransitionTime"), p + ".lastTransitionTime")))
    rs = status.get("replicaStatuses")
    if rs is not None:
        if not isinstance(rs, dict):
            raise ConversionError("replicaStatuses: expected object")
        for k, v in rs.items():
            if v is None:
                continue
            if not isinstance(v, dict):
                raise ConversionError(f"replicaStatuses.{k}: expected object")
            p = f"replicaStatuses.{k}"
            sel = v.get("labelSelector")
            if sel is not None and not isinstance(sel, dict):
                raise ConversionError(p + ".labelSelector: expected object")
            js.replica_statuses[k] = ReplicaStatus(active=_int(v.get("active"), p + ".active"),
                                                   succeeded=_int(v.get("succeeded"), p + ".succeeded"),
                                                   failed=_int(v.get("failed"), p + ".failed"),
                                                   selector=_str(v.get("selector"), p + ".selector"),
                                                   label_selector=sel)
    js.start_time = _time(status.get("startTime"), "startTime")
    js.completion_time = _time(status.get("completionTime"), "completionTime")
    js.last_reconcile_time = _time(status.get("lastReconcileTime"), "lastReconcileTime")
    return js


def get_job_status(workload: Dict[str, Any]) -> JobStatus:
    """``getJobStatus`` (``cron_util.go:90-114``)."""
    st = workload.get("status")
    if not isinstance(st, dict):
        return JobStatus()
    return job_status_from_unstructured(st)


def has_condition(status: JobStatus, cond_type: str) -> bool:
    for c in status.conditions:
        if c.type == cond_type and c.status == ConditionTrue:
            return True
    return False


def is_succeeded(status: JobStatus) -> bool:
    return has_condition(status, JobSucceeded)


def is_failed(status: JobStatus) -> bool:
    return has_condition(status, JobFailed)


def terminal_condition(status: JobStatus) -> Optional[JobCondition]:
    for c in reversed(status.conditions):
        if c.type in (JobSucceeded, JobFailed) and c.status == ConditionTrue:
            return c
    return None
