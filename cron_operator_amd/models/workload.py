"""Workload adapter (reference layer L3b: ``internal/controller/cron_util.go:37-129``).

A Cron's ``template.workload`` is an opaque manifest of any kind.  This module
turns it into an object to create, names it, and classifies existing children
as active or terminated.

Reference behaviour (kept bit-for-bit, including error strings the reference
tests assert on, ``cron_util_test.go:44-118``):

* :func:`new_empty_workload` -- ``workload template is missing in Cron spec`` for
  a nil template; JSON decode errors (including a missing ``kind``, which the
  unstructured decoder rejects) are ``failed to unmarshal workload template: ...``;
  an empty group/version/kind is ``workload template is missing apiVersion or kind``.
* :func:`get_default_job_name` -- ``<cron>-<unix seconds>``.
* :func:`is_workload_finished` -- (last condition type, Succeeded||Failed).
* :func:`sort_by_creation_timestamp` -- stable ascending sort.

Adapters beyond the reference (each switchable, see :class:`WorkloadPolicy`):

* ``allow_core_group`` -- accept ``apiVersion: v1`` templates such as a Pod (the
  reference rejects them although its doc comment promises Pod support,
  SURVEY Appendix B #7; BASELINE config 1 schedules a busybox Pod);
* ``builtin_status`` -- classify ``batch/v1`` Jobs by ``Complete``/``Failed``
  conditions and core Pods by ``status.phase``;
* ``mpi_launcher_status`` -- classify kubeflow MPIJob v1alpha1, whose status has
  no conditions, by ``status.launcherStatus`` (the reference never sees it finish,
  SURVEY section 3.4).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

from ..api.meta import GroupVersionKind, creation_timestamp
from ..utils import jsonutil
from ..utils.gotime import GoTime, parse_rfc3339
from . import kubeflow as kf


class WorkloadError(ValueError):
    pass


@dataclass
class WorkloadPolicy:
    allow_core_group: bool = True
    builtin_status: bool = True
    mpi_launcher_status: bool = True

    @staticmethod
    def reference() -> "WorkloadPolicy":
        """Exactly the reference's behaviour."""
        return WorkloadPolicy(allow_core_group=False, builtin_status=False, mpi_launcher_status=False)


def _decode(workload: Any) -> Dict[str, Any]:
    """``json.Unmarshal(raw, &unstructured.Unstructured{})``."""
    if isinstance(workload, (bytes, bytearray, str)):
        try:
            obj = jsonutil.loads(workload)
        except ValueError as e:
            raise WorkloadError(f"failed to unmarshal workload template: {e}") from None
    else:
        obj = jsonutil.deepcopy(workload)
    return _check_decoded(obj)


def _check_decoded(obj: Any) -> Dict[str, Any]:
    if not isinstance(obj, dict):
        raise WorkloadError("failed to unmarshal workload template: cannot unmarshal into Object: "
                           f"unexpected {type(obj).__name__}")
    kind = obj.get("kind")
    if not isinstance(kind, str) or kind == "":
        raise WorkloadError(f"failed to unmarshal workload template: Object 'Kind' is missing in "
                           f"'{jsonutil.dumps(obj)}'")
    av = obj.get("apiVersion")
    if av is not None and not isinstance(av, str):
        raise WorkloadError("failed to unmarshal workload template: apiVersion must be a string")
    return obj


def new_empty_workload(workload: Any, policy: Optional[WorkloadPolicy] = None) -> Dict[str, Any]:
    """``newEmptyWorkload`` (``cron_util.go:37-56``): a fresh, mutable copy."""
    if workload is None:
        raise WorkloadError("workload template is missing in Cron spec")
    obj = _decode(workload)
    gvk = GroupVersionKind.from_object(obj)
    allow_core = policy.allow_core_group if policy is not None else False
    if (gvk.group == "" and not allow_core) or gvk.version == "" or gvk.kind == "":
        raise WorkloadError("workload template is missing apiVersion or kind")
    return obj


def get_workload_gvk(workload: Any, policy: Optional[WorkloadPolicy] = None) -> GroupVersionKind:
    """``getWorkloadGVK`` (``cron_util.go:58-65``): the same checks and errors as
    :func:`new_empty_workload`, without copying a parsed (dict) template."""
    if workload is None:
        raise WorkloadError("workload template is missing in Cron spec")
    obj = _check_decoded(workload) if isinstance(workload, dict) else _decode(workload)
    gvk = GroupVersionKind.from_object(obj)
    allow_core = policy.allow_core_group if policy is not None else False
    if (gvk.group == "" and not allow_core) or gvk.version == "" or gvk.kind == "":
        raise WorkloadError("workload template is missing apiVersion or kind")
    return gvk


def get_default_job_name(cron_name: str, schedule_time: GoTime) -> str:
    """``getDefaultJobName`` (``cron_util.go:67-71``)."""
    return f"{cron_name}-{schedule_time.sec}"


def is_workload_finished(workload: Dict[str, Any]) -> Tuple[str, bool]:
    """``isWorkloadFinished`` (``cron_util.go:73-88``); conversion errors -> ("", False)."""
    try:
        st = kf.get_job_status(workload)
    except kf.ConversionError:
        return "", False
    finished = kf.is_failed(st) or kf.is_succeeded(st)
    if st.conditions:
        return st.conditions[-1].type, finished
    return "", finished


def sort_by_creation_timestamp(workloads: List[Dict[str, Any]]) -> None:
    """``sortByCreationTimestamp``: stable, ascending (``cron_util.go:116-129``)."""
    workloads.sort(key=lambda w: creation_timestamp(w).key())


@dataclass(slots=True, frozen=True)
class Classification:
    finished: bool
    status: str                      # history.status: last condition type (or phase)
    finished_at: Optional[GoTime]    # completion instant when the workload records one


def _parse_time(v: Any) -> Optional[GoTime]:
    if isinstance(v, str) and v:
        try:
            return parse_rfc3339(v)
        except ValueError:
            return None
    return None


def _kubeflow_summary_py(raw: Any):
    return None


def _native_summary():
    from ..utils import jsonutil

    if not jsonutil.NATIVE:
        return _kubeflow_summary_py
    from ..ops import fastjson_native

    return getattr(fastjson_native.load(), "kubeflow_summary", _kubeflow_summary_py)


# status dict -> (finished, last condition type, #conditions, completionTime, terminal
# lastTransitionTime) for exactly-typed statuses, else None (ops/csrc/fastjson.cpp)
_summary = _native_summary()


_FINISHED: Dict[Tuple[Any, Any], "Classification"] = {}


def classify(workload: Dict[str, Any], gvk: GroupVersionKind, policy: WorkloadPolicy) -> Classification:
    """Active/terminated decision for one child.  Raises ``kf.ConversionError``
    when the status does not convert (the reconciler then skips the child)."""
    raw = workload.get("status")
    sm = _summary(raw) if raw.__class__ is dict else None
    if sm is not None:  # a well-typed kubeflow status, read natively without building a JobStatus
        finished, last, nconds, comp, tltt = sm
        if finished:
            t = comp if comp is not None else tltt
            # one shared (read-only) classification per outcome and completion second: the jobs a
            # tick started mostly finish together, and every finished child is cached
            key = (last, t)
            c = _FINISHED.get(key)
            if c is None:
                if len(_FINISHED) >= 4096:
                    _FINISHED.clear()
                c = _FINISHED[key] = Classification(True, last, parse_rfc3339(t) if t is not None else None)
            return c
        has_conditions = nconds > 0
    else:
        st = kf.get_job_status(workload)
        finished = kf.is_succeeded(st) or kf.is_failed(st)
        last = st.conditions[-1].type if st.conditions else ""
        if finished:
            at = st.completion_time
            if at is None:
                tc = kf.terminal_condition(st)
                at = tc.last_transition_time if tc is not None else None
            return Classification(True, last, at)
        has_conditions = bool(st.conditions)
    raw = raw if isinstance(raw, dict) else {}
    if policy.builtin_status:
        if gvk.group == "batch" and gvk.kind == "Job":
            for c in reversed(raw.get("conditions") or []):
                if isinstance(c, dict) and c.get("status") == "True" and c.get("type") in ("Complete", "Failed"):
                    at = _parse_time(raw.get("completionTime")) or _parse_time(c.get("lastTransitionTime"))
                    return Classification(True, c.get("type"), at)
        if gvk.group == "" and gvk.kind == "Pod":
            phase = raw.get("phase")
            if phase in ("Succeeded", "Failed"):
                return Classification(True, phase, None)
            return _unfinished(phase or last)
    if policy.mpi_launcher_status and gvk.kind == "MPIJob" and not has_conditions:
        ls = raw.get("launcherStatus")
        if ls in (kf.JobSucceeded, kf.JobFailed):
            return Classification(True, ls, _parse_time(raw.get("completionTime")))
    return _unfinished(last)


def _unfinished(status: Any) -> Classification:
    """The shared classification of a child still running with last condition ``status``."""
    if status.__class__ is not str:
        return Classification(False, status, None)
    c = _UNFINISHED.get(status)
    if c is None:
        c = Classification(False, status, None)
        if len(_UNFINISHED) < 256:
            _UNFINISHED[status] = c
    return c


_UNFINISHED: Dict[Any, Classification] = {}
