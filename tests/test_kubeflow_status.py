"""The kubeflow JobStatus conversion's fast path (exactly-typed JSON) is the strict converter:
same JobStatus for every input the strict path accepts, and the strict path's exact
ConversionError for every input it rejects (``models/kubeflow.py``; reference converter
``internal/controller/cron_util.go:90-114``)."""
from __future__ import annotations

from hypothesis import given, settings
from hypothesis import strategies as st

from cron_operator_amd.models import kubeflow as kf

_scalar = st.one_of(st.none(), st.booleans(), st.integers(-3, 3), st.floats(-2, 2, allow_nan=False),
                    st.sampled_from(["", "True", "Succeeded", "Running", "x"]),
                    st.sampled_from(["2026-01-01T12:00:00Z", "2026-01-01T12:00:00.5+02:00", "2026-13-01T00:00:00Z",
                                     "not a time"]),
                    st.just([]), st.just({}))
_time = st.one_of(st.none(), st.just(""), st.integers(0, 2), st.sampled_from([
    "2026-01-01T12:00:00Z", "2026-02-30T01:02:03Z", "2026-01-01T12:00:00.123456789-07:00", "bad"]))
_cond = st.one_of(
    st.fixed_dictionaries({}, optional={"type": _scalar, "status": _scalar, "reason": _scalar, "message": _scalar,
                                        "lastUpdateTime": _time, "lastTransitionTime": _time}),
    _scalar)
_replica = st.one_of(st.none(), _scalar, st.fixed_dictionaries({}, optional={
    "active": _scalar, "succeeded": _scalar, "failed": _scalar, "selector": _scalar,
    "labelSelector": st.one_of(st.none(), st.just({"matchLabels": {"a": "b"}}), _scalar)}))
_status = st.fixed_dictionaries({}, optional={
    "conditions": st.one_of(st.lists(_cond, max_size=4), _scalar),
    "replicaStatuses": st.one_of(st.dictionaries(st.sampled_from(["Master", "Worker"]), _replica, max_size=2), _scalar),
    "startTime": _time, "completionTime": _time, "lastReconcileTime": _time})


def _outcome(fn, s):
    try:
        return "ok", fn(s)
    except kf.ConversionError as e:
        return "err", str(e)


@settings(max_examples=600, deadline=None)
@given(_status)
def test_fast_path_equals_strict_converter(status):
    assert _outcome(kf.job_status_from_unstructured, status) == _outcome(kf._strict_job_status, status)


def test_fast_path_taken_for_a_typical_finished_job():
    s = {"conditions": [{"type": "Created", "status": "True", "lastTransitionTime": "2026-01-01T12:00:00Z"},
                        {"type": "Succeeded", "status": "True", "reason": "Done",
                         "lastUpdateTime": "2026-01-01T12:01:00Z", "lastTransitionTime": "2026-01-01T12:01:00Z"}],
         "replicaStatuses": {"Master": {"succeeded": 1}}, "startTime": "2026-01-01T12:00:00Z",
         "completionTime": "2026-01-01T12:01:00Z"}
    fast = kf._fast_job_status(s)
    assert fast is not None and fast == kf._strict_job_status(s)
    assert kf.is_succeeded(fast) and fast.completion_time is not None
    assert kf._fast_job_status({"replicaStatuses": {"Master": {"active": True}}}) is None  # bool: strict path


_kinds = st.sampled_from([("kubeflow.org", "v1", "PyTorchJob"), ("kubeflow.org", "v1", "MPIJob"),
                          ("batch", "v1", "Job"), ("", "v1", "Pod")])


def _classify_outcome(workload, gvk):
    from cron_operator_amd.models.workload import WorkloadPolicy, classify

    try:
        c = classify(workload, gvk, WorkloadPolicy())
        return "ok", (c.finished, c.status, c.finished_at)
    except kf.ConversionError as e:
        return "err", str(e)


@settings(max_examples=600, deadline=None)
@given(st.one_of(_status, st.fixed_dictionaries({}, optional={"phase": st.sampled_from(["Succeeded", "Running"]),
                                                             "launcherStatus": st.sampled_from(["Succeeded", "x"]),
                                                             "conditions": st.lists(_cond, max_size=3)}),
                 _scalar), _kinds)
def test_native_status_summary_classifies_like_the_converter(status, kind):
    """classify() with the native kubeflow summary (``_fastjson.kubeflow_summary``) equals
    classify() on the Python converter for every status, typed or not."""
    import pytest

    from cron_operator_amd.api.meta import GroupVersionKind
    from cron_operator_amd.models import workload as wl

    if wl._summary is wl._kubeflow_summary_py:
        pytest.skip("_fastjson not built")
    gvk = GroupVersionKind(*kind)
    w = {"apiVersion": gvk.api_version, "kind": gvk.kind, "metadata": {"name": "j"}, "status": status}
    native = _classify_outcome(w, gvk)
    saved, wl._summary = wl._summary, wl._kubeflow_summary_py
    try:
        python = _classify_outcome(w, gvk)
    finally:
        wl._summary = saved
    assert native == python


def test_native_summary_is_taken_for_a_typical_finished_job():
    from cron_operator_amd.models import workload as wl

    if wl._summary is wl._kubeflow_summary_py:
        return
    s = {"conditions": [{"type": "Created", "status": "True", "lastTransitionTime": "2026-01-01T12:00:00Z"},
                        {"type": "Succeeded", "status": "True", "lastTransitionTime": "2026-01-01T12:01:00.5+02:00"}],
         "replicaStatuses": {"Master": {"succeeded": 1}}, "completionTime": ""}
    assert wl._summary(s) == (True, "Succeeded", 2, None, "2026-01-01T12:01:00.5+02:00")
    assert wl._summary({"replicaStatuses": {"M": {"active": True}}}) is None  # bool count: strict path
    assert wl._summary({"startTime": "2026-01-01T12:00:00Z\n"}) is None       # not ASCII-exact: strict path
