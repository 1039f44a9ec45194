"""Unit tests mirroring the reference's pure-function tier.

``internal/controller/cron_util_test.go:38-251`` (newEmptyWorkload, getWorkloadGVK,
getDefaultJobName, getJobStatus, isWorkloadFinished, sortByCreationTimestamp) and
``internal/controller/util_test.go:28-63`` (logConstructor), plus JSON shape tests
for the API types (``api/v1alpha1/cron_types.go``).
"""
from __future__ import annotations

import io
import sys
import json

import pytest

from cron_operator_amd.api.meta import GroupVersionKind
from cron_operator_amd.api.v1alpha1 import (
    CRON_GVK,
    Cron,
    CronHistory,
    CronStatus,
    ObjectReference,
    TypedLocalObjectReference,
    new_cron,
)
from cron_operator_amd.models import kubeflow as kf
from cron_operator_amd.models.workload import (
    WorkloadError,
    WorkloadPolicy,
    get_default_job_name,
    get_workload_gvk,
    is_workload_finished,
    new_empty_workload,
    sort_by_creation_timestamp,
)
from cron_operator_amd.runtime.controller import Request
from cron_operator_amd.utils.gotime import MINUTE, UTC, GoTime, parse_rfc3339
from cron_operator_amd.utils.logging import log_constructor, new_from_options

# ---------------------------------------------------------------- newEmptyWorkload (cron_util_test.go:44-118)


def test_new_empty_workload_valid():
    obj = new_empty_workload(b'{"apiVersion":"kubeflow.org/v1","kind":"PyTorchJob"}')
    assert GroupVersionKind.from_object(obj) == GroupVersionKind("kubeflow.org", "v1", "PyTorchJob")


def test_new_empty_workload_missing_template():
    with pytest.raises(WorkloadError) as e:
        new_empty_workload(None)
    assert str(e.value) == "workload template is missing in Cron spec"


def test_new_empty_workload_invalid_json():
    with pytest.raises(WorkloadError, match="failed to unmarshal workload template"):
        new_empty_workload(b"{invalid json}")


def test_new_empty_workload_missing_api_version():
    with pytest.raises(WorkloadError) as e:
        new_empty_workload(b'{"kind":"PyTorchJob"}')
    assert str(e.value) == "workload template is missing apiVersion or kind"


def test_new_empty_workload_missing_kind_fails_at_unmarshal():
    with pytest.raises(WorkloadError, match="failed to unmarshal workload template"):
        new_empty_workload(b'{"apiVersion":"kubeflow.org/v1"}')


def test_new_empty_workload_core_group_policy():
    pod = {"apiVersion": "v1", "kind": "Pod"}
    with pytest.raises(WorkloadError, match="missing apiVersion or kind"):
        new_empty_workload(pod)  # reference behaviour (no policy)
    with pytest.raises(WorkloadError):
        new_empty_workload(pod, WorkloadPolicy.reference())
    assert new_empty_workload(pod, WorkloadPolicy())["kind"] == "Pod"


def test_new_empty_workload_returns_private_copy():
    tmpl = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"labels": {"a": "b"}}}
    w = new_empty_workload(tmpl)
    w["metadata"]["labels"]["x"] = "y"
    assert tmpl["metadata"]["labels"] == {"a": "b"}


def test_get_workload_gvk_tfjob():
    assert get_workload_gvk(b'{"apiVersion":"kubeflow.org/v1","kind":"TFJob"}') == \
        GroupVersionKind("kubeflow.org", "v1", "TFJob")


def test_get_default_job_name_deterministic():
    assert get_default_job_name("cron-test", GoTime(1234567890, 0, UTC)) == "cron-test-1234567890"


# ---------------------------------------------------------------- getJobStatus / isWorkloadFinished


def _with_conditions(*conds):
    return {"status": {"conditions": [{"type": t, "status": s} for t, s in conds]}}


def test_get_job_status_extracts_conditions():
    st = kf.get_job_status(_with_conditions(("Succeeded", "True")))
    assert len(st.conditions) == 1 and st.conditions[0].type == "Succeeded"


def test_get_job_status_missing_or_non_map_status_is_empty():
    assert kf.get_job_status({}).conditions == []
    assert kf.get_job_status({"status": "weird"}).conditions == []


def test_get_job_status_ignores_unknown_fields():
    st = kf.get_job_status({"status": {"launcherStatus": "Succeeded", "conditions": []}})
    assert st.conditions == []


def test_get_job_status_conversion_error():
    with pytest.raises(kf.ConversionError):
        kf.get_job_status({"status": {"conditions": "nope"}})
    with pytest.raises(kf.ConversionError):
        kf.get_job_status({"status": {"startTime": "yesterday"}})


@pytest.mark.parametrize("ctype,finished", [("Succeeded", True), ("Failed", True), ("Running", False)])
def test_is_workload_finished(ctype, finished):
    cond, fin = is_workload_finished(_with_conditions((ctype, "True")))
    assert fin == finished and cond == ctype


def test_is_workload_finished_requires_true_status_and_reports_last_type():
    cond, fin = is_workload_finished(_with_conditions(("Succeeded", "False"), ("Running", "True")))
    assert not fin and cond == "Running"
    cond, fin = is_workload_finished(_with_conditions(("Created", "True"), ("Succeeded", "True"),
                                                      ("Restarting", "True")))
    assert fin and cond == "Restarting"


def test_sort_by_creation_timestamp_stable_ascending():
    now = GoTime(1_800_000_000, 0, UTC)

    def w(name, delta):
        return {"metadata": {"name": name, "creationTimestamp": now.add(delta * MINUTE).rfc3339()}}

    ws = [w("w1", -10), w("w2", -20), w("w3", -5), w("w4", -10)]
    sort_by_creation_timestamp(ws)
    assert [x["metadata"]["name"] for x in ws] == ["w2", "w1", "w4", "w3"]


# ---------------------------------------------------------------- logConstructor (util_test.go:29-62)


def test_log_constructor_with_and_without_request():
    buf = io.StringIO()
    base = new_from_options(encoder="json", level="info", stream=buf)
    ctor = log_constructor(base, "Cron")
    ctor(None).info("hello")
    ctor(Request("ns", "n")).info("hi")
    lines = [json.loads(x) for x in buf.getvalue().splitlines()]
    assert lines[0]["controller"] == "cron" and "Cron" not in lines[0]
    assert lines[1]["Cron"] == {"name": "n", "namespace": "ns"} and lines[1]["controller"] == "cron"
    assert lines[1]["level"] == "info" and lines[1]["msg"] == "hi"


def test_log_levels_and_verbosity():
    buf = io.StringIO()
    log = new_from_options(encoder="json", level="1", stream=buf)
    log.v(1).info("shown")
    log.v(2).info("hidden")
    log.error(ValueError("x"), "err")
    out = buf.getvalue()
    assert "shown" in out and "hidden" not in out and '"error":"x"' in out


def test_console_encoder_format():
    buf = io.StringIO()
    log = new_from_options(encoder="console", level="info", stream=buf)
    log.with_values(controller="cron").info("Start reconciling Cron")
    parts = buf.getvalue().rstrip("\n").split("\t")
    assert parts[1] == "INFO" and parts[3] == "Start reconciling Cron" and json.loads(parts[4]) == {
        "controller": "cron"}
    assert parts[0].endswith("Z") and "T" in parts[0]


# ---------------------------------------------------------------- API types JSON (cron_types.go)


def test_cron_json_omission_rules():
    c = new_cron("c", "ns", "*/5 * * * *", {"apiVersion": "kubeflow.org/v1", "kind": "TFJob"})
    d = c.to_dict()
    assert d["apiVersion"] == "apps.kubedl.io/v1alpha1" and d["kind"] == "Cron"
    assert "status" not in d  # omitzero
    assert d["spec"] == {"schedule": "*/5 * * * *", "template": {"workload": {"apiVersion": "kubeflow.org/v1",
                                                                              "kind": "TFJob"}}}
    c.spec.suspend = False
    c.spec.history_limit = 0
    d = c.to_dict()
    assert d["spec"]["suspend"] is False and d["spec"]["historyLimit"] == 0  # pointers: present when set


def test_cron_status_roundtrip_and_semantic_equal():
    t = parse_rfc3339("2026-01-01T12:00:00Z", UTC)
    st = CronStatus(active=[ObjectReference(kind="PyTorchJob", namespace="ns", name="j", uid="u",
                                            api_version="kubeflow.org/v1", resource_version="7")],
                    history=[CronHistory(object=TypedLocalObjectReference(kind="PyTorchJob", name="h",
                                                                          api_group="kubeflow.org/v1"),
                                         status="Succeeded", uid="u2", created=t, finished=t)],
                    last_schedule_time=t)
    d = st.to_dict()
    assert d["active"][0] == {"kind": "PyTorchJob", "namespace": "ns", "name": "j", "uid": "u",
                              "apiVersion": "kubeflow.org/v1", "resourceVersion": "7"}
    assert d["history"][0] == {"uid": "u2", "object": {"apiGroup": "kubeflow.org/v1", "kind": "PyTorchJob",
                                                       "name": "h"},
                               "status": "Succeeded", "created": "2026-01-01T12:00:00Z",
                               "finished": "2026-01-01T12:00:00Z"}
    back = CronStatus.from_dict(json.loads(json.dumps(d)))
    assert back.semantic_equal(st)
    # nanosecond difference is a semantic difference (metav1.Time compares full precision)
    st2 = st.deepcopy()
    st2.last_schedule_time = t.add(1)
    assert not st2.semantic_equal(st)
    # nil == empty
    assert CronStatus().semantic_equal(CronStatus(active=[], history=[]))


def test_cron_from_dict_roundtrip():
    c = new_cron("c", "ns", "@daily", {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob"},
                 concurrency_policy="Replace", history_limit=3,
                 deadline=parse_rfc3339("2027-01-01T00:00:00Z", UTC))
    d = c.to_dict()
    c2 = Cron.from_dict(d)
    assert c2.to_dict() == d and c2.gvk() == CRON_GVK


def test_log_caller_is_the_log_call_site():
    """zap's ``caller`` field names the line of the log call itself (AddCaller)."""
    from cron_operator_amd.utils.logging import new_from_options

    buf = io.StringIO()
    log = new_from_options(encoder="json", level="info", stream=buf)
    line = sys._getframe().f_lineno + 1
    log.info("here")
    rec = json.loads(buf.getvalue().strip().splitlines()[-1])
    assert rec["caller"] == f"tests/test_util_parity.py:{line}"
