"""Reconciler behaviour: the reference's envtest + unit tests, plus SURVEY Appendix A (B1-B24).

Mirrors ``internal/controller/cron_controller_test.go`` (reconcile succeeds,
creates a workload on a missed tick, suspend creates nothing, template metadata,
getNextSchedule vectors) and ``cron_util_test.go``, and adds the behaviours the
reference never tested (Forbid/Replace, history GC, deadline, status patching,
clock skew) -- each test names the Appendix A row it pins.  The reconciler is
called directly on a fake apiserver with an injected clock, like the reference
calls ``r.Reconcile(ctx, req)`` against envtest.
"""
from __future__ import annotations

import pytest

from cron_operator_amd.api import errors
from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.api.v1alpha1 import CRON_GVR, LABEL_CRON_NAME, Cron, new_cron
from cron_operator_amd.controller.reconciler import CronReconciler, ReconcilerOptions
from cron_operator_amd.cron.engine import NativeEngine, PythonEngine
from cron_operator_amd.runtime.controller import Request
from cron_operator_amd.runtime.events import FakeRecorder
from cron_operator_amd.testing.env import TestEnv
from cron_operator_amd.trainingop.operator import finished_status, running_status
from cron_operator_amd.utils.gotime import MINUTE, UTC, GoTime, parse_rfc3339
from cron_operator_amd.utils.logging import get_logger

PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
TF = GroupVersionResource("kubeflow.org", "v1", "tfjobs")
NS = "default"
NAME = "cron-test"
PT_TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"labels": {"test-label": "true"}}}
LOG = get_logger()

MODES = {"optimized": ReconcilerOptions(list_mode="live"), "reference": ReconcilerOptions.reference()}


def T(s: str) -> GoTime:
    return parse_rfc3339(s, UTC)


class Rig:
    """envtest-style rig: fake apiserver + a directly-called reconciler."""

    def __init__(self, options: ReconcilerOptions = None, engine=None):
        self.env = TestEnv()
        self.server = self.env.server
        self.clock = self.env.clock
        self.rec_events = FakeRecorder()
        self.r = CronReconciler(self.env.client, None, self.rec_events, self.clock, engine or NativeEngine(),
                                options or ReconcilerOptions(list_mode="live"))

    async def create(self, schedule="*/1 * * * *", workload=None, **kw):
        c = new_cron(NAME, NS, schedule, PT_TMPL if workload is None else workload, **kw)
        return await self.env.create_cron(c)

    async def reconcile(self):
        return await self.r.reconcile(Request(NS, NAME), LOG)

    def cron(self):
        return self.server.get(CRON_GVR, NS, NAME)

    def jobs(self, gvr=PT):
        return self.server.list(gvr, NS, label_selector=f"{LABEL_CRON_NAME}={NAME}")["items"]

    def set_status(self, **status):
        obj = self.cron()
        obj["status"] = dict(obj.get("status") or {}, **status)
        self.server.update(CRON_GVR, NS, NAME, obj, "status")

    def finish(self, name, ok=True, ts="2026-01-01T11:00:00Z"):
        self.server.patch(PT, NS, name, {"status": finished_status("PyTorchJob", name, ts, ok)}, "merge", "status")

    def advance(self, seconds):
        self.clock.advance(seconds)


# ---------------------------------------------------------------- reference envtest cases


@pytest.mark.parametrize("mode", MODES)
async def test_reconcile_succeeds(mode):
    rig = Rig(MODES[mode])
    await rig.create(concurrency_policy="Forbid")
    res = await rig.reconcile()
    assert res.after_ns() > 0  # cron_controller_test.go:84-88


@pytest.mark.parametrize("mode", MODES)
async def test_creates_workload_when_tick_missed(mode):
    # cron_controller_test.go:90-109: lastScheduleTime = now-2m -> a job with the cron label
    rig = Rig(MODES[mode])
    await rig.create(concurrency_policy="Forbid")
    now = rig.clock.now(UTC)
    rig.set_status(lastScheduleTime=now.add(-2 * MINUTE).utc().rfc3339())
    await rig.reconcile()
    jobs = rig.jobs()
    assert len(jobs) == 1
    assert jobs[0]["metadata"]["labels"][LABEL_CRON_NAME] == NAME
    assert jobs[0]["metadata"]["labels"]["test-label"] == "true"


@pytest.mark.parametrize("mode", MODES)
async def test_suspend_creates_nothing(mode):
    # cron_controller_test.go:111-129 (B10)
    rig = Rig(MODES[mode])
    await rig.create(suspend=True)
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    res = await rig.reconcile()
    assert rig.jobs() == []
    assert res.is_zero()  # no requeue


async def test_new_workload_from_template_populates_metadata():
    # cron_controller_test.go:139-159 (B18)
    rig = Rig()
    c = new_cron(NAME, NS, "*/1 * * * *", {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob"})
    c.metadata["uid"] = "u-1"
    t = GoTime(1767268800, 5, UTC)
    w = rig.r.new_workload_from_template(c, t)
    assert w["metadata"]["name"] == f"{NAME}-1767268800"
    assert w["metadata"]["namespace"] == NS
    assert w["metadata"]["labels"][LABEL_CRON_NAME] == NAME
    ref = w["metadata"]["ownerReferences"][0]
    assert ref == {"apiVersion": "apps.kubedl.io/v1alpha1", "kind": "Cron", "name": NAME, "uid": "u-1",
                   "controller": True, "blockOwnerDeletion": True}


@pytest.mark.parametrize("engine", [PythonEngine(), NativeEngine()], ids=["python", "native"])
def test_get_next_schedule_reference_vectors(engine):
    # cron_controller_test.go:162-223 (B12, B21)
    from cron_operator_amd.cron.engine import ScheduleError

    now = T("2026-01-01T12:00:00Z")
    rig = Rig(engine=engine)

    def cron(spec):
        c = new_cron(NAME, NS, spec, PT_TMPL)
        c.metadata["creationTimestamp"] = now.add(-5 * MINUTE).rfc3339()
        return c

    with pytest.raises(ScheduleError, match="unparsable cron"):
        rig.r.get_next_schedule(cron("60 31 30 2 *"), now)
    with pytest.raises(ScheduleError, match="unschedulable cron"):
        rig.r.get_next_schedule(cron("0 0 30 2 *"), now)
    last, nxt = rig.r.get_next_schedule(cron("*/1 * * * *"), now)
    assert last == now and nxt.sec == now.add(MINUTE).sec


# ---------------------------------------------------------------- Appendix A


async def test_b1_not_found_is_noop():
    rig = Rig()
    res = await rig.reconcile()
    assert res.is_zero()


@pytest.mark.parametrize("mode", MODES)
async def test_b2_status_written_only_via_status_patch(mode):
    rig = Rig(MODES[mode])
    await rig.create()
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    before = rig.server.stats.by_verb.get("patch", 0)
    updates_before = rig.server.stats.by_verb.get("update", 0)
    await rig.reconcile()
    assert rig.server.stats.by_verb.get("patch", 0) == before + 1
    assert rig.server.stats.by_verb.get("update", 0) == updates_before
    st = rig.cron()["status"]
    assert st["lastScheduleTime"] == rig.clock.now(UTC).utc().rfc3339()


async def test_parsed_status_memo_reused_only_for_identical_status(monkeypatch):
    """The status parsed on the last write is reused only while the stored status equals it."""
    from cron_operator_amd.api.v1alpha1 import types

    calls = []
    orig = types.CronStatus.from_dict
    monkeypatch.setattr(types.CronStatus, "from_dict", staticmethod(lambda d: calls.append(d) or orig(d)))
    rig = Rig()
    await rig.create(concurrency_policy="Forbid")
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    await rig.reconcile()
    job = rig.jobs()[0]["metadata"]["name"]
    n = len(calls)
    await rig.reconcile()  # status unchanged since our write: no re-parse
    assert len(calls) == n
    assert [a["name"] for a in rig.cron()["status"]["active"]] == [job]
    # an out-of-band edit (active cleared) must be parsed, not masked by the memo
    obj = rig.cron()
    obj["status"].pop("active", None)
    rig.server.update(CRON_GVR, NS, NAME, obj, "status")
    await rig.reconcile()
    assert len(calls) == n + 1
    assert [a["name"] for a in rig.cron()["status"]["active"]] == [job]  # re-derived from the child


async def test_b2_patch_error_is_joined_and_result_cleared():
    rig = Rig()
    await rig.create()
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    rig.server.faults.add(verb="patch", resource="crons", subresource="status", code=500, times=1)
    with pytest.raises(Exception, match="failed to patch Cron status"):
        await rig.reconcile()
    assert len(rig.jobs()) == 1  # the create itself went through


@pytest.mark.parametrize("workload,msg", [
    (None, "missing in Cron spec"),
    ({"kind": "PyTorchJob"}, "missing apiVersion or kind"),
])
async def test_b3_bad_template_no_requeue(workload, msg):
    rig = Rig()
    c = new_cron(NAME, NS, "*/1 * * * *", workload)
    if workload is None:
        c.spec.template.workload = None
    await rig.env.create_cron(c)
    res = await rig.reconcile()
    assert res.is_zero()
    assert rig.server.stats.by_resource_verb.get(("pytorchjobs", "create"), 0) == 0


@pytest.mark.parametrize("mode", MODES)
async def test_b4_children_selected_by_label_only(mode):
    rig = Rig(MODES[mode])
    await rig.create()
    # an unrelated PyTorchJob (no label) and one labelled for another cron
    rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": "x"}})
    rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "y", "labels": {LABEL_CRON_NAME: "other"}}})
    # labelled for us but without an ownerRef: still counted (B4: ownerRef not checked)
    rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "z", "labels": {LABEL_CRON_NAME: NAME}}})
    await rig.reconcile()
    st = rig.cron()["status"]
    assert [a["name"] for a in st["active"]] == ["z"]


@pytest.mark.parametrize("mode", MODES)
async def test_b5_b6_classification_and_active_refs(mode):
    rig = Rig(MODES[mode])
    await rig.create()
    for i, st in enumerate([None, "running", "succeeded", "failed"]):
        name = f"{NAME}-{i}"
        rig.clock.advance(1)
        rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                   "metadata": {"name": name, "labels": {LABEL_CRON_NAME: NAME}}})
        if st == "running":
            rig.server.patch(PT, NS, name, {"status": running_status("PyTorchJob", name, "2026-01-01T12:00:00Z")},
                             "merge", "status")
        elif st:
            rig.finish(name, ok=(st == "succeeded"))
    # unconvertible status: skipped entirely (B5)
    rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "bad", "labels": {LABEL_CRON_NAME: NAME}}})
    rig.server._bucket(rig.server.resource(PT))[NS]["bad"]["status"] = {"conditions": "oops"}
    await rig.reconcile()
    st = rig.cron()["status"]
    assert [a["name"] for a in st["active"]] == [f"{NAME}-0", f"{NAME}-1"]
    a0 = st["active"][0]
    assert a0["apiVersion"] == "kubeflow.org/v1" and a0["kind"] == "PyTorchJob" and a0["uid"] and \
        a0["resourceVersion"] and a0["namespace"] == NS
    assert [(h["object"]["name"], h["status"]) for h in st["history"]] == [(f"{NAME}-2", "Succeeded"),
                                                                          (f"{NAME}-3", "Failed")]
    assert st["history"][0]["object"]["apiGroup"] == "kubeflow.org/v1"  # group/version, back-compat


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("limit,kept", [(None, 5), (3, 3), (0, 0), (-1, 0)])
async def test_b7_history_limit_gc(mode, limit, kept):
    rig = Rig(MODES[mode])
    await rig.create(history_limit=limit)
    for i in range(5):
        rig.clock.advance(1)
        name = f"{NAME}-{i}"
        rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                   "metadata": {"name": name, "labels": {LABEL_CRON_NAME: NAME}}})
        rig.finish(name)
    await rig.reconcile()
    remaining = sorted(j["metadata"]["name"] for j in rig.jobs())
    assert remaining == [f"{NAME}-{i}" for i in range(5 - kept, 5)]  # oldest deleted first
    hist = (rig.cron().get("status") or {}).get("history") or []
    assert [h["object"]["name"] for h in hist] == remaining


async def test_b7_gc_deletes_overlap_the_status_patch():
    """``overlap_gc_deletes``: under apiserver latency the GC DELETEs and the status PATCH
    take one round trip together, not one each -- and the reconcile still returns only after
    every DELETE finished; a failed DELETE is only logged, as in the reference."""
    import time

    async def run(opts):
        rig = Rig(opts)
        await rig.create(history_limit=1)
        for i in range(4):
            rig.clock.advance(1)
            name = f"{NAME}-{i}"
            rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                       "metadata": {"name": name, "labels": {LABEL_CRON_NAME: NAME}}})
            rig.finish(name)
        rig.server.faults.add(verb="delete", resource="pytorchjobs", name=f"{NAME}-1", code=500)
        rig.server.faults.latency.update({"delete": 0.08, "patch": 0.08})
        t0 = time.perf_counter()
        await rig.reconcile()
        dt = time.perf_counter() - t0
        rig.server.faults.clear()
        assert sorted(j["metadata"]["name"] for j in rig.jobs()) == [f"{NAME}-1", f"{NAME}-3"]
        assert [h["object"]["name"] for h in rig.cron()["status"]["history"]] == [f"{NAME}-3"]
        return dt

    seq = await run(ReconcilerOptions(list_mode="live", overlap_gc_deletes=False))
    par = await run(ReconcilerOptions(list_mode="live"))
    assert seq >= 0.3  # 3 DELETEs + 1 PATCH, one after the other
    assert par < 0.2, (seq, par)


async def test_b7_finished_time_now_vs_completion():
    ref = Rig(ReconcilerOptions.reference())
    opt = Rig(ReconcilerOptions(list_mode="live"))
    for rig in (ref, opt):
        await rig.create()
        rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                   "metadata": {"name": "j", "labels": {LABEL_CRON_NAME: NAME}}})
        rig.finish("j", ts="2026-01-01T11:00:00Z")
        await rig.reconcile()
    assert ref.cron()["status"]["history"][0]["finished"] == ref.clock.now(UTC).utc().rfc3339()
    assert opt.cron()["status"]["history"][0]["finished"] == "2026-01-01T11:00:00Z"


@pytest.mark.parametrize("mode", MODES)
async def test_b8_b9_status_synced_before_deletion_stop(mode):
    rig = Rig(MODES[mode])
    obj = await rig.create()
    obj["metadata"]["finalizers"] = ["test/hold"]
    rig.server.update(CRON_GVR, NS, NAME, obj)
    rig.server.delete(CRON_GVR, NS, NAME)  # -> deletionTimestamp set, object kept
    rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "j", "labels": {LABEL_CRON_NAME: NAME}}})
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-5 * MINUTE).utc().rfc3339())
    res = await rig.reconcile()
    assert res.is_zero()
    st = rig.cron()["status"]
    assert [a["name"] for a in st["active"]] == ["j"]  # synced ...
    assert len(rig.jobs()) == 1  # ... but nothing scheduled


@pytest.mark.parametrize("mode", MODES)
async def test_b11_deadline_event_and_stop(mode):
    rig = Rig(MODES[mode])
    past = rig.clock.now(UTC).add(-MINUTE)
    await rig.create(deadline=GoTime(past.sec, 0, UTC))
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-5 * MINUTE).utc().rfc3339())
    res = await rig.reconcile()
    assert res.is_zero() and rig.jobs() == []
    assert rig.rec_events.reasons() == ["Deadline"]
    assert rig.rec_events.events[0][1] == "Normal"


async def test_b12_schedule_error_logged_not_requeued():
    rig = Rig()
    await rig.create(schedule="61 * * * *")
    res = await rig.reconcile()
    assert res.is_zero() and rig.jobs() == []


@pytest.mark.parametrize("mode", MODES)
async def test_unrunnable_cron_explained_by_a_warning_event(mode):
    """B3/B12 errors are only logged by the reference (``cron_controller.go:122-126,184-190``);
    the default mode also records a Warning event on the Cron, so ``kubectl describe cron``
    says why it never runs.  Reference mode stays silent, as the reference is."""
    rig = Rig(MODES[mode])
    await rig.create(schedule="61 * * * *")
    await rig.reconcile()
    tmpl = Rig(MODES[mode])
    c = new_cron(NAME, NS, "*/1 * * * *", {"kind": "PyTorchJob"})
    await tmpl.env.create_cron(c)
    await tmpl.reconcile()
    got = [(e[1], e[2]) for e in rig.rec_events.events + tmpl.rec_events.events]
    if mode == "optimized":
        assert got == [("Warning", "InvalidSchedule"), ("Warning", "InvalidTemplate")]
        assert "unparsable cron" in rig.rec_events.events[0][3]
        assert "missing apiVersion or kind" in tmpl.rec_events.events[0][3]
    else:
        assert got == []


@pytest.mark.parametrize("mode", MODES)
async def test_b13_b14_requeue_after_next_tick(mode):
    rig = Rig(MODES[mode])
    await rig.create()  # created at 12:00:05, clock at 12:00:05
    res = await rig.reconcile()
    now = rig.clock.now(UTC)
    assert res.after_ns() == T("2026-01-01T12:01:00Z").sub(now)
    assert rig.jobs() == []


@pytest.mark.parametrize("mode", MODES)
async def test_b15_forbid_skips_without_advancing(mode):
    rig = Rig(MODES[mode])
    await rig.create(concurrency_policy="Forbid")
    last = rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339()
    rig.set_status(lastScheduleTime=last)
    rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "running", "labels": {LABEL_CRON_NAME: NAME}}})
    res = await rig.reconcile()
    assert [j["metadata"]["name"] for j in rig.jobs()] == ["running"]
    assert rig.cron()["status"]["lastScheduleTime"] == last  # not advanced
    assert res.after_ns() > 0
    # once the running job finishes, the delayed run fires
    rig.finish("running")
    await rig.reconcile()
    assert len(rig.jobs()) == 2


@pytest.mark.parametrize("mode", MODES)
async def test_b16_replace_deletes_active(mode):
    rig = Rig(MODES[mode])
    await rig.create(concurrency_policy="Replace")
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "old", "labels": {LABEL_CRON_NAME: NAME}}})
    await rig.reconcile()
    names = [j["metadata"]["name"] for j in rig.jobs()]
    assert "old" not in names and len(names) == 1


async def test_b16_replace_delete_error_returned():
    rig = Rig()
    await rig.create(concurrency_policy="Replace")
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "old", "labels": {LABEL_CRON_NAME: NAME}}})
    rig.server.faults.add(verb="delete", resource="pytorchjobs", code=500)
    with pytest.raises(errors.ApiError):
        await rig.reconcile()
    assert [j["metadata"]["name"] for j in rig.jobs()] == ["old"]  # nothing created


@pytest.mark.parametrize("policy", ["", "Allow"])
async def test_b17_allow_creates_alongside_active(policy):
    rig = Rig()
    await rig.create(concurrency_policy=policy)
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "running", "labels": {LABEL_CRON_NAME: NAME}}})
    await rig.reconcile()
    assert len(rig.jobs()) == 2


async def test_b18_named_template_overrides_policy_in_memory():
    rig = Rig()
    tmpl = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
            "metadata": {"name": "fixed", "generateName": "gen-"}}
    await rig.create(workload=tmpl)
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    await rig.reconcile()
    jobs = rig.jobs()
    assert [j["metadata"]["name"] for j in jobs] == ["fixed"]
    assert "generateName" not in jobs[0]["metadata"]
    assert "OverridePolicy" in rig.rec_events.reasons()
    assert rig.cron()["spec"]["concurrencyPolicy"] == "Allow"  # never persisted


async def test_parsed_spec_memo_follows_the_spec_object_and_is_never_mutated():
    """With a Cron informer the parsed CronSpec is reused while the cached spec object is the
    same (the wire codec hands back one object per spec bytes); a new spec object is parsed
    again; the named-template override replaces the spec instead of mutating the memo."""
    rig = Rig(ReconcilerOptions())
    tmpl = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": {"name": "fixed"}}
    await rig.create(workload=tmpl)
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())

    class Inf:
        obj = rig.cron()

        def get(self, ns, name, copy=True):
            return self.obj

    inf = Inf()
    rig.r.cron_informer = inf
    key = f"{NS}/{NAME}"
    await rig.reconcile()
    spec1 = rig.r._spec_memo[key][1]
    assert spec1.concurrency_policy == "Allow"  # the override went to a copy
    inf.obj = rig.cron()
    inf.obj["spec"] = rig.r._spec_memo[key][0]  # same spec object, newer status
    await rig.reconcile()
    assert rig.r._spec_memo[key][1] is spec1 and spec1.concurrency_policy == "Allow"
    inf.obj = dict(inf.obj, spec=dict(inf.obj["spec"], suspend=True))
    await rig.reconcile()
    assert rig.r._spec_memo[key][1] is not spec1 and rig.r._spec_memo[key][1].suspend is True
    rig.r.forget_cron(key)
    assert key not in rig.r._spec_memo


@pytest.mark.parametrize("mode", MODES)
async def test_b18_job_name_uses_next_run(mode):
    rig = Rig(MODES[mode])
    await rig.create()
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    await rig.reconcile()
    # now = 12:00:05 -> missed tick 12:00:00, next run 12:01:00 names the job
    assert rig.jobs()[0]["metadata"]["name"] == f"{NAME}-{T('2026-01-01T12:01:00Z').sec}"


@pytest.mark.parametrize("mode", MODES)
async def test_b19_b20_already_exists_is_success(mode):
    rig = Rig(MODES[mode])
    await rig.create(concurrency_policy="Allow")
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    name = f"{NAME}-{T('2026-01-01T12:01:00Z').sec}"
    rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": name}})  # same name, not labelled
    await rig.reconcile()
    assert rig.cron()["status"]["lastScheduleTime"] == rig.clock.now(UTC).utc().rfc3339()


async def test_b19_create_error_emits_failed_create():
    rig = Rig()
    await rig.create()
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
    rig.server.faults.add(verb="create", resource="pytorchjobs", code=500, message="boom")
    with pytest.raises(errors.ApiError):
        await rig.reconcile()
    assert rig.rec_events.reasons() == ["FailedCreate"]
    assert rig.rec_events.events[0][1] == "Warning"
    assert "Error creating PyTorchJob" in rig.rec_events.events[0][3]
    assert "lastScheduleTime" in rig.cron()["status"]  # unchanged from set_status (not advanced)


async def test_b21_collapse_missed_and_too_many_event():
    rig = Rig()
    await rig.create()
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-300 * MINUTE).utc().rfc3339())
    await rig.reconcile()
    assert len(rig.jobs()) == 1  # only the last missed tick runs
    assert "TooManyMissedTimes" in rig.rec_events.reasons()
    msg = [e for e in rig.rec_events.events if e[2] == "TooManyMissedTimes"][0][3]
    assert msg == "too many missed start times: 300. Check clock skew"


async def test_b21_future_earliest_means_nothing_missed():
    rig = Rig()
    await rig.create()
    rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(10 * MINUTE).utc().rfc3339())  # clock skew
    res = await rig.reconcile()
    assert rig.jobs() == [] and res.after_ns() > 0


async def test_core_group_pod_template_supported_in_optimized_mode():
    opt = Rig()
    ref = Rig(ReconcilerOptions.reference())
    pod = {"apiVersion": "v1", "kind": "Pod", "spec": {"containers": [{"name": "c", "image": "busybox"}]}}
    for rig in (opt, ref):
        await rig.create(workload=pod)
        rig.set_status(lastScheduleTime=rig.clock.now(UTC).add(-2 * MINUTE).utc().rfc3339())
        await rig.reconcile()
    pods = GroupVersionResource("", "v1", "pods")
    assert len(opt.server.list(pods, NS)["items"]) == 1
    assert len(ref.server.list(pods, NS)["items"]) == 0  # reference rejects core-group templates


async def test_mpijob_v1alpha1_launcher_status_finishes():
    mpi = GroupVersionResource("kubeflow.org", "v1alpha1", "mpijobs")
    for opts, finished in ((ReconcilerOptions(list_mode="live"), True), (ReconcilerOptions.reference(), False)):
        rig = Rig(opts)
        await rig.create(workload={"apiVersion": "kubeflow.org/v1alpha1", "kind": "MPIJob"})
        rig.server.create(mpi, NS, {"apiVersion": "kubeflow.org/v1alpha1", "kind": "MPIJob",
                                    "metadata": {"name": "m", "labels": {LABEL_CRON_NAME: NAME}}})
        rig.server.patch(mpi, NS, "m", {"status": {"launcherStatus": "Succeeded"}}, "merge", "status")
        await rig.reconcile()
        st = rig.cron().get("status") or {}
        assert bool(st.get("history")) == finished
        assert bool(st.get("active")) != finished


async def test_noop_reconcile_sends_no_patch_optimized_but_does_in_reference():
    for opts, expect_patch in ((ReconcilerOptions(list_mode="live"), False), (ReconcilerOptions.reference(), True)):
        rig = Rig(opts)
        await rig.create()
        rig.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                   "metadata": {"name": "j", "labels": {LABEL_CRON_NAME: NAME}}})
        rig.finish("j")
        await rig.reconcile()
        rig.clock.advance(2)  # a later second: reference rewrites finished=now
        before = rig.server.stats.by_verb.get("patch", 0)
        await rig.reconcile()
        patched = rig.server.stats.by_verb.get("patch", 0) > before
        assert patched == expect_patch


async def test_child_cache_is_slimmed_in_optimized_mode_only():
    """``slim_child_cache``: cached children drop ``spec`` and ``managedFields`` (never read by a
    reconcile); the reference's typed informers cache whole objects."""
    from cron_operator_amd.testing.env import TestEnv as _Env

    for opts, slim in ((ReconcilerOptions(), True), (ReconcilerOptions.reference(), False)):
        env = _Env()
        await env.create_cron(new_cron(NAME, NS, "*/1 * * * *", PT_TMPL))
        env.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                   "metadata": {"name": "j", "labels": {LABEL_CRON_NAME: NAME},
                                                "managedFields": [{"manager": "kubectl"}]},
                                   "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}})
        await env.start_manager(opts)
        await env.settle()
        from cron_operator_amd.api.meta import GroupVersionKind

        inf = env.reconciler.child_informers.get(GroupVersionKind("kubeflow.org", "v1", "PyTorchJob"))
        if inf is None:  # reference mode: the static Owns() informer
            inf = next(i for i in env.manager.cache.informers() if i.name.startswith("pytorchjobs"))
        cached = inf.get(NS, "j", copy=False)
        assert ("spec" not in cached) is slim and ("managedFields" not in cached["metadata"]) is slim
        st = env.server.get(CRON_GVR, NS, NAME).get("status") or {}
        assert [a["name"] for a in st.get("active") or []] == ["j"]
        await env.stop()
