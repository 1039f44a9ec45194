"""A realistic job lifecycle costs the optimized operator no extra API requests.

The Kubeflow training-operator writes a job's status several times while it runs: ``Created``,
``replicaStatuses`` as each pod starts, ``Running``, then ``Succeeded`` with ``completionTime``
(the ``JobStatus`` schema of ``/root/reference/test/crds/kubeflow.org_pytorchjobs.yaml:4739-4828``).
The reference rebuilds ``status.active`` with each child's *current* resourceVersion on every
reconcile (``/root/reference/internal/controller/cron_controller.go:284-304``) and requeues the
Cron on every owned-child event (``:70-77``), so each of those writes costs it a reconcile, a live
LIST and a status PATCH.  Here an active ref keeps the resourceVersion the child entered
``status.active`` with (``ReconcilerOptions.active_ref_resource_version="first"``, Kubernetes
CronJob semantics) and child updates that change nothing a reconcile reads are dropped
(``skip_unchanged_child_updates``).
"""
from __future__ import annotations

from cron_operator_amd.api.meta import GroupVersionKind, GroupVersionResource
from cron_operator_amd.api.v1alpha1 import CRON_GVR, LABEL_CRON_NAME, new_cron
from cron_operator_amd.bench.harness import BenchConfig, lifecycle_stages, pytorchjob_template, run
from cron_operator_amd.controller.reconciler import ReconcilerOptions
from cron_operator_amd.controller.setup import child_update_matters
from cron_operator_amd.models.workload import WorkloadPolicy
from cron_operator_amd.testing.env import TestEnv
from cron_operator_amd.trainingop.operator import lifecycle_status, lifecycle_statuses, replica_counts

NS = "default"
PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
PT_GVK = GroupVersionKind("kubeflow.org", "v1", "PyTorchJob")


def _job(name="j-1", rv="5", status=None, labels=None):
    o = dict(pytorchjob_template())
    o["metadata"] = {"name": name, "namespace": NS, "uid": "u1", "resourceVersion": rv,
                     "labels": labels if labels is not None else {LABEL_CRON_NAME: "j"},
                     "creationTimestamp": "2026-01-01T12:00:01Z"}
    if status is not None:
        o["status"] = status
    return o


def test_lifecycle_statuses_follow_the_training_operator_sequence():
    job = _job()
    assert replica_counts(job) == [("Master", 1), ("Worker", 1)]
    seq = lifecycle_statuses(job, "2026-01-01T12:00:01Z", "2026-01-01T12:00:30Z")
    # Created; Master pod active; Worker pod active; Running; Succeeded
    assert len(seq) == 5
    assert [c["type"] for c in seq[0]["conditions"]] == ["Created"]
    assert seq[0]["replicaStatuses"] == {"Master": {}, "Worker": {}}
    assert seq[1]["replicaStatuses"] == {"Master": {"active": 1}, "Worker": {}}
    assert seq[2]["replicaStatuses"] == {"Master": {"active": 1}, "Worker": {"active": 1}}
    assert [c["type"] for c in seq[3]["conditions"]] == ["Created", "Running"]
    last = seq[4]
    assert [(c["type"], c["status"]) for c in last["conditions"]] == [
        ("Created", "True"), ("Running", "False"), ("Succeeded", "True")]
    assert last["completionTime"] == "2026-01-01T12:00:30Z"
    assert last["replicaStatuses"] == {"Master": {"succeeded": 1}, "Worker": {"succeeded": 1}}
    for st in seq:  # every stage fits the reference's PyTorchJob status schema
        assert set(st) <= {"conditions", "replicaStatuses", "startTime", "completionTime", "lastReconcileTime"}
    for i in range(-len(seq), len(seq)):  # one stage at a time, as the bench writes them
        assert lifecycle_status(job, i, "2026-01-01T12:00:01Z", "2026-01-01T12:00:30Z") == seq[i], i
    three = _job()
    three["spec"]["pytorchReplicaSpecs"]["Worker"]["replicas"] = 3
    seq3 = lifecycle_statuses(three, "s", "e")
    assert len(seq3) == 7 and [lifecycle_status(three, i, "s", "e") for i in range(7)] == seq3
    assert lifecycle_stages(BenchConfig()) == 4 and lifecycle_stages(BenchConfig(lifecycle="instant")) == 0


def test_child_update_predicate_drops_only_running_status_churn():
    pol = WorkloadPolicy()
    seq = lifecycle_statuses(_job(), "2026-01-01T12:00:01Z", "2026-01-01T12:00:30Z")
    a, b = _job(rv="5", status=seq[0]), _job(rv="6", status=seq[1])
    assert not child_update_matters(a, b, PT_GVK, pol)               # replica count while running
    assert not child_update_matters(b, _job(rv="7", status=seq[3]), PT_GVK, pol)  # Running
    assert child_update_matters(_job(rv="7", status=seq[3]), _job(rv="8", status=seq[4]), PT_GVK, pol)
    assert child_update_matters(a, _job(rv="6", status=seq[1], labels={LABEL_CRON_NAME: "other"}), PT_GVK, pol)
    gone = _job(rv="6", status=seq[1])
    gone["metadata"]["deletionTimestamp"] = "2026-01-01T12:00:09Z"
    assert child_update_matters(a, gone, PT_GVK, pol)
    bad = _job(rv="6", status={"conditions": "not-a-list"})
    assert child_update_matters(a, bad, PT_GVK, pol)  # an unreadable status is reported by a reconcile


async def _lifecycle_cost(opts):
    """One Cron fires, then its job goes through the four pre-completion writes: API requests
    and reconciles the operator spends on them, and the active ref's resourceVersion after."""
    env = TestEnv()
    await env.create_cron(new_cron("j", NS, "*/1 * * * *", pytorchjob_template(), history_limit=2))
    await env.start_manager(opts)
    await env.settle()
    await env.advance(60)
    job = env.server.list(PT, NS, label_selector=f"{LABEL_CRON_NAME}=j")["items"][0]
    created_rv = job["metadata"]["resourceVersion"]
    req0, rec0 = env.client.requests, env.controller.reconciles
    for st in lifecycle_statuses(job, "2026-01-01T12:01:01Z", "2026-01-01T12:01:30Z")[:-1]:
        env.server.patch(PT, NS, job["metadata"]["name"], {"status": st}, "merge", "status")
        await env.settle()
    cost = (env.client.requests - req0, env.controller.reconciles - rec0,
            env.server.get(CRON_GVR, NS, "j")["status"]["active"][0]["resourceVersion"], created_rv,
            env.server.get(PT, NS, job["metadata"]["name"])["metadata"]["resourceVersion"])
    await env.stop()
    return cost


async def test_running_job_status_writes_cost_no_requests():
    reqs, recs, active_rv, created_rv, _ = await _lifecycle_cost(ReconcilerOptions())
    assert (reqs, recs) == (0, 0)
    assert active_rv == created_rv  # the ref keeps the version the job entered status.active with


async def test_reference_pays_a_patch_per_running_job_status_write():
    reqs, recs, active_rv, _, job_rv = await _lifecycle_cost(ReconcilerOptions.reference())
    assert recs >= 4 and reqs >= 8  # a live LIST + a status PATCH for each of the four writes
    assert active_rv == job_rv      # the ref follows the job's current resourceVersion


async def test_bench_realistic_lifecycle_requests_per_fire():
    """The done-when of the round-4 verdict: under the realistic sequence the optimized operator
    spends <= 4.5 API requests per fire (it spends 4.0: CREATE, the fire's status PATCH, the
    completion's status PATCH, the history-GC DELETE); the reference algorithm pays for every
    training-operator write."""
    opt = await run(BenchConfig(n_crons=20, steps=2, warmup=1, transport="memory", lifecycle="realistic"))
    assert opt.api_requests_per_fire <= 4.5, opt.api_requests_by_verb
    assert opt.reconciles_per_fire <= 2.0
    ref = await run(BenchConfig(n_crons=20, steps=2, warmup=1, transport="memory", lifecycle="realistic",
                                mode="reference"))
    assert ref.api_requests_per_fire >= 2 * opt.api_requests_per_fire, ref.api_requests_by_verb
