"""Parity pins against fixtures the reference itself ships (skipped when it is not mounted).

The reference's envtest suite (``internal/controller/suite_test.go:53-124``) installs the
Cron CRD from ``charts/cron-operator/crds`` and the Kubeflow CRDs from ``test/crds``.
Here the fake apiserver is given exactly those files (not this repo's CRD generator or
its slim training-operator schemas), and the reference's own example Crons
(``examples/v1alpha1/cron/cron-{pytorch,tf,mpi}.yaml``) run through several schedule
ticks in both reconciler modes.  Every object the operator writes -- the workloads built
from the templates, the Cron status patches -- is admitted by the reference's structural
schemas, and the fake training-operator's finished-status writes are too.
"""
from __future__ import annotations

import os

import pytest
import yaml

from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.api.v1alpha1 import CRON_GVR, LABEL_CRON_NAME
from cron_operator_amd.controller.reconciler import ReconcilerOptions
from cron_operator_amd.testing.env import TestEnv
from cron_operator_amd.trainingop.operator import FakeTrainingOperator

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "test", "crds")),
                                reason="reference checkout not mounted")

EXAMPLES = {
    "cron-pytorch.yaml": GroupVersionResource("kubeflow.org", "v1", "pytorchjobs"),
    "cron-tf.yaml": GroupVersionResource("kubeflow.org", "v1", "tfjobs"),
    "cron-mpi.yaml": GroupVersionResource("kubeflow.org", "v1alpha1", "mpijobs"),
}
MODES = {"optimized": ReconcilerOptions(), "reference": ReconcilerOptions.reference()}
NS = "default"


def _load(path: str):
    with open(path) as fh:
        return [d for d in yaml.safe_load_all(fh) if d]


def _reference_env() -> TestEnv:
    env = TestEnv(install_kubeflow=False)
    # the reference's CRDs replace this repo's: the Cron CRD as the chart ships it ...
    for d in _load(os.path.join(REF, "charts", "cron-operator", "crds", "apps.kubedl.io_crons.yaml")):
        env.server.install_crd(d)
    # ... and the Kubeflow CRDs its envtest installs
    for name in sorted(os.listdir(os.path.join(REF, "test", "crds"))):
        for d in _load(os.path.join(REF, "test", "crds", name)):
            env.server.install_crd(d)
    return env


@pytest.mark.parametrize("mode", MODES)
async def test_reference_examples_run_against_reference_crds(mode):
    env = _reference_env()
    trainer = FakeTrainingOperator(env.new_client(), env.clock, mode="timed", duration=20)
    await trainer.start()
    crons = {}
    for fname in EXAMPLES:
        (cron,) = _load(os.path.join(REF, "examples", "v1alpha1", "cron", fname))
        cron["metadata"]["namespace"] = NS
        await env.client.create(CRON_GVR, cron, NS)
        crons[fname] = cron["metadata"]["name"]
    await env.start_manager(MODES[mode])
    await env.settle()
    for _ in range(8):  # four one-minute ticks; every job finishes 20 s after it starts
        await env.advance(30)
    for fname, gvr in EXAMPLES.items():
        name = crons[fname]
        items = env.server.list(gvr, NS, label_selector=f"{LABEL_CRON_NAME}={name}")["items"]
        assert items, f"{fname}: no {gvr.resource} created"
        for w in items:
            # the template's labels/annotations are carried over, the owner is the Cron
            assert w["metadata"]["labels"]["key1"] == "value1"
            assert w["metadata"]["annotations"]["key2"] == "value2"
            ref = w["metadata"]["ownerReferences"][0]
            assert (ref["kind"], ref["name"], ref["controller"]) == ("Cron", name, True)
        st = env.server.get(CRON_GVR, NS, name)["status"]
        assert st.get("lastScheduleTime"), fname
        hist = st.get("history") or []
        if fname == "cron-mpi.yaml" and mode == "reference":
            # MPIJob v1alpha1 reports only status.launcherStatus, no conditions: the reference's
            # condition-based isWorkloadFinished never sees it finish, so
            # under Forbid its first job stays active and nothing else runs
            assert hist == [] and len(items) == 1 and len(st.get("active") or []) == 1
            continue
        assert hist and all(h["status"] == "Succeeded" for h in hist), (fname, hist)
        assert len(hist) <= 3  # the examples' historyLimit
    await trainer.stop()
    await env.stop()


async def test_mi355x_examples_are_valid_kubeflow_jobs_under_reference_crds():
    """This repo's MI355X example Crons (``examples/mi355x``: the smoke job, the torchrun DDP
    job and the Master + 7 Worker DDP job, with ``amd.com/gpu`` limits and RCCL env) produce
    PyTorchJobs the reference's ``kubeflow.org_pytorchjobs.yaml`` schema admits, on their own
    schedules (two of them ``CRON_TZ=Asia/Shanghai 30 2 * * *``)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = _reference_env()
    trainer = FakeTrainingOperator(env.new_client(), env.clock, mode="timed", duration=60)
    await trainer.start()
    pt = EXAMPLES["cron-pytorch.yaml"]
    crons = []
    for fname in sorted(os.listdir(os.path.join(root, "examples", "mi355x"))):
        for cron in _load(os.path.join(root, "examples", "mi355x", fname)):
            if cron.get("kind") != "Cron":
                continue
            cron["metadata"]["namespace"] = NS
            await env.client.create(CRON_GVR, cron, NS)
            crons.append(cron["metadata"]["name"])
    await env.start_manager(ReconcilerOptions())
    await env.settle()
    for _ in range(16):  # 8 hours: 02:30 Asia/Shanghai is 18:30 UTC, the env starts at 12:00 UTC
        await env.advance(1800)
    for name in crons:
        items = env.server.list(pt, NS, label_selector=f"{LABEL_CRON_NAME}={name}")["items"]
        assert items, f"{name}: no PyTorchJob admitted"
        st = env.server.get(CRON_GVR, NS, name)["status"]
        assert any(h["status"] == "Succeeded" for h in st.get("history") or []), (name, st)
    await trainer.stop()
    await env.stop()


def test_chart_rbac_grants_every_rule_of_the_reference_chart():
    """A Cron whose template names any kind the reference's Helm ClusterRole grants
    (``charts/cron-operator/templates/cluster_role.yaml``: kubeflow.org jobs, KubeDL's XDLJob,
    the xgboost-operator's XGBoostJob, events, leases, Crons) is creatable by this chart's
    operator too, so a switch-over keeps every working Cron working.  Child ``/status``
    subresources are read only here (the reference grants ``update`` it never uses)."""
    from cron_operator_amd.controller.rbac import RULES

    with open(os.path.join(REF, "charts", "cron-operator", "templates", "cluster_role.yaml")) as fh:
        ref_rules = yaml.safe_load(fh.read().split("\nrules:\n", 1)[1])
    granted = {(g, r, v) for rule in RULES for g in rule["apiGroups"] for r in rule["resources"]
               for v in rule["verbs"]}
    missing = []
    for rule in ref_rules:
        for g in rule["apiGroups"]:
            for r in rule["resources"]:
                child_status = r.endswith("/status") and not r.startswith("crons")
                for v in (["get"] if child_status else rule["verbs"]):
                    if (g, r, v) not in granted:
                        missing.append((g, r, v))
    assert not missing, missing


def test_chart_values_have_every_key_of_the_reference_chart():
    """A values file written for the reference chart keeps working: every key (nested) of its
    ``values.yaml`` exists here with the same type (docs/migration.md)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(REF, "charts", "cron-operator", "values.yaml")) as fh:
        ref = yaml.safe_load(fh)
    with open(os.path.join(root, "charts", "cron-operator", "values.yaml")) as fh:
        ours = yaml.safe_load(fh)

    def walk(a, b, path):
        for k, v in a.items():
            assert k in b, f"missing value {path}{k}"
            if isinstance(v, dict) and v:
                assert isinstance(b[k], dict), f"{path}{k} is not a map here"
                walk(v, b[k], f"{path}{k}.")
            elif v is not None and b[k] is not None:
                assert type(b[k]) is type(v) or {type(b[k]), type(v)} <= {int, float}, f"{path}{k} changed type"

    walk(ref, ours, "")
