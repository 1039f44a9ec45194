"""RBAC: the shipped roles really let the operator run (reference Appendix B #1).

The reference's kustomize ClusterRole grants ``kubedl.io`` instead of
``apps.kubedl.io`` (``internal/controller/cron_controller.go:79-85`` ->
``config/rbac/role.yaml:7-32``); no reference test catches it because envtest
runs as admin.  Here the fake apiserver enforces RBAC and the operator runs
under the ServiceAccount that each install method creates:

* ``deploy/kustomize/default`` (our ``make build-installer`` output),
* the Helm chart (``charts/cron-operator``),

and the reference's own ``config/rbac/role.yaml`` (read as YAML text when the
checkout is present) is shown to be denied.
"""
from __future__ import annotations

import asyncio
import os
from typing import Any, Dict, Optional

import pytest
import yaml

from cron_operator_amd.api import errors
from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.api.v1alpha1 import CRON_GVR, LABEL_CRON_NAME
from cron_operator_amd.api.v1alpha1.crd import crd as cron_crd
from cron_operator_amd.apiserver.http import APIServerApp
from cron_operator_amd.apiserver.rbac import RBACAuthorizer, forbidden_message, rule_allows, service_account_user
from cron_operator_amd.apiserver.server import APIServer
from cron_operator_amd.controller.setup import setup_with_manager
from cron_operator_amd.runtime.client import Client
from cron_operator_amd.runtime.http import HttpTransport
from cron_operator_amd.runtime.kubeconfig import RestConfig
from cron_operator_amd.runtime.manager import Manager, ManagerOptions
from cron_operator_amd.testing.env import aligned_start
from cron_operator_amd.trainingop.crds import kubeflow_crds
from cron_operator_amd.utils.clock import FakeClock
from cron_operator_amd.utils.gotemplate import render_chart
from cron_operator_amd.utils.kustomize import build_sorted

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_ROLE = "/root/reference/config/rbac/role.yaml"
PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
PLURALS = {"Namespace": ("", "namespaces"), "ServiceAccount": ("", "serviceaccounts"),
           "ClusterRole": ("rbac.authorization.k8s.io", "clusterroles"),
           "ClusterRoleBinding": ("rbac.authorization.k8s.io", "clusterrolebindings"),
           "Role": ("rbac.authorization.k8s.io", "roles"),
           "RoleBinding": ("rbac.authorization.k8s.io", "rolebindings"),
           "Deployment": ("apps", "deployments"), "Service": ("", "services")}


# ------------------------------------------------------------------ rule semantics
def test_rule_matching():
    r = {"apiGroups": ["apps.kubedl.io"], "resources": ["crons", "crons/status"], "verbs": ["get", "patch"]}
    a = {"verb": "get", "group": "apps.kubedl.io", "resource": "crons", "namespace": "n", "name": "x"}
    assert rule_allows(r, a)
    assert rule_allows(r, dict(a, subresource="status", verb="patch"))
    assert not rule_allows(r, dict(a, subresource="finalizers", verb="patch"))
    assert not rule_allows(r, dict(a, group="kubedl.io"))  # the reference's wrong group
    assert not rule_allows(r, dict(a, verb="list"))
    star = {"apiGroups": ["*"], "resources": ["*/status"], "verbs": ["*"]}
    assert rule_allows(star, dict(a, subresource="status", verb="update"))
    assert not rule_allows(star, a)
    named = {"apiGroups": ["coordination.k8s.io"], "resources": ["leases"], "verbs": ["get", "list"],
             "resourceNames": ["619a52b8.kubedl.io"]}
    lease = {"verb": "get", "group": "coordination.k8s.io", "resource": "leases", "name": "619a52b8.kubedl.io"}
    assert rule_allows(named, lease)
    assert not rule_allows(named, dict(lease, name="other"))
    assert not rule_allows(named, dict(lease, verb="list", name=""))  # names never match collections
    nr = {"nonResourceURLs": ["/metrics", "/debug/*"], "verbs": ["get"]}
    assert rule_allows(nr, {"verb": "get", "path": "/metrics"})
    assert rule_allows(nr, {"verb": "get", "path": "/debug/pprof"})
    assert not rule_allows(nr, {"verb": "get", "path": "/healthz"})
    assert not rule_allows(nr, a)


def test_bindings_scope_and_aggregation():
    srv = APIServer(FakeClock(0), authorization="RBAC")
    rb = GroupVersionResource("rbac.authorization.k8s.io", "v1", "rolebindings")
    role = GroupVersionResource("rbac.authorization.k8s.io", "v1", "roles")
    cr = GroupVersionResource("rbac.authorization.k8s.io", "v1", "clusterroles")
    crb = GroupVersionResource("rbac.authorization.k8s.io", "v1", "clusterrolebindings")
    srv.create_namespace("a")
    srv.create_namespace("b")
    srv.create(role, "a", {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "Role",
                           "metadata": {"name": "pods", "namespace": "a"},
                           "rules": [{"apiGroups": [""], "resources": ["pods"], "verbs": ["list"]}]})
    srv.create(rb, "a", {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
                         "metadata": {"name": "pods", "namespace": "a"},
                         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "Role", "name": "pods"},
                         "subjects": [{"kind": "ServiceAccount", "name": "sa"}]})
    # aggregated ClusterRole picks up labelled roles
    srv.create(cr, "", {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                        "metadata": {"name": "view"},
                        "aggregationRule": {"clusterRoleSelectors": [{"matchLabels": {"agg": "view"}}]}})
    srv.create(cr, "", {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
                        "metadata": {"name": "cron-viewer", "labels": {"agg": "view"}},
                        "rules": [{"apiGroups": ["apps.kubedl.io"], "resources": ["crons"], "verbs": ["get"]}]})
    srv.create(crb, "", {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
                         "metadata": {"name": "view"},
                         "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": "view"},
                         "subjects": [{"kind": "Group", "name": "viewers"}]})
    az = RBACAuthorizer(srv)
    sa = service_account_user("a", "sa")
    pods = {"verb": "list", "group": "", "resource": "pods"}
    assert az.authorize(sa["username"], sa["groups"], dict(pods, namespace="a"))
    assert not az.authorize(sa["username"], sa["groups"], dict(pods, namespace="b"))
    assert not az.authorize("system:serviceaccount:b:sa", [], dict(pods, namespace="a"))
    get_cron = {"verb": "get", "group": "apps.kubedl.io", "resource": "crons", "namespace": "x", "name": "c"}
    assert az.authorize("alice", ["viewers"], get_cron)
    assert not az.authorize("alice", [], get_cron)
    assert az.authorize("root", ["system:masters"], dict(get_cron, verb="delete"))
    # SubjectAccessReview goes through the same authorizer
    assert srv.authorizer({"user": "alice", "groups": ["viewers"]}, {"resourceAttributes": get_cron})
    assert not srv.authorizer({"user": "alice", "groups": []}, {"resourceAttributes": get_cron})
    msg = forbidden_message("bob", get_cron)
    assert msg == ('crons.apps.kubedl.io "c" is forbidden: User "bob" cannot get resource "crons" in API group '
                   '"apps.kubedl.io" in the namespace "x"')


# ------------------------------------------------------------------ installs under RBAC
def _server(sa_ns: str, sa_name: str):
    clock = FakeClock(aligned_start())
    srv = APIServer(clock, gc=True, authorization="RBAC",
                    tokens={"admin": {"username": "admin", "groups": ["system:masters"]},
                            "sa": service_account_user(sa_ns, sa_name)})
    srv.install_crd(cron_crd())
    for c in kubeflow_crds():
        srv.install_crd(c)
    return clock, srv


def _apply(srv: APIServer, objs):
    for o in objs:
        if o["kind"] == "CustomResourceDefinition":
            continue  # installed above
        g, r = PLURALS[o["kind"]]
        gvr = GroupVersionResource(g, o["apiVersion"].rpartition("/")[2], r)
        ns = o["metadata"].get("namespace", "")
        if o["kind"] == "Namespace":
            try:
                srv.create(gvr, "", o)
            except errors.ApiError as e:
                assert errors.is_already_exists(e)
            continue
        if ns:
            try:
                srv.create_namespace(ns)
            except errors.ApiError:
                pass
        srv.create(gvr, ns, o)


async def _operator_fires_under(srv: APIServer, clock: FakeClock, lease_ns: str,
                                workload: Optional[Dict[str, Any]] = None,
                                gvr: GroupVersionResource = PT) -> None:
    app = APIServerApp(srv)
    port = await app.start("127.0.0.1", 0)
    admin = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}", bearer_token="admin")), qps=-1)
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}", bearer_token="sa")), qps=-1)
    mgr = Manager(client, ManagerOptions(clock=clock, leader_election=True, leader_election_namespace=lease_ns,
                                         health_probe_bind_address="0", metrics_bind_address="0"))
    task = None
    try:
        ctrl, rec = await setup_with_manager(mgr)
        task = asyncio.get_running_loop().create_task(mgr.start())
        await asyncio.wait_for(mgr.started.wait(), 20)
        cron = {"apiVersion": "apps.kubedl.io/v1alpha1", "kind": "Cron",
                "metadata": {"name": "rbac", "namespace": "default"},
                "spec": {"schedule": "* * * * *", "concurrencyPolicy": "Replace", "historyLimit": 0,
                         "template": {"workload": workload or {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                                               "spec": {"pytorchReplicaSpecs": {}}}}}}
        await admin.create(CRON_GVR, cron, "default")

        async def advance(seconds: int) -> None:
            # step the fake clock like wall time so the leader keeps renewing its Lease
            for _ in range(seconds):
                clock.advance(1)
                await asyncio.sleep(0.002)

        await advance(60)
        for _ in range(400):
            items = (await admin.list(gvr, "default", label_selector=f"{LABEL_CRON_NAME}=rbac"))["items"]
            if items:
                break
            await asyncio.sleep(0.01)
        assert items, f"no job created; reconcile errors={ctrl.errors}"
        # Replace: the next tick deletes the active job and creates a new one (delete verb granted)
        first = items[0]["metadata"]["name"]
        await advance(60)
        for _ in range(400):
            names = [o["metadata"]["name"] for o in
                     (await admin.list(gvr, "default", label_selector=f"{LABEL_CRON_NAME}=rbac"))["items"]]
            if names and first not in names:
                break
            await asyncio.sleep(0.01)
        assert names and first not in names
        st = (await admin.get(CRON_GVR, "default", "rbac")).get("status") or {}
        assert st.get("lastScheduleTime") and len(st.get("active") or []) == 1  # status subresource granted
        assert ctrl.errors == 0
    finally:
        mgr.stop()
        if task is not None:
            try:
                await asyncio.wait_for(task, 10)
            except Exception:  # noqa: BLE001
                pass
        await admin.close()
        await client.close()
        srv.close_all_watches()
        await app.stop()


async def test_kustomize_install_rbac_suffices():
    clock, srv = _server("cron-operator-system", "cron-operator-controller-manager")
    _apply(srv, build_sorted(os.path.join(ROOT, "deploy", "kustomize", "default")))
    await _operator_fires_under(srv, clock, "cron-operator-system")


async def test_helm_install_rbac_suffices():
    docs = render_chart(os.path.join(ROOT, "charts", "cron-operator"), {}, release="cron-operator",
                        namespace="cron-operator")
    objs = [o for lst in docs.values() for o in lst]
    sa = next(o for o in objs if o["kind"] == "ServiceAccount")
    for o in objs:
        o.setdefault("metadata", {}).setdefault("namespace", "cron-operator") \
            if o["kind"] not in ("ClusterRole", "ClusterRoleBinding") else None
    clock, srv = _server("cron-operator", sa["metadata"]["name"])
    srv.create_namespace("cron-operator")
    _apply(srv, objs)
    await _operator_fires_under(srv, clock, "cron-operator")


async def test_helm_install_rbac_covers_the_reference_charts_other_job_groups():
    """The reference chart grants KubeDL's ``xdl.kubedl.io`` XDLJob (``charts/cron-operator/
    templates/cluster_role.yaml:89-106``): a Cron templating one fires and replaces it under
    this chart's RBAC alone."""
    from cron_operator_amd.trainingop.crds import job_crd

    docs = render_chart(os.path.join(ROOT, "charts", "cron-operator"), {}, release="cron-operator",
                        namespace="cron-operator")
    objs = [o for lst in docs.values() for o in lst]
    sa = next(o for o in objs if o["kind"] == "ServiceAccount")
    for o in objs:
        if o["kind"] not in ("ClusterRole", "ClusterRoleBinding"):
            o.setdefault("metadata", {}).setdefault("namespace", "cron-operator")
    clock, srv = _server("cron-operator", sa["metadata"]["name"])
    srv.install_crd(job_crd("xdl.kubedl.io", "v1alpha1", "xdljobs", "XDLJob"))
    srv.create_namespace("cron-operator")
    _apply(srv, objs)
    await _operator_fires_under(srv, clock, "cron-operator",
                                workload={"apiVersion": "xdl.kubedl.io/v1alpha1", "kind": "XDLJob",
                                          "spec": {"xdlReplicaSpecs": {}}},
                                gvr=GroupVersionResource("xdl.kubedl.io", "v1alpha1", "xdljobs"))


async def test_operator_denied_without_binding():
    clock, srv = _server("cron-operator-system", "nobody")
    app = APIServerApp(srv)
    port = await app.start("127.0.0.1", 0)
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}", bearer_token="sa")), qps=-1)
    try:
        with pytest.raises(errors.ApiError) as ei:
            await client.list(CRON_GVR, "default")
        assert ei.value.code == 403 and "cannot list resource \"crons\"" in str(ei.value)
    finally:
        await client.close()
        await app.stop()


@pytest.mark.skipif(not os.path.exists(REF_ROLE), reason="reference checkout not present")
async def test_reference_kustomize_role_is_denied():
    """Reference Appendix B #1 reproduced: its manager-role cannot read Crons."""
    with open(REF_ROLE) as fh:
        ref_role = yaml.safe_load(fh)
    clock, srv = _server("cron-operator-system", "controller-manager")
    srv.create_namespace("cron-operator-system")
    binding = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
               "metadata": {"name": "manager-rolebinding"},
               "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                           "name": ref_role["metadata"]["name"]},
               "subjects": [{"kind": "ServiceAccount", "name": "controller-manager",
                             "namespace": "cron-operator-system"}]}
    _apply(srv, [ref_role, binding])
    app = APIServerApp(srv)
    port = await app.start("127.0.0.1", 0)
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}", bearer_token="sa")), qps=-1)
    try:
        with pytest.raises(errors.ApiError) as ei:
            await client.list(CRON_GVR, "default")
        assert ei.value.code == 403
        # ...while the kubeflow job rules in the same role do work
        await client.list(PT, "default")
    finally:
        await client.close()
        await app.stop()
