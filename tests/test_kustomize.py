"""``kustomize build`` of the shipped tree (reference: ``make build-installer``,
``Makefile:112-150``, which renders ``config/default`` into ``dist/install.yaml``).

Checks the transformers the install relies on -- namespace, namePrefix with
reference fix-ups, image override, JSON6902 patch -- plus strategic-merge and
6902 semantics on small inputs, and that every rendered object is accepted by
the fake apiserver (the "kubectl apply" smoke of the installer).
"""
from __future__ import annotations

import os

import pytest
import yaml

from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.apiserver.server import APIServer
from cron_operator_amd.cmd.main import main as cli
from cron_operator_amd.utils.clock import FakeClock
from cron_operator_amd.utils.kustomize import KustomizeError, apply_json6902, build, build_sorted, strategic_merge

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = os.path.join(ROOT, "deploy", "kustomize", "default")


def by_kind(objs, kind):
    return [o for o in objs if o["kind"] == kind]


def test_default_install_namespace_prefix_and_refs():
    objs = build_sorted(DEFAULT)
    kinds = [o["kind"] for o in objs]
    assert kinds[:2] == ["Namespace", "CustomResourceDefinition"]  # legacy order, as `kubectl apply` needs
    assert kinds[-2:] == ["Service", "Deployment"]
    crd = objs[1]
    assert crd["metadata"]["name"] == "crons.apps.kubedl.io"  # CRDs are never prefixed
    ns = by_kind(objs, "Namespace")
    assert [n["metadata"]["name"] for n in ns] == ["cron-operator-system"]
    for o in objs:
        if o["kind"] not in ("CustomResourceDefinition", "ClusterRole", "ClusterRoleBinding", "Namespace"):
            assert o["metadata"]["namespace"] == "cron-operator-system", o["metadata"]
        if o["kind"] != "CustomResourceDefinition":
            assert o["metadata"]["name"].startswith("cron-operator-")
    names = {(o["kind"], o["metadata"]["name"]) for o in objs}
    sa = by_kind(objs, "ServiceAccount")[0]["metadata"]["name"]
    for b in by_kind(objs, "ClusterRoleBinding") + by_kind(objs, "RoleBinding"):
        assert (b["roleRef"]["kind"], b["roleRef"]["name"]) in names
        for s in b["subjects"]:
            if s["kind"] == "ServiceAccount":
                assert s["name"] == sa and s["namespace"] == "cron-operator-system"
    dep = by_kind(objs, "Deployment")[0]
    pod = dep["spec"]["template"]["spec"]
    assert pod["serviceAccountName"] == sa
    c = pod["containers"][0]
    assert c["image"] == "docker.io/cron-operator-amd/cron-operator:0.3.0"
    # metrics patch (config/default/manager_metrics_patch.yaml analog) applied
    assert "--metrics-bind-address=:8443" in c["args"]
    assert "--leader-elect" in c["args"]
    assert {"name": "https", "containerPort": 8443} in c["ports"]
    # the user-facing aggregated roles keep the reference names under the prefix
    assert {"cron-operator-cron-admin-role", "cron-operator-cron-editor-role", "cron-operator-cron-viewer-role"} <= \
        {o["metadata"]["name"] for o in by_kind(objs, "ClusterRole")}
    # the manager role grants the right group (reference Appendix B #1 fixed)
    mgr = next(o for o in by_kind(objs, "ClusterRole") if o["metadata"]["name"] == "cron-operator-manager-role")
    assert any("apps.kubedl.io" in r.get("apiGroups", []) for r in mgr["rules"])


@pytest.mark.parametrize("overlay", ["prometheus", "network-policy", "crd", "rbac", "manager"])
def test_component_dirs_build(overlay):
    assert build(os.path.join(ROOT, "deploy", "kustomize", overlay))


def test_examples_kustomization_builds():
    objs = build(os.path.join(ROOT, "examples"))
    assert {o["kind"] for o in objs} == {"Cron"}
    assert len(objs) >= 5


def test_install_objects_accepted_by_apiserver():
    """`kubectl apply -f dist/install.yaml` against the fake apiserver."""
    srv = APIServer(FakeClock(0), gc=False)
    objs = build_sorted(DEFAULT)
    plural = {"CustomResourceDefinition": ("apiextensions.k8s.io", "customresourcedefinitions"),
              "Namespace": ("", "namespaces"), "ServiceAccount": ("", "serviceaccounts"),
              "ClusterRole": ("rbac.authorization.k8s.io", "clusterroles"),
              "ClusterRoleBinding": ("rbac.authorization.k8s.io", "clusterrolebindings"),
              "Role": ("rbac.authorization.k8s.io", "roles"),
              "RoleBinding": ("rbac.authorization.k8s.io", "rolebindings"),
              "Deployment": ("apps", "deployments"), "Service": ("", "services")}
    for o in objs:
        g, r = plural[o["kind"]]
        gvr = GroupVersionResource(g, o["apiVersion"].rpartition("/")[2], r)
        if o["kind"] == "CustomResourceDefinition":
            srv.install_crd(o)
            continue
        srv.create(gvr, o["metadata"].get("namespace", ""), o)
    # the CRD from the installer is live: a Cron can be created
    srv.create_namespace("d")
    srv.create(GroupVersionResource("apps.kubedl.io", "v1alpha1", "crons"),
               "d", {"apiVersion": "apps.kubedl.io/v1alpha1", "kind": "Cron",
                     "metadata": {"name": "c", "namespace": "d"},
                     "spec": {"schedule": "@hourly", "template": {"workload": {"apiVersion": "kubeflow.org/v1",
                                                                                "kind": "PyTorchJob"}}}})


def test_cli_kustomize_writes_installer(tmp_path, capsys):
    out = tmp_path / "dist" / "install.yaml"
    assert cli(["kustomize", DEFAULT, "-o", str(out)]) == 0
    docs = [d for d in yaml.safe_load_all(out.read_text()) if d]
    assert docs == build_sorted(DEFAULT)


def test_cli_helm_template_set(capsys):
    assert cli(["helm-template", os.path.join(ROOT, "charts", "cron-operator"), "--set", "qps=99",
                "--set", "leaderElection.enable=false"]) == 0
    text = capsys.readouterr().out
    assert "--qps=99" in text and "--leader-elect=false" in text


def test_json6902_ops():
    doc = {"a": {"b": [1, 2]}, "c": 1}
    out = apply_json6902(doc, [
        {"op": "add", "path": "/a/b/-", "value": 3},
        {"op": "add", "path": "/a/b/0", "value": 0},
        {"op": "replace", "path": "/c", "value": 2},
        {"op": "copy", "from": "/c", "path": "/d"},
        {"op": "move", "from": "/d", "path": "/e"},
        {"op": "remove", "path": "/a/b/1"},
        {"op": "test", "path": "/e", "value": 2},
        {"op": "add", "path": "/x~1y", "value": True},
    ])
    assert out == {"a": {"b": [0, 2, 3]}, "c": 2, "e": 2, "x/y": True}
    assert doc == {"a": {"b": [1, 2]}, "c": 1}  # input untouched
    with pytest.raises(KustomizeError):
        apply_json6902(doc, [{"op": "replace", "path": "/nope", "value": 1}])
    with pytest.raises(KustomizeError):
        apply_json6902(doc, [{"op": "test", "path": "/c", "value": 5}])


def test_strategic_merge_containers_by_name():
    base = {"spec": {"containers": [{"name": "a", "image": "x", "args": ["1"]}, {"name": "b", "image": "y"}],
                     "nodeSelector": {"k": "v"}}}
    patch = {"spec": {"containers": [{"name": "a", "image": "x2"}, {"name": "c", "image": "z"},
                                     {"name": "b", "$patch": "delete"}],
                      "nodeSelector": {"k": None, "k2": "v2"}}}
    out = strategic_merge(base, patch)
    assert out["spec"]["containers"] == [{"name": "a", "image": "x2", "args": ["1"]}, {"name": "c", "image": "z"}]
    assert out["spec"]["nodeSelector"] == {"k2": "v2"}


def test_overlay_with_labels_images_and_inline_patch(tmp_path):
    base = tmp_path / "base"
    base.mkdir()
    (base / "kustomization.yaml").write_text("resources: [dep.yaml]\n")
    (base / "dep.yaml").write_text(yaml.safe_dump({
        "apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "m"},
        "spec": {"selector": {"matchLabels": {"app": "m"}}, "template": {"metadata": {"labels": {"app": "m"}},
                 "spec": {"containers": [{"name": "c", "image": "controller:latest"}]}}}}))
    ov = tmp_path / "ov"
    ov.mkdir()
    (ov / "kustomization.yaml").write_text(yaml.safe_dump({
        "resources": ["../base"], "nameSuffix": "-x", "namespace": "n",
        "labels": [{"pairs": {"tier": "ops"}, "includeSelectors": True}],
        "images": [{"name": "controller", "newName": "reg/op", "newTag": "v9"}],
        "patches": [{"patch": "apiVersion: apps/v1\nkind: Deployment\nmetadata: {name: m}\nspec: {replicas: 3}\n"}]}))
    (o,) = build(str(ov))
    assert o["metadata"] == {"name": "m-x", "namespace": "n", "labels": {"tier": "ops"}}
    assert o["spec"]["replicas"] == 3
    assert o["spec"]["selector"]["matchLabels"] == {"app": "m", "tier": "ops"}
    assert o["spec"]["template"]["spec"]["containers"][0]["image"] == "reg/op:v9"


def test_patch_target_must_match(tmp_path):
    (tmp_path / "kustomization.yaml").write_text(yaml.safe_dump({
        "resources": [], "patches": [{"patch": "[]", "target": {"kind": "Deployment"}}]}))
    with pytest.raises(KustomizeError):
        build(str(tmp_path))


# ---------------------------------------------------------------- optional TLS pieces


def test_default_keeps_optional_sections_off():
    kinds = {o["kind"] for o in build(DEFAULT)}
    assert not kinds & {"Certificate", "Issuer", "ServiceMonitor", "NetworkPolicy"}
    dep = by_kind(build(DEFAULT), "Deployment")[0]["spec"]["template"]["spec"]
    assert dep["volumes"] == [] and dep["containers"][0]["volumeMounts"] == []


def test_cert_manager_metrics_and_servicemonitor_tls(tmp_path):
    """The reference's [METRICS-WITH-CERTS] + [PROMETHEUS] TLS variant
    (config/default/cert_metrics_manager_patch.yaml, config/prometheus/monitor_tls_patch.yaml):
    the Deployment mounts the cert-manager Secret and serves it; the ServiceMonitor verifies it
    against the prefixed Service's DNS name; the Certificate covers those names and points at
    the prefixed Issuer."""
    from cron_operator_amd.utils.kustomize import enable_optional

    objs = build_sorted(enable_optional(DEFAULT, str(tmp_path / "tree")))
    svc = [o for o in by_kind(objs, "Service") if "metrics" in o["metadata"]["name"]][0]
    host = f"{svc['metadata']['name']}.cron-operator-system.svc"
    assert host == "cron-operator-controller-manager-metrics-service.cron-operator-system.svc"
    cert = by_kind(objs, "Certificate")[0]
    assert cert["spec"]["dnsNames"] == [host, host + ".cluster.local"]
    assert cert["spec"]["secretName"] == "metrics-server-cert"
    issuer = by_kind(objs, "Issuer")[0]
    assert cert["spec"]["issuerRef"] == {"kind": "Issuer", "name": issuer["metadata"]["name"]}
    assert issuer["metadata"]["namespace"] == cert["metadata"]["namespace"] == "cron-operator-system"
    pod = by_kind(objs, "Deployment")[0]["spec"]["template"]["spec"]
    c = pod["containers"][0]
    assert "--metrics-cert-path=/tmp/k8s-metrics-server/metrics-certs" in c["args"]
    assert "--metrics-bind-address=:8443" in c["args"]
    assert c["volumeMounts"] == [{"name": "metrics-certs", "mountPath": "/tmp/k8s-metrics-server/metrics-certs",
                                  "readOnly": True}]
    vol = pod["volumes"][0]
    assert vol["secret"]["secretName"] == "metrics-server-cert"
    assert sorted(i["key"] for i in vol["secret"]["items"]) == ["ca.crt", "tls.crt", "tls.key"]
    mon = by_kind(objs, "ServiceMonitor")[0]
    tls = mon["spec"]["endpoints"][0]["tlsConfig"]
    assert tls["serverName"] == host and tls["insecureSkipVerify"] is False
    assert tls["ca"]["secret"] == {"name": "metrics-server-cert", "key": "ca.crt"}
    assert tls["keySecret"] == {"name": "metrics-server-cert", "key": "tls.key"}
    assert by_kind(objs, "NetworkPolicy")


def test_cli_enable_optional_renders_certs(tmp_path):
    out = tmp_path / "install-certs.yaml"
    assert cli(["kustomize", "--enable-optional", DEFAULT, "-o", str(out)]) == 0
    kinds = [d["kind"] for d in yaml.safe_load_all(out.read_text())]
    assert "Certificate" in kinds and "ServiceMonitor" in kinds


def test_replacements_semantics(tmp_path):
    (tmp_path / "kustomization.yaml").write_text(yaml.safe_dump({
        "namePrefix": "p-",
        "resources": ["objs.yaml"],
        "replacements": [
            {"source": {"kind": "Service", "name": "svc", "fieldPath": "metadata.name"},
             "targets": [{"select": {"kind": "ConfigMap"},
                          "fieldPaths": ["data.host", "data.[a.b/c]"],
                          "options": {"delimiter": ".", "index": 0, "create": True}},
                         {"select": {"kind": "Deployment"},
                          "fieldPaths": ["spec.template.spec.containers.[name=app].env.[name=SVC].value"]}]},
            {"source": {"kind": "ConfigMap", "name": "cm", "fieldPath": "data.host",
                        "options": {"delimiter": ".", "index": 1}},
             "targets": [{"select": {"kind": "Deployment"}, "fieldPaths": ["metadata.annotations.zone"],
                          "options": {"create": True}}]},
        ]}))
    (tmp_path / "objs.yaml").write_text(yaml.safe_dump_all([
        {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "svc"}},
        {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cm"}, "data": {"host": "X.zone1.svc"}},
        {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d"},
         "spec": {"template": {"spec": {"containers": [{"name": "app", "env": [{"name": "SVC", "value": ""}]}]}}}},
    ]))
    objs = {o["kind"]: o for o in build(str(tmp_path))}
    assert objs["ConfigMap"]["data"] == {"host": "p-svc.zone1.svc", "a.b/c": "p-svc"}
    assert objs["Deployment"]["spec"]["template"]["spec"]["containers"][0]["env"][0]["value"] == "p-svc"
    assert objs["Deployment"]["metadata"]["annotations"] == {"zone": "zone1"}
    # a source that matches nothing is an error, as in kustomize
    k = yaml.safe_load((tmp_path / "kustomization.yaml").read_text())
    k["replacements"][0]["source"]["name"] = "nope"
    (tmp_path / "kustomization.yaml").write_text(yaml.safe_dump(k))
    with pytest.raises(KustomizeError):
        build(str(tmp_path))


REF_CONFIG = "/root/reference/config/default"


@pytest.mark.skipif(not os.path.isdir(REF_CONFIG), reason="reference checkout not mounted")
def test_reference_config_tree_builds_with_this_renderer():
    """Parity pin for the kustomize subset: the reference's own ``config/default`` tree
    (``make build-installer``, Makefile) renders with ``utils/kustomize.py``: the
    ``cron-operator-`` name prefix and ``cron-operator-system`` namespace land on every object,
    the metrics JSON6902 patch inserts ``--metrics-bind-address=:8443`` at ``args[0]``
    (``config/default/manager_metrics_patch.yaml``), and this CLI parses the resulting args."""
    from cron_operator_amd.cmd.main import build_parser, cobra_order

    objs = build_sorted(REF_CONFIG)
    kinds = sorted(o["kind"] for o in objs)
    assert kinds.count("ClusterRole") == 6 and kinds.count("Deployment") == 1 \
        and kinds.count("CustomResourceDefinition") == 1
    for o in objs:
        m = o["metadata"]
        if o["kind"] not in ("Namespace", "CustomResourceDefinition"):
            assert m["name"].startswith("cron-operator-"), m["name"]
        if o["kind"] in ("Deployment", "Service", "ServiceAccount", "Role", "RoleBinding"):
            assert m["namespace"] == "cron-operator-system", (o["kind"], m)
    (dep,) = by_kind(objs, "Deployment")
    args = dep["spec"]["template"]["spec"]["containers"][0]["args"]
    assert args[0] == "--metrics-bind-address=:8443" and "start" in args and "--leader-elect" in args
    ns = build_parser().parse_args(cobra_order(args))
    assert ns.metrics_bind_address == ":8443" and ns.leader_elect


def test_alert_rules_use_metrics_the_operator_exports():
    """``deploy/kustomize/prometheus/rules.yaml``: every series an alert expression reads is one
    this operator registers (a renamed metric would leave an alert silently never firing), and
    the Lease name is the operator's."""
    import re

    import cron_operator_amd.runtime.metrics as m
    from cron_operator_amd.runtime.manager import DEFAULT_LEADER_ELECTION_ID as LEADER_ELECTION_ID

    objs = build(os.path.join(ROOT, "deploy", "kustomize", "prometheus"))
    (rule,) = [o for o in objs if o["kind"] == "PrometheusRule"]
    exported = set(m.REGISTRY._names)
    alerts = [r for g in rule["spec"]["groups"] for r in g["rules"]]
    assert {a["alert"] for a in alerts} >= {"CronOperatorMissedTicks", "CronOperatorClientThrottled",
                                           "CronOperatorNoLeader"}
    promql = {"sum", "rate", "increase", "max", "by", "le", "histogram_quantile"}
    for a in alerts:
        names = {n for n in re.findall(r"[a-z_][a-z0-9_]*(?=[\[{(\s]|$)", a["expr"]) if n not in promql}
        names = {re.sub(r"_(bucket|sum|count)$", "", n) if n.endswith(("_bucket", "_sum", "_count")) and
                 re.sub(r"_(bucket|sum|count)$", "", n) in exported else n for n in names}
        assert names and names <= exported, (a["alert"], names - exported)
        assert a["labels"]["severity"] in ("warning", "critical") and a["annotations"]["summary"]
    assert LEADER_ELECTION_ID in next(a["expr"] for a in alerts if a["alert"] == "CronOperatorNoLeader")


@pytest.mark.skipif(not os.path.isdir("/root/reference/config/default"), reason="reference checkout not mounted")
def test_default_install_names_every_object_as_the_reference_does():
    """``make deploy`` over a cluster the reference's kustomize install runs replaces its objects
    in place (docs/migration.md): the default overlay renders the same (kind, name) set -- the
    ServiceAccount, the leader-election and metrics-auth roles and bindings, the metrics Service."""
    ref = {(o["kind"], o["metadata"]["name"]) for o in build("/root/reference/config/default")}
    ours = {(o["kind"], o["metadata"]["name"]) for o in build(os.path.join(ROOT, "deploy", "kustomize", "default"))}
    assert ref == ours, (sorted(ref - ours), sorted(ours - ref))
