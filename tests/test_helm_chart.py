"""Helm chart rendering tests (helm-unittest analog).

The reference tests its chart with helm-unittest
(``charts/cron-operator/tests/{deployment,service,cluster_role,cluster_role_binding}_test.yaml``):
image composition, replicas, pull policy, zap flags, leader election on/off,
concurrency/QPS/burst flags, resources, nodeSelector merge and override,
affinity, tolerations concatenation, host-timezone mount, the Edge profile,
service type/port, RBAC rules and the binding.  Helm is not installed here, so
the templates are rendered with :mod:`cron_operator_amd.utils.gotemplate`.
"""
from __future__ import annotations

import os

import pytest

from cron_operator_amd.controller.rbac import RULES
from cron_operator_amd.utils.gotemplate import Engine, TemplateError, render_chart

CHART = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "charts", "cron-operator")


def deployment(values=None, release="cron-operator"):
    return render_chart(CHART, values, release=release)["deployment.yaml"][0]


def container(values=None):
    d = deployment(values)
    return [c for c in d["spec"]["template"]["spec"]["containers"] if c["name"] == "cron-operator"][0]


def test_image_composition():
    c = container({"image": {"registry": "test-registry", "repository": "test-repository", "tag": "test-tag"}})
    assert c["image"] == "test-registry/test-repository:test-tag"
    assert container()["image"].endswith(":0.3.0")  # defaults to appVersion


def test_replicas_and_pull_policy():
    d = deployment({"replicas": 3, "image": {"pullPolicy": "Always"}})
    assert d["spec"]["replicas"] == 3
    assert d["spec"]["template"]["spec"]["containers"][0]["imagePullPolicy"] == "Always"


@pytest.mark.parametrize("values,arg", [
    ({"logEncoder": "json"}, "--zap-encoder=json"),
    ({"logLevel": "debug"}, "--zap-log-level=debug"),
    ({"leaderElection": {"enable": True}}, "--leader-elect=true"),
    ({"leaderElection": {"enable": False}}, "--leader-elect=false"),
    ({"maxConcurrentReconciles": 20}, "--max-concurrent-reconciles=20"),
    ({"qps": 100}, "--qps=100"),
    ({"burst": 200}, "--burst=200"),
    ({}, "--qps=150"),
    ({}, "--burst=300"),
    ({}, "--max-inflight-requests=128"),
    ({"maxInflightRequests": 0}, "--max-inflight-requests=0"),
    ({"compatMode": "reference"}, "--compat-mode=reference"),
    ({"extraArgs": ["--namespace=team-a"]}, "--namespace=team-a"),
    ({"sharding": {"processes": 4, "routing": "labels"}}, "--shard-processes=4"),
    ({"sharding": {"processes": 4}}, "--shard-routing=labels"),
    ({"sharding": {"count": 2, "routing": "hash"}}, "--shard-routing=hash"),
    ({"sharding": {"count": 2, "index": 1}}, "--shard-index=1"),
])
def test_args(values, arg):
    assert arg in container(values)["args"]


def test_sharding_args_absent_by_default():
    args = container()["args"]
    assert not [a for a in args if a.startswith("--shard")]


def test_args_are_parsed_by_the_cli():
    from cron_operator_amd.cmd.main import build_parser

    args = container()["args"]
    a = build_parser().parse_args(args)
    assert a.command == "start" and a.leader_elect is True and a.metrics_secure is False
    assert a.metrics_bind_address == ":8080" and a.health_probe_bind_address == ":8081"


def test_resources():
    res = {"requests": {"cpu": "1", "memory": "1Gi"}, "limits": {"cpu": "2", "memory": "2Gi"}}
    assert container({"resources": res})["resources"] == res


def spec(values):
    return deployment(values)["spec"]["template"]["spec"]


def test_node_selector_merge_and_override():
    assert "nodeSelector" not in spec({})
    assert spec({"global": {"nodeSelector": {"key1": "value1"}}})["nodeSelector"] == {"key1": "value1"}
    assert spec({"nodeSelector": {"key2": "value2"}})["nodeSelector"] == {"key2": "value2"}
    both = spec({"global": {"nodeSelector": {"key1": "value1", "key2": "value2"}},
                 "nodeSelector": {"key1": "value1-override", "key3": "value3"}})["nodeSelector"]
    assert both == {"key1": "value1-override", "key2": "value2", "key3": "value3"}


def test_affinity():
    aff = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
        {"matchExpressions": [{"key": "k", "operator": "In", "values": ["v"]}]}]}}}
    assert spec({"affinity": aff})["affinity"] == aff


def test_tolerations_concat():
    g = [{"key": "key1", "operator": "Equal", "value": "value1", "effect": "NoSchedule"}]
    t = [{"key": "key2", "operator": "Exists", "effect": "NoExecute"}]
    assert "tolerations" not in spec({})
    assert spec({"global": {"tolerations": g}})["tolerations"] == g
    assert spec({"global": {"tolerations": g}, "tolerations": t})["tolerations"] == g + t


def test_host_timezone_mount():
    s = spec({"useHostTimezone": True})
    assert s["volumes"] == [{"name": "volume-localtime", "hostPath": {"path": "/etc/localtime"}}]
    assert s["containers"][0]["volumeMounts"][0]["mountPath"] == "/etc/localtime"
    assert "volumes" not in spec({})


def test_edge_profile():
    s = spec({"global": {"clusterProfile": "Edge"}, "tolerations": [{"key": "x", "operator": "Exists"}]})
    assert s["nodeSelector"] == {"alibabacloud.com/is-edge-worker": "false"}
    assert {"key": "node-role.alibabacloud.com/addon", "operator": "Exists", "effect": "NoSchedule"} in \
        s["tolerations"]
    assert {"key": "x", "operator": "Exists"} in s["tolerations"]


def test_probes_and_security_context():
    c = container()
    assert c["livenessProbe"]["httpGet"]["path"] == "/healthz"
    assert c["readinessProbe"]["httpGet"]["path"] == "/readyz"
    assert c["securityContext"]["readOnlyRootFilesystem"] is True
    assert c["securityContext"]["runAsNonRoot"] is True


def test_service():
    out = render_chart(CHART, {"service": {"type": "NodePort"}})["service.yaml"][0]
    assert out["spec"]["type"] == "NodePort"
    assert out["spec"]["ports"] == [{"name": "metrics", "port": 8080, "targetPort": "metrics", "protocol": "TCP"}]


def test_rbac_rules_match_generator_and_group_is_correct():
    out = render_chart(CHART)
    role = out["cluster_role.yaml"][0]
    assert role["kind"] == "ClusterRole"
    assert role["rules"] == RULES
    assert any("apps.kubedl.io" in r["apiGroups"] and "crons" in r["resources"] for r in role["rules"])
    binding = out["cluster_role_binding.yaml"][0]
    assert binding["roleRef"] == {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                                  "name": "cron-operator"}
    assert binding["subjects"] == [{"kind": "ServiceAccount", "name": "cron-operator", "namespace": "cron-operator"}]


def test_extra_workload_rules():
    docs = render_chart(CHART, {"rbac": {"extraWorkloadRules": [{"apiGroups": ["ray.io"],
                                                                 "resources": ["rayjobs"]}]}})["cluster_role.yaml"]
    role = docs[0]
    assert role["rules"][-1]["apiGroups"] == ["ray.io"]


def test_fullname_rules():
    assert deployment(release="cron-operator")["metadata"]["name"] == "cron-operator"
    assert deployment(release="prod")["metadata"]["name"] == "prod-cron-operator"
    assert render_chart(CHART, {"fullnameOverride": "x"})["deployment.yaml"][0]["metadata"]["name"] == "x"


# ---------------------------------------------------------------- the template engine itself


def _r(src, dot=None):
    e = Engine()
    return e.render(e.add_template(src), dot if dot is not None else {})


def test_engine_basics():
    assert _r("{{ .a }}-{{ .b.c }}", {"a": 1, "b": {"c": "x"}}) == "1-x"
    assert _r("{{- if .a }}yes{{ else }}no{{ end -}}", {"a": ""}) == "no"
    assert _r("{{ range $i, $v := .l }}{{ $i }}={{ $v }};{{ end }}", {"l": ["a", "b"]}) == "0=a;1=b;"
    assert _r("{{ range $k, $v := .m }}{{ $k }}{{ $v }}{{ end }}", {"m": {"b": 2, "a": 1}}) == "a1b2"
    assert _r('{{ printf "%s-%d" "x" 3 | upper }}') == "X-3"
    assert _r('{{ $x := 1 }}{{ if true }}{{ $x = 2 }}{{ end }}{{ $x }}') == "2"
    assert _r('{{ define "t" }}[{{ . }}]{{ end }}{{ include "t" "v" }}') == "[v]"
    assert _r("{{ .missing }}") == "<no value>"
    assert _r('{{ default "d" .x }}', {"x": ""}) == "d"
    assert _r("{{ and 1 0 }}{{ or 0 2 }}") == "02"
    with pytest.raises(TemplateError):
        _r('{{ required "need x" .x }}')


# ---------------------------------------------------------------- helm-unittest suites (charts/cron-operator/tests)


def test_helm_unittest_suites_pass():
    """The chart's helm-unittest suites (reference tier: charts/cron-operator/tests, Makefile:158-160)."""
    from cron_operator_amd.utils.helmunittest import run_all

    passed, failed, results = run_all(CHART)
    assert failed == 0, [(r.suite, r.name, r.failures) for r in results if not r.passed]
    assert passed >= 25


def test_helm_unittest_runner_detects_failures(tmp_path):
    from cron_operator_amd.utils.helmunittest import get_path, run_suite

    doc = {"spec": {"containers": [{"name": "a", "args": ["x"]}, {"name": "b"}]},
           "metadata": {"labels": {"app.kubernetes.io/name": "n"}}}
    assert get_path(doc, "spec.containers[?(@.name=='b')].name") == "b"
    assert get_path(doc, 'metadata.labels["app.kubernetes.io/name"]') == "n"
    suite = tmp_path / "bad_test.yaml"
    suite.write_text("""
suite: negative
templates: [deployment.yaml]
tests:
  - it: wrong replicas
    asserts:
      - equal: {path: spec.replicas, value: 7}
  - it: negated assertion
    asserts:
      - isKind: {of: Deployment}
        not: true
""")
    res = run_suite(str(suite), CHART)
    assert [r.passed for r in res] == [False, False]


REF_CHART_TESTS = "/root/reference/charts/cron-operator/tests"


@pytest.mark.skipif(not os.path.isdir(REF_CHART_TESTS), reason="reference checkout not mounted")
def test_reference_helm_unittest_suites_pass_against_this_chart(tmp_path):
    """Parity pin: the reference's OWN helm-unittest suites (``charts/cron-operator/tests/*_test.yaml``,
    run by its ``make helm-unittest``) assert against this chart, unmodified.  The template files carry
    the reference's names (``cluster_role.yaml``, ``cluster_role_binding.yaml``,
    ``service_account.yaml``) so every suite resolves its templates."""
    import shutil

    from cron_operator_amd.utils.helmunittest import run_all

    chart = tmp_path / "chart"
    shutil.copytree(CHART, chart, ignore=shutil.ignore_patterns("tests"))
    (chart / "tests").mkdir()
    for name in sorted(os.listdir(REF_CHART_TESTS)):
        if name.endswith("_test.yaml"):
            shutil.copy(os.path.join(REF_CHART_TESTS, name), chart / "tests" / name)
    passed, failed, results = run_all(str(chart))
    assert failed == 0, [(r.suite, r.name, r.failures) for r in results if not r.passed]
    assert passed >= 20


def test_monitoring_objects_are_off_by_default_and_match_the_kustomize_ones():
    """``metrics.serviceMonitor`` / ``metrics.prometheusRule`` (new): nothing by default (the
    reference chart has neither); enabled, the ServiceMonitor scrapes the metrics Service's
    port and the PrometheusRule carries exactly the alerts of
    ``deploy/kustomize/prometheus/rules.yaml``, with Prometheus's ``{{ $value }}`` left for
    Prometheus to expand."""
    import yaml

    kinds = {o["kind"] for lst in render_chart(CHART, {}).values() for o in lst}
    assert not kinds & {"ServiceMonitor", "PrometheusRule"}
    docs = render_chart(CHART, {"metrics": {"serviceMonitor": {"enabled": True, "labels": {"release": "kp"}},
                                            "prometheusRule": {"enabled": True}}})
    objs = {o["kind"]: o for lst in docs.values() for o in lst}
    sm = objs["ServiceMonitor"]
    svc = objs["Service"]
    assert sm["metadata"]["labels"]["release"] == "kp"
    assert sm["spec"]["selector"]["matchLabels"].items() <= svc["metadata"]["labels"].items()
    assert sm["spec"]["endpoints"][0]["port"] == svc["spec"]["ports"][0]["name"] == "metrics"
    with open(os.path.join(os.path.dirname(os.path.dirname(CHART)), "deploy", "kustomize", "prometheus",
                           "rules.yaml")) as fh:
        want = yaml.safe_load(fh)["spec"]
    assert objs["PrometheusRule"]["spec"] == want
    assert "{{ $value }}" in objs["PrometheusRule"]["spec"]["groups"][0]["rules"][0]["annotations"]["description"]


def test_action_ends_outside_string_literals():
    """Go's lexer: ``}}`` inside a quoted string does not end the action."""
    e = Engine()
    t = e.add_template('a {{ "{{" }} $v {{ "}}" }} b {{- " x" -}} c {{ `}}` }}')
    assert e.render(t, {}) == "a {{ $v }} b xc }}"


def test_subfield_of_a_parenthesised_pipeline_as_an_argument():
    e = Engine()
    t = e.add_template('{{ printf "%s!" (.m).k }}')
    assert e.render(t, {"m": {"k": "v"}}) == "v!"


@pytest.mark.skipif(not os.path.isdir("/root/reference/charts/cron-operator"), reason="reference checkout not mounted")
@pytest.mark.parametrize("release", ["cron-operator", "nightly"])
def test_helm_upgrade_over_the_reference_release_keeps_names_and_selector(release):
    """``helm upgrade <release> charts/cron-operator`` over a reference release: the same
    objects by (kind, name), and the same Deployment selector -- a Deployment's selector is
    immutable, so a different one would make the upgrade fail (docs/migration.md)."""
    ref = render_chart("/root/reference/charts/cron-operator", {}, release=release, namespace="ns")
    ours = render_chart(CHART, {}, release=release, namespace="ns")

    def names(docs):
        return {(o["kind"], o["metadata"]["name"]) for lst in docs.values() for o in lst}

    def dep(docs):
        return next(o for lst in docs.values() for o in lst if o["kind"] == "Deployment")

    assert names(ref) == names(ours)
    assert dep(ref)["spec"]["selector"] == dep(ours)["spec"]["selector"]
    assert dep(ref)["spec"]["template"]["spec"]["serviceAccountName"] == \
        dep(ours)["spec"]["template"]["spec"]["serviceAccountName"]
