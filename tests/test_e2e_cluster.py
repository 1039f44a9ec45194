"""Real-cluster e2e tier: the operator deployed into a kind (or any) cluster, driven by kubectl.

The behavioural analog of the reference's Ginkgo suite (``test/e2e/e2e_test.go:156-277``, run
by ``make test-e2e`` against kind): the manager pod reaches Running and Ready, it logs
"Serving metrics server", a ServiceAccount bound to the ``metrics-reader`` ClusterRole reads
``/metrics`` through the authenticated HTTPS endpoint from a curl pod inside the cluster, the
scrape carries ``controller_runtime_reconcile_total``, and (beyond the reference) a Cron applied
to the cluster fires and records ``status.lastScheduleTime``.

This container has no kind, kubectl or network, so the tier SKIPS unless it is pointed at a
cluster: ``E2E_CLUSTER=1`` with ``kubectl`` on PATH and a kubeconfig whose current context is
the target (``make test-e2e-cluster`` creates a kind cluster, loads the image and deploys the
``deploy/kustomize/default`` overlay first).  Everything it creates is removed at the end
unless ``E2E_KEEP=1``.  The process-level analog that does run here is ``tests/test_e2e.py``.
"""

from __future__ import annotations

import json
import os
import shutil
import subprocess
import time
from typing import Callable, List

import pytest

pytestmark = [
    pytest.mark.slow,
    pytest.mark.skipif(
        os.environ.get("E2E_CLUSTER") != "1" or shutil.which("kubectl") is None,
        reason="real-cluster e2e: set E2E_CLUSTER=1 with kubectl pointed at a cluster (make test-e2e-cluster)",
    ),
]

# names rendered by deploy/kustomize/default (namePrefix cron-operator-, namespace below)
NAMESPACE = os.environ.get("E2E_NAMESPACE", "cron-operator-system")
PREFIX = "cron-operator-"
SERVICE_ACCOUNT = PREFIX + "controller-manager"
METRICS_SERVICE = PREFIX + "controller-manager-metrics-service"
METRICS_ROLE = PREFIX + "metrics-reader"
METRICS_BINDING = PREFIX + "e2e-metrics-binding"
POD_SELECTOR = "app.kubernetes.io/name=cron-operator"
CURL_POD = "curl-metrics"
CRON_EXAMPLE = os.path.join(os.path.dirname(__file__), "..", "examples", "v1alpha1", "cron", "cron-pod.yaml")
CRON_NAMESPACE = os.environ.get("E2E_CRON_NAMESPACE", "default")


def kubectl(*args: str, check: bool = True, stdin: str | None = None) -> str:
    p = subprocess.run(["kubectl", *args], input=stdin, capture_output=True, text=True, timeout=120)
    if check and p.returncode != 0:
        raise AssertionError(f"kubectl {' '.join(args)} failed ({p.returncode}): {p.stderr.strip()}")
    return p.stdout


def eventually(probe: Callable[[], None], timeout: float = 120.0, interval: float = 1.0) -> None:
    """Retry ``probe`` until it stops raising (Gomega's ``Eventually(...).Should(Succeed())``)."""
    deadline = time.monotonic() + timeout
    while True:
        try:
            probe()
            return
        except AssertionError:
            if time.monotonic() >= deadline:
                raise
            time.sleep(interval)


def lines(s: str) -> List[str]:
    return [ln for ln in s.splitlines() if ln.strip()]


@pytest.fixture(scope="module")
def controller_pod():
    found: List[str] = []

    def up() -> None:
        names = lines(kubectl("get", "pods", "-n", NAMESPACE, "-l", POD_SELECTOR,
                              "-o", "custom-columns=NAME:.metadata.name", "--no-headers"))
        assert len(names) == 1, f"expected one controller pod, got {names}"
        phase = kubectl("get", "pod", names[0], "-n", NAMESPACE, "-o", "jsonpath={.status.phase}")
        assert phase == "Running", f"controller pod phase {phase!r}"
        found[:] = names

    eventually(up, timeout=120)
    return found[0]


@pytest.fixture(scope="module")
def cleanup():
    yield
    if os.environ.get("E2E_KEEP") == "1":
        return
    kubectl("delete", "pod", CURL_POD, "-n", NAMESPACE, "--ignore-not-found", check=False)
    kubectl("delete", "clusterrolebinding", METRICS_BINDING, "--ignore-not-found", check=False)
    kubectl("delete", "-n", CRON_NAMESPACE, "-f", CRON_EXAMPLE, "--ignore-not-found", check=False)


def test_manager_runs(controller_pod):
    assert controller_pod.startswith("cron-operator")


def test_metrics_endpoint_serves_reconcile_metrics(controller_pod, cleanup):
    kubectl("delete", "clusterrolebinding", METRICS_BINDING, "--ignore-not-found")
    kubectl("create", "clusterrolebinding", METRICS_BINDING, f"--clusterrole={METRICS_ROLE}",
            f"--serviceaccount={NAMESPACE}:{SERVICE_ACCOUNT}")
    kubectl("get", "service", METRICS_SERVICE, "-n", NAMESPACE)
    token = kubectl("create", "token", SERVICE_ACCOUNT, "-n", NAMESPACE).strip()
    assert token

    def ready() -> None:
        st = kubectl("get", "pod", controller_pod, "-n", NAMESPACE,
                     "-o", "jsonpath={.status.conditions[?(@.type=='Ready')].status}")
        assert st == "True", f"controller pod Ready={st!r}"

    eventually(ready, timeout=180)

    def serving() -> None:
        assert "Serving metrics server" in kubectl("logs", controller_pod, "-n", NAMESPACE)

    eventually(serving, timeout=180)

    url = f"https://{METRICS_SERVICE}.{NAMESPACE}.svc.cluster.local:8443/metrics"
    overrides = {"spec": {
        "serviceAccountName": SERVICE_ACCOUNT,
        "containers": [{
            "name": "curl", "image": "curlimages/curl:latest", "command": ["/bin/sh", "-c"],
            "args": [f"curl -sS -k -H 'Authorization: Bearer {token}' {url}"],
            "securityContext": {
                "readOnlyRootFilesystem": True, "allowPrivilegeEscalation": False,
                "capabilities": {"drop": ["ALL"]}, "runAsNonRoot": True, "runAsUser": 1000,
                "seccompProfile": {"type": "RuntimeDefault"},
            },
        }],
    }}
    kubectl("delete", "pod", CURL_POD, "-n", NAMESPACE, "--ignore-not-found")
    kubectl("run", CURL_POD, "--restart=Never", "-n", NAMESPACE, "--image=curlimages/curl:latest",
            "--overrides", json.dumps(overrides))

    def done() -> None:
        phase = kubectl("get", "pod", CURL_POD, "-n", NAMESPACE, "-o", "jsonpath={.status.phase}")
        assert phase == "Succeeded", f"curl pod phase {phase!r}"

    eventually(done, timeout=300)
    scrape = kubectl("logs", CURL_POD, "-n", NAMESPACE)
    assert "controller_runtime_reconcile_total" in scrape


def test_cron_fires_in_cluster(controller_pod, cleanup):
    kubectl("apply", "-n", CRON_NAMESPACE, "-f", CRON_EXAMPLE)

    def fired() -> None:
        last = kubectl("get", "cron", "heartbeat-pod", "-n", CRON_NAMESPACE,
                       "-o", "jsonpath={.status.lastScheduleTime}")
        assert last, "Cron has not fired yet"

    # `*/1 * * * *`: the first fire is at most one minute (plus scheduling slack) away
    eventually(fired, timeout=150, interval=2)
    active = kubectl("get", "cron", "heartbeat-pod", "-n", CRON_NAMESPACE, "-o", "json")
    status = json.loads(active).get("status", {})
    assert status.get("active") or status.get("history"), status
