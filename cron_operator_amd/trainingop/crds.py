"""Schema-level CRDs for Kubeflow training jobs (the envtest "fake workload CRDs").

The reference's integration tests install 15k lines of third-party CRD YAML
just so the apiserver serves ``kubeflow.org`` kinds (``test/crds/*.yaml``,
loaded at ``internal/controller/suite_test.go:73-79``).  The operator only needs
the kinds to exist and their ``.status`` to have the kubeflow JobStatus shape
(``test/crds/kubeflow.org_pytorchjobs.yaml:4739-4828``), so these definitions are
generated: ``spec`` preserves unknown fields, ``status`` is structured.

MPIJob is served as ``v1alpha1`` with the old ``launcherStatus`` status shape
(no conditions, ``test/crds/kubeflow.org_mpijobs.yaml:6003-6017``) and as ``v1``
with conditions, so both behaviours can be exercised.
"""
from __future__ import annotations

from typing import Any, Dict, List, Tuple

KUBEFLOW_GROUP = "kubeflow.org"


def _time() -> Dict[str, Any]:
    return {"type": "string", "format": "date-time"}


def job_status_schema() -> Dict[str, Any]:
    return {
        "type": "object",
        "properties": {
            "conditions": {"type": "array", "items": {"type": "object", "properties": {
                "type": {"type": "string"}, "status": {"type": "string"}, "reason": {"type": "string"},
                "message": {"type": "string"}, "lastUpdateTime": _time(), "lastTransitionTime": _time()}}},
            "replicaStatuses": {"type": "object", "additionalProperties": {"type": "object", "properties": {
                "active": {"type": "integer"}, "succeeded": {"type": "integer"}, "failed": {"type": "integer"},
                "selector": {"type": "string"},
                "labelSelector": {"type": "object", "x-kubernetes-preserve-unknown-fields": True}}}},
            "startTime": _time(),
            "completionTime": _time(),
            "lastReconcileTime": _time(),
        },
    }


def mpi_v1alpha1_status_schema() -> Dict[str, Any]:
    return {
        "type": "object",
        "properties": {
            "launcherStatus": {"type": "string"},
            "workerReplicas": {"type": "integer"},
            "startTime": _time(),
            "completionTime": _time(),
        },
    }


def _version(name: str, status: Dict[str, Any], storage: bool) -> Dict[str, Any]:
    return {"name": name, "served": True, "storage": storage, "subresources": {"status": {}},
            "schema": {"openAPIV3Schema": {"type": "object", "properties": {
                "apiVersion": {"type": "string"}, "kind": {"type": "string"}, "metadata": {"type": "object"},
                "spec": {"type": "object", "x-kubernetes-preserve-unknown-fields": True},
                "status": status}}}}


def _crd(plural: str, kind: str, versions: List[Dict[str, Any]], group: str = KUBEFLOW_GROUP) -> Dict[str, Any]:
    return {"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
            "metadata": {"name": f"{plural}.{group}"},
            "spec": {"group": group, "scope": "Namespaced",
                     "names": {"kind": kind, "listKind": kind + "List", "plural": plural,
                               "singular": kind.lower()},
                     "versions": versions}}


JOB_KINDS: List[Tuple[str, str]] = [
    ("pytorchjobs", "PyTorchJob"),
    ("tfjobs", "TFJob"),
    ("xgboostjobs", "XGBoostJob"),
    ("paddlejobs", "PaddleJob"),
    ("jaxjobs", "JAXJob"),
]


def kubeflow_crds() -> List[Dict[str, Any]]:
    out = [_crd(p, k, [_version("v1", job_status_schema(), True)]) for p, k in JOB_KINDS]
    out.append(_crd("mpijobs", "MPIJob", [_version("v1alpha1", mpi_v1alpha1_status_schema(), False),
                                          _version("v1", job_status_schema(), True)]))
    return out


def job_crd(group: str, version: str, plural: str, kind: str) -> Dict[str, Any]:
    """A job kind of another operator with the kubeflow JobStatus shape -- e.g. KubeDL's
    ``xdl.kubedl.io`` XDLJob, which the reference chart's ClusterRole grants."""
    return _crd(plural, kind, [_version(version, job_status_schema(), True)], group)
