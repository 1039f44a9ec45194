"""Resource registry of the fake apiserver (what discovery advertises).

Built-in resources cover what the operator and its tests touch: namespaces,
pods, events, configmaps, leases (leader election), batch Jobs, events.k8s.io
Events, TokenReview/SubjectAccessReview (metrics authn/authz filter),
CustomResourceDefinitions, the RBAC kinds (enforced with
``authorization="RBAC"``, see :mod:`.rbac`) and the Deployment /
NetworkPolicy kinds an install applies.  Custom resources are added by creating a CRD
object (exactly how envtest installs ``charts/cron-operator/crds`` and
``test/crds``, reference ``internal/controller/suite_test.go:73-79``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

from ..api.meta import GroupVersionKind, GroupVersionResource


@dataclass
class ResourceInfo:
    group: str
    version: str
    resource: str
    kind: str
    namespaced: bool = True
    singular: str = ""
    status_subresource: bool = False
    schema: Optional[Dict[str, Any]] = None
    short_names: List[str] = field(default_factory=list)
    verbs: Tuple[str, ...] = ("create", "delete", "deletecollection", "get", "list", "patch", "update", "watch")
    virtual: bool = False          # create-only review resources, not persisted
    is_crd: bool = False
    printer_columns: List[Dict[str, Any]] = field(default_factory=list)

    @property
    def gvr(self) -> GroupVersionResource:
        return GroupVersionResource(self.group, self.version, self.resource)

    @property
    def gvk(self) -> GroupVersionKind:
        return GroupVersionKind(self.group, self.version, self.kind)

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    @property
    def list_kind(self) -> str:
        return self.kind + "List"

    def discovery_entry(self) -> Dict[str, Any]:
        e: Dict[str, Any] = {"name": self.resource, "singularName": self.singular or self.kind.lower(),
                             "namespaced": self.namespaced, "kind": self.kind, "verbs": list(self.verbs)}
        if self.short_names:
            e["shortNames"] = list(self.short_names)
        return e


def builtin_resources() -> List[ResourceInfo]:
    R = ResourceInfo
    return [
        R("", "v1", "namespaces", "Namespace", namespaced=False, status_subresource=True),
        R("", "v1", "pods", "Pod", status_subresource=True, short_names=["po"]),
        R("", "v1", "events", "Event", short_names=["ev"]),
        R("", "v1", "configmaps", "ConfigMap", short_names=["cm"]),
        R("", "v1", "secrets", "Secret"),
        R("", "v1", "services", "Service", status_subresource=True, short_names=["svc"]),
        R("", "v1", "serviceaccounts", "ServiceAccount", short_names=["sa"]),
        R("coordination.k8s.io", "v1", "leases", "Lease"),
        R("batch", "v1", "jobs", "Job", status_subresource=True),
        R("events.k8s.io", "v1", "events", "Event", short_names=["ev"]),
        R("authentication.k8s.io", "v1", "tokenreviews", "TokenReview", namespaced=False, virtual=True,
          verbs=("create",)),
        R("authorization.k8s.io", "v1", "subjectaccessreviews", "SubjectAccessReview", namespaced=False,
          virtual=True, verbs=("create",)),
        R("apiextensions.k8s.io", "v1", "customresourcedefinitions", "CustomResourceDefinition", namespaced=False,
          status_subresource=True, short_names=["crd", "crds"]),
        R("rbac.authorization.k8s.io", "v1", "roles", "Role"),
        R("rbac.authorization.k8s.io", "v1", "rolebindings", "RoleBinding"),
        R("rbac.authorization.k8s.io", "v1", "clusterroles", "ClusterRole", namespaced=False),
        R("rbac.authorization.k8s.io", "v1", "clusterrolebindings", "ClusterRoleBinding", namespaced=False),
        R("apps", "v1", "deployments", "Deployment", status_subresource=True, short_names=["deploy"]),
        R("networking.k8s.io", "v1", "networkpolicies", "NetworkPolicy", short_names=["netpol"]),
    ]


def resources_from_crd(crd: Dict[str, Any]) -> List[ResourceInfo]:
    spec = crd.get("spec") or {}
    names = spec.get("names") or {}
    group = spec.get("group", "")
    out = []
    for v in spec.get("versions") or []:
        if not v.get("served", True):
            continue
        schema = ((v.get("schema") or {}).get("openAPIV3Schema")) or None
        out.append(ResourceInfo(
            group=group, version=v.get("name", ""), resource=names.get("plural", ""), kind=names.get("kind", ""),
            namespaced=(spec.get("scope", "Namespaced") == "Namespaced"),
            singular=names.get("singular", ""),
            status_subresource="status" in (v.get("subresources") or {}),
            schema=schema, short_names=list(names.get("shortNames") or []), is_crd=True,
            printer_columns=list(v.get("additionalPrinterColumns") or [])))
    return out
