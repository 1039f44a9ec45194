"""RBAC authorization for the fake apiserver.

A real cluster evaluates every request of the operator's ServiceAccount against
the ClusterRole the deployment installs.  The reference's kustomize role grants
the wrong API group (``kubedl.io`` instead of ``apps.kubedl.io``,
``internal/controller/cron_controller.go:79-85`` -> ``config/rbac/role.yaml:7-32``,
SURVEY Appendix B #1) and nothing in its test tiers catches that, because
envtest runs as an admin and the e2e run uses the Helm chart's hand-written
ClusterRole instead.  With ``APIServer(authorization="RBAC")`` the fake
apiserver enforces the stored Roles/ClusterRoles/(Cluster)RoleBindings the
way kube-apiserver's RBAC authorizer does, so a test can run the operator
under exactly the RBAC objects an install ships and see a ``403`` if they are
wrong.

Semantics implemented (k8s ``plugin/pkg/auth/authorizer/rbac``):

* subjects: ``User`` (name), ``Group`` (name), ``ServiceAccount``
  (``system:serviceaccount:<ns>:<name>``);
* ClusterRoleBindings grant cluster-wide; RoleBindings grant inside their
  namespace and may reference a Role (same namespace) or a ClusterRole;
* rule matching: ``verbs``, ``apiGroups``, ``resources`` (``res``,
  ``res/sub``, ``*``, ``*/sub``), ``resourceNames`` (never matches list/
  watch/create/deletecollection without a name), ``nonResourceURLs``
  (exact or trailing ``*`` prefix);
* ClusterRole ``aggregationRule`` (labels of other ClusterRoles);
* the ``system:masters`` group is always allowed (the superuser shortcut).
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional

from ..api.meta import GroupVersionResource
from ..api.selectors import matches_labels, parse_label_selector

RBAC = "rbac.authorization.k8s.io"
ROLES = GroupVersionResource(RBAC, "v1", "roles")
CLUSTER_ROLES = GroupVersionResource(RBAC, "v1", "clusterroles")
ROLE_BINDINGS = GroupVersionResource(RBAC, "v1", "rolebindings")
CLUSTER_ROLE_BINDINGS = GroupVersionResource(RBAC, "v1", "clusterrolebindings")


def service_account_user(namespace: str, name: str) -> Dict[str, Any]:
    """The user info a ServiceAccount token authenticates as."""
    return {"username": f"system:serviceaccount:{namespace}:{name}",
            "groups": ["system:serviceaccounts", f"system:serviceaccounts:{namespace}", "system:authenticated"]}


def _subject_matches(s: Dict[str, Any], user: str, groups: Iterable[str], binding_ns: str) -> bool:
    kind = s.get("kind")
    if kind == "User":
        return s.get("name") == user
    if kind == "Group":
        return s.get("name") in set(groups)
    if kind == "ServiceAccount":
        ns = s.get("namespace") or binding_ns
        return user == f"system:serviceaccount:{ns}:{s.get('name')}"
    return False


def _has(values: Iterable[str], want: str) -> bool:
    vs = list(values or [])
    return "*" in vs or want in vs


def rule_allows(rule: Dict[str, Any], attrs: Dict[str, Any]) -> bool:
    verb = attrs.get("verb", "")
    if not _has(rule.get("verbs"), verb):
        return False
    url = attrs.get("path")
    if url is not None:  # non-resource request
        for pat in rule.get("nonResourceURLs") or []:
            if pat == "*" or pat == url or (pat.endswith("*") and url.startswith(pat[:-1])):
                return True
        return False
    if rule.get("nonResourceURLs") and not rule.get("resources"):
        return False
    if not _has(rule.get("apiGroups"), attrs.get("group", "")):
        return False
    res = attrs.get("resource", "")
    sub = attrs.get("subresource", "")
    full = f"{res}/{sub}" if sub else res
    ok = False
    for r in rule.get("resources") or []:
        if r == "*" or r == full or (sub and r == f"*/{sub}"):
            ok = True
            break
    if not ok:
        return False
    names = rule.get("resourceNames") or []
    if names:
        name = attrs.get("name", "")
        return bool(name) and name in names
    return True


class RBACAuthorizer:
    def __init__(self, server: Any):
        self.server = server

    def _objs(self, gvr: GroupVersionResource, ns: Optional[str] = None) -> List[Dict[str, Any]]:
        try:
            return list(self.server.objects(gvr, ns))
        except Exception:  # noqa: BLE001 - resource not registered
            return []

    def _cluster_role_rules(self, name: str) -> List[Dict[str, Any]]:
        roles = {(r.get("metadata") or {}).get("name"): r for r in self._objs(CLUSTER_ROLES)}
        role = roles.get(name)
        if role is None:
            return []
        rules = list(role.get("rules") or [])
        agg = role.get("aggregationRule") or {}
        for sel in agg.get("clusterRoleSelectors") or []:
            match = sel.get("matchLabels") or {}
            reqs = parse_label_selector(",".join(f"{k}={v}" for k, v in match.items()))
            for other in roles.values():
                if other is role:
                    continue
                if matches_labels(reqs, (other.get("metadata") or {}).get("labels") or {}):
                    rules.extend(other.get("rules") or [])
        return rules

    def rules_for(self, user: str, groups: Iterable[str], namespace: str) -> List[Dict[str, Any]]:
        groups = list(groups or [])
        rules: List[Dict[str, Any]] = []
        for b in self._objs(CLUSTER_ROLE_BINDINGS):
            if any(_subject_matches(s, user, groups, "") for s in b.get("subjects") or []):
                ref = b.get("roleRef") or {}
                if ref.get("kind") == "ClusterRole":
                    rules.extend(self._cluster_role_rules(ref.get("name", "")))
        if namespace:
            for b in self._objs(ROLE_BINDINGS, namespace):
                if not any(_subject_matches(s, user, groups, namespace) for s in b.get("subjects") or []):
                    continue
                ref = b.get("roleRef") or {}
                if ref.get("kind") == "ClusterRole":
                    rules.extend(self._cluster_role_rules(ref.get("name", "")))
                elif ref.get("kind") == "Role":
                    for r in self._objs(ROLES, namespace):
                        if (r.get("metadata") or {}).get("name") == ref.get("name"):
                            rules.extend(r.get("rules") or [])
        return rules

    def authorize(self, user: str, groups: Iterable[str], attrs: Dict[str, Any]) -> bool:
        groups = list(groups or [])
        if "system:masters" in groups:
            return True
        ns = attrs.get("namespace", "") if attrs.get("path") is None else ""
        return any(rule_allows(r, attrs) for r in self.rules_for(user, groups, ns))

    # signature of APIServer.authorizer (SubjectAccessReview)
    def __call__(self, who: Dict[str, Any], spec: Dict[str, Any]) -> bool:
        ra = spec.get("resourceAttributes")
        nra = spec.get("nonResourceAttributes")
        if ra:
            attrs = {"verb": ra.get("verb", ""), "group": ra.get("group", ""), "resource": ra.get("resource", ""),
                     "subresource": ra.get("subresource", ""), "namespace": ra.get("namespace", ""),
                     "name": ra.get("name", "")}
        elif nra:
            attrs = {"verb": nra.get("verb", ""), "path": nra.get("path", "")}
        else:
            return False
        return self.authorize(who.get("user") or "", who.get("groups") or [], attrs)


def forbidden_message(user: str, attrs: Dict[str, Any]) -> str:
    """kube-apiserver's wording for a denied request."""
    if attrs.get("path") is not None:
        return f'forbidden: User "{user}" cannot {attrs["verb"]} path "{attrs["path"]}"'
    res = attrs.get("resource", "")
    sub = attrs.get("subresource", "")
    group = attrs.get("group", "")
    what = f"{res}.{group}" if group else res
    name = attrs.get("name", "")
    head = f'{what} "{name}" is forbidden' if name else f"{what} is forbidden"
    rtext = f"{res}/{sub}" if sub else res
    scope = f' in the namespace "{attrs["namespace"]}"' if attrs.get("namespace") else " at the cluster scope"
    return f'{head}: User "{user}" cannot {attrs["verb"]} resource "{rtext}" in API group "{group}"{scope}'
