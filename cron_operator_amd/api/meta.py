"""Kubernetes meta types used by the API and the runtime.

Python counterparts of the apimachinery pieces the reference leans on:
``schema.GroupVersionKind`` / ``GroupVersionResource``, ``corev1.ObjectReference``,
``corev1.TypedLocalObjectReference``, ``metav1.OwnerReference`` and the
``metav1.Object`` accessors over unstructured objects.  Objects themselves stay
plain JSON trees (``dict``); these helpers read and write their metadata.
"""
from __future__ import annotations

from typing import Any, Dict, List, NamedTuple, Optional, Tuple

from ..utils.gotime import GoTime, format_rfc3339_utc, parse_rfc3339


class GroupVersion(NamedTuple):
    """``schema.GroupVersion``.  This and the GVK/GVR types are named tuples: they key the
    REST mapper, the informer cache and the path memo, so hashing runs in C."""

    group: str
    version: str

    def __str__(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    @staticmethod
    def parse(api_version: str) -> "GroupVersion":
        """``schema.ParseGroupVersion``; raises ValueError on ``a/b/c``."""
        if api_version == "" or api_version == "/":
            return GroupVersion("", "")
        parts = api_version.split("/")
        if len(parts) == 1:
            return GroupVersion("", parts[0])
        if len(parts) == 2:
            return GroupVersion(parts[0], parts[1])
        raise ValueError(f"unexpected GroupVersion string: {api_version}")

    def with_kind(self, kind: str) -> "GroupVersionKind":
        return GroupVersionKind(self.group, self.version, kind)

    def with_resource(self, resource: str) -> "GroupVersionResource":
        return GroupVersionResource(self.group, self.version, resource)


class GroupVersionKind(NamedTuple):
    group: str
    version: str
    kind: str

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    def group_version(self) -> GroupVersion:
        return GroupVersion(self.group, self.version)

    def __str__(self) -> str:
        return f"{self.api_version}, Kind={self.kind}"

    @staticmethod
    def from_object(obj: Dict[str, Any]) -> "GroupVersionKind":
        """``Unstructured.GroupVersionKind()``: an unparsable apiVersion yields empty.
        Memoised per (apiVersion, kind): a handful of kinds recur on every event."""
        av = obj.get("apiVersion") or ""
        kind = obj.get("kind") or ""
        hit = _GVK_MEMO.get((av, kind))
        if hit is not None:
            return hit
        try:
            gv = GroupVersion.parse(av)
            hit = GroupVersionKind(gv.group, gv.version, kind)
        except ValueError:
            hit = GroupVersionKind("", "", "")
        if len(_GVK_MEMO) < 4096:
            _GVK_MEMO[(av, kind)] = hit
        return hit


_GVK_MEMO: Dict[Tuple[str, str], GroupVersionKind] = {}


class GroupVersionResource(NamedTuple):
    group: str
    version: str
    resource: str

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    def __str__(self) -> str:
        return f"{self.api_version}/{self.resource}"


class NamespacedName(NamedTuple):
    """``types.NamespacedName`` -- the work-queue key.  A named tuple so that hashing and
    equality (every queue, dirty-set and rate-limiter lookup) run in C."""

    namespace: str
    name: str

    def __str__(self) -> str:
        return f"{self.namespace}/{self.name}" if self.namespace else self.name


# --------------------------------------------------------------------------- metav1.Time


def time_to_json(t: Optional[GoTime]) -> Optional[str]:
    if t is None or t.is_zero():
        return None
    return format_rfc3339_utc(t)


def time_from_json(s: Optional[str]) -> Optional[GoTime]:
    if s is None or s == "":
        return None
    return parse_rfc3339(s)



# --------------------------------------------------------------------------- metadata accessors


def meta(obj: Dict[str, Any]) -> Dict[str, Any]:
    m = obj.get("metadata")
    if m is None:
        m = obj["metadata"] = {}
    return m



def creation_timestamp(obj: Dict[str, Any]) -> GoTime:
    s = (obj.get("metadata") or {}).get("creationTimestamp")
    t = time_from_json(s)
    return t if t is not None else GoTime.zero()


def deletion_timestamp(obj: Dict[str, Any]) -> Optional[GoTime]:
    return time_from_json((obj.get("metadata") or {}).get("deletionTimestamp"))


def key_of(obj: Dict[str, Any]) -> str:
    m = obj.get("metadata") or {}
    ns = m.get("namespace", "")
    return f"{ns}/{m.get('name', '')}" if ns else m.get("name", "")


def controller_ref(obj: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    """``metav1.GetControllerOf``."""
    for ref in (obj.get("metadata") or {}).get("ownerReferences") or []:
        if ref.get("controller"):
            return ref
    return None


def new_controller_ref(owner: Dict[str, Any], gvk: GroupVersionKind) -> Dict[str, Any]:
    """``metav1.NewControllerRef`` (controller + blockOwnerDeletion true)."""
    m = owner.get("metadata") or {}
    return {
        "apiVersion": gvk.api_version,
        "kind": gvk.kind,
        "name": m.get("name", ""),
        "uid": m.get("uid", ""),
        "controller": True,
        "blockOwnerDeletion": True,
    }


class AlreadyOwnedError(ValueError):
    pass


def set_controller_reference(owner: Dict[str, Any], owner_gvk: GroupVersionKind, obj: Dict[str, Any]) -> None:
    """``controllerutil.SetControllerReference``.

    Fails if the object already has a different controller; cluster-scoped
    owners of namespaced objects and cross-namespace owners are rejected like
    upstream.
    """
    om = owner.get("metadata") or {}
    m = meta(obj)
    owner_ns = om.get("namespace", "")
    obj_ns = m.get("namespace", "")
    if owner_ns and owner_ns != obj_ns:
        raise ValueError(f"cross-namespace owner references are disallowed, owner's namespace {owner_ns}, "
                         f"obj's namespace {obj_ns}")
    ref = new_controller_ref(owner, owner_gvk)
    refs: List[Dict[str, Any]] = list(m.get("ownerReferences") or [])
    existing = None
    for r in refs:
        if r.get("controller"):
            existing = r
            break
    if existing is not None and not _same_owner(existing, ref):
        raise AlreadyOwnedError(
            f"Object {obj_ns}/{m.get('name', '')} is already owned by another {existing.get('kind')} "
            f"controller {existing.get('name')}")
    out = []
    replaced = False
    for r in refs:
        if _same_owner(r, ref):
            out.append(ref)
            replaced = True
        else:
            out.append(r)
    if not replaced:
        out.append(ref)
    m["ownerReferences"] = out


def _same_owner(a: Dict[str, Any], b: Dict[str, Any]) -> bool:
    try:
        ga = GroupVersion.parse(a.get("apiVersion", "")).group
        gb = GroupVersion.parse(b.get("apiVersion", "")).group
    except ValueError:
        return False
    return ga == gb and a.get("kind") == b.get("kind") and a.get("name") == b.get("name")


