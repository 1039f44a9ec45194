"""A small ``kustomize build`` for the manifests this repo ships.

The reference installs with ``make build-installer`` / ``make deploy``, i.e.
``kustomize build config/default`` (``Makefile:112-150``, kustomize v5.7.1
pinned at ``Makefile:243-262``).  kustomize is not available here, so this
module implements the subset of its transformers the ``deploy/kustomize`` tree
(and typical user overlays) use:

* ``resources`` -- files (multi-document YAML) and directories holding a
  ``kustomization.yaml`` (built recursively, depth first, in order);
* ``namespace`` -- set on every namespaced object, and on ``ServiceAccount``
  subjects of (Cluster)RoleBindings;
* ``namePrefix`` / ``nameSuffix`` -- on every object except CRDs, with the
  name references kustomize fixes up (roleRef, ServiceAccount subjects,
  ``serviceAccountName``, Service/ServiceMonitor/NetworkPolicy don't need it);
* ``labels`` (with ``includeSelectors``) and legacy ``commonLabels``;
* ``images`` -- ``newName`` / ``newTag`` / ``digest`` by image name;
* ``patches`` -- JSON 6902 op lists or strategic-merge documents, inline
  (``patch``) or from a file (``path``), selected by ``target``
  (group/version/kind/name/namespace/labelSelector) or by the patch's own
  kind+name.

Output uses kustomize's default ``legacy`` sort: Namespaces, CRDs,
ServiceAccounts and RBAC before workloads, webhooks last (stable within a
kind), so ``kubectl apply -f`` of the result never references a namespace or
role that comes later in the file.
"""
from __future__ import annotations

import copy
import os
import re
from typing import Any, Dict, Iterable, List, Optional

import yaml

from ..api.selectors import matches_labels, parse_label_selector

CLUSTER_SCOPED = {
    "CustomResourceDefinition", "ClusterRole", "ClusterRoleBinding", "Namespace", "PersistentVolume",
    "StorageClass", "PriorityClass", "APIService", "MutatingWebhookConfiguration",
    "ValidatingWebhookConfiguration", "ClusterIssuer", "IngressClass", "RuntimeClass",
}
NO_PREFIX = {"CustomResourceDefinition", "APIService"}
# kustomize api/resource/legacy ordering (first group, then last group)
_ORDER_FIRST = ["Namespace", "ResourceQuota", "StorageClass", "CustomResourceDefinition", "ServiceAccount",
                "PodSecurityPolicy", "Role", "ClusterRole", "RoleBinding", "ClusterRoleBinding", "ConfigMap",
                "Secret", "Endpoints", "Service", "LimitRange", "PriorityClass", "PersistentVolume",
                "PersistentVolumeClaim", "Deployment", "StatefulSet", "CronJob", "PodDisruptionBudget"]
_ORDER_LAST = ["MutatingWebhookConfiguration", "ValidatingWebhookConfiguration"]


def legacy_sort(objs: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    def key(o: Dict[str, Any]):
        k = o.get("kind", "")
        if k in _ORDER_FIRST:
            return (0, _ORDER_FIRST.index(k))
        if k in _ORDER_LAST:
            return (2, _ORDER_LAST.index(k))
        return (1, 0)

    return sorted(objs, key=key)


class KustomizeError(Exception):
    pass


def _load_docs(path: str) -> List[Dict[str, Any]]:
    with open(path) as fh:
        return [d for d in yaml.safe_load_all(fh) if d]


def _kfile(d: str) -> str:
    for n in ("kustomization.yaml", "kustomization.yml", "Kustomization"):
        p = os.path.join(d, n)
        if os.path.exists(p):
            return p
    raise KustomizeError(f"no kustomization file in {d}")


# ------------------------------------------------------------------ patches
def _ptr_tokens(path: str) -> List[str]:
    if path == "":
        return []
    if not path.startswith("/"):
        raise KustomizeError(f"bad JSON pointer {path!r}")
    return [t.replace("~1", "/").replace("~0", "~") for t in path[1:].split("/")]


def _walk(doc: Any, toks: List[str]) -> Any:
    cur = doc
    for t in toks:
        if isinstance(cur, list):
            cur = cur[int(t)]
        elif isinstance(cur, dict):
            if t not in cur:
                raise KustomizeError(f"path segment {t!r} not found")
            cur = cur[t]
        else:
            raise KustomizeError(f"cannot descend into {type(cur).__name__} at {t!r}")
    return cur


def apply_json6902(doc: Dict[str, Any], ops: Iterable[Dict[str, Any]]) -> Dict[str, Any]:
    """RFC 6902 add/remove/replace/move/copy/test."""
    doc = copy.deepcopy(doc)
    for op in ops:
        kind = op.get("op")
        toks = _ptr_tokens(op.get("path", ""))
        if kind == "test":
            if _walk(doc, toks) != op.get("value"):
                raise KustomizeError(f"test failed at {op.get('path')}")
            continue
        if kind in ("move", "copy"):
            src = _ptr_tokens(op["from"])
            val = copy.deepcopy(_walk(doc, src))
            if kind == "move":
                parent = _walk(doc, src[:-1])
                if isinstance(parent, list):
                    parent.pop(int(src[-1]))
                else:
                    del parent[src[-1]]
            kind, value = "add", val
        else:
            value = copy.deepcopy(op.get("value"))
        if not toks:
            if kind in ("add", "replace"):
                doc = value
                continue
            raise KustomizeError("cannot remove the document root")
        parent = _walk(doc, toks[:-1])
        last = toks[-1]
        if isinstance(parent, list):
            if kind == "add":
                if last == "-":
                    parent.append(value)
                else:
                    parent.insert(int(last), value)
            elif kind == "replace":
                parent[int(last)] = value
            elif kind == "remove":
                parent.pop(int(last))
            else:
                raise KustomizeError(f"unsupported op {kind!r}")
        elif isinstance(parent, dict):
            if kind == "add":
                parent[last] = value
            elif kind == "replace":
                if last not in parent:
                    raise KustomizeError(f"replace: {op.get('path')} does not exist")
                parent[last] = value
            elif kind == "remove":
                if last not in parent:
                    raise KustomizeError(f"remove: {op.get('path')} does not exist")
                del parent[last]
            else:
                raise KustomizeError(f"unsupported op {kind!r}")
        else:
            raise KustomizeError(f"cannot patch into {type(parent).__name__}")
    return doc


# list fields merged by key in strategic merge patch (the ones manifests use)
_MERGE_KEYS = {"containers": "name", "initContainers": "name", "ports": "containerPort", "env": "name",
               "volumes": "name", "volumeMounts": "mountPath", "tolerations": None, "args": None}


def strategic_merge(base: Any, patch: Any, field: str = "") -> Any:
    if isinstance(base, dict) and isinstance(patch, dict):
        out = dict(base)
        for k, v in patch.items():
            if k == "$patch":
                continue
            if v is None:
                out.pop(k, None)
            elif isinstance(v, dict) and v.get("$patch") == "delete":
                out.pop(k, None)
            elif k in out:
                out[k] = strategic_merge(out[k], v, k)
            else:
                out[k] = copy.deepcopy(v)
        return out
    if isinstance(base, list) and isinstance(patch, list):
        key = _MERGE_KEYS.get(field)
        if key and all(isinstance(x, dict) for x in base + patch):
            out = [copy.deepcopy(x) for x in base]
            for item in patch:
                idx = next((i for i, b in enumerate(out) if b.get(key) == item.get(key)), None)
                if item.get("$patch") == "delete":
                    if idx is not None:
                        out.pop(idx)
                elif idx is None:
                    out.append(copy.deepcopy(item))
                else:
                    out[idx] = strategic_merge(out[idx], item, field)
            return out
        return copy.deepcopy(patch)
    return copy.deepcopy(patch)


def _gvk(obj: Dict[str, Any]):
    av = obj.get("apiVersion", "")
    group, _, version = av.rpartition("/")
    return group, version, obj.get("kind", "")


def _matches(obj: Dict[str, Any], target: Dict[str, Any]) -> bool:
    group, version, kind = _gvk(obj)
    md = obj.get("metadata") or {}
    for k, have in (("group", group), ("version", version), ("kind", kind), ("name", md.get("name", "")),
                    ("namespace", md.get("namespace", ""))):
        want = target.get(k)
        if want is not None and not re.fullmatch(str(want), have or ""):
            return False
    if target.get("labelSelector"):
        if not matches_labels(parse_label_selector(target["labelSelector"]), md.get("labels") or {}):
            return False
    if target.get("annotationSelector"):
        if not matches_labels(parse_label_selector(target["annotationSelector"]), md.get("annotations") or {}):
            return False
    return True


# ------------------------------------------------------------------ build
def _images(objs: List[Dict[str, Any]], images: List[Dict[str, Any]]) -> None:
    def fix(ref: str) -> str:
        for im in images:
            name = im["name"]
            base, tag, digest = ref, "", ""
            if "@" in base:
                base, digest = base.split("@", 1)
            if ":" in base.rsplit("/", 1)[-1]:
                base, tag = base.rsplit(":", 1)
            if base != name:
                continue
            base = im.get("newName", base)
            if im.get("digest"):
                return f"{base}@{im['digest']}"
            tag = str(im.get("newTag", tag))
            return f"{base}:{tag}" if tag else (f"{base}@{digest}" if digest else base)
        return ref

    def walk(x: Any) -> None:
        if isinstance(x, dict):
            for k in ("containers", "initContainers"):
                for c in x.get(k) or []:
                    if isinstance(c, dict) and isinstance(c.get("image"), str):
                        c["image"] = fix(c["image"])
            for v in x.values():
                walk(v)
        elif isinstance(x, list):
            for v in x:
                walk(v)

    for o in objs:
        walk(o)


def _set_labels(objs: List[Dict[str, Any]], labels: Dict[str, str], selectors: bool) -> None:
    for o in objs:
        md = o.setdefault("metadata", {})
        md.setdefault("labels", {}).update(labels)
        if not selectors:
            continue
        spec = o.get("spec") or {}
        if o.get("kind") in ("Deployment", "StatefulSet", "DaemonSet", "ReplicaSet", "Job"):
            spec.setdefault("selector", {}).setdefault("matchLabels", {}).update(labels)
            tmpl = spec.setdefault("template", {}).setdefault("metadata", {})
            tmpl.setdefault("labels", {}).update(labels)
        elif o.get("kind") == "Service":
            spec.setdefault("selector", {}).update(labels)


def _rename(objs: List[Dict[str, Any]], prefix: str, suffix: str, namespace: Optional[str]) -> None:
    renamed: Dict[tuple, str] = {}
    for o in objs:
        kind = o.get("kind", "")
        md = o.setdefault("metadata", {})
        if kind not in NO_PREFIX and (prefix or suffix):
            new = f"{prefix}{md.get('name', '')}{suffix}"
            renamed[(kind, md.get("name", ""))] = new
            md["name"] = new
    for o in objs:
        kind = o.get("kind", "")
        md = o["metadata"]
        if namespace is not None and kind not in CLUSTER_SCOPED:
            md["namespace"] = namespace
        if kind in ("RoleBinding", "ClusterRoleBinding"):
            ref = o.get("roleRef") or {}
            if (ref.get("kind"), ref.get("name")) in renamed:
                ref["name"] = renamed[(ref["kind"], ref["name"])]
            for s in o.get("subjects") or []:
                if s.get("kind") == "ServiceAccount":
                    if ("ServiceAccount", s.get("name")) in renamed:
                        s["name"] = renamed[("ServiceAccount", s["name"])]
                    if namespace is not None:
                        s["namespace"] = namespace
        pod = ((o.get("spec") or {}).get("template") or {}).get("spec") if kind in (
            "Deployment", "StatefulSet", "DaemonSet", "Job") else None
        if isinstance(pod, dict) and ("ServiceAccount", pod.get("serviceAccountName")) in renamed:
            pod["serviceAccountName"] = renamed[("ServiceAccount", pod["serviceAccountName"])]
        if kind == "CustomResourceDefinition" and namespace is not None:
            conv = ((o.get("spec") or {}).get("conversion") or {}).get("webhook", {}).get("clientConfig", {})
            if conv.get("service"):
                conv["service"]["namespace"] = namespace


def build(directory: str) -> List[Dict[str, Any]]:
    """``kustomize build <directory>`` -> list of objects."""
    kpath = _kfile(directory)
    with open(kpath) as fh:
        k = yaml.safe_load(fh) or {}
    objs: List[Dict[str, Any]] = []
    for r in k.get("resources") or []:
        p = os.path.normpath(os.path.join(directory, r))
        if os.path.isdir(p):
            objs.extend(build(p))
        elif os.path.exists(p):
            objs.extend(_load_docs(p))
        else:
            raise KustomizeError(f"{kpath}: resource {r!r} not found")
    for r in k.get("crds") or []:
        objs.extend(_load_docs(os.path.join(directory, r)))

    for ent in k.get("patches") or []:
        if "path" in ent:
            docs = _load_docs(os.path.join(directory, ent["path"]))
            body = docs[0] if len(docs) == 1 else docs
        else:
            body = yaml.safe_load(ent["patch"])
        target = ent.get("target")
        is_6902 = isinstance(body, list)
        if target is None:
            if is_6902:
                raise KustomizeError("a JSON6902 patch needs a target")
            md = body.get("metadata") or {}
            target = {"kind": body.get("kind"), "name": md.get("name")}
        hit = False
        for i, o in enumerate(objs):
            if _matches(o, target):
                objs[i] = apply_json6902(o, body) if is_6902 else strategic_merge(o, body)
                hit = True
        if not hit:
            raise KustomizeError(f"{kpath}: patch target {target} matched nothing")
    for ent in k.get("patchesStrategicMerge") or []:
        body = _load_docs(os.path.join(directory, ent))[0]
        md = body.get("metadata") or {}
        for i, o in enumerate(objs):
            if _matches(o, {"kind": body.get("kind"), "name": md.get("name")}):
                objs[i] = strategic_merge(o, body)

    if k.get("images"):
        _images(objs, k["images"])
    if k.get("commonLabels"):
        _set_labels(objs, k["commonLabels"], True)
    for ent in k.get("labels") or []:
        _set_labels(objs, ent.get("pairs") or {}, bool(ent.get("includeSelectors")))
    _rename(objs, k.get("namePrefix", ""), k.get("nameSuffix", ""), k.get("namespace"))
    return objs


def build_sorted(directory: str) -> List[Dict[str, Any]]:
    """``kustomize build`` output order (legacy sort)."""
    return legacy_sort(build(directory))


def build_yaml(directory: str) -> str:
    return "---\n".join(yaml.safe_dump(o, sort_keys=False) for o in build_sorted(directory))


if __name__ == "__main__":
    import sys

    sys.stdout.write(build_yaml(sys.argv[1] if len(sys.argv) > 1 else "deploy/kustomize/default"))
