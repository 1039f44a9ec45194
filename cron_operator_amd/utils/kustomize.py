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
  ``serviceAccountName``, Service/ServiceMonitor/NetworkPolicy don't need it)
  plus the ``nameReference`` entries of ``configurations`` files (for CRD
  fields such as a Certificate's ``spec.issuerRef.name``);
* ``labels`` (with ``includeSelectors``) and legacy ``commonLabels``;
* ``images`` -- ``newName`` / ``newTag`` / ``digest`` by image name;
* ``patches`` -- JSON 6902 op lists or strategic-merge documents, inline
  (``patch``) or from a file (``path``), selected by ``target``
  (group/version/kind/name/namespace/labelSelector) or by the patch's own
  kind+name;
* ``replacements`` -- copy a field of one object (``source``: selected by
  group/version/kind/name/namespace, matching the name before or after
  ``namePrefix``) into fields of others (``targets``: ``fieldPaths`` with
  ``[key=value]`` list selectors and ``[dotted.key]`` map keys, ``options``
  ``delimiter``/``index``/``create``), run last as kustomize does.

:func:`enable_optional` un-comments the optional sections of a kustomization
(the reference's ``[CERTMANAGER]``-style toggles) into a copy of the tree.

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


def _load_name_refs(directory: str, files: List[str]) -> List[Dict[str, Any]]:
    """``configurations:`` files -> their ``nameReference`` entries (how kustomize learns that a
    CRD field, e.g. a cert-manager Certificate's ``spec.issuerRef.name``, names another object)."""
    refs: List[Dict[str, Any]] = []
    for f in files:
        for doc in _load_docs(os.path.join(directory, f)):
            refs.extend(doc.get("nameReference") or [])
    return refs


def _fix_name_refs(objs: List[Dict[str, Any]], renamed: Dict[tuple, str], refs: List[Dict[str, Any]]) -> None:
    for ref in refs:
        kind = ref.get("kind")
        for fs in ref.get("fieldSpecs") or []:
            for o in objs:
                if fs.get("kind") is not None and fs["kind"] != o.get("kind"):
                    continue
                if fs.get("group") is not None and fs["group"] != _gvk(o)[0]:
                    continue
                node: Any = o
                toks = [t for t in str(fs.get("path", "")).split("/") if t]
                for t in toks[:-1]:
                    node = node.get(t) if isinstance(node, dict) else None
                if isinstance(node, dict) and toks and (kind, node.get(toks[-1])) in renamed:
                    node[toks[-1]] = renamed[(kind, node[toks[-1]])]


def _rename(objs: List[Dict[str, Any]], prefix: str, suffix: str, namespace: Optional[str],
            name_refs: Optional[List[Dict[str, Any]]] = None) -> None:
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
    if name_refs:
        _fix_name_refs(objs, renamed, name_refs)


# ------------------------------------------------------------------ replacements
def _field_tokens(path: str) -> List[str]:
    """``spec.endpoints.0.tlsConfig.serverName`` / ``.metadata.annotations.[a.b/c]`` /
    ``spec.containers.[name=manager].args`` -> tokens (brackets keep their dots)."""
    toks: List[str] = []
    i, cur, n = 0, "", len(path)
    while i < n:
        c = path[i]
        if c == "[":
            j = path.index("]", i)
            toks.append(path[i:j + 1])
            i = j + 1
            continue
        if c == ".":
            if cur:
                toks.append(cur)
            cur = ""
        else:
            cur += c
        i += 1
    if cur:
        toks.append(cur)
    return toks


def _step(node: Any, tok: str, create: bool, last: bool) -> Any:
    """One path step; with ``create`` missing maps (or the final key) are made."""
    if tok.startswith("[") and tok.endswith("]"):
        inner = tok[1:-1]
        if "=" in inner and isinstance(node, list):
            k, v = inner.split("=", 1)
            for it in node:
                if isinstance(it, dict) and str(it.get(k)) == v:
                    return it
            if not create:
                raise KeyError(tok)
            it = {k: v}
            node.append(it)
            return it
        tok = inner
    if isinstance(node, list):
        idx = int(tok)
        if idx < len(node):
            return node[idx]
        raise KeyError(tok)
    if not isinstance(node, dict):
        raise KeyError(tok)
    if tok not in node:
        if not create:
            raise KeyError(tok)
        if not last:
            node[tok] = {}
    return node.get(tok)


def _get_field(obj: Dict[str, Any], path: str) -> Any:
    node: Any = obj
    for t in _field_tokens(path):
        node = _step(node, t, False, False)
    return node


def _set_field(obj: Dict[str, Any], path: str, value: Any, opts: Dict[str, Any]) -> bool:
    toks = _field_tokens(path)
    create = bool(opts.get("create"))
    node: Any = obj
    try:
        for t in toks[:-1]:
            node = _step(node, t, create, False)
    except KeyError:
        return False
    last = toks[-1]
    if last.startswith("[") and "=" not in last:
        last = last[1:-1]
    if isinstance(node, list):
        idx = int(last)
        if idx >= len(node):
            return False
        cur, setter = node[idx], (lambda v: node.__setitem__(idx, v))
    elif isinstance(node, dict):
        if last not in node and not create:
            return False
        cur, setter = node.get(last), (lambda v: node.__setitem__(last, v))
    else:
        return False
    if "delimiter" in opts:
        d = str(opts["delimiter"])
        parts = str(cur).split(d) if cur not in (None, "") else []
        at = int(opts.get("index", 0))
        if at < 0:
            parts.insert(0, str(value))
        elif at >= len(parts):
            parts.append(str(value))
        else:
            parts[at] = str(value)
        setter(d.join(parts))
    else:
        setter(copy.deepcopy(value))
    return True


def _select(objs: List[Dict[str, Any]], sel: Dict[str, Any], orig: Dict[int, str]) -> List[Dict[str, Any]]:
    out = []
    for o in objs:
        group, version, kind = _gvk(o)
        md = o.get("metadata") or {}
        if sel.get("kind") is not None and sel["kind"] != kind:
            continue
        if sel.get("group") is not None and sel["group"] != group:
            continue
        if sel.get("version") is not None and sel["version"] != version:
            continue
        if sel.get("namespace") is not None and sel["namespace"] != md.get("namespace", ""):
            continue
        if sel.get("name") is not None and sel["name"] not in (md.get("name"), orig.get(id(o))):
            continue
        out.append(o)
    return out


def _replacements(objs: List[Dict[str, Any]], reps: List[Dict[str, Any]], orig: Dict[int, str],
                  where: str) -> None:
    for rep in reps:
        src = rep.get("source") or {}
        found = _select(objs, src, orig)
        if len(found) != 1:
            raise KustomizeError(f"{where}: replacement source {src} matched {len(found)} objects")
        try:
            value = _get_field(found[0], src.get("fieldPath") or "metadata.name")
        except KeyError:
            raise KustomizeError(f"{where}: source fieldPath {src.get('fieldPath')} not found") from None
        sopts = src.get("options") or {}
        if "delimiter" in sopts:
            parts = str(value).split(str(sopts["delimiter"]))
            value = parts[int(sopts.get("index", 0))]
        for tgt in rep.get("targets") or []:
            hits = _select(objs, tgt.get("select") or {}, orig)
            for rej in tgt.get("reject") or []:
                bad = {id(o) for o in _select(objs, rej, orig)}
                hits = [o for o in hits if id(o) not in bad]
            for o in hits:
                for fp in tgt.get("fieldPaths") or ["metadata.name"]:
                    if not _set_field(o, fp, value, tgt.get("options") or {}):
                        raise KustomizeError(f"{where}: target field {fp} missing in "
                                             f"{o.get('kind')}/{(o.get('metadata') or {}).get('name')}")


def enable_optional(directory: str, dest: str) -> str:
    """Copy the kustomize tree holding ``directory`` to ``dest`` with every optional section
    of its kustomization files un-commented, and return the copied ``directory``.

    A toggle is a comment whose text is YAML at its own indentation -- ``#  - ../x``,
    ``#patches:``, ``#    target:`` -- i.e. ``#`` followed by a key at column 0 or by two or
    more spaces; prose comments are ``# `` plus one space and stay comments."""
    import shutil

    root = os.path.dirname(os.path.abspath(directory))
    shutil.copytree(root, dest, dirs_exist_ok=True)
    toggle = re.compile(r"^#(?:[A-Za-z_][\w-]*:| {2,}\S)")
    for dirpath, _, files in os.walk(dest):
        for f in files:
            if f not in ("kustomization.yaml", "kustomization.yml", "Kustomization"):
                continue
            p = os.path.join(dirpath, f)
            with open(p) as fh:
                lines = fh.read().splitlines()
            with open(p, "w") as fh:
                fh.write("\n".join(ln[1:] if toggle.match(ln) else ln for ln in lines) + "\n")
    return os.path.join(dest, os.path.basename(os.path.abspath(directory)))


def _collect_name_refs(directory: str) -> List[Dict[str, Any]]:
    """``configurations`` of this kustomization and of every kustomization it includes
    (kustomize merges them, so a base's configuration applies to the overlay's prefix)."""
    with open(_kfile(directory)) as fh:
        k = yaml.safe_load(fh) or {}
    refs = _load_name_refs(directory, k.get("configurations") or [])
    for r in k.get("resources") or []:
        p = os.path.normpath(os.path.join(directory, r))
        if os.path.isdir(p):
            refs.extend(_collect_name_refs(p))
    return refs


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
    orig = {id(o): (o.get("metadata") or {}).get("name", "") for o in objs}
    _rename(objs, k.get("namePrefix", ""), k.get("nameSuffix", ""), k.get("namespace"),
            _collect_name_refs(directory))
    if k.get("replacements"):
        _replacements(objs, k["replacements"], orig, kpath)
    return objs


def build_sorted(directory: str) -> List[Dict[str, Any]]:
    """``kustomize build`` output order (legacy sort)."""
    return legacy_sort(build(directory))


def build_yaml(directory: str) -> str:
    return "---\n".join(yaml.safe_dump(o, sort_keys=False) for o in build_sorted(directory))


if __name__ == "__main__":
    import sys

    sys.stdout.write(build_yaml(sys.argv[1] if len(sys.argv) > 1 else "deploy/kustomize/default"))
