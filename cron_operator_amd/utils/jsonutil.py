"""JSON-tree helpers: copy, semantic equality, RFC 7386 merge patch.

Kubernetes objects travel as JSON object trees (``dict``/``list``/``str``/
``int``/``float``/``bool``/``None``) everywhere in this framework: the fake
apiserver stores them, the informer caches them, the reconciler reads them.
These helpers are on the hot path of every request, so the native
``_fastjson`` extension (``ops/csrc/fastjson.cpp``) provides drop-in versions
of :func:`deepcopy`, :func:`json_equal` and :func:`create_merge_patch`; the
pure-Python implementations below are the fallback and the test oracle.

``create_merge_patch(old, new)`` reproduces what controller-runtime's
``client.MergeFrom(old)`` sends (``CreateMergePatch`` of the two JSON
documents), which the reference uses for its deferred status write
(``internal/controller/cron_controller.go:107-120``).
"""
from __future__ import annotations

import json
from typing import Any, Dict

_SCALARS = (str, int, float, bool, type(None))


def py_deepcopy(x: Any) -> Any:
    t = type(x)
    if t is dict:
        return {k: (v if type(v) in _SCALARS else py_deepcopy(v)) for k, v in x.items()}
    if t is list:
        return [v if type(v) in _SCALARS else py_deepcopy(v) for v in x]
    return x


def py_json_equal(a: Any, b: Any) -> bool:
    if a is b:
        return True
    ta, tb = type(a), type(b)
    if ta is dict and tb is dict:
        if len(a) != len(b):
            return False
        for k, v in a.items():
            if k not in b or not py_json_equal(v, b[k]):
                return False
        return True
    if ta is list and tb is list:
        if len(a) != len(b):
            return False
        return all(py_json_equal(x, y) for x, y in zip(a, b))
    if ta is bool or tb is bool:
        return ta is tb and a == b
    return a == b


def py_create_merge_patch(old: Any, new: Any, share: bool = False) -> Any:
    """Minimal RFC 7386 patch turning ``old`` into ``new`` (objects only recurse).
    ``share=True``: the patch references ``new``'s subtrees instead of copies (for a patch
    that is only serialised; ``new`` must not change while it lives)."""
    cp = (lambda x: x) if share else py_deepcopy
    if type(old) is not dict or type(new) is not dict:
        return cp(new)
    patch = {}
    for k, v in new.items():
        if k not in old:
            patch[k] = cp(v)
        else:
            ov = old[k]
            if type(ov) is dict and type(v) is dict:
                sub = py_create_merge_patch(ov, v, share)
                if sub:
                    patch[k] = sub
            elif not py_json_equal(ov, v):
                patch[k] = cp(v)
    for k in old:
        if k not in new:
            patch[k] = None
    return patch


def apply_merge_patch(target: Any, patch: Any, share: bool = False) -> Any:
    """RFC 7386 apply; returns a new tree (inputs untouched).

    ``share=True`` (structural sharing): only the dicts on the patch's paths are
    copied (shallowly) and every untouched subtree -- and the patch's own values --
    is shared with the inputs.  For callers that treat both inputs as immutable,
    e.g. the apiserver merging a freshly decoded request body into a stored object.
    """
    if type(patch) is not dict:
        return patch if share else deepcopy(patch)
    if type(target) is dict:
        out = dict(target) if share else deepcopy(target)
    else:
        out = {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        elif type(v) is dict:
            out[k] = apply_merge_patch(out.get(k), v, share)
        else:
            out[k] = v if share else deepcopy(v)
    return out


def apply_json_patch(target: Any, ops: list) -> Any:
    """RFC 6902 JSON patch (add/remove/replace/test/move/copy)."""
    doc = deepcopy(target)

    def parse_ptr(p: str):
        if p == "":
            return []
        if not p.startswith("/"):
            raise ValueError(f"invalid JSON pointer {p!r}")
        return [s.replace("~1", "/").replace("~0", "~") for s in p[1:].split("/")]

    def walk(d, parts):
        for s in parts:
            if type(d) is list:
                d = d[int(s)]
            else:
                d = d[s]
        return d

    for op in ops:
        kind = op.get("op")
        path = parse_ptr(op.get("path", ""))
        if kind == "test":
            if not py_json_equal(walk(doc, path), op.get("value")):
                raise ValueError(f"test operation failed at {op.get('path')}")
            continue
        if kind in ("move", "copy"):
            src = parse_ptr(op["from"])
            val = deepcopy(walk(doc, src))
            if kind == "move":
                parent = walk(doc, src[:-1])
                if type(parent) is list:
                    parent.pop(int(src[-1]))
                else:
                    del parent[src[-1]]
            kind, op = "add", {"value": val}
        if not path:
            if kind in ("add", "replace"):
                doc = deepcopy(op.get("value"))
                continue
            raise ValueError("cannot remove the document root")
        parent = walk(doc, path[:-1])
        last = path[-1]
        if kind == "add":
            if type(parent) is list:
                if last == "-":
                    parent.append(deepcopy(op.get("value")))
                else:
                    parent.insert(int(last), deepcopy(op.get("value")))
            else:
                parent[last] = deepcopy(op.get("value"))
        elif kind == "remove":
            if type(parent) is list:
                parent.pop(int(last))
            else:
                del parent[last]
        elif kind == "replace":
            if type(parent) is list:
                parent[int(last)] = deepcopy(op.get("value"))
            else:
                if last not in parent:
                    raise KeyError(last)
                parent[last] = deepcopy(op.get("value"))
        else:
            raise ValueError(f"unsupported JSON patch op {kind!r}")
    return doc


def py_dumps(x: Any) -> str:
    return json.dumps(x, separators=(",", ":"), ensure_ascii=False)


def py_dumpb(x: Any) -> bytes:
    return json.dumps(x, separators=(",", ":"), ensure_ascii=False).encode()


dumps = py_dumps
dumpb = py_dumpb


py_loads = json.loads
loads = json.loads

# --------------------------------------------------------------------------- native dispatch

def dumpb_shared(obj: Any, cache: Dict[int, Any], volatile_keys: Any = ()) -> bytes:
    """``dumpb`` of a tree that is never mutated, reusing the bytes of its top-level
    containers (except under ``volatile_keys``) cached by identity in ``cache`` (native);
    the Python twin ignores the cache."""
    return dumpb(obj)


class PyMemo:
    """Python twin of the native ``Memo`` (no reuse: every value is built afresh)."""

    def __init__(self, slots: int = 1 << 14, max_slots: int = 1 << 19):
        self.slots = slots
        self.max_slots = max(slots, max_slots)

    def stats(self) -> Dict[str, int]:
        return {"hits": 0, "misses": 0, "stores": 0, "reuses": 0, "evictions": 0, "grows": 0, "used": 0,
                "slots": self.slots, "max_slots": self.max_slots}

    def forget(self, obj: Any) -> bool:
        return False

    def clear(self) -> None:
        pass


def _drop(v: Any, path: Any) -> None:
    if not path:
        return
    head, rest = path[0], path[1:]
    if head == "*":
        if type(v) is list:
            for x in v:
                _drop(x, rest)
        return
    if type(v) is not dict:
        return
    if not rest:
        v.pop(head, None)
    elif head in v:
        _drop(v[head], rest)


def _rawify(v: Any, path: Any) -> None:
    """Replace the value at ``path`` ("*" = any list element) by its JSON text (bytes)."""
    head, rest = path[0], path[1:]
    if head == "*":
        if type(v) is list:
            for i, x in enumerate(v):
                if rest:
                    _rawify(x, rest)
                else:
                    v[i] = dumpb(x)
        return
    if type(v) is not dict or head not in v:
        return
    if rest:
        _rawify(v[head], rest)
    else:
        v[head] = dumpb(v[head])


def _route_foreign(meta: Any, route: Any) -> bool:
    """The native codec's route test: True only when ``meta`` surely hashes to another shard
    (FNV-1a of ``namespace/key``, as ``runtime.controller.shard_of``)."""
    index, count, label = route
    if count <= 1 or type(meta) is not dict:
        return False
    ns = meta.get("namespace", "")
    if type(ns) is not str:
        return False
    if label is not None:
        labels = meta.get("labels")
        if type(labels) is not dict or label not in labels:
            return False
        key = labels[label]
    else:
        key = meta.get("name", "")
    if type(key) is not str:
        return False
    try:
        raw = f"{ns}/{key}".encode()
    except UnicodeEncodeError:
        return False
    h = 0x811C9DC5
    for b in raw:
        h = ((h ^ b) * 0x01000193) & 0xFFFFFFFF
    return h % count != index


def _route(v: Any, path: Any, route: Any) -> None:
    """At ``path``: an object of another shard keeps its members up to ``metadata``."""
    if not path:
        if type(v) is dict and "metadata" in v and _route_foreign(v["metadata"], route):
            keys = list(v)
            for k in keys[keys.index("metadata") + 1:]:
                del v[k]
        return
    head, rest = path[0], path[1:]
    if head == "*":
        if type(v) is list:
            for x in v:
                _route(x, rest, route)
        return
    if type(v) is dict and head in v:
        _route(v[head], rest, route)


def _unraw(v: Any, path: Any) -> None:
    head, rest = path[0], path[1:]
    if head == "*":
        if type(v) is list:
            for i, x in enumerate(v):
                if rest:
                    _unraw(x, rest)
                elif isinstance(x, (bytes, bytearray)):
                    v[i] = loads(x)
        return
    if type(v) is not dict or head not in v:
        return
    if rest:
        _unraw(v[head], rest)
    elif isinstance(v[head], (bytes, bytearray)):
        v[head] = loads(v[head])


class PyCodec:
    """Python twin of the native ``Codec(skip, memo_paths, memo, raw_paths, route_paths, route)``:
    ``loads`` decodes, cuts another shard's objects at route paths after their ``metadata``,
    removes the skipped paths ("*" = any list element) and turns the values at raw paths into
    their JSON text (bytes; re-encoded compactly here, the input's own text natively); memo
    paths change nothing but speed, so they are ignored here.  Calling it
    decodes one watch event line into ``(type, object)``."""

    def __init__(self, skip: Any = (), memo_paths: Any = (), memo: Any = None, raw_paths: Any = (),
                 route_paths: Any = None, route: Any = None):
        self.skip = [tuple(p) for p in skip or ()]
        self.raw = [tuple(p) for p in raw_paths or ()]
        self.memo = memo
        self.route_paths = [tuple(p) for p in route_paths] if route_paths is not None else []
        if route_paths is not None:
            index, count, label = route
            if not (isinstance(index, int) and isinstance(count, int) and 0 <= index < count) or \
                    not (label is None or isinstance(label, str)):
                raise ValueError("route must be (index, count, label or None) with 0 <= index < count")
        self.route = route

    def loads(self, data: Any) -> Any:
        v = loads(data)
        for path in self.route_paths:
            _route(v, path, self.route)
        for path in self.skip:
            _drop(v, path)
        for path in self.raw:
            _rawify(v, path)
        return v

    def __call__(self, line: Any) -> Any:
        ev = self.loads(line)
        return ev.get("type", "") or "", ev.get("object") or {}

    def dumpb(self, tree: Any) -> bytes:
        if self.raw:  # raw values (bytes) go back as the JSON they hold
            tree = deepcopy(tree)
            for path in self.raw:
                _unraw(tree, path)
        return dumpb(tree)


deepcopy = py_deepcopy
json_equal = py_json_equal
create_merge_patch = py_create_merge_patch
Codec: Any = PyCodec
Memo: Any = PyMemo
NATIVE = False
# informer-event bookkeeping (runtime/informer.py); None without the native module
store_apply: Any = None


def py_pick(d: Dict[Any, Any], keys: Any) -> list:
    """``[d[k] for k in keys]``."""
    return [d[k] for k in keys]


pick: Any = py_pick


def _try_native() -> None:
    global deepcopy, json_equal, create_merge_patch, loads, dumps, dumpb, dumpb_shared, Codec, Memo, NATIVE
    global store_apply, pick
    import os

    if os.environ.get("CRON_OPERATOR_FASTJSON", "auto").lower() == "python":
        return
    try:
        from ..ops import fastjson_native

        mod = fastjson_native.load()
    except Exception:  # noqa: BLE001 - fall back to Python
        if os.environ.get("CRON_OPERATOR_FASTJSON", "auto").lower() == "native":
            raise
        return
    deepcopy = mod.deepcopy
    json_equal = mod.json_equal
    create_merge_patch = mod.create_merge_patch
    loads = mod.loads
    dumps = mod.dumps
    dumpb = mod.dumpb
    dumpb_shared = mod.dumpb_shared
    Codec = mod.Codec
    Memo = mod.Memo
    store_apply = getattr(mod, "store_apply", None)
    pick = getattr(mod, "pick", py_pick)
    NATIVE = True


_try_native()
