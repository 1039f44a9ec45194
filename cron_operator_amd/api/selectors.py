"""Label and field selectors (``k8s.io/apimachinery/pkg/labels`` / ``fields`` syntax).

Used by the fake apiserver's LIST/WATCH filtering and by the informer indexers.
The reference lists children with ``client.MatchingLabels{kubedl.io/cron-name:
<name>}`` (``internal/controller/cron_controller.go:252-258``), i.e. the selector
``kubedl.io/cron-name=<name>``.
"""
from __future__ import annotations

import re
from functools import lru_cache
from typing import Any, Callable, Dict, List, Optional, Tuple

Requirement = Tuple[str, str, Tuple[str, ...]]  # (key, op, values); op in = != in notin exists !exists

_TOKEN_RE = re.compile(r"\s*(!=|==|=|\(|\)|,|!|[^\s!=(),]+)")


class SelectorError(ValueError):
    pass


def _tokens(s: str) -> List[str]:
    out = []
    pos = 0
    while pos < len(s):
        m = _TOKEN_RE.match(s, pos)
        if not m:
            if s[pos:].strip() == "":
                break
            raise SelectorError(f"unable to parse requirement: {s!r}")
        out.append(m.group(1))
        pos = m.end()
    return out


def parse_label_selector(s: Optional[str]) -> List[Requirement]:
    if not s or not s.strip():
        return []
    toks = _tokens(s)
    reqs: List[Requirement] = []
    i = 0
    while i < len(toks):
        if toks[i] == "!":
            if i + 1 >= len(toks):
                raise SelectorError("missing key after '!'")
            reqs.append((toks[i + 1], "!exists", ()))
            i += 2
        else:
            key = toks[i]
            i += 1
            if i >= len(toks) or toks[i] == ",":
                reqs.append((key, "exists", ()))
            elif toks[i] in ("=", "=="):
                if i + 1 >= len(toks) or toks[i + 1] == ",":
                    reqs.append((key, "=", ("",)))
                    i += 1
                else:
                    reqs.append((key, "=", (toks[i + 1],)))
                    i += 2
            elif toks[i] == "!=":
                if i + 1 >= len(toks) or toks[i + 1] == ",":
                    reqs.append((key, "!=", ("",)))
                    i += 1
                else:
                    reqs.append((key, "!=", (toks[i + 1],)))
                    i += 2
            elif toks[i] in ("in", "notin"):
                op = toks[i]
                i += 1
                if i >= len(toks) or toks[i] != "(":
                    raise SelectorError(f"expected '(' after {op}")
                i += 1
                vals = []
                while i < len(toks) and toks[i] != ")":
                    if toks[i] != ",":
                        vals.append(toks[i])
                    i += 1
                if i >= len(toks):
                    raise SelectorError("unterminated value list")
                i += 1
                reqs.append((key, op, tuple(vals)))
            else:
                raise SelectorError(f"unexpected token {toks[i]!r} in selector {s!r}")
        if i < len(toks):
            if toks[i] != ",":
                raise SelectorError(f"expected ',' in selector {s!r}")
            i += 1
    return reqs


def matches_labels(reqs: List[Requirement], labels: Dict[str, str]) -> bool:
    for key, op, vals in reqs:
        has = key in labels
        if op == "=":
            if not has or labels[key] != vals[0]:
                return False
        elif op == "!=":
            if has and labels[key] == vals[0]:
                return False
        elif op == "in":
            if not has or labels[key] not in vals:
                return False
        elif op == "notin":
            if has and labels[key] in vals:
                return False
        elif op == "exists":
            if not has:
                return False
        elif op == "!exists":
            if has:
                return False
    return True



def _field_value(obj: Dict[str, Any], path: str) -> Optional[str]:
    cur: Any = obj
    for part in path.split("."):
        if not isinstance(cur, dict):
            return None
        cur = cur.get(part)
    if cur is None:
        return ""
    return cur if isinstance(cur, str) else str(cur)


def parse_field_selector(s: Optional[str]) -> List[Tuple[str, str, str]]:
    if not s or not s.strip():
        return []
    out = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "!=" in part:
            k, v = part.split("!=", 1)
            out.append((k.strip(), "!=", v.strip()))
        elif "==" in part:
            k, v = part.split("==", 1)
            out.append((k.strip(), "=", v.strip()))
        elif "=" in part:
            k, v = part.split("=", 1)
            out.append((k.strip(), "=", v.strip()))
        else:
            raise SelectorError(f"invalid field selector: {part!r}")
    return out


def matches_fields(reqs: List[Tuple[str, str, str]], obj: Dict[str, Any]) -> bool:
    for path, op, val in reqs:
        got = _field_value(obj, path)
        if op == "=" and got != val:
            return False
        if op == "!=" and got == val:
            return False
    return True


def _requirement_check(key: str, op: str, vals: Tuple[str, ...]) -> Callable[[Dict[str, str]], bool]:
    if op == "=":
        v = vals[0]
        return lambda labels: labels.get(key) == v
    if op == "!=":
        v = vals[0]
        return lambda labels: labels.get(key) != v
    if op == "in":
        vs = frozenset(vals)
        return lambda labels: key in labels and labels[key] in vs
    if op == "notin":
        vs = frozenset(vals)
        return lambda labels: labels.get(key) not in vs if key in labels else True
    if op == "exists":
        return lambda labels: key in labels
    return lambda labels: key not in labels


class Selector:
    """A compiled label + field selector: ``sel(obj) -> bool``.

    ``pinned`` is the first ``key=value`` label requirement, if any: every matching
    object carries that label value, which lets the fake apiserver index watchers by it.
    Instances are shared per selector string (:func:`compile_selectors` memoises), so
    watchers with equal selectors can share one evaluation per event.
    """

    __slots__ = ("label_selector", "field_selector", "pinned", "_fn")

    def __init__(self, label_selector: Optional[str], field_selector: Optional[str]):
        self.label_selector = label_selector or ""
        self.field_selector = field_selector or ""
        lreq = parse_label_selector(label_selector)
        freq = parse_field_selector(field_selector)
        self.pinned: Optional[Tuple[str, str]] = next(((k, vals[0]) for k, op, vals in lreq if op == "="), None)
        checks = tuple(_requirement_check(*r) for r in lreq)
        if not checks and not freq:
            self._fn: Callable[[Dict[str, Any]], bool] = lambda obj: True
        elif len(checks) == 1 and not freq:
            c = checks[0]
            self._fn = lambda obj: c((obj.get("metadata") or {}).get("labels") or {})
        else:
            def fn(obj: Dict[str, Any]) -> bool:
                if checks:
                    labels = (obj.get("metadata") or {}).get("labels") or {}
                    for c in checks:
                        if not c(labels):
                            return False
                return not freq or matches_fields(freq, obj)
            self._fn = fn

    def __call__(self, obj: Dict[str, Any]) -> bool:
        return self._fn(obj)


@lru_cache(maxsize=4096)
def compile_selectors(label_selector: Optional[str], field_selector: Optional[str]) -> Selector:
    return Selector(label_selector, field_selector)
