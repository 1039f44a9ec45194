"""Label and field selectors (``k8s.io/apimachinery/pkg/labels`` / ``fields`` syntax).

Used by the fake apiserver's LIST/WATCH filtering and by the informer indexers.
The reference lists children with ``client.MatchingLabels{kubedl.io/cron-name:
<name>}`` (``internal/controller/cron_controller.go:252-258``), i.e. the selector
``kubedl.io/cron-name=<name>``.
"""
from __future__ import annotations

import re
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


def format_label_selector(match: Dict[str, str]) -> str:
    return ",".join(f"{k}={v}" for k, v in sorted(match.items()))


def equality_value(reqs: List[Requirement], key: str) -> Optional[str]:
    """The value ``key`` is pinned to by an ``=`` requirement, if any (index lookups)."""
    for k, op, vals in reqs:
        if k == key and op == "=":
            return vals[0]
    return None


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


def compile_selectors(label_selector: Optional[str], field_selector: Optional[str]) -> Callable[[Dict[str, Any]], bool]:
    lreq = parse_label_selector(label_selector)
    freq = parse_field_selector(field_selector)
    if not lreq and not freq:
        return lambda obj: True

    def pred(obj: Dict[str, Any]) -> bool:
        if lreq and not matches_labels(lreq, (obj.get("metadata") or {}).get("labels") or {}):
            return False
        return not freq or matches_fields(freq, obj)

    return pred
