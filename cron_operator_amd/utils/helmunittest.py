"""A helm-unittest compatible runner on top of the in-repo chart renderer.

The reference unit-tests its chart with the helm-unittest plugin (v0.8.2,
``Makefile:158-160``): YAML suites under ``charts/cron-operator/tests`` that
render templates with ``set`` values and assert on paths of the output.  helm
and the plugin are not available here, so this runs the same suite format with
:func:`cron_operator_amd.utils.gotemplate.render_chart`:

suite keys
    ``suite``, ``templates``, ``release`` (name, namespace), ``values`` (files),
    ``set`` (suite-wide), ``tests`` (list).
test keys
    ``it``, ``set``, ``values``, ``template`` / ``templates``, ``documentIndex``,
    ``release``, ``asserts``.
assertions
    ``equal``, ``notEqual``, ``contains`` (``content``, ``count``), ``notContains``,
    ``isNull``, ``isNotNull``, ``isNotEmpty``, ``isEmpty``, ``isKind`` (``of``),
    ``isAPIVersion`` (``of``), ``hasDocuments`` (``count``), ``matchRegex``
    (``pattern``), ``notMatchRegex``, ``isSubset`` (``content``), ``exists``,
    ``notExists``, ``lengthEqual`` (``count``); each may carry ``not: true``,
    ``template`` and ``documentIndex``.
paths
    ``a.b[0].c``, ``a["key.with.dots"]``, ``a['k']`` and the filter
    ``list[?(@.name=='x')]`` (first match), as helm-unittest's JSONPath.

``python -m cron_operator_amd.utils.helmunittest [suite.yaml ...]`` runs every
suite of the chart and exits non-zero on failure (``make helm-unittest``).
"""
from __future__ import annotations

import copy
import glob
import os
import re
import sys
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import yaml

from .gotemplate import render_chart

_MISSING = object()
_TOKEN = re.compile(r"""\.?([A-Za-z0-9_\-$]+)"""              # .key
                    r"""|\[(\d+)\]"""                            # [0]
                    r"""|\[\s*["']([^"']+)["']\s*\]"""             # ["dotted.key"]
                    r"""|\[\?\(@\.([A-Za-z0-9_\-.]+)\s*==\s*["']([^"']*)["']\)\]""")  # [?(@.k=='v')]


def get_path(doc: Any, path: str) -> Any:
    """Resolve a helm-unittest path; ``_MISSING`` when any segment is absent."""
    cur = doc
    pos = 0
    path = path.strip()
    while pos < len(path):
        m = _TOKEN.match(path, pos)
        if not m or m.end() == pos:
            raise ValueError(f"unsupported path syntax at {path[pos:]!r} in {path!r}")
        pos = m.end()
        key, idx, qkey, fkey, fval = m.groups()
        if key is not None or qkey is not None:
            k = key if key is not None else qkey
            if not isinstance(cur, dict) or k not in cur:
                return _MISSING
            cur = cur[k]
        elif idx is not None:
            i = int(idx)
            if not isinstance(cur, list) or i >= len(cur):
                return _MISSING
            cur = cur[i]
        else:
            if not isinstance(cur, list):
                return _MISSING
            hit = _MISSING
            for it in cur:
                if isinstance(it, dict) and str(get_path(it, fkey)) == fval:
                    hit = it
                    break
            if hit is _MISSING:
                return _MISSING
            cur = hit
    return cur


def _merge(dst: Dict[str, Any], src: Dict[str, Any]) -> Dict[str, Any]:
    for k, v in (src or {}).items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)
    return dst


def _set_values(sets: Dict[str, Any]) -> Dict[str, Any]:
    """``set`` accepts nested maps and dotted keys (``image.tag: x``)."""
    out: Dict[str, Any] = {}
    for k, v in (sets or {}).items():
        cur = out
        parts = k.split(".")
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        if isinstance(v, dict) and isinstance(cur.get(parts[-1]), dict):
            _merge(cur[parts[-1]], v)
        else:
            cur[parts[-1]] = copy.deepcopy(v)
    return out


@dataclass
class Result:
    suite: str
    name: str
    passed: bool
    failures: List[str] = field(default_factory=list)


def _assert(kind: str, spec: Dict[str, Any], docs: List[Dict[str, Any]]) -> Optional[str]:
    negate = bool(spec.get("not"))
    if kind == "hasDocuments":
        ok = len(docs) == int(spec.get("count", 0))
        return None if ok != negate else f"hasDocuments: expected {spec.get('count')}, got {len(docs)}"
    idx = spec.get("documentIndex")
    targets = [docs[idx]] if idx is not None and idx < len(docs) else ([] if idx is not None else docs)
    if not targets:
        return f"{kind}: no document to assert on"
    for d in targets:
        err = _assert_one(kind, spec, d)
        if (err is None) == negate:
            return err or f"{kind} (negated) unexpectedly passed on {spec}"
    return None


def _assert_one(kind: str, spec: Dict[str, Any], doc: Dict[str, Any]) -> Optional[str]:
    if kind == "isKind":
        return None if doc.get("kind") == spec.get("of") else f"isKind: {doc.get('kind')} != {spec.get('of')}"
    if kind == "isAPIVersion":
        ok = doc.get("apiVersion") == spec.get("of")
        return None if ok else f"isAPIVersion: {doc.get('apiVersion')} != {spec.get('of')}"
    path = spec.get("path", "")
    val = get_path(doc, path)
    if kind == "exists":
        return None if val is not _MISSING else f"exists: {path} missing"
    if kind == "notExists":
        return None if val is _MISSING else f"notExists: {path} = {val!r}"
    if kind == "isNull":
        return None if val is _MISSING or val is None else f"isNull: {path} = {val!r}"
    if kind == "isNotNull":
        return None if val is not _MISSING and val is not None else f"isNotNull: {path} is null"
    if kind == "isEmpty":
        return None if val is _MISSING or not val else f"isEmpty: {path} = {val!r}"
    if kind == "isNotEmpty":
        return None if val is not _MISSING and val else f"isNotEmpty: {path} is empty"
    if val is _MISSING:
        return f"{kind}: {path} missing"
    if kind == "equal":
        return None if val == spec.get("value") else f"equal: {path} = {val!r}, want {spec.get('value')!r}"
    if kind == "notEqual":
        return None if val != spec.get("value") else f"notEqual: {path} = {val!r}"
    if kind in ("contains", "notContains"):
        if not isinstance(val, list):
            return f"{kind}: {path} is not a list"
        want = spec.get("content")
        n = sum(1 for it in val if it == want or (isinstance(want, dict) and isinstance(it, dict)
                                                  and all(it.get(k) == v for k, v in want.items())))
        if kind == "notContains":
            return None if n == 0 else f"notContains: {path} contains {want!r}"
        cnt = spec.get("count")
        if cnt is not None:
            return None if n == int(cnt) else f"contains: {path} has {n} x {want!r}, want {cnt}"
        return None if n > 0 else f"contains: {path} = {val!r} lacks {want!r}"
    if kind in ("matchRegex", "notMatchRegex"):
        hit = re.search(spec.get("pattern", ""), str(val)) is not None
        if kind == "matchRegex":
            return None if hit else f"matchRegex: {path} = {val!r} !~ {spec.get('pattern')}"
        return None if not hit else f"notMatchRegex: {path} = {val!r} =~ {spec.get('pattern')}"
    if kind == "isSubset":
        want = spec.get("content") or {}
        ok = isinstance(val, dict) and all(val.get(k) == v for k, v in want.items())
        return None if ok else f"isSubset: {path} = {val!r} lacks {want!r}"
    if kind == "lengthEqual":
        return None if len(val) == int(spec.get("count", 0)) else f"lengthEqual: len({path}) = {len(val)}"
    return f"unsupported assertion {kind}"


def run_suite(path: str, chart_dir: str) -> List[Result]:
    with open(path) as fh:
        suite = yaml.safe_load(fh) or {}
    sname = suite.get("suite", os.path.basename(path))
    base_values: Dict[str, Any] = {}
    for vf in suite.get("values") or []:
        with open(os.path.join(os.path.dirname(path), vf)) as fh:
            _merge(base_values, yaml.safe_load(fh) or {})
    _merge(base_values, _set_values(suite.get("set") or {}))
    srel = suite.get("release") or {}
    results = []
    for t in suite.get("tests") or []:
        values = copy.deepcopy(base_values)
        for vf in t.get("values") or []:
            with open(os.path.join(os.path.dirname(path), vf)) as fh:
                _merge(values, yaml.safe_load(fh) or {})
        _merge(values, _set_values(t.get("set") or {}))
        rel = dict(srel, **(t.get("release") or {}))
        templates = t.get("templates") or ([t["template"]] if t.get("template") else None) or \
            suite.get("templates") or []
        failures: List[str] = []
        try:
            rendered = render_chart(chart_dir, values, release=rel.get("name", "cron-operator"),
                                    namespace=rel.get("namespace", "default"))
        except Exception as e:  # noqa: BLE001 - a render error fails the test
            results.append(Result(sname, t.get("it", ""), False, [f"render failed: {e}"]))
            continue
        for a in t.get("asserts") or []:
            (kind, spec), = ((k, v) for k, v in a.items() if k not in ("template", "documentIndex", "not"))
            spec = dict(spec or {})
            for k in ("documentIndex", "not"):
                if k in a:
                    spec[k] = a[k]
            if "documentIndex" in t and "documentIndex" not in spec:
                spec["documentIndex"] = t["documentIndex"]
            tmpl_names = [a["template"]] if a.get("template") else templates
            docs: List[Dict[str, Any]] = []
            for tn in tmpl_names:
                key = os.path.basename(tn)
                if key not in rendered:
                    failures.append(f"template {tn} not found")
                    continue
                docs.extend(rendered[key])
            err = _assert(kind, spec, docs)
            if err:
                failures.append(err)
        results.append(Result(sname, t.get("it", ""), not failures, failures))
    return results


def run_all(chart_dir: str, suites: Optional[List[str]] = None) -> Tuple[int, int, List[Result]]:
    paths = suites or sorted(glob.glob(os.path.join(chart_dir, "tests", "*_test.yaml")))
    results: List[Result] = []
    for p in paths:
        results.extend(run_suite(p, chart_dir))
    failed = sum(1 for r in results if not r.passed)
    return len(results) - failed, failed, results


def main(argv: List[str]) -> int:
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    chart = os.path.join(root, "charts", "cron-operator")
    passed, failed, results = run_all(chart, argv or None)
    for r in results:
        mark = "PASS" if r.passed else "FAIL"
        print(f"{mark}  {r.suite} :: {r.name}")
        for f in r.failures:
            print(f"      - {f}")
    print(f"\nCharts: 1 passed, 1 total\nTest Suites/Tests: {passed} passed, {failed} failed, {passed + failed} total")
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
