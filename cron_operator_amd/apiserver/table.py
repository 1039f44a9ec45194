"""Server-side printing: ``meta.k8s.io/v1`` Table responses for ``kubectl get``.

kubectl asks the apiserver for ``Accept: application/json;as=Table;v=v1;g=meta.k8s.io``
and prints the returned columns.  For custom resources the columns are ``Name``
plus the CRD's ``additionalPrinterColumns`` -- for ``Cron`` that is SCHEDULE,
SUSPEND, LAST_SCHEDULE and AGE (``charts/cron-operator/crds/apps.kubedl.io_crons.yaml:17-29``),
the "kubectl UX" the reference promises.  This module implements what
kube-apiserver's CRD table convertor does:

* each column's ``jsonPath`` is evaluated with the kubectl JSONPath subset
  (``.a.b``, ``.a[0].b``, ``{.a.b}``); a missing value is an empty cell;
* ``date`` columns become a human age relative to *now* (``5m``, ``3h12m``,
  ``2d``: k8s ``duration.HumanDuration``); ``integer``/``number``/``boolean``
  cells keep their JSON type, arrays/objects are JSON-encoded;
* every row carries ``PartialObjectMetadata`` (``includeObject=Metadata``).

:func:`render` formats a Table the way kubectl prints it.
"""
from __future__ import annotations

import json
import re
from typing import Any, Dict, List, Optional

from ..utils.gotime import NANOS, parse_rfc3339

_SEG = re.compile(r"\.?([^.\[\]]+)|\[(\d+)\]")


def jsonpath(obj: Any, path: str) -> Any:
    """Evaluate the kubectl JSONPath subset used by printer columns; ``None`` if absent."""
    p = path.strip()
    if p.startswith("{") and p.endswith("}"):
        p = p[1:-1]
    if p in ("", "."):
        return obj
    cur = obj
    pos = 0
    while pos < len(p):
        m = _SEG.match(p, pos)
        if not m or m.end() == pos:
            return None
        pos = m.end()
        if m.group(1) is not None:
            if not isinstance(cur, dict) or m.group(1) not in cur:
                return None
            cur = cur[m.group(1)]
        else:
            i = int(m.group(2))
            if not isinstance(cur, list) or i >= len(cur):
                return None
            cur = cur[i]
    return cur


def human_duration(seconds: float) -> str:
    """k8s ``apimachinery/pkg/util/duration.HumanDuration``."""
    s = int(seconds)
    if s < -1:
        return "<invalid>"
    if s < 0:
        return "0s"
    if s < 60 * 2:
        return f"{s}s"
    m = s // 60
    if m < 10:
        rs = s % 60
        return f"{m}m{rs}s" if rs else f"{m}m"
    if m < 60 * 3:
        return f"{m}m"
    h = s // 3600
    if h < 8:
        rm = (s // 60) % 60
        return f"{h}h{rm}m" if rm else f"{h}h"
    if h < 48:
        return f"{h}h"
    if h < 24 * 8:
        rh = h % 24
        return f"{h // 24}d{rh}h" if rh else f"{h // 24}d"
    if h < 24 * 365 * 2:
        return f"{h // 24}d"
    if h < 24 * 365 * 8:
        dy = (h // 24) % 365
        return f"{h // 24 // 365}y{dy}d" if dy else f"{h // 24 // 365}y"
    return f"{h // 24 // 365}y"


def _cell(v: Any, col_type: str, now_ns: int) -> Any:
    if v is None:
        return None
    if col_type == "date":
        try:
            t = parse_rfc3339(str(v))
        except ValueError:
            return str(v)
        return human_duration((now_ns - t.unix_nano()) / NANOS)
    if col_type in ("integer", "number", "boolean"):
        return v
    if isinstance(v, (dict, list)):
        return json.dumps(v, separators=(",", ":"))
    return v if isinstance(v, str) else str(v)


def columns_for(printer_columns: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    cols = [{"name": "Name", "type": "string", "format": "name",
             "description": "Name must be unique within a namespace.", "priority": 0}]
    for c in printer_columns:
        cols.append({"name": c.get("name", ""), "type": c.get("type", "string"), "format": c.get("format", ""),
                     "description": c.get("description", ""), "priority": int(c.get("priority") or 0)})
    return cols


def to_table(printer_columns: List[Dict[str, Any]], objects: List[Dict[str, Any]], now_ns: int,
             resource_version: str = "", include_object: str = "Metadata") -> Dict[str, Any]:
    if not printer_columns:  # built-in kinds without a convertor: kube-apiserver's default columns
        printer_columns = [{"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"}]
    rows = []
    for o in objects:
        cells: List[Any] = [(o.get("metadata") or {}).get("name", "")]
        for c in printer_columns:
            cells.append(_cell(jsonpath(o, c.get("jsonPath", "")), c.get("type", "string"), now_ns))
        row: Dict[str, Any] = {"cells": cells}
        if include_object == "Object":
            row["object"] = o
        elif include_object != "None":
            row["object"] = {"kind": "PartialObjectMetadata", "apiVersion": "meta.k8s.io/v1",
                             "metadata": o.get("metadata") or {}}
        rows.append(row)
    return {"kind": "Table", "apiVersion": "meta.k8s.io/v1", "metadata": {"resourceVersion": resource_version},
            "columnDefinitions": columns_for(printer_columns), "rows": rows}


def wants_table(accept: str) -> bool:
    """``Accept: application/json;as=Table;v=v1;g=meta.k8s.io[, application/json]``."""
    for part in accept.split(","):
        params = {k.strip(): v.strip() for k, _, v in (x.partition("=") for x in part.split(";")[1:])}
        if params.get("as") == "Table" and params.get("g", "meta.k8s.io") == "meta.k8s.io":
            return True
    return False


def render(table: Dict[str, Any], wide: bool = False, namespace_column: bool = False,
           no_headers: bool = False) -> str:
    """kubectl's human-readable printer: upper-case headers, 3-space gaps, ``<none>`` for empty."""
    cols = [(i, c) for i, c in enumerate(table.get("columnDefinitions") or []) if wide or not c.get("priority")]
    header = [c["name"].upper() for _, c in cols]
    lines: List[List[str]] = []
    for row in table.get("rows") or []:
        cells = row.get("cells") or []
        out = []
        for i, _ in cols:
            v = cells[i] if i < len(cells) else None
            if v is None or v == "":
                out.append("<none>")
            elif isinstance(v, bool):
                out.append("true" if v else "false")
            else:
                out.append(str(v))
        if namespace_column:
            ns = (((row.get("object") or {}).get("metadata")) or {}).get("namespace", "")
            out.insert(0, ns)
        lines.append(out)
    if namespace_column:
        header.insert(0, "NAMESPACE")
    grid = ([header] if not no_headers else []) + lines
    if not grid:
        return ""
    widths = [max(len(r[i]) for r in grid) for i in range(len(grid[0]))]
    text = []
    for r in grid:
        text.append("   ".join(v.ljust(widths[i]) for i, v in enumerate(r)).rstrip())
    return "\n".join(text) + "\n"


def printer_columns_of(resource_info: Any) -> Optional[List[Dict[str, Any]]]:
    return list(getattr(resource_info, "printer_columns", None) or [])
