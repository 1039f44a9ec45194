"""A Go ``text/template`` + Sprig subset, enough to render Helm charts in tests.

The reference unit-tests its chart with helm-unittest (``charts/cron-operator/tests/*.yaml``,
``Makefile:158-160``).  Neither helm nor Go exists in this image, so the chart's
templates are rendered by this interpreter and the rendered manifests are
asserted on (``tests/test_helm_chart.py``).  Supported:

* actions with trim markers (``{{-``/``-}}``) and comments (``{{/* */}}``);
* ``if/else if/else``, ``with/else``, ``range`` (lists and maps, ``$i, $v :=``),
  ``define``/``include``/``template``, variables (``$x :=`` / ``$x =``, ``$``);
* pipelines ``a | f b``, parenthesised sub-expressions, field chains
  (``.Values.image.tag``, ``$.Release.Name``), string/number/bool/nil literals;
* functions: default, empty, coalesce, ternary, quote, squote, printf, print,
  trunc, trimSuffix, trimPrefix, trim, lower, upper, title, replace, contains,
  hasPrefix, hasSuffix, toYaml, toJson, indent, nindent, list, dict, get, set,
  hasKey, keys, merge, mergeOverwrite, deepCopy, concat, append, len, eq, ne,
  lt, le, gt, ge, and, or, not, required, fail, b64enc, int, toString, join,
  semverCompare (>=, <=, = only), tpl.

Semantics follow Go where it matters for charts: truthiness (empty
string/map/list, 0, nil and false are false), ``and``/``or`` returning operands,
``printf`` with Go verbs (%s %d %v %q), and ``toYaml`` producing block YAML.
"""
from __future__ import annotations

import base64
import copy
import json
import re
from collections import ChainMap
from typing import Any, Callable, Dict, List, Optional, Tuple

import yaml


class TemplateError(Exception):
    pass


# --------------------------------------------------------------------------- lexing


# an action ends at the first "}}" outside a string literal ({{ "}}" }} prints "}}", as in Go)
_ACTION = re.compile(r"\{\{(-\s)?((?:\"(?:[^\"\\]|\\.)*\"|`[^`]*`|.)*?)(\s-)?\}\}", re.S)


def _split(src: str) -> List[Tuple[str, str]]:
    """-> [("text", s) | ("action", body)] with trim markers applied."""
    out: List[Tuple[str, str]] = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip(" \t\r\n")
        out.append(("text", text))
        body = m.group(2).strip()
        out.append(("action", body))
        pos = m.end()
        if m.group(3):
            rest = src[pos:]
            stripped = rest.lstrip(" \t\r\n")
            pos += len(rest) - len(stripped)
    out.append(("text", src[pos:]))
    return out


_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<str>"(?:[^"\\]|\\.)*"|`[^`]*`)
  | (?P<char>'(?:[^'\\]|\\.)')
  | (?P<num>-?\d+(?:\.\d+)?)
  | (?P<decl>:=)
  | (?P<assign>=)
  | (?P<pipe>\|)
  | (?P<lp>\()
  | (?P<rp>\))
  | (?P<comma>,)
  | (?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)
  | (?P<field>(?:\.[A-Za-z0-9_]+)+|\.)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)
""", re.X)


def _tokens(s: str) -> List[Tuple[str, str]]:
    out = []
    pos = 0
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise TemplateError(f"unexpected character in action: {s[pos:]!r}")
        kind = m.lastgroup
        if kind != "ws":
            out.append((kind, m.group(kind)))
        pos = m.end()
    return out


# --------------------------------------------------------------------------- AST


class Node:
    pass


class Text(Node):
    def __init__(self, s: str):
        self.s = s


class Action(Node):
    def __init__(self, pipe):
        self.pipe = pipe


class If(Node):
    def __init__(self, branches, else_body):
        self.branches = branches  # [(pipe, body)]
        self.else_body = else_body


class With(Node):
    def __init__(self, pipe, body, else_body):
        self.pipe, self.body, self.else_body = pipe, body, else_body


class Range(Node):
    def __init__(self, pipe, body, else_body, vars_):
        self.pipe, self.body, self.else_body, self.vars = pipe, body, else_body, vars_


class TemplateCall(Node):
    def __init__(self, name, pipe):
        self.name, self.pipe = name, pipe


def _parse_pipe(toks: List[Tuple[str, str]]):
    """A pipeline: optional variable declaration, then commands separated by ``|``."""
    decl = None
    if len(toks) >= 2 and toks[0][0] == "var" and toks[1][0] in ("decl", "assign"):
        decl = (toks[0][1], toks[1][0])
        toks = toks[2:]
    elif len(toks) >= 4 and toks[0][0] == "var" and toks[1][0] == "comma" and toks[2][0] == "var" and \
            toks[3][0] == "decl":
        decl = ((toks[0][1], toks[2][1]), "decl2")
        toks = toks[4:]
    cmds: List[List[Any]] = [[]]
    i = 0
    while i < len(toks):
        k, v = toks[i]
        if k == "pipe":
            cmds.append([])
            i += 1
            continue
        if k == "lp":
            depth = 1
            j = i + 1
            while j < len(toks) and depth:
                if toks[j][0] == "lp":
                    depth += 1
                elif toks[j][0] == "rp":
                    depth -= 1
                j += 1
            cmds[-1].append(("sub", _parse_pipe(toks[i + 1:j - 1])))
            i = j
            # allow (.x).field chains
            if i < len(toks) and toks[i][0] == "field" and toks[i][1] != ".":
                cmds[-1][-1] = ("subfield", cmds[-1][-1][1], toks[i][1])
                i += 1
            continue
        cmds[-1].append((k, v))
        i += 1
    return (decl, cmds)


def _parse(src: str, defines: Dict[str, List[Node]]) -> List[Node]:
    parts = _split(src)
    pos = 0

    def block(stop: Tuple[str, ...]):
        nonlocal pos
        nodes: List[Node] = []
        while pos < len(parts):
            kind, body = parts[pos]
            pos += 1
            if kind == "text":
                if body:
                    nodes.append(Text(body))
                continue
            if body.startswith("/*"):
                continue
            word = body.split(None, 1)[0] if body else ""
            rest = body[len(word):].strip()
            if word in stop:
                return nodes, word, rest
            if word == "if":
                branches = []
                else_body = None
                cond = rest
                while True:
                    sub, w, r = block(("else", "end"))
                    branches.append((_parse_pipe(_tokens(cond)), sub))
                    if w == "end":
                        break
                    if r.startswith("if "):
                        cond = r[3:].strip()
                        continue
                    else_body, w2, _ = block(("end",))
                    break
                nodes.append(If(branches, else_body))
            elif word == "with":
                sub, w, r = block(("else", "end"))
                else_body = None
                if w == "else":
                    else_body, _, _ = block(("end",))
                nodes.append(With(_parse_pipe(_tokens(rest)), sub, else_body))
            elif word == "range":
                toks = _tokens(rest)
                vars_ = None
                if len(toks) >= 4 and toks[0][0] == "var" and toks[1][0] == "comma" and toks[3][0] == "decl":
                    vars_ = (toks[0][1], toks[2][1])
                    toks = toks[4:]
                elif len(toks) >= 2 and toks[0][0] == "var" and toks[1][0] == "decl":
                    vars_ = (None, toks[0][1])
                    toks = toks[2:]
                sub, w, r = block(("else", "end"))
                else_body = None
                if w == "else":
                    else_body, _, _ = block(("end",))
                nodes.append(Range(_parse_pipe(toks), sub, else_body, vars_))
            elif word == "define":
                name = json.loads(rest)
                sub, _, _ = block(("end",))
                defines[name] = sub
            elif word == "template":
                toks = _tokens(rest)
                name = json.loads(toks[0][1])
                nodes.append(TemplateCall(name, _parse_pipe(toks[1:]) if len(toks) > 1 else None))
            elif word in ("end", "else"):
                raise TemplateError(f"unexpected {{{{{word}}}}}")
            else:
                nodes.append(Action(_parse_pipe(_tokens(body))))
        if stop:
            raise TemplateError(f"missing {{{{end}}}} (expected one of {stop})")
        return nodes, None, ""

    nodes, _, _ = block(())
    return nodes


# --------------------------------------------------------------------------- values / helpers


def truthy(v: Any) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return True


def _go_str(v: Any) -> str:
    if v is None:
        return "<no value>"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{_go_str(x)}" for k, x in sorted(v.items())) + "]"
    if isinstance(v, list):
        return "[" + " ".join(_go_str(x) for x in v) + "]"
    return str(v)


def _printf(fmt: str, *args: Any) -> str:
    out = []
    i = 0
    ai = 0
    while i < len(fmt):
        c = fmt[i]
        if c == "%" and i + 1 < len(fmt):
            verb = fmt[i + 1]
            i += 2
            if verb == "%":
                out.append("%")
                continue
            a = args[ai] if ai < len(args) else None
            ai += 1
            if verb in ("s", "v"):
                out.append(_go_str(a))
            elif verb == "d":
                out.append(str(int(a)))
            elif verb == "q":
                out.append(json.dumps(_go_str(a)))
            else:
                out.append(_go_str(a))
            continue
        out.append(c)
        i += 1
    return "".join(out)


def to_yaml(v: Any) -> str:
    if v is None:
        return "null"
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=True).rstrip("\n")


def _indent(n: int, s: str) -> str:
    pad = " " * int(n)
    return "\n".join(pad + line for line in str(s).split("\n"))


def _merge(dst: Dict[str, Any], *srcs: Dict[str, Any], overwrite: bool) -> Dict[str, Any]:
    for src in srcs:
        for k, v in (src or {}).items():
            if k in dst and isinstance(dst[k], dict) and isinstance(v, dict):
                _merge(dst[k], v, overwrite=overwrite)
            elif k not in dst or overwrite:
                dst[k] = copy.deepcopy(v)
    return dst


def _cmp(a: Any, b: Any) -> int:
    return (a > b) - (a < b)


def _semver_compare(constraint: str, version: str) -> bool:
    def parse(v: str):
        v = v.lstrip("v").split("-")[0].split("+")[0]
        return tuple(int(x) for x in (v.split(".") + ["0", "0"])[:3])
    m = re.match(r"^\s*(>=|<=|=|>|<)?\s*(.+)$", constraint)
    op, ver = (m.group(1) or "="), m.group(2)
    a, b = parse(version), parse(ver)
    return {">=": a >= b, "<=": a <= b, "=": a == b, ">": a > b, "<": a < b}[op]


# --------------------------------------------------------------------------- engine


class Engine:
    def __init__(self):
        self.defines: Dict[str, List[Node]] = {}
        self.funcs: Dict[str, Callable[..., Any]] = {
            "default": lambda d, v=None: v if truthy(v) else d,
            "empty": lambda v: not truthy(v),
            "coalesce": lambda *a: next((x for x in a if truthy(x)), None),
            "ternary": lambda a, b, c: a if truthy(c) else b,
            "quote": lambda *a: " ".join(json.dumps(_go_str(x) if x is not None else "") for x in a),
            "squote": lambda *a: " ".join(f"'{_go_str(x)}'" for x in a),
            "printf": _printf,
            "print": lambda *a: "".join(_go_str(x) for x in a),
            "trunc": lambda n, s: s[:int(n)] if int(n) >= 0 else s[int(n):],
            "trimSuffix": lambda suf, s: s[:-len(suf)] if suf and s.endswith(suf) else s,
            "trimPrefix": lambda pre, s: s[len(pre):] if pre and s.startswith(pre) else s,
            "trim": lambda s: str(s).strip(),
            "lower": lambda s: str(s).lower(),
            "upper": lambda s: str(s).upper(),
            "title": lambda s: str(s).title(),
            "replace": lambda old, new, s: str(s).replace(old, new),
            "contains": lambda sub, s: sub in str(s),
            "hasPrefix": lambda p, s: str(s).startswith(p),
            "hasSuffix": lambda p, s: str(s).endswith(p),
            "toYaml": to_yaml,
            "toJson": lambda v: json.dumps(v, separators=(",", ":")),
            "indent": _indent,
            "nindent": lambda n, s: "\n" + _indent(n, s),
            "list": lambda *a: list(a),
            "dict": lambda *a: {a[i]: a[i + 1] for i in range(0, len(a) - 1, 2)},
            "get": lambda d, k: (d or {}).get(k, ""),
            "set": lambda d, k, v: (d.__setitem__(k, v), d)[1],
            "hasKey": lambda d, k: k in (d or {}),
            "keys": lambda *ds: sorted(k for d in ds for k in (d or {})),
            "merge": lambda d, *s: _merge(d, *s, overwrite=False),
            "mergeOverwrite": lambda d, *s: _merge(d, *s, overwrite=True),
            "deepCopy": lambda v: copy.deepcopy(v),
            "concat": lambda *ls: [x for lst in ls for x in (lst or [])],
            "append": lambda lst, v: list(lst or []) + [v],
            "len": lambda v: len(v or []),
            "eq": lambda a, *bs: any(a == b for b in bs),
            "ne": lambda a, b: a != b,
            "lt": lambda a, b: _cmp(a, b) < 0,
            "le": lambda a, b: _cmp(a, b) <= 0,
            "gt": lambda a, b: _cmp(a, b) > 0,
            "ge": lambda a, b: _cmp(a, b) >= 0,
            "not": lambda v: not truthy(v),
            "required": self._required,
            "fail": self._fail,
            "b64enc": lambda s: base64.b64encode(str(s).encode()).decode(),
            "int": lambda v: int(float(v)) if v not in (None, "") else 0,
            "toString": _go_str,
            "join": lambda sep, lst: sep.join(_go_str(x) for x in (lst or [])),
            "semverCompare": _semver_compare,
        }

    @staticmethod
    def _required(msg: str, v: Any) -> Any:
        if v is None or v == "":
            raise TemplateError(msg)
        return v

    @staticmethod
    def _fail(msg: str) -> Any:
        raise TemplateError(msg)

    def add_template(self, src: str) -> List[Node]:
        return _parse(src, self.defines)

    # -- evaluation
    def _field(self, base: Any, path: str) -> Any:
        cur = base
        for part in [p for p in path.split(".") if p]:
            if isinstance(cur, dict):
                cur = cur.get(part)
            else:
                cur = getattr(cur, part, None)
            if cur is None:
                return None
        return cur

    def _arg(self, tok, dot, scope):
        k, v = tok[0], tok[1]  # ("subfield", pipe, field) carries a third element
        if k == "str":
            return json.loads(v) if v.startswith('"') else v[1:-1]
        if k == "char":
            return ord(json.loads('"' + v[1:-1] + '"'))
        if k == "num":
            return float(v) if "." in v else int(v)
        if k == "field":
            return dot if v == "." else self._field(dot, v)
        if k == "var":
            name, _, rest = v.partition(".")
            if name not in scope:
                raise TemplateError(f"undefined variable {name}")
            base = scope[name]
            return self._field(base, rest) if rest else base
        if k == "ident":
            if v in ("true", "false"):
                return v == "true"
            if v == "nil":
                return None
            if v in self.funcs or v in ("include", "tpl"):
                return self._call(v, [], dot, scope)
            raise TemplateError(f'function "{v}" not defined')
        if k == "sub":
            return self._pipe(v, dot, scope)
        if k == "subfield":
            return self._field(self._pipe(v, dot, scope), tok[2])
        raise TemplateError(f"bad token {tok}")

    def _call(self, name: str, args: List[Any], dot, scope):
        if name == "include":
            return self.render_define(args[0], args[1] if len(args) > 1 else None)
        if name == "tpl":
            nodes = _parse(args[0], self.defines)
            return self._exec(nodes, args[1], ChainMap({"$": args[1]}))
        if name == "and":
            r = None
            for a in args:
                r = a
                if not truthy(a):
                    return a
            return r
        if name == "or":
            r = None
            for a in args:
                r = a
                if truthy(a):
                    return a
            return r
        fn = self.funcs.get(name)
        if fn is None:
            raise TemplateError(f'function "{name}" not defined')
        return fn(*args)

    def _command(self, cmd, dot, scope, piped=False, pv=None):
        if not cmd:
            raise TemplateError("empty command")
        head = cmd[0]
        if head[0] == "ident" and head[1] not in ("true", "false", "nil"):
            args = [self._arg(t, dot, scope) for t in cmd[1:]]
            if piped:
                args.append(pv)
            return self._call(head[1], args, dot, scope)
        if len(cmd) > 1 or piped:
            raise TemplateError(f"can't give argument to non-function {head}")
        return self._arg(head, dot, scope)

    def _pipe(self, pipe, dot, scope):
        decl, cmds = pipe
        val = None
        for i, cmd in enumerate(cmds):
            val = self._command(cmd, dot, scope, piped=i > 0, pv=val)
        if decl is not None:
            names, kind = decl
            if kind == "decl2":
                raise TemplateError("two-variable declaration outside range")
            if kind == "assign":
                for m in scope.maps:  # assignment updates the nearest enclosing declaration
                    if names in m:
                        m[names] = val
                        break
                else:
                    raise TemplateError(f"undefined variable {names}")
            else:
                scope.maps[0][names] = val
            return None  # declarations print nothing
        return val

    def _exec(self, nodes: List[Node], dot, scope) -> str:
        out: List[str] = []
        for n in nodes:
            if isinstance(n, Text):
                out.append(n.s)
            elif isinstance(n, Action):
                decl = n.pipe[0]
                v = self._pipe(n.pipe, dot, scope)
                if decl is None:
                    out.append(_go_str(v))  # nil prints "<no value>", stripped like Helm does
            elif isinstance(n, If):
                for pipe, body in n.branches:
                    if truthy(self._pipe(pipe, dot, scope)):
                        out.append(self._exec(body, dot, scope.new_child()))
                        break
                else:
                    if n.else_body is not None:
                        out.append(self._exec(n.else_body, dot, scope.new_child()))
            elif isinstance(n, With):
                v = self._pipe(n.pipe, dot, scope)
                if truthy(v):
                    out.append(self._exec(n.body, v, scope.new_child()))
                elif n.else_body is not None:
                    out.append(self._exec(n.else_body, dot, scope.new_child()))
            elif isinstance(n, Range):
                v = self._pipe(n.pipe, dot, scope)
                items: List[Tuple[Any, Any]]
                if isinstance(v, dict):
                    items = sorted(v.items())
                elif isinstance(v, (list, tuple)):
                    items = list(enumerate(v))
                elif isinstance(v, int) and not isinstance(v, bool):
                    items = list(enumerate(range(v)))
                else:
                    items = []
                if not items:
                    if n.else_body is not None:
                        out.append(self._exec(n.else_body, dot, scope.new_child()))
                    continue
                for k, item in items:
                    sc = scope.new_child()
                    if n.vars:
                        if n.vars[0]:
                            sc[n.vars[0]] = k
                        sc[n.vars[1]] = item
                    out.append(self._exec(n.body, item, sc))
            elif isinstance(n, TemplateCall):
                arg = self._pipe(n.pipe, dot, scope) if n.pipe is not None else None
                out.append(self.render_define(n.name, arg))
        return "".join(out)

    def render_define(self, name: str, dot: Any) -> str:
        if name not in self.defines:
            raise TemplateError(f'no template "{name}" associated with template')
        return self._exec(self.defines[name], dot, ChainMap({"$": dot}))

    def render(self, nodes: List[Node], dot: Any) -> str:
        return self._exec(nodes, dot, ChainMap({"$": dot}))


def _no_value_cleanup(s: str) -> str:
    return s.replace("<no value>", "")


def render_chart(chart_dir: str, values_override: Optional[Dict[str, Any]] = None, release: str = "cron-operator",
                 namespace: str = "cron-operator", only: Optional[str] = None) -> Dict[str, List[Dict[str, Any]]]:
    """Render every template of a chart; returns ``{template_file: [documents]}``."""
    import os

    with open(os.path.join(chart_dir, "Chart.yaml")) as fh:
        chart = yaml.safe_load(fh)
    with open(os.path.join(chart_dir, "values.yaml")) as fh:
        values = yaml.safe_load(fh) or {}
    _merge(values, values_override or {}, overwrite=True)
    ctx = {
        "Values": values,
        "Chart": {"Name": chart.get("name"), "Version": chart.get("version"), "AppVersion": chart.get("appVersion")},
        "Release": {"Name": release, "Namespace": namespace, "Service": "Helm", "IsInstall": True,
                    "IsUpgrade": False, "Revision": 1},
        "Capabilities": {"KubeVersion": {"Version": "v1.34.0", "Major": "1", "Minor": "34"}},
    }
    eng = Engine()
    tdir = os.path.join(chart_dir, "templates")
    files = sorted(os.listdir(tdir))
    parsed = {}
    for f in files:  # helpers first so defines exist
        with open(os.path.join(tdir, f)) as fh:
            parsed[f] = eng.add_template(fh.read())
    out: Dict[str, List[Dict[str, Any]]] = {}
    for f in files:
        if f.startswith("_") or not f.endswith((".yaml", ".yml")):
            continue
        if only and f != only:
            continue
        ctx["Template"] = {"Name": f"{chart.get('name')}/templates/{f}", "BasePath": f"{chart.get('name')}/templates"}
        text = _no_value_cleanup(eng.render(parsed[f], ctx))
        docs = [d for d in yaml.safe_load_all(text) if d]
        out[f] = docs
    return out
