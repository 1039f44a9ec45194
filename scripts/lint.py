#!/usr/bin/env python3
"""Stdlib-only lint (``make lint``; ``--fix`` for ``make fmt``).

The reference lints with golangci-lint (``.golangci.yml:1-52``) and gofmt
(``.github/workflows/integration.yaml:25-45``).  ruff/flake8 are not in the
build image, so this checks the rules that matter for this codebase with
``ast`` + text scanning:

* F401 unused import (names imported but never referenced; ``__init__`` re-exports,
  ``__all__`` members and ``# noqa`` lines are exempt),
* F811-ish duplicate top-level function/class definitions,
* E501 line longer than 120 columns,
* W291/W293 trailing whitespace, W292 missing final newline, tabs in indentation,
* B006 mutable default arguments,
* D001 (documentation evidence): in ``docs/*.md``, ``README.md`` and ``BASELINE.md`` every
  paragraph, list item or table row that states a *measured* figure (throughput in
  cron-reconciles/s or fires/s, latency as p50/p99, operator CPU per fire, RSS in MiB/KiB,
  busy fractions) cites its evidence -- a ``profiles/...`` file, a driver record
  (``BENCH_rNN.json`` etc.) or a test/script that produces it (a table row may rely on the
  paragraph that introduces its table) -- and every ``profiles/...``
  path the docs name exists.  ``profiles/`` itself holds at most ``MAX_PROFILES`` files,
  each cited somewhere in the docs (D002).
"""
from __future__ import annotations

import ast
import os
import re
import sys
from typing import List, Set, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIRS = ["cron_operator_amd", "tests", "scripts"]
FILES = ["bench.py", "__graft_entry__.py"]
MAX_LINE = 120
DOCS = ["README.md", "BASELINE.md"]
MAX_PROFILES = 30


def py_files() -> List[str]:
    out = [os.path.join(ROOT, f) for f in FILES]
    for d in DIRS:
        for dp, dns, fns in os.walk(os.path.join(ROOT, d)):
            dns[:] = [x for x in dns if x != "__pycache__"]
            out.extend(os.path.join(dp, f) for f in fns if f.endswith(".py"))
    return sorted(out)


class _Names(ast.NodeVisitor):
    def __init__(self) -> None:
        self.used: Set[str] = set()

    def visit_Name(self, node: ast.Name) -> None:
        self.used.add(node.id)

    def visit_Attribute(self, node: ast.Attribute) -> None:
        root = node
        while isinstance(root, ast.Attribute):
            root = root.value
        if isinstance(root, ast.Name):
            self.used.add(root.id)
        self.generic_visit(node)


def _string_names(tree: ast.AST) -> Set[str]:
    """Names referenced from string annotations / __all__."""
    out: Set[str] = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str) and node.value.isidentifier():
            out.add(node.value)
        elif isinstance(node, ast.Constant) and isinstance(node.value, str) and len(node.value) < 200:
            for tok in node.value.replace("[", " ").replace("]", " ").replace(",", " ").replace(".", " ").split():
                if tok.isidentifier():
                    out.add(tok)
    return out


def check_file(path: str) -> List[Tuple[int, str, str]]:
    errs: List[Tuple[int, str, str]] = []
    with open(path, encoding="utf-8") as fh:
        text = fh.read()
    lines = text.split("\n")
    for i, line in enumerate(lines, 1):
        if len(line) > MAX_LINE and "http" not in line:
            errs.append((i, "E501", f"line too long ({len(line)} > {MAX_LINE})"))
        if line.rstrip() != line:
            errs.append((i, "W291", "trailing whitespace"))
        if line[: len(line) - len(line.lstrip())].count("\t"):
            errs.append((i, "W191", "tab in indentation"))
    if text and not text.endswith("\n"):
        errs.append((len(lines), "W292", "no newline at end of file"))
    try:
        tree = ast.parse(text, path)
    except SyntaxError as e:
        return errs + [(e.lineno or 0, "E999", f"syntax error: {e.msg}")]

    is_init = os.path.basename(path) == "__init__.py"
    imported: List[Tuple[str, int]] = []
    for node in tree.body:
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            for a in node.names:
                name = (a.asname or a.name).split(".")[0]
                imported.append((name, node.lineno))
    # function-level imports too
    for node in ast.walk(tree):
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)):
            for sub in ast.walk(node):
                if isinstance(sub, (ast.Import, ast.ImportFrom)):
                    for a in sub.names:
                        imported.append(((a.asname or a.name).split(".")[0], sub.lineno))
    v = _Names()
    v.visit(tree)
    used = v.used | _string_names(tree)
    if not is_init:
        for name, ln in imported:
            if name == "*" or name in used:
                continue
            if "noqa" in lines[ln - 1]:
                continue
            errs.append((ln, "F401", f"'{name}' imported but unused"))

    seen = {}
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            if node.name in seen and not any(isinstance(d, ast.Name) and d.id == "overload"
                                             for d in getattr(node, "decorator_list", [])):
                errs.append((node.lineno, "F811", f"redefinition of '{node.name}' from line {seen[node.name]}"))
            seen[node.name] = node.lineno
    for node in ast.walk(tree):
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)):
            for d in node.args.defaults + [x for x in node.args.kw_defaults if x is not None]:
                if isinstance(d, (ast.List, ast.Dict, ast.Set)):
                    errs.append((node.lineno, "B006", f"mutable default argument in '{node.name}'"))
    return errs


def fix_file(path: str) -> bool:
    with open(path, encoding="utf-8") as fh:
        text = fh.read()
    new = "\n".join(line.rstrip() for line in text.split("\n")).rstrip("\n") + "\n"
    if new != text:
        with open(path, "w", encoding="utf-8") as fh:
            fh.write(new)
        return True
    return False


# a measured figure: a number with a measurement unit, or a p50/p99 value
_MEASURE = re.compile(r"\d[\d,.]*\s*(?:cron-reconciles/s|fires/s|MiB\b|KiB\b|ms (?:of )?(?:operator )?CPU)"
                      r"|\bp(?:50|99)\b[^|]{0,20}?\d[\d,.]*\s*m?s\b|\b\d\.\d+ busy|busy \d\.\d+")
_EVIDENCE = re.compile(r"profiles/[\w.\-/*]+|\b(?:BENCH|SCALE|GPUTEST|MULTICHIP)_r\d+\.json|tests/test_\w+\.py"
                       r"|scripts/\w+\.py|test_\w+")
_PROFILE_REF = re.compile(r"profiles/[\w.\-]+")


def doc_files() -> List[str]:
    out = [os.path.join(ROOT, f) for f in DOCS]
    d = os.path.join(ROOT, "docs")
    out.extend(os.path.join(d, f) for f in sorted(os.listdir(d)) if f.endswith(".md"))
    return out


def _blocks(text: str) -> List[Tuple[int, str]]:
    """(first line number, text) of each paragraph, list item and table row."""
    out: List[Tuple[int, str]] = []
    cur: List[str] = []
    start = 0
    in_code = False
    for i, line in enumerate(text.splitlines(), 1):
        if line.startswith("```"):
            in_code = not in_code
            continue
        if in_code:
            continue
        s = line.strip()
        new_item = s.startswith(("|", "* ", "- ", "#")) or re.match(r"\d+\. ", s) is not None
        if not s or new_item:
            if cur:
                out.append((start, " ".join(cur)))
            cur = []
        if s:
            if not cur:
                start = i
            cur.append(s)
            if s.startswith(("|", "#")):
                out.append((start, " ".join(cur)))
                cur = []
    if cur:
        out.append((start, " ".join(cur)))
    return out


def check_docs() -> List[Tuple[str, int, str, str]]:
    problems: List[Tuple[str, int, str, str]] = []
    cited: Set[str] = set()
    for path in doc_files():
        with open(path, encoding="utf-8") as fh:
            text = fh.read()
        rel = os.path.relpath(path, ROOT)
        caption = False  # the paragraph introducing the current table cites evidence
        for ln, block in _blocks(text):
            for ref in _PROFILE_REF.findall(block):
                ref = ref.rstrip(".")
                cited.add(ref)
                if not os.path.exists(os.path.join(ROOT, ref)):
                    problems.append((rel, ln, "D001", f"cites missing {ref}"))
            has = _EVIDENCE.search(block) is not None
            row = block.startswith("|")
            if not row and not block.startswith("#"):
                caption = has
            if _MEASURE.search(block) and not has and not (row and caption):
                problems.append((rel, ln, "D001", f"measured figure without evidence: {block[:90]!r}"))
    problems.extend(check_current_tables())
    pdir = os.path.join(ROOT, "profiles")
    files = sorted(f for f in os.listdir(pdir) if not f.startswith("."))
    if len(files) > MAX_PROFILES:
        problems.append(("profiles", 0, "D002", f"{len(files)} files (at most {MAX_PROFILES})"))
    for f in files:
        if f"profiles/{f}" not in cited:
            problems.append(("profiles", 0, "D002", f"{f} is not cited by any doc"))
    return problems


def latest_driver_record() -> str:
    """``BENCH_rNN.json`` of the latest round the driver has recorded ("" if none)."""
    rounds = [int(m.group(1)) for f in os.listdir(ROOT) for m in [re.match(r"BENCH_r(\d+)\.json$", f)] if m]
    return f"BENCH_r{max(rounds):02d}.json" if rounds else ""


def check_current_tables() -> List[Tuple[str, int, str, str]]:
    """D003: a section headed "Current ..." must rest on the latest driver record -- cite
    ``BENCH_r<latest>.json`` -- so a "current" table cannot outlive the run that superseded it."""
    latest = latest_driver_record()
    if not latest:
        return []
    out: List[Tuple[str, int, str, str]] = []
    for path in doc_files():
        with open(path, encoding="utf-8") as fh:
            lines = fh.read().splitlines()
        rel = os.path.relpath(path, ROOT)
        for i, line in enumerate(lines):
            m = re.match(r"(#+)\s+(.*)", line)
            if not m or not re.search(r"\bcurrent\b", m.group(2), re.I):
                continue
            level = len(m.group(1))
            body = []
            for nxt in lines[i + 1:]:
                h = re.match(r"(#+)\s", nxt)
                if h and len(h.group(1)) <= level:
                    break
                body.append(nxt)
            if latest not in "\n".join(body):
                out.append((rel, i + 1, "D003", f"'{m.group(2)}' does not cite the latest driver record {latest}"))
    return out


def main(argv: List[str]) -> int:
    files = py_files()
    if "--fix" in argv:
        changed = [f for f in files if fix_file(f)]
        for f in changed:
            print(f"fixed {os.path.relpath(f, ROOT)}")
        return 0
    n = 0
    for f in files:
        for ln, code, msg in check_file(f):
            print(f"{os.path.relpath(f, ROOT)}:{ln}: {code} {msg}")
            n += 1
    for rel, ln, code, msg in check_docs():
        print(f"{rel}:{ln}: {code} {msg}")
        n += 1
    if n:
        print(f"{n} problem(s)")
        return 1
    print(f"lint ok ({len(files)} files, {len(doc_files())} docs)")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
