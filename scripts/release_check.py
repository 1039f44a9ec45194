#!/usr/bin/env python3
"""Release guards, run by ``.github/workflows/release.yaml`` before anything is tagged.

Mirrors the reference release workflow's checks
(``/root/reference/.github/workflows/release.yaml:30-63``):

1. ``VERSION`` is semver with a leading ``v`` (``v1.2.3``, optionally ``-rc.1``);
2. the chart's ``version`` **and** ``appVersion`` equal it without the ``v``;
3. the Python package's ``__version__`` equals it too (this repo ships a package);
4. the tag does not exist yet -- a release is never re-cut over an existing tag.

Prints ``VERSION=<v>`` and ``RAW_VERSION=<v without v>`` lines on success (append them to
``$GITHUB_ENV`` / ``$GITHUB_OUTPUT``); exits 1 with one ``Error:`` line per failed check.
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
from typing import List, Optional

SEMVER = re.compile(r"^v(0|[1-9]\d*)\.(0|[1-9]\d*)\.(0|[1-9]\d*)(-[0-9A-Za-z.-]+)?(\+[0-9A-Za-z.-]+)?$")


def _field(text: str, key: str) -> Optional[str]:
    m = re.search(rf"^{re.escape(key)}:\s*['\"]?([^'\"\s#]+)", text, re.M)
    return m.group(1) if m else None


def tag_exists(root: str, tag: str) -> bool:
    r = subprocess.run(["git", "-C", root, "rev-parse", "-q", "--verify", f"refs/tags/{tag}"],
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return r.returncode == 0


def check(root: str, check_tag: bool = True) -> List[str]:
    errs: List[str] = []
    try:
        version = open(os.path.join(root, "VERSION")).read().strip()
    except OSError as e:
        return [f"Error: cannot read VERSION: {e}"]
    if not SEMVER.match(version):
        return [f"Error: Version '{version}' does not match semver pattern (e.g. v1.2.3)."]
    raw = version[1:]
    chart = open(os.path.join(root, "charts", "cron-operator", "Chart.yaml")).read()
    for key, label in (("version", "Chart version"), ("appVersion", "Chart appVersion")):
        got = _field(chart, key)
        if got != raw:
            errs.append(f"Error: {label} '{got}' does not match VERSION '{raw}'.")
    init = open(os.path.join(root, "cron_operator_amd", "__init__.py")).read()
    m = re.search(r"__version__\s*=\s*['\"]([^'\"]+)['\"]", init)
    if m is None or m.group(1) != raw:
        errs.append(f"Error: package __version__ '{m.group(1) if m else None}' does not match VERSION '{raw}'.")
    if check_tag and tag_exists(root, version):
        errs.append(f"Error: Tag '{version}' already exists.")
    return errs


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--root", default=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    ap.add_argument("--no-tag-check", action="store_true")
    a = ap.parse_args(argv)
    errs = check(a.root, check_tag=not a.no_tag_check)
    if errs:
        print("\n".join(errs), file=sys.stderr)
        return 1
    version = open(os.path.join(a.root, "VERSION")).read().strip()
    print(f"VERSION={version}\nRAW_VERSION={version[1:]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
