"""Release guards (``scripts/release_check.py``) and packaging parity files.

Reference: ``/root/reference/.github/workflows/release.yaml:30-63`` (semver VERSION, chart
version and appVersion equal to it, tag must not exist), ``/root/reference/LICENSE`` and
``/root/reference/charts/cron-operator/.helmignore``.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import release_check  # noqa: E402


def _tree(tmp_path, version="v1.2.3", chart="1.2.3", app="1.2.3", pkg="1.2.3"):
    (tmp_path / "charts" / "cron-operator").mkdir(parents=True)
    (tmp_path / "cron_operator_amd").mkdir()
    (tmp_path / "VERSION").write_text(version + "\n")
    (tmp_path / "charts" / "cron-operator" / "Chart.yaml").write_text(
        f"apiVersion: v2\nname: cron-operator\nversion: {chart}\nappVersion: \"{app}\"\n")
    (tmp_path / "cron_operator_amd" / "__init__.py").write_text(f'__version__ = "{pkg}"\n')
    return str(tmp_path)


def test_repo_passes_its_own_release_guards():
    assert release_check.check(ROOT, check_tag=False) == []


def test_consistent_tree_passes(tmp_path):
    assert release_check.check(_tree(tmp_path), check_tag=False) == []


@pytest.mark.parametrize("kw,needle", [
    ({"version": "1.2.3"}, "semver"),
    ({"version": "v1.2"}, "semver"),
    ({"chart": "1.2.4"}, "Chart version '1.2.4'"),
    ({"app": "1.2.2"}, "Chart appVersion '1.2.2'"),
    ({"pkg": "0.0.1"}, "package __version__ '0.0.1'"),
])
def test_mismatches_fail(tmp_path, kw, needle):
    errs = release_check.check(_tree(tmp_path, **kw), check_tag=False)
    assert errs and any(needle in e for e in errs), errs


@pytest.mark.skipif(shutil.which("git") is None, reason="git not installed")
def test_existing_tag_fails(tmp_path):
    root = _tree(tmp_path)
    env = dict(os.environ, GIT_AUTHOR_NAME="t", GIT_AUTHOR_EMAIL="t@e", GIT_COMMITTER_NAME="t",
               GIT_COMMITTER_EMAIL="t@e")
    for cmd in (["init", "-q"], ["add", "-A"], ["commit", "-qm", "x"]):
        subprocess.run(["git", "-C", root] + cmd, check=True, env=env)
    assert release_check.check(root) == []
    subprocess.run(["git", "-C", root, "tag", "v1.2.3"], check=True, env=env)
    assert release_check.check(root) == ["Error: Tag 'v1.2.3' already exists."]
    assert release_check.main(["--root", root]) == 1


def test_license_and_helmignore_present():
    lic = open(os.path.join(ROOT, "LICENSE")).read()
    assert "Apache License" in lic and "Version 2.0" in lic
    assert 'license = { text = "Apache-2.0" }' in open(os.path.join(ROOT, "pyproject.toml")).read()
    ignore = open(os.path.join(ROOT, "charts", "cron-operator", ".helmignore")).read().split()
    for pat in (".git/", "*.swp", "*.bak", "*.orig", "*~", ".idea/", ".vscode/", ".DS_Store"):
        assert pat in ignore, pat
