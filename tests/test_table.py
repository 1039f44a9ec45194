"""kubectl UX: server-side Table printing with the Cron printer columns, and `cron-operator get`."""
from __future__ import annotations

import asyncio
import os
import subprocess
import sys

from cron_operator_amd.api.v1alpha1 import CRON_GVR, new_cron
from cron_operator_amd.apiserver.http import APIServerApp
from cron_operator_amd.apiserver.table import human_duration, jsonpath, render, wants_table
from cron_operator_amd.runtime.client import Client
from cron_operator_amd.runtime.http import HttpTransport
from cron_operator_amd.runtime.kubeconfig import RestConfig, write_kubeconfig
from cron_operator_amd.testing.env import TestEnv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob"}


def test_jsonpath_subset():
    o = {"spec": {"schedule": "* * * * *", "l": [{"n": "a"}, {"n": "b"}]}, "metadata": {"name": "x"}}
    assert jsonpath(o, ".spec.schedule") == "* * * * *"
    assert jsonpath(o, "{.spec.l[1].n}") == "b"
    assert jsonpath(o, ".spec.missing") is None and jsonpath(o, ".spec.l[5].n") is None
    assert jsonpath(o, ".metadata") == {"name": "x"}


def test_human_duration_matches_k8s():
    cases = {0: "0s", 59: "59s", 119: "119s", 120: "2m", 150: "2m30s", 600: "10m", 10799: "179m", 10800: "3h",
             3 * 3600 + 25 * 60: "3h25m", 8 * 3600: "8h", 47 * 3600: "47h", 48 * 3600: "2d", 50 * 3600: "2d2h",
             8 * 86400: "8d", 400 * 86400: "400d", 800 * 86400: "2y70d", 9 * 365 * 86400: "9y", -5: "<invalid>"}
    for s, want in cases.items():
        assert human_duration(s) == want, (s, human_duration(s), want)


def test_wants_table():
    assert wants_table("application/json;as=Table;v=v1;g=meta.k8s.io,application/json")
    assert wants_table("application/json;as=Table;v=v1;g=meta.k8s.io")
    assert not wants_table("application/json")
    assert not wants_table("application/json;as=PartialObjectMetadataList;v=v1;g=meta.k8s.io")


async def _serve_crons():
    env = TestEnv()
    await env.create_cron(new_cron("nightly", "default", "0 2 * * *", TMPL, suspend=True))
    await env.create_cron(new_cron("hourly", "default", "@hourly", TMPL))
    env.server.patch(CRON_GVR, "default", "hourly", {"status": {"lastScheduleTime": "2026-01-01T12:00:00Z"}},
                     "merge", "status")
    env.server.create_namespace("other")
    await env.create_cron(new_cron("elsewhere", "other", "*/5 * * * *", TMPL))
    env.clock.advance(3 * 3600 + 25 * 60)
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    return env, app, port


async def test_table_over_http_and_in_memory():
    env, app, port = await _serve_crons()
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)
    try:
        for c in (client, env.client):
            t = await c.table(CRON_GVR, "default")
            assert t["kind"] == "Table"
            assert [d["name"] for d in t["columnDefinitions"]] == ["Name", "SCHEDULE", "SUSPEND", "LAST_SCHEDULE",
                                                                   "AGE"]
            rows = {r["cells"][0]: r["cells"] for r in t["rows"]}
            assert rows["nightly"] == ["nightly", "0 2 * * *", True, None, "3h25m"]
            assert rows["hourly"] == ["hourly", "@hourly", None, "2026-01-01T12:00:00Z", "3h25m"]
            assert t["rows"][0]["object"]["kind"] == "PartialObjectMetadata"
            one = await c.table(CRON_GVR, "default", "nightly")
            assert len(one["rows"]) == 1
        text = render(await client.table(CRON_GVR, ""), namespace_column=True)
        lines = text.splitlines()
        assert lines[0].split() == ["NAMESPACE", "NAME", "SCHEDULE", "SUSPEND", "LAST_SCHEDULE", "AGE"]
        assert any(line.startswith("other") and "*/5 * * * *" in line for line in lines[1:])
        assert any("nightly" in line and "true" in line and "<none>" in line for line in lines)
        # plain JSON still served when Table is not asked for
        lst = await client.list(CRON_GVR, "default")
        assert lst["kind"] == "CronList" or "items" in lst
    finally:
        await client.close()
        await app.stop()


async def test_cli_get(tmp_path):
    env, app, port = await _serve_crons()
    kc = tmp_path / "kc"
    write_kubeconfig(str(kc), f"http://127.0.0.1:{port}", "")
    envv = dict(os.environ, PYTHONPATH=ROOT)

    async def run(*args):
        p = await asyncio.create_subprocess_exec(sys.executable, "-m", "cron_operator_amd", "get", *args,
                                                 "--kubeconfig", str(kc), env=envv, stdout=subprocess.PIPE,
                                                 stderr=subprocess.PIPE)
        out, err = await asyncio.wait_for(p.communicate(), 120)
        return p.returncode, out.decode(), err.decode()

    try:
        rc, out, _ = await run("crons")
        assert rc == 0
        assert out.splitlines()[0].split() == ["NAME", "SCHEDULE", "SUSPEND", "LAST_SCHEDULE", "AGE"]
        assert len(out.splitlines()) == 3
        rc, out, _ = await run("cron", "-A", "-o", "name")
        assert rc == 0 and sorted(out.split()) == ["cron.apps.kubedl.io/elsewhere", "cron.apps.kubedl.io/hourly",
                                                   "cron.apps.kubedl.io/nightly"]
        rc, out, _ = await run("cron", "hourly", "-o", "json")
        assert rc == 0 and '"schedule": "@hourly"' in out
        rc, _, err = await run("cron", "missing")
        assert rc == 1 and "NotFound" in err
        rc, _, err = await run("pods")
        assert rc == 1
    finally:
        await app.stop()
