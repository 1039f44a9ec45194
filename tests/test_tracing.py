"""Tracing subsystem: per-reconcile span trees and their exports."""
from __future__ import annotations

import json

from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.api.v1alpha1 import new_cron
from cron_operator_amd.runtime import tracing
from cron_operator_amd.runtime.servers import ProbeServer
from cron_operator_amd.testing.env import TestEnv

PT_TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}}
PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")


def test_disabled_is_noop():
    t = tracing.Tracer(enabled=False)
    old = tracing.set_tracer(t)
    try:
        with tracing.span("x", a=1) as s:
            s.set(b=2)
        assert s is tracing.NOOP and t.spans() == []
    finally:
        tracing.set_tracer(old)


def test_nesting_errors_and_sampling(tmp_path):
    f = tmp_path / "spans.jsonl"
    t = tracing.Tracer(enabled=True, file=str(f))
    old = tracing.set_tracer(t)
    try:
        with tracing.span("root", k="v") as r:
            with tracing.span("child"):
                pass
            try:
                with tracing.span("boom"):
                    raise ValueError("bad")
            except ValueError:
                pass
            r.event("mark", n=1)
        spans = {s["name"]: s for s in t.spans()}
        assert spans["child"]["parentSpanId"] == spans["root"]["spanId"]
        assert spans["child"]["traceId"] == spans["root"]["traceId"]
        assert spans["boom"]["status"] == "error" and "ValueError: bad" in spans["boom"]["attributes"]["error"]
        assert spans["root"]["events"][0]["name"] == "mark"
        assert len(f.read_text().strip().splitlines()) == 3
        ct = t.chrome_trace()
        assert {e["name"] for e in ct["traceEvents"] if e["ph"] == "X"} == {"root", "child", "boom"}
        json.dumps(ct)
    finally:
        tracing.set_tracer(old)
        t.close()
    t0 = tracing.Tracer(enabled=True, sample_rate=0.0)
    with t0.span("root"):
        pass
    assert t0.spans() == []


async def test_reconcile_span_tree_has_tick_to_create():
    t = tracing.Tracer(enabled=True)
    old = tracing.set_tracer(t)
    env = TestEnv()
    try:
        await env.create_cron(new_cron("tr", "default", "*/1 * * * *", PT_TMPL))
        await env.start_manager()
        await env.settle()
        t.clear()
        await env.advance(60)
        spans = t.spans()
        creates = [s for s in spans if s["name"] == "create_workload"]
        assert len(creates) == 1
        c = creates[0]
        assert c["attributes"]["kind"] == "PyTorchJob" and c["attributes"]["tick_to_create_ms"] >= 0
        by_id = {s["spanId"]: s for s in spans}
        parent = by_id[c["parentSpanId"]]
        assert parent["name"] == "reconcile" and parent["attributes"]["name"] == "tr"
        kids = {s["name"] for s in spans if s["parentSpanId"] == parent["spanId"]}
        assert {"list_children", "sync_status", "create_workload", "patch_status"} <= kids
        http = [s for s in spans if s["parentSpanId"] == c["spanId"]]
        assert [s["name"] for s in http] == ["http.create"]
        assert http[0]["attributes"]["resource"] == "pytorchjobs"
        # the probe server exposes the same data
        ps = ProbeServer("127.0.0.1:0")
        await ps.start()
        try:
            import aiohttp

            async with aiohttp.ClientSession() as s:
                async with s.get(f"http://127.0.0.1:{ps.port}/debug/traces") as r:
                    assert r.status == 200
                    body = await r.json()
            assert any(e["name"] == "create_workload" for e in body["traceEvents"])
        finally:
            await ps.stop()
    finally:
        await env.stop()
        tracing.set_tracer(old)
