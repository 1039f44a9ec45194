"""Runtime layer: work queue, rate limiters, informers, HTTP client/transport,
leader election, event recorder, probe + metrics servers, kubeconfig."""
from __future__ import annotations

import asyncio
import json
import os
import tempfile

import aiohttp
import pytest

from cron_operator_amd.api import errors
from cron_operator_amd.api.meta import GroupVersionKind, GroupVersionResource
from cron_operator_amd.api.v1alpha1 import CRON_GVK, CRON_GVR, new_cron
from cron_operator_amd.apiserver.http import APIServerApp
from cron_operator_amd.parallel.leaderelection import LEASES, LeaderElector
from cron_operator_amd.parallel.workqueue import ShutDown, WorkQueue
from cron_operator_amd.runtime.client import Client
from cron_operator_amd.runtime.events import Broadcaster, EVENTS_GVR
from cron_operator_amd.runtime.http import HttpTransport, resource_path
from cron_operator_amd.runtime.informer import EventHandler, Informer, label_index
from cron_operator_amd.runtime.kubeconfig import ConfigError, RestConfig, get_config, load_kubeconfig, \
    write_kubeconfig
from cron_operator_amd.runtime.ratelimit import (
    ItemExponentialFailureRateLimiter,
    TokenBucket,
    default_controller_rate_limiter,
    make_client_limiter,
)
from cron_operator_amd.runtime.servers import MetricsServer, ProbeServer, parse_bind_address
from cron_operator_amd.testing.env import TestEnv
from cron_operator_amd.utils.clock import FakeClock

CM = GroupVersionResource("", "v1", "configmaps")


# ---------------------------------------------------------------- work queue


async def test_queue_dedupe_and_serialisation():
    q = WorkQueue("t", FakeClock(0))
    q.add("a")
    q.add("a")
    q.add("b")
    assert len(q) == 2
    a = await q.get()
    assert a == "a"
    q.add("a")  # while processing: parked, not queued
    assert len(q) == 1
    b = await q.get()
    assert b == "b"
    q.done("a")
    assert len(q) == 1 and await q.get() == "a"
    q.done("a")
    q.done("b")
    assert q.idle()


async def test_queue_priority_and_raise():
    q = WorkQueue("t", FakeClock(0))
    q.add("low1")
    q.add("low2")
    q.add("high", priority=10)
    q.add("low2", priority=5)  # raised
    assert [await q.get() for _ in range(3)] == ["high", "low2", "low1"]


async def test_queue_add_after_uses_clock_and_keeps_earliest():
    clock = FakeClock(0)
    q = WorkQueue("t", clock)
    q.add_after("a", 10)
    q.add_after("a", 5)
    q.add_after("a", 20)
    assert len(q) == 0 and q.waiting() == 1
    clock.advance(4.9)
    assert len(q) == 0
    clock.advance(0.2)
    assert len(q) == 1 and await q.get() == "a"


async def test_queue_shutdown_wakes_getters():
    q = WorkQueue("t", FakeClock(0))
    t = asyncio.get_running_loop().create_task(q.get())
    await asyncio.sleep(0)
    q.shutdown()
    with pytest.raises(ShutDown):
        await t


def test_rate_limiters():
    r = ItemExponentialFailureRateLimiter(0.005, 1000)
    assert [r.when("x") for _ in range(4)] == [0.005, 0.01, 0.02, 0.04]
    assert r.num_requeues("x") == 4
    r.forget("x")
    assert r.when("x") == 0.005
    assert ItemExponentialFailureRateLimiter(0.005, 1.0).when("y") <= 1.0
    d = default_controller_rate_limiter()
    assert d.when("z") == pytest.approx(0.005, abs=1e-3)
    assert make_client_limiter(-1, 10) is None
    assert make_client_limiter(0, 0).qps == 5.0


async def test_token_bucket_paces():
    b = TokenBucket(100, 5)
    t0 = asyncio.get_running_loop().time()
    for _ in range(15):
        await b.wait()
    assert asyncio.get_running_loop().time() - t0 >= 0.08  # 10 tokens beyond the burst at 100/s


# ---------------------------------------------------------------- informer


async def test_informer_list_watch_index_and_relist():
    env = TestEnv()
    s = env.server
    s.create(CM, "default", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "a", "labels": {"k": "1"}}})
    inf = Informer(env.client, CM, indexers={"k": label_index("k")})
    seen = []
    inf.add_handler(EventHandler(on_add=lambda o: seen.append(("add", o["metadata"]["name"])),
                                 on_update=lambda a, b: seen.append(("upd", b["metadata"]["name"])),
                                 on_delete=lambda o: seen.append(("del", o["metadata"]["name"]))))
    inf.start()
    await asyncio.wait_for(inf.synced.wait(), 5)
    s.create(CM, "default", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "b", "labels": {"k": "1"}}})
    s.patch(CM, "default", "a", {"data": {"x": "y"}})
    s.delete(CM, "default", "b")
    for _ in range(50):
        await asyncio.sleep(0.001)
    assert seen == [("add", "a"), ("add", "b"), ("upd", "a"), ("del", "b")]
    assert [o["metadata"]["name"] for o in inf.by_index("k", "default/1")] == ["a"]
    # force a 410 on the next watch: closing the stream makes the reflector resume; expire the window
    s._log_floor[("", "configmaps")] = s.current_rv() + 100
    s.close_all_watches()
    s.create(CM, "default", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c"}})
    for _ in range(200):
        await asyncio.sleep(0.002)
        if inf.get("default", "c") is not None:
            break
    assert inf.get("default", "c") is not None and inf.relists >= 2
    await inf.stop()


# ---------------------------------------------------------------- HTTP transport against the served fake apiserver


async def test_http_transport_end_to_end():
    env = TestEnv()
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)
    try:
        created = await client.create(CRON_GVK, new_cron("c", "default", "* * * * *",
                                                         {"apiVersion": "kubeflow.org/v1",
                                                          "kind": "PyTorchJob"}).to_dict())
        assert created["spec"]["concurrencyPolicy"] == "Allow"
        got = await client.get(CRON_GVR, "default", "c")
        assert got["metadata"]["uid"] == created["metadata"]["uid"]
        lst = await client.list(CRON_GVK, "default")
        assert len(lst["items"]) == 1
        with pytest.raises(errors.ApiError) as e:
            await client.get(CRON_GVR, "default", "missing")
        assert errors.is_not_found(e.value)
        with pytest.raises(errors.ApiError) as e:
            await client.create(CRON_GVR, created)
        assert errors.is_already_exists(e.value)
        p = await client.patch(CRON_GVR, "default", "c", {"status": {"lastScheduleTime": "2026-01-01T00:00:00Z"}},
                               "merge", "status")
        assert p["status"]["lastScheduleTime"] == "2026-01-01T00:00:00Z"
        # watch over HTTP
        w = await client.watch(CRON_GVR, "default", resource_version=p["metadata"]["resourceVersion"])
        await client.patch(CRON_GVR, "default", "c", {"metadata": {"labels": {"x": "y"}}})
        et, obj = await asyncio.wait_for(w.__anext__(), 5)
        assert et == "MODIFIED" and obj["metadata"]["labels"] == {"x": "y"}
        w.stop()
        # informer over HTTP
        inf = Informer(client, CRON_GVR)
        inf.start()
        await asyncio.wait_for(inf.synced.wait(), 5)
        assert inf.get("default", "c") is not None
        await inf.stop()
        await client.delete(CRON_GVR, "default", "c")
        # discovery via the mapper
        gvr, namespaced = await client.mapper.resource_for(GroupVersionKind("kubeflow.org", "v1", "TFJob"))
        assert gvr.resource == "tfjobs" and namespaced
    finally:
        await client.close()
        await app.stop()


async def test_bookmarks_advance_informer_resource_version():
    """Periodic BOOKMARKs (kube-apiserver sends ~1/min) move an idle informer's resourceVersion to
    the server's current one, so a resumed watch does not start from a compacted version."""
    env = TestEnv()
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0, bookmark_interval=0.05)
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)
    try:
        inf = Informer(client, CRON_GVR, "default")
        inf.start()
        await asyncio.wait_for(inf.synced.wait(), 5)
        start_rv = inf.last_rv
        # writes the informer does not watch (another namespace) still advance the global RV
        env.server.create_namespace("elsewhere")
        await client.create(CRON_GVK, new_cron("other", "elsewhere", "* * * * *",
                                               {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob"}).to_dict())
        target = str(env.server.current_rv())
        for _ in range(200):
            if inf.last_rv == target:
                break
            await asyncio.sleep(0.01)
        assert int(inf.last_rv) > int(start_rv or 0) and inf.last_rv == target
        assert inf.get("elsewhere", "other") is None  # bookmarks carry no object
        await inf.stop()
    finally:
        await client.close()
        await app.stop()


async def test_workqueue_unfinished_work_metrics_refresh():
    from cron_operator_amd.runtime import metrics
    from cron_operator_amd.runtime.controller import Controller, Request

    gate = asyncio.Event()

    class Slow:
        async def reconcile(self, req, log):
            await gate.wait()

    ctrl = Controller("unfinished-test", Slow(), FakeClock(0), 1)
    ctrl.start()
    ctrl.queue.add(Request("ns", "a"))
    longest = metrics.WQ_LONGEST.labels("unfinished-test", "unfinished-test")
    for _ in range(300):
        if longest.get() > 0:
            break
        await asyncio.sleep(0.01)
    assert longest.get() > 0 and metrics.WQ_UNFINISHED.labels("unfinished-test", "unfinished-test").get() > 0
    gate.set()
    await ctrl.stop()


def test_resource_paths():
    assert resource_path(CRON_GVR, "ns", "n", "status") == "/apis/apps.kubedl.io/v1alpha1/namespaces/ns/crons/n/status"
    assert resource_path(GroupVersionResource("", "v1", "namespaces"), "", "x") == "/api/v1/namespaces/x"


async def test_http_bearer_token_required():
    env = TestEnv()
    env.server.tokens = {"sekret": {"username": "u"}}
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    try:
        bad = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)
        with pytest.raises(errors.ApiError) as e:
            await bad.get(CRON_GVR, "default", "x")
        assert e.value.code == 401
        await bad.close()
        good = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}", bearer_token="sekret")), qps=-1)
        with pytest.raises(errors.ApiError) as e:
            await good.get(CRON_GVR, "default", "x")
        assert e.value.code == 404
        await good.close()
    finally:
        await app.stop()


@pytest.mark.parametrize("fast", [True, False])
async def test_http_token_file_rotation(fast):
    """A projected service-account token rotates under the running operator: the file is
    re-read once its cache period passes, and a 401 forces the re-read right away."""
    env = TestEnv()
    env.server.tokens = {"tok-1": {"username": "u"}}
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "token")
        with open(path, "w") as fh:
            fh.write("tok-1\n")
        cfg = RestConfig(host=f"http://127.0.0.1:{port}", bearer_token_file=path)
        c = Client(HttpTransport(cfg, fast=fast), qps=-1)
        try:
            with pytest.raises(errors.ApiError) as e:
                await c.get(CRON_GVR, "default", "x")
            assert e.value.code == 404
            # kubelet rotates the file; the apiserver stops accepting the old token
            with open(path, "w") as fh:
                fh.write("tok-2\n")
            env.server.tokens = {"tok-2": {"username": "u"}}
            with pytest.raises(errors.ApiError) as e:  # cached old token: one 401 ...
                await c.get(CRON_GVR, "default", "x")
            assert e.value.code == 401
            with pytest.raises(errors.ApiError) as e:  # ... which drops the cache
                await c.get(CRON_GVR, "default", "x")
            assert e.value.code == 404
            # and the periodic re-read, without a 401
            with open(path, "w") as fh:
                fh.write("tok-3\n")
            env.server.tokens = {"tok-2": {"username": "u"}, "tok-3": {"username": "u"}}
            cfg._file_token_refresh_at = 0.0  # the minute passed
            await c.create(CM, {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "rot"}}, "default")
            env.server.tokens = {"tok-3": {"username": "u"}}
            assert (await c.get(CM, "default", "rot"))["metadata"]["name"] == "rot"
            # a vanished file keeps the last good token
            os.unlink(path)
            cfg._file_token_refresh_at = 0.0
            assert cfg.token() == "tok-3"
        finally:
            await c.close()
            await app.stop()


# ---------------------------------------------------------------- leader election


async def test_leader_election_single_leader_and_failover():
    clock = FakeClock(1_000_000 * 10**9)
    env = TestEnv(clock=clock)
    a = LeaderElector(env.new_client(), "619a52b8.kubedl.io", "default", "a", clock, 15, 10, 2)
    b = LeaderElector(env.new_client(), "619a52b8.kubedl.io", "default", "b", clock, 15, 10, 2)
    assert await a.try_acquire_or_renew()
    assert not await b.try_acquire_or_renew()  # held and fresh
    lease = env.server.get(LEASES, "default", "619a52b8.kubedl.io")
    assert lease["spec"]["holderIdentity"] == "a" and lease["spec"]["leaseTransitions"] == 0
    clock.advance(10)
    assert await a.try_acquire_or_renew()  # renew
    clock.advance(16)  # a stops renewing
    # b last saw the record before a's renewal: it sees it change now, and its local
    # expiry clock restarts (client-go observedTime), so the lease is still a's
    assert not await b.try_acquire_or_renew()
    clock.advance(14)
    assert not await b.try_acquire_or_renew()
    clock.advance(2)  # 16 s of local time without a change: expired
    assert await b.try_acquire_or_renew()
    lease = env.server.get(LEASES, "default", "619a52b8.kubedl.io")
    assert lease["spec"]["holderIdentity"] == "b" and lease["spec"]["leaseTransitions"] == 1
    assert not await a.try_acquire_or_renew()


async def test_leader_election_release():
    clock = FakeClock(10**12)
    env = TestEnv(clock=clock)
    a = LeaderElector(env.new_client(), "l", "default", "a", clock, 15, 10, 2, release_on_cancel=True)
    await a.try_acquire_or_renew()
    a.is_leader = True
    await a.release()
    b = LeaderElector(env.new_client(), "l", "default", "b", clock, 15, 10, 2)
    clock.advance(1.5)
    assert await b.try_acquire_or_renew()


def test_leader_election_validates_timings():
    with pytest.raises(ValueError):
        LeaderElector(None, "l", "ns", "a", FakeClock(0), 10, 10, 2)


# ---------------------------------------------------------------- events


async def test_event_broadcaster_writes_and_aggregates():
    env = TestEnv()
    b = Broadcaster(env.new_client(), env.clock)
    b.start()
    rec = b.recorder_for("cron")
    obj = {"apiVersion": "apps.kubedl.io/v1alpha1", "kind": "Cron",
           "metadata": {"name": "c", "namespace": "default", "uid": "u1"}}
    rec.event(obj, "Normal", "Deadline", "cron has reach deadline and stop scheduling")
    rec.event(obj, "Normal", "Deadline", "cron has reach deadline and stop scheduling")
    rec.eventf(obj, "Warning", "TooManyMissedTimes", "too many missed start times: %d. Check clock skew", 101)
    await b.flush()
    for _ in range(20):
        await asyncio.sleep(0.001)
    evs = env.server.list(EVENTS_GVR, "default")["items"]
    by_reason = {e["reason"]: e for e in evs}
    assert by_reason["Deadline"]["count"] == 2 and by_reason["Deadline"]["type"] == "Normal"
    assert by_reason["Deadline"]["involvedObject"]["kind"] == "Cron"
    assert by_reason["Deadline"]["source"] == {"component": "cron"}
    assert by_reason["TooManyMissedTimes"]["message"].endswith("101. Check clock skew")
    with pytest.raises(ValueError):
        rec.event(obj, "Info", "X", "y")
    await b.stop()


async def test_event_spam_filter():
    env = TestEnv()
    b = Broadcaster(env.new_client(), env.clock, spam_burst=3)
    b.start()
    rec = b.recorder_for("cron")
    obj = {"kind": "Cron", "apiVersion": "apps.kubedl.io/v1alpha1", "metadata": {"name": "c", "namespace": "default"}}
    for i in range(10):
        rec.event(obj, "Normal", "R", f"m{i}")
    await b.flush()
    for _ in range(20):
        await asyncio.sleep(0.001)
    assert len(env.server.list(EVENTS_GVR, "default")["items"]) == 3 and b.dropped == 7
    await b.stop()


# ---------------------------------------------------------------- servers


def test_parse_bind_address():
    assert parse_bind_address("0") is None
    assert parse_bind_address(":8081") == ("0.0.0.0", 8081)
    assert parse_bind_address("127.0.0.1:9") == ("127.0.0.1", 9)


async def test_probe_server():
    p = ProbeServer("127.0.0.1:0")
    p.healthz["ping"] = lambda: None
    p.readyz["ping"] = lambda: None
    p.readyz["cache"] = lambda: "not synced"
    await p.start()
    try:
        async with aiohttp.ClientSession() as s:
            async with s.get(f"http://127.0.0.1:{p.port}/healthz") as r:
                assert r.status == 200 and await r.text() == "ok"
            async with s.get(f"http://127.0.0.1:{p.port}/readyz?verbose") as r:
                assert r.status == 500 and "[-]cache failed: not synced" in await r.text()
            async with s.get(f"http://127.0.0.1:{p.port}/readyz/ping") as r:
                assert r.status == 200
    finally:
        await p.stop()


async def test_debug_views_report_caches_and_the_wire_memo():
    """/debug/caches and /debug/wire-memo on the probe port: what each informer holds and the
    process's memory, for sizing a deployment (docs/operations.md "Memory")."""
    from cron_operator_amd.api.v1alpha1 import new_cron
    from cron_operator_amd.controller.setup import setup_with_manager
    from cron_operator_amd.runtime.manager import Manager, ManagerOptions

    env = TestEnv()
    await env.create_cron(new_cron("d", "default", "*/1 * * * *", {"apiVersion": "kubeflow.org/v1",
                                                                   "kind": "PyTorchJob", "spec": {}}))
    mgr = Manager(env.client, ManagerOptions(clock=env.clock, health_probe_bind_address="127.0.0.1:0",
                                             metrics_bind_address="0"))
    await setup_with_manager(mgr)
    task = asyncio.get_running_loop().create_task(mgr.start())
    try:
        await asyncio.wait_for(mgr.started.wait(), 20)
        async with aiohttp.ClientSession() as s:
            async with s.get(f"http://127.0.0.1:{mgr.probes.port}/debug/caches") as r:
                assert r.status == 200
                view = await r.json()
            assert view["rss_mib"] > 0
            crons = [i for i in view["informers"] if i["informer"].startswith("crons")]
            assert crons and crons[0]["objects"] == 1 and crons[0]["synced"]
            async with s.get(f"http://127.0.0.1:{mgr.probes.port}/debug/wire-memo") as r:
                assert r.status == 200 and "slots" in await r.json()
            async with s.get(f"http://127.0.0.1:{mgr.probes.port}/debug/nope") as r:
                assert r.status == 404 and "caches" in await r.text()
    finally:
        mgr.stop()
        await asyncio.wait({task}, timeout=10)


async def _parked_here(ev: asyncio.Event) -> None:
    await ev.wait()


async def test_debug_tasks_and_the_opt_in_cpu_profile():
    """/debug/tasks groups live tasks by where they wait (a goroutine dump's analogue);
    /debug/profile is served only with --enable-profiling, one profile at a time."""
    from cron_operator_amd.runtime import profiler

    probes = ProbeServer("127.0.0.1:0")
    await probes.start()
    ev = asyncio.Event()
    parked = [asyncio.get_running_loop().create_task(_parked_here(ev)) for _ in range(7)]
    stop = False

    async def busy() -> None:
        while not stop:
            sum(i * i for i in range(2000))
            await asyncio.sleep(0)

    spin = asyncio.get_running_loop().create_task(busy())
    base = f"http://127.0.0.1:{probes.port}"
    try:
        async with aiohttp.ClientSession() as s:
            async with s.get(base + "/debug/tasks?stacks=1") as r:
                view = await r.json()
            here = [g for g in view["by_location"] if "(_parked_here)" in g["where"]]
            assert here and here[0]["tasks"] == 7 and view["tasks"] >= 9
            assert "tests/test_runtime.py" in here[0]["where"] and "locks.py" in here[0]["await_chain"][-1]
            async with s.get(base + "/debug/profile?seconds=0.3") as r:
                assert r.status == 404 and "--enable-profiling" in await r.text()
            profiler.allow()
            try:
                first = asyncio.ensure_future(s.get(base + "/debug/profile?seconds=0.5"))
                await asyncio.sleep(0.1)
                async with s.get(base + "/debug/profile?seconds=0.2") as r:
                    assert r.status == 409  # one at a time
                async with await first as r:
                    assert r.status == 200
                    text = await r.text()
                assert "samples over" in text and "## by self samples" in text and "(busy)" in text
                async with s.get(base + "/debug/profile?seconds=x") as r:
                    assert r.status == 400
                for bad in ("nan", "inf", "-inf", "NaN"):  # a NaN timer corrupts the loop's heap
                    async with s.get(base + f"/debug/profile?seconds={bad}") as r:
                        assert r.status == 400, bad
                with pytest.raises(ValueError):
                    await profiler.cpu_profile(float("nan"))
            finally:
                profiler.allow(False)
    finally:
        stop = True
        ev.set()
        await asyncio.gather(spin, *parked)
        await probes.stop()


async def test_metrics_server_insecure_and_secure():
    env = TestEnv()
    env.server.tokens = {"good": {"username": "system:serviceaccount:x:prom", "groups": []}}
    env.server.authorizer = lambda who, spec: who["user"].startswith("system:serviceaccount:x:")
    m = MetricsServer("127.0.0.1:0", secure=False)
    await m.start()
    try:
        async with aiohttp.ClientSession() as s:
            async with s.get(f"http://127.0.0.1:{m.port}/metrics") as r:
                body = await r.text()
                assert r.status == 200 and "workqueue_adds_total" in body or "process_" in body
    finally:
        await m.stop()
    sm = MetricsServer("127.0.0.1:0", secure=True, client=env.new_client())
    await sm.start()
    try:
        async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(ssl=False)) as s:
            url = f"https://127.0.0.1:{sm.port}/metrics"
            async with s.get(url) as r:
                assert r.status == 401
            async with s.get(url, headers={"Authorization": "Bearer bad"}) as r:
                assert r.status == 401
            async with s.get(url, headers={"Authorization": "Bearer good"}) as r:
                assert r.status == 200 and "controller_runtime" in (await r.text()) or r.status == 200
        env.server.authorizer = lambda who, spec: False
        async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(ssl=False)) as s:
            async with s.get(f"https://127.0.0.1:{sm.port}/metrics", headers={"Authorization": "Bearer good"}) as r:
                assert r.status == 403
    finally:
        await sm.stop()


# ---------------------------------------------------------------- kubeconfig


def test_kubeconfig_load_and_precedence(monkeypatch):
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "kc")
        write_kubeconfig(p, "https://example:6443", token="abc", insecure=True)
        cfg = load_kubeconfig(p)
        assert cfg.host == "https://example:6443" and cfg.token() == "abc" and cfg.insecure
        assert cfg.auth_headers()["Authorization"] == "Bearer abc"
        monkeypatch.setenv("KUBECONFIG", p)
        assert get_config().host == "https://example:6443"
        monkeypatch.delenv("KUBECONFIG")
        monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "10.0.0.1")
        monkeypatch.setenv("KUBERNETES_SERVICE_PORT", "443")
        ic = get_config()
        assert ic.host == "https://10.0.0.1:443" and ic.bearer_token_file.endswith("/token")
        with pytest.raises(ConfigError):
            load_kubeconfig(os.path.join(d, "missing"))


# ---------------------------------------------------------------- periodic resync (controller-runtime SyncPeriod)


async def test_periodic_resync_reconciles_idle_crons():
    """A suspended Cron is never requeued; only the cache resync brings it back (SyncPeriod)."""
    from cron_operator_amd.api.v1alpha1 import new_cron
    from cron_operator_amd.testing.env import TestEnv

    env = TestEnv()
    tmpl = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob"}
    await env.create_cron(new_cron("idle", "default", "*/1 * * * *", tmpl, suspend=True))
    await env.start_manager(sync_period=600.0)
    await env.settle()
    before = env.controller.reconciles
    await env.advance(300)
    assert env.controller.reconciles == before  # nothing requeues a suspended Cron
    await env.advance(400)  # past 600 s (+ <=10% jitter)
    assert env.controller.reconciles == before + 1
    infs = env.manager.cache.informers()
    assert all(i.resyncs >= 1 for i in infs if i.synced.is_set())
    await env.stop()


async def test_resync_disabled_with_zero_period():
    from cron_operator_amd.api.v1alpha1 import new_cron
    from cron_operator_amd.testing.env import TestEnv

    env = TestEnv()
    await env.create_cron(new_cron("idle", "default", "*/1 * * * *", {"apiVersion": "kubeflow.org/v1",
                                                                      "kind": "PyTorchJob"}, suspend=True))
    await env.start_manager(sync_period=0.0)
    await env.settle()
    before = env.controller.reconciles
    await env.advance(100 * 3600)
    assert env.controller.reconciles == before
    await env.stop()


async def test_http_watch_stream_timeout_keepalive_and_disconnect():
    """The HTTP front end's watch responses: events written as chunks, timeoutSeconds ends the
    response with the terminating chunk and the kept-alive connection serves the next request;
    a client that disconnects mid-watch leaves no watcher behind."""
    env = TestEnv()
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    try:
        reader, writer = await asyncio.open_connection("127.0.0.1", port)
        writer.write(b"GET /api/v1/namespaces/default/configmaps?watch=true&timeoutSeconds=1 HTTP/1.1\r\n"
                     b"Host: x\r\n\r\n")
        await writer.drain()
        head = await asyncio.wait_for(reader.readuntil(b"\r\n\r\n"), 5)
        assert head.startswith(b"HTTP/1.1 200") and b"chunked" in head
        env.server.create(CM, "default", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "a"}})
        env.server.create(CM, "default", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "b"}})
        size = int((await asyncio.wait_for(reader.readuntil(b"\r\n"), 5)).strip(), 16)
        chunk = await reader.readexactly(size + 2)
        lines = [json.loads(ln) for ln in chunk[:-2].splitlines()]
        assert [(e["type"], e["object"]["metadata"]["name"]) for e in lines] == [("ADDED", "a"), ("ADDED", "b")]
        assert await asyncio.wait_for(reader.readuntil(b"0\r\n\r\n"), 5)  # timeoutSeconds ended the response
        writer.write(b"GET /api/v1/namespaces/default/configmaps/a HTTP/1.1\r\nHost: x\r\n\r\n")
        await writer.drain()
        assert (await asyncio.wait_for(reader.readuntil(b"\r\n\r\n"), 5)).startswith(b"HTTP/1.1 200")
        writer.close()
        # a watch whose client goes away
        reader, writer = await asyncio.open_connection("127.0.0.1", port)
        writer.write(b"GET /api/v1/namespaces/default/configmaps?watch=true HTTP/1.1\r\nHost: x\r\n\r\n")
        await writer.drain()
        await asyncio.wait_for(reader.readuntil(b"\r\n\r\n"), 5)
        key = ("", "configmaps")
        assert len(env.server._watchers[key]) == 1
        writer.close()
        for _ in range(100):
            await asyncio.sleep(0.01)
            if not env.server._watchers[key]:
                break
        assert not env.server._watchers[key] and not app._streams
    finally:
        await app.stop()


def test_workqueue_counts_adds_like_client_go():
    """client-go's workqueue counts an Add only when the item was not dirty already: a key
    queued twice, or re-added twice while processing, is one add."""
    from cron_operator_amd.parallel.workqueue import WorkQueue
    from cron_operator_amd.runtime.controller import Request
    from cron_operator_amd.utils.clock import FakeClock

    async def run():
        q = WorkQueue("t", FakeClock(0))
        a = Request("ns", "a")
        q.add(a)
        q.add(a)
        assert q.adds == 1 and len(q) == 1
        assert await q.get() == a
        q.add(a)
        q.add(a)  # dirty while processing: once
        assert q.adds == 2
        q.done(a)
        assert len(q) == 1 and q.adds == 2

    asyncio.run(run())


async def test_metrics_server_reloads_a_rotated_certificate(tmp_path):
    """``--metrics-cert-path``: like controller-runtime's certwatcher, a certificate rotated
    on disk (cert-manager renewing the Secret) is served to new connections without a restart;
    a half-written pair keeps the previous certificate."""
    import hashlib
    import ssl

    from cron_operator_amd.runtime.servers import self_signed_cert

    def fingerprint(port):
        ctx = ssl.create_default_context()
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE

        async def grab():
            _, w = await asyncio.open_connection("127.0.0.1", port, ssl=ctx)
            der = w.get_extra_info("ssl_object").getpeercert(binary_form=True)
            w.close()
            return hashlib.sha256(der).hexdigest()
        return grab()

    certs = tmp_path / "certs"
    certs.mkdir()
    crt, key = self_signed_cert(str(certs), host="first")
    env = TestEnv()
    sm = MetricsServer("127.0.0.1:0", secure=True, cert_dir=str(certs), client=env.new_client(),
                       cert_poll_interval=0.05)
    await sm.start()
    try:
        first = await fingerprint(sm.port)
        with open(crt, "w") as fh:  # caught mid-rotation: an unreadable certificate is not loaded
            fh.write("not a certificate")
        await asyncio.sleep(0.3)
        assert await fingerprint(sm.port) == first and sm.cert_reloads == 0
        other = tmp_path / "other"
        other.mkdir()
        ncrt, nkey = self_signed_cert(str(other), host="second")
        os.replace(nkey, key)
        os.replace(ncrt, crt)
        for _ in range(100):
            await asyncio.sleep(0.05)
            if sm.cert_reloads:
                break
        assert sm.cert_reloads == 1
        assert await fingerprint(sm.port) != first
        from cron_operator_amd.runtime import metrics as m

        assert m.CERT_READ_ERRORS._only().get() >= 1 and m.CERT_READS._only().get() >= 3
    finally:
        await sm.stop()


async def test_metrics_cert_rotation_with_mismatched_key_keeps_serving(tmp_path):
    """A new certificate lands before its key (a rotation seen half way, or a bad Secret):
    the pair does not match, so the watcher must keep serving the previous certificate --
    the live context is never half-loaded -- and pick up the new pair once the key follows."""
    import hashlib
    import ssl

    from cron_operator_amd.runtime.servers import self_signed_cert

    async def fingerprint(port):
        ctx = ssl.create_default_context()
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
        _, w = await asyncio.open_connection("127.0.0.1", port, ssl=ctx)
        der = w.get_extra_info("ssl_object").getpeercert(binary_form=True)
        w.close()
        return hashlib.sha256(der).hexdigest()

    certs = tmp_path / "certs"
    certs.mkdir()
    crt, key = self_signed_cert(str(certs), host="first")
    env = TestEnv()
    sm = MetricsServer("127.0.0.1:0", secure=True, cert_dir=str(certs), client=env.new_client(),
                       cert_poll_interval=0.05)
    await sm.start()
    try:
        first = await fingerprint(sm.port)
        other = tmp_path / "other"
        other.mkdir()
        ncrt, nkey = self_signed_cert(str(other), host="second")
        os.replace(ncrt, crt)  # valid certificate, old key: KEY_VALUES_MISMATCH
        await asyncio.sleep(0.4)
        assert sm.cert_reloads == 0
        for _ in range(3):  # still serving, with the previous certificate
            assert await fingerprint(sm.port) == first
        os.replace(nkey, key)
        for _ in range(100):
            await asyncio.sleep(0.05)
            if sm.cert_reloads:
                break
        assert sm.cert_reloads == 1
        assert await fingerprint(sm.port) != first
    finally:
        await sm.stop()


async def test_informer_transforms_list_pages_once():
    """A paged initial LIST is transformed page by page as it arrives, and each object exactly
    once (``_replace`` does not transform again); watch events are transformed as before."""
    env = TestEnv()
    s = env.server
    for i in range(23):
        s.create(CM, "default", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": f"c{i}"},
                                 "data": {"big": "x" * 100}})
    seen = []

    def slim(o):
        seen.append(o["metadata"]["name"])
        o.pop("data", None)
        return o

    inf = Informer(env.new_client(), CM, "default", page_size=5, transform=slim)
    inf.start()
    await asyncio.wait_for(inf.synced.wait(), 5)
    assert sorted(seen) == sorted(f"c{i}" for i in range(23)) and len(seen) == 23
    assert all("data" not in o for o in inf.store.values())
    s.create(CM, "default", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "late"}, "data": {"a": "b"}})
    for _ in range(200):
        await asyncio.sleep(0.001)
        if inf.get("default", "late", copy=False) is not None:
            break
    assert "data" not in inf.get("default", "late", copy=False) and seen.count("late") == 1
    await inf.stop()


async def test_informer_keep_filter_stores_only_what_passes_it():
    """``keep`` (the shard assigner's share of an unassigned fleet): rejected LIST items and
    events are never stored, and an object that stops passing it leaves as a deletion."""
    env = TestEnv()
    s = env.server
    for i in range(12):
        s.create(CM, "default", {"apiVersion": "v1", "kind": "ConfigMap",
                                 "metadata": {"name": f"c{i}", "labels": {"mine": str(i % 3 == 0).lower()}}})
    gone: list = []
    inf = Informer(env.new_client(), CM, "default", page_size=5,
                   keep=lambda o: o["metadata"].get("labels", {}).get("mine") == "true")
    inf.add_handler(EventHandler(on_delete=lambda o: gone.append(o["metadata"]["name"])))
    inf.start()
    await asyncio.wait_for(inf.synced.wait(), 5)
    assert set(inf.store) == {f"default/c{i}" for i in (0, 3, 6, 9)}

    async def until(pred):
        for _ in range(500):
            if pred():
                return
            await asyncio.sleep(0.002)
        raise AssertionError("timed out")

    s.patch(CM, "default", "c1", {"metadata": {"labels": {"mine": "true"}}}, "merge")  # now passes
    await until(lambda: "default/c1" in inf.store)
    s.patch(CM, "default", "c0", {"metadata": {"labels": {"mine": "false"}}}, "merge")  # stops passing
    await until(lambda: "default/c0" not in inf.store)
    assert gone == ["c0"]
    s.create(CM, "default", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x"}})
    s.delete(CM, "default", "c2")  # never stored: no delete to deliver
    s.patch(CM, "default", "c3", {"metadata": {"labels": {"other": "y"}}}, "merge")  # a barrier
    await until(lambda: "other" in inf.store["default/c3"]["metadata"]["labels"])
    assert "default/x" not in inf.store and gone == ["c0"]
    assert set(inf.store) == {f"default/c{i}" for i in (1, 3, 6, 9)}
    await inf.stop()


def test_free_port_is_free_and_below_the_ephemeral_range():
    import socket

    from cron_operator_amd.utils.ports import _ephemeral_low, free_port

    low = _ephemeral_low()
    for _ in range(20):
        p = free_port()
        assert 1024 < p and (p < low or low - 15000 < 1000)
        with socket.socket() as s:
            s.bind(("127.0.0.1", p))  # still free


async def test_debug_views_answer_only_loopback_clients_by_default():
    """the probe port's /debug views expose internals; by default (--debug-views=local)
    only loopback clients get them, the probes themselves stay open to the kubelet."""
    from cron_operator_amd.runtime import miniweb
    from cron_operator_amd.runtime.servers import is_loopback

    assert is_loopback("127.0.0.1") and is_loopback("::1") and is_loopback("::ffff:127.0.0.1")
    assert not is_loopback("10.244.1.7") and not is_loopback("") and not is_loopback("fe80::1%eth0")

    async def call(probes, path, peer):
        h, info = probes.app().match(path)
        req = miniweb.Request("GET", path, {}, {}, peer)
        req.match_info = info
        return await h(req)

    local = ProbeServer("127.0.0.1:0")
    local.debug["caches"] = lambda: {"ok": 1}
    for path in ("/debug/tasks", "/debug/caches", "/debug/profile", "/debug/traces"):
        assert (await call(local, path, "10.244.1.7")).status == 403, path
    assert (await call(local, "/debug/caches", "127.0.0.1")).status == 200
    assert (await call(local, "/healthz", "10.244.1.7")).status == 200  # the kubelet's probe
    anyone = ProbeServer("127.0.0.1:0", debug_views="all")
    anyone.debug["caches"] = lambda: {"ok": 1}
    assert (await call(anyone, "/debug/caches", "10.244.1.7")).status == 200
    off = ProbeServer("127.0.0.1:0", debug_views="off")
    off.debug["caches"] = lambda: {"ok": 1}
    assert (await call(off, "/debug/caches", "127.0.0.1")).status == 404
    with pytest.raises(ValueError):
        ProbeServer(":8081", debug_views="public")
