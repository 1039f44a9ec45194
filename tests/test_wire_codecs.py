"""Plan-driven watch decoding over real HTTP (``ReconcilerOptions.wire_codecs``).

The operator talks to the apiserver as the reference does -- REST + watch streams
(``/root/reference/internal/controller/cron_controller.go:70-77`` watches Crons and owned
jobs; ``:107-120`` writes status with a merge patch).  Here the Cron informer decodes its
watch through the same memo the status write was encoded with, so the echo of our own
write carries the reconciler's own history-entry objects, and the child informers never
build the job ``spec`` they drop anyway.
"""
from __future__ import annotations

import asyncio

from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.api.v1alpha1 import CRON_GVR, LABEL_CRON_NAME, new_cron
from cron_operator_amd.controller.reconciler import ReconcilerOptions
from cron_operator_amd.controller.setup import setup_with_manager
from cron_operator_amd.runtime.manager import Manager, ManagerOptions
from cron_operator_amd.testing.env import TestEnv
from cron_operator_amd.trainingop.operator import finished_status
from cron_operator_amd.utils import jsonutil
from cron_operator_amd.utils.gotime import NANOS, UTC, GoTime

PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
NS = "default"
PT_TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "template": {"spec": {"containers": [
               {"name": "pytorch", "image": "rocm/pytorch:latest"}]}}}}}}


async def _until(pred, what: str, timeout: float = 10.0) -> None:
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while loop.time() < end:
        if pred():
            return
        await asyncio.sleep(0.01)
    raise AssertionError(f"timed out waiting for {what}")


async def _run(opts: ReconcilerOptions):
    from cron_operator_amd.apiserver.http import APIServerApp
    from cron_operator_amd.runtime.client import Client
    from cron_operator_amd.runtime.http import HttpTransport
    from cron_operator_amd.runtime.kubeconfig import RestConfig

    env = TestEnv()
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)
    mgr = Manager(client, ManagerOptions(clock=env.clock, health_probe_bind_address="0", metrics_bind_address="0"))
    ctrl, rec = await setup_with_manager(mgr, opts)
    task = asyncio.get_running_loop().create_task(mgr.start())
    try:
        await asyncio.wait_for(mgr.started.wait(), 20)
        await env.create_cron(new_cron("c", NS, "*/1 * * * *", PT_TMPL, history_limit=2))
        seen: set = set()
        for tick in range(1, 5):
            env.clock.advance(60)

            def new_jobs():
                return {o["metadata"]["name"] for o in env.server.list(PT, NS)["items"]} - seen

            await _until(lambda: new_jobs(), f"job of tick {tick}")
            job = sorted(new_jobs())[-1]
            seen.add(job)
            ts = GoTime(env.clock.now_ns() // NANOS, 0, UTC).rfc3339()
            env.server.patch(PT, NS, job, {"status": finished_status("PyTorchJob", job, ts, True)}, "merge",
                             "status")
            want = min(tick, 2)
            await _until(lambda: len((rec.cron_informer.get(NS, "c", copy=False) or {}).get("status", {})
                                     .get("history") or []) == want and ctrl.queue.idle(), f"history after {tick}")
        cached = rec.cron_informer.get(NS, "c", copy=False)
        stored = env.server.get(CRON_GVR, NS, "c")
        child_inf = next(iter(rec.child_informers.values()))
        children = child_inf.list(NS, copy=False)
        return rec, cached, stored, children
    finally:
        mgr.stop()
        await asyncio.wait({task}, timeout=10)
        await client.close()
        await app.stop()


async def test_cron_events_carry_the_reconcilers_own_history_entries():
    rec, cached, stored, children = await _run(ReconcilerOptions())
    assert jsonutil.json_equal(cached["status"], stored["status"])  # exactly what a plain decode gives
    # the template is cached as its JSON text; every job of the 4 ticks was built from it
    wl = cached["spec"]["template"]["workload"]
    assert isinstance(wl, bytes) and jsonutil.loads(wl) == stored["spec"]["template"]["workload"]
    key = f"{NS}/c"
    parsed = rec._parsed_status[key][1]
    hist = cached["status"]["history"]
    assert len(hist) == 2
    if jsonutil.NATIVE:
        # the echo of our status write holds the very dicts the write encoded
        assert all(h is e._json for h, e in zip(hist, parsed.history)), "history entries were rebuilt"
        st = rec.codecs.memo.stats()
        assert st["hits"] > 0 and st["stores"] > 0
    # the echo of our last status write is cached as the very status dict written (active refs
    # and lists are held once per Cron, not twice)
    assert cached["status"] is rec._parsed_status[key][0]
    # children: spec never built, everything the reconciler reads is there
    assert children and all("spec" not in c and c["metadata"]["labels"][LABEL_CRON_NAME] == "c" for c in children)


async def test_reference_mode_decodes_plainly():
    rec, cached, stored, children = await _run(ReconcilerOptions(list_mode="cache", wire_codecs=False,
                                                                 slim_child_cache=False))
    assert rec.codecs is None
    assert jsonutil.json_equal(cached["status"], stored["status"])
    assert cached["spec"]["template"]["workload"] == stored["spec"]["template"]["workload"]  # a dict
    assert children and all("spec" in c for c in children)


async def test_initial_list_shares_labels_and_owners_and_trims_status():
    """A starting operator over an existing fleet: the child informer's first LIST is decoded with
    the same memo plans as its watch events (``WireCodecs.child_list``), so the jobs of one Cron
    share one labels dict and one ownerReferences list, no spec is built, and each job's status is
    trimmed to what classifies it (``compact_child``) -- the memory a 10,000-Cron fleet caches."""
    from cron_operator_amd.api.meta import new_controller_ref
    from cron_operator_amd.api.v1alpha1 import CRON_GVK
    from cron_operator_amd.apiserver.http import APIServerApp
    from cron_operator_amd.runtime.client import Client
    from cron_operator_amd.runtime.http import HttpTransport
    from cron_operator_amd.runtime.kubeconfig import RestConfig

    env = TestEnv()
    cron = await env.create_cron(new_cron("c", NS, "*/1 * * * *", PT_TMPL, history_limit=5))
    for i in range(4):
        name = f"c-{1767268800 + 60 * i}"
        job = jsonutil.deepcopy(PT_TMPL)
        job["metadata"] = {"name": name, "namespace": NS, "labels": {LABEL_CRON_NAME: "c"},
                           "annotations": {"kubectl.kubernetes.io/last-applied-configuration": "{}" * 200},
                           "ownerReferences": [new_controller_ref(cron, CRON_GVK)]}
        env.server.create(PT, NS, job)
        env.server.patch(PT, NS, name, {"status": finished_status("PyTorchJob", name, "2026-01-01T12:00:30Z", True)},
                         "merge", "status")
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)
    mgr = Manager(client, ManagerOptions(clock=env.clock, health_probe_bind_address="0", metrics_bind_address="0"))
    ctrl, rec = await setup_with_manager(mgr, ReconcilerOptions())
    task = asyncio.get_running_loop().create_task(mgr.start())
    try:
        await asyncio.wait_for(mgr.started.wait(), 20)
        inf = next(iter(rec.child_informers.values()))
        kids = inf.list(NS, copy=False)
        assert len(kids) == 4 and all("spec" not in k for k in kids)
        # metadata: only what is read (no annotations, generation, managedFields)
        assert all(set(k["metadata"]) <= {"name", "namespace", "uid", "resourceVersion", "creationTimestamp",
                                          "labels", "ownerReferences"} for k in kids), kids[0]["metadata"]
        for k in kids:
            st = k["status"]
            assert set(st) <= {"conditions", "completionTime"}, st
            assert [c["type"] for c in st["conditions"]] == ["Succeeded"]  # the terminal (= last) one
            assert set(st["conditions"][0]) <= {"type", "status", "lastTransitionTime"}
        # every finished job shares one read-only status; its memo has the completion time
        assert len({id(k["status"]) for k in kids}) == 1
        for info in inf.derived.values():
            assert info.finished and info.cls.status == "Succeeded"
            assert info.cls.finished_at is not None and info.cls.finished_at.rfc3339() == "2026-01-01T12:00:30Z"
        if jsonutil.NATIVE:
            assert len({id(k["metadata"]["labels"]) for k in kids}) == 1
            assert len({id(k["metadata"]["ownerReferences"]) for k in kids}) == 1
    finally:
        mgr.stop()
        await asyncio.wait({task}, timeout=10)
        await client.close()
        await app.stop()


def test_compacting_codecs_never_build_the_child_metadata_the_cache_drops():
    """With the compact child cache, the keys compact_child() would drop from a child's metadata
    (generation, annotations such as kubectl's last-applied manifest, finalizers, ...) are
    skipped while decoding: the cached child keeps its decoded metadata dict, no filtered copy."""
    import json

    from cron_operator_amd.controller.reconciler import CHILD_METADATA, CHILD_METADATA_DROPPED, WireCodecs

    meta = {"name": "j", "namespace": "ns", "uid": "u", "resourceVersion": "5", "generation": 1,
            "creationTimestamp": "2026-01-01T00:00:00Z", "labels": {"a": "b"},
            "annotations": {"kubectl.kubernetes.io/last-applied-configuration": "{}"}, "finalizers": ["x"],
            "ownerReferences": [{"kind": "Cron", "name": "c", "uid": "cu", "controller": True}]}
    obj = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": meta, "spec": {"x": 1}}
    line = json.dumps({"type": "ADDED", "object": obj}).encode()
    _, got = WireCodecs(compact_metadata=True).child_event(line)
    assert set(got["metadata"]) == {k for k in CHILD_METADATA if k in meta}
    assert not set(got["metadata"]) & set(CHILD_METADATA_DROPPED) and "spec" not in got
    page = json.dumps({"kind": "List", "metadata": {}, "items": [obj]}).encode()
    assert set(WireCodecs(compact_metadata=True).child_list.loads(page)["items"][0]["metadata"]) == set(got["metadata"])
    _, full = WireCodecs().child_event(line)  # without the compact cache: all of it
    assert set(full["metadata"]) == set(meta)


def test_a_fixed_name_template_kept_as_text_still_runs_as_forbid():
    """A template with ``metadata.name`` (cron_controller.go:355-362: every run reuses that name,
    so the ran-tick dedupe must not look for a generated one) is recognised whether the cached
    template is a dict or its JSON text."""
    from cron_operator_amd.controller.reconciler import _template_fixed_name

    named = dict(PT_TMPL, metadata={"name": "fixed"})
    assert _template_fixed_name(jsonutil.dumpb(named)) and not _template_fixed_name(jsonutil.dumpb(PT_TMPL))
    assert _template_fixed_name(named) and not _template_fixed_name(b"not json")


def test_hash_routed_codecs_build_only_their_shards_objects():
    """With hash routing every shard watches the whole fleet: its decoders (``WireCodecs(shard=)``)
    build another shard's Crons and jobs only up to their metadata, which the informers' keep
    filter then drops; its own decode whole."""
    import json

    from cron_operator_amd.controller.reconciler import WireCodecs
    from cron_operator_amd.runtime.controller import shard_of

    names = [f"c{i}" for i in range(8)]
    mine = {n for n in names if shard_of(NS, n, 2) == 0}
    assert mine and len(mine) < len(names)
    c = WireCodecs(shard=(0, 2))
    for n in names:
        cron = {"apiVersion": "apps.kubedl.io/v1alpha1", "kind": "Cron", "metadata": {"name": n, "namespace": NS},
                "spec": {"schedule": "* * * * *", "template": {"workload": PT_TMPL}}, "status": {"history": []}}
        _, got = c.cron_event(json.dumps({"type": "MODIFIED", "object": cron}).encode())
        assert ("spec" in got and "status" in got) == (n in mine)
        job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
               "metadata": {"name": f"{n}-1", "namespace": NS, "labels": {LABEL_CRON_NAME: n}},
               "status": {"conditions": [{"type": "Succeeded", "status": "True"}]}}
        _, got = c.child_event(json.dumps({"type": "MODIFIED", "object": job}).encode())
        assert ("status" in got) == (n in mine)
        page = c.cron_list.loads(json.dumps({"kind": "List", "metadata": {}, "items": [cron]}).encode())
        assert ("spec" in page["items"][0]) == (n in mine)
    # a job without the cron-name label is routed to every shard (as without sharding)
    _, got = c.child_event(json.dumps({"type": "ADDED", "object": {"metadata": {"name": "x", "namespace": NS},
                                                                  "status": {}}}).encode())
    assert "status" in got
    assert "spec" in WireCodecs().cron_event(json.dumps({"type": "ADDED", "object": {
        "metadata": {"name": next(n for n in names if n not in mine)}, "spec": {}}}).encode())[1]


async def test_hash_routed_shards_over_http_fire_every_cron_once():
    """Two hash-routed shards against the HTTP apiserver (route-path decoders + keep-filtered
    informers): every Cron fires once per tick, by its own shard, and each shard caches only
    its own Crons and jobs."""
    from cron_operator_amd.apiserver.http import APIServerApp
    from cron_operator_amd.runtime.client import Client
    from cron_operator_amd.runtime.controller import shard_of
    from cron_operator_amd.runtime.http import HttpTransport
    from cron_operator_amd.runtime.kubeconfig import RestConfig

    env = TestEnv()
    names = [f"h{i}" for i in range(8)]
    for n in names:
        await env.create_cron(new_cron(n, NS, "*/1 * * * *", PT_TMPL, history_limit=2))
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    clients, mgrs, recs, tasks = [], [], [], []
    try:
        for idx in range(2):
            client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)
            mgr = Manager(client, ManagerOptions(clock=env.clock, health_probe_bind_address="0",
                                                 metrics_bind_address="0", shard_index=idx, shard_count=2,
                                                 shard_routing="hash"))
            _, rec = await setup_with_manager(mgr, ReconcilerOptions())
            clients.append(client)
            mgrs.append(mgr)
            recs.append(rec)
            tasks.append(asyncio.get_running_loop().create_task(mgr.start()))
        for mgr in mgrs:
            await asyncio.wait_for(mgr.started.wait(), 20)
        env.clock.advance(60)
        await _until(lambda: len(env.server.list(PT, NS)["items"]) == len(names), "a job per Cron")
        await asyncio.sleep(0.2)  # a second CREATE would show up by now
        jobs = env.server.list(PT, NS)["items"]
        assert sorted(j["metadata"]["labels"][LABEL_CRON_NAME] for j in jobs) == sorted(names)
        for idx, rec in enumerate(recs):
            mine = {n for n in names if shard_of(NS, n, 2) == idx}
            await _until(lambda r=rec, m=mine: {o["metadata"]["labels"][LABEL_CRON_NAME] for inf in
                                                r.child_informers.values() for o in inf.store.values()} == m,
                         f"shard {idx}'s jobs cached")
            assert {o["metadata"]["name"] for o in rec.cron_informer.store.values()} == mine
            assert rec.codecs is not None
    finally:
        for mgr in mgrs:
            mgr.stop()
        await asyncio.wait(set(tasks), timeout=10)
        for client in clients:
            await client.close()
        await app.stop()
