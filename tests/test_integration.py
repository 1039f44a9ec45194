"""Manager-level integration: the controller running against the fake apiserver
through informers, the work queue and timers, over many virtual minutes.

Covers the BASELINE.json configs at small scale (PyTorchJob Forbid + historyLimit,
TFJob Replace + deadline, suspend/resume cycle, Pod template), the no-duplicate
guarantee under many workers and duplicated events, fail-over via
leader election with deterministic names, and both reconciler modes.
"""
from __future__ import annotations

import asyncio

import pytest

from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.api.v1alpha1 import CRON_GVR, LABEL_CRON_NAME, new_cron
from cron_operator_amd.controller.reconciler import ReconcilerOptions
from cron_operator_amd.testing.env import TestEnv
from cron_operator_amd.trainingop.operator import FakeTrainingOperator
from cron_operator_amd.utils.clock import FakeClock
from cron_operator_amd.utils.gotime import UTC, GoTime

PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
TF = GroupVersionResource("kubeflow.org", "v1", "tfjobs")
PODS = GroupVersionResource("", "v1", "pods")
NS = "default"

PT_TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}, "Worker": {"replicas": 1}}}}
TF_TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob",
           "spec": {"tfReplicaSpecs": {"PS": {"replicas": 1}, "Worker": {"replicas": 2}}}}

MODES = {"optimized": ReconcilerOptions(), "reference": ReconcilerOptions.reference()}


async def _quiesce(env, ctrls, timeout: float = 15.0) -> None:
    """Wait until every controller's queue is idle, its shard assigner has nothing pending and
    no watch event is in flight, for a stretch of consecutive polls (a fixed sleep is too
    short on a loaded CI host)."""
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    stable = 0
    while loop.time() < end:
        await asyncio.sleep(0.002)
        if env._watches_drained() and all(c.queue.idle() for c in ctrls) and all(
                c.reconciler.shard_assigner is None or not c.reconciler.shard_assigner.pending() for c in ctrls):
            stable += 1
            if stable >= 25:
                return
        else:
            stable = 0
    raise TimeoutError("controllers did not go idle")


def names(server, gvr, cron):
    items = server.list(gvr, NS, label_selector=f"{LABEL_CRON_NAME}={cron}")["items"]
    return sorted(o["metadata"]["name"] for o in items)


@pytest.mark.parametrize("mode", MODES)
async def test_pytorchjob_forbid_history_limit(mode):
    env = TestEnv()
    trainer = FakeTrainingOperator(env.new_client(), env.clock, mode="timed", duration=90)
    await trainer.start()
    await env.create_cron(new_cron("pt", NS, "*/1 * * * *", PT_TMPL, concurrency_policy="Forbid", history_limit=3))
    await env.start_manager(MODES[mode])
    await env.settle()
    created = []
    for _ in range(12):
        await env.advance(30)
        for n in names(env.server, PT, "pt"):
            if n not in created:
                created.append(n)
        active = [o for o in env.server.list(PT, NS)["items"] if not (o.get("status") or {}).get("completionTime")]
        assert len(active) <= 1  # Forbid: never two running jobs
    st = env.server.get(CRON_GVR, NS, "pt")["status"]
    assert len(created) >= 3
    assert len(st.get("history") or []) <= 3
    assert len(names(env.server, PT, "pt")) <= 4  # history limit GC (3 finished + at most 1 running)
    await trainer.stop()
    await env.stop()


@pytest.mark.parametrize("mode", MODES)
async def test_tfjob_replace_and_deadline(mode):
    env = TestEnv()
    start = env.clock.now(UTC)
    deadline = GoTime(start.sec + 5 * 60, 0, UTC)
    await env.create_cron(new_cron("tf", NS, "*/1 * * * *", TF_TMPL, concurrency_policy="Replace",
                                   deadline=deadline))
    await env.start_manager(MODES[mode])
    await env.settle()
    seen = set()
    for _ in range(9):
        await env.advance(60)
        cur = names(env.server, TF, "tf")
        assert len(cur) <= 1  # Replace: the previous run is deleted first
        seen.update(cur)
    assert 4 <= len(seen) <= 5  # only ticks before the deadline fired
    await env.stop()


@pytest.mark.parametrize("mode", MODES)
async def test_suspend_resume_collapses_missed_runs(mode):
    env = TestEnv()
    await env.create_cron(new_cron("s", NS, "*/1 * * * *", PT_TMPL))
    await env.start_manager(MODES[mode])
    await env.settle()
    await env.advance(60)
    assert len(names(env.server, PT, "s")) == 1
    env.server.patch(CRON_GVR, NS, "s", {"spec": {"suspend": True}})
    await env.settle()
    for _ in range(5):
        await env.advance(60)
    assert len(names(env.server, PT, "s")) == 1
    env.server.patch(CRON_GVR, NS, "s", {"spec": {"suspend": False}})
    await env.settle()
    assert len(names(env.server, PT, "s")) == 2  # one immediate run for all missed ticks
    await env.advance(60)
    assert len(names(env.server, PT, "s")) == 3
    await env.stop()


@pytest.mark.timeout(300)
async def test_mi355x_ddp_example_suspend_resume_cycle_cpu():
    """BASELINE config 5 with the real example Cron (examples/mi355x): its torchrun DDP job
    runs for real (2 gloo ranks on CPU here, RCCL on the GPU box -- tests/test_gpu.py), then
    a suspend/resume cycle collapses the missed ticks into one more run."""
    from cron_operator_amd.bench.ddp_cycle import run_ddp_cycle

    res = await run_ddp_cycle(2, cpu=True, timeout=240)
    assert [s for _, s in res["history"]] == ["Succeeded", "Succeeded"] and res["active"] == 0
    assert all(codes == [0] for codes in res["exit_codes"].values())
    assert all(r["world"] == 2 for r in res["ddp"].values())


@pytest.mark.timeout(400)
async def test_mi355x_ddp_8_replica_cron_suspend_resume_cycle_cpu():
    """BASELINE config 5 as written: the Master + 7 Worker example PyTorchJob
    (examples/mi355x/cron-pytorch-ddp-8worker-mi355x.yaml, the reference examples' replica
    topology).  The fake training-operator starts 8 replica processes with the PyTorchJob
    env (WORLD_SIZE=8, RANK 0..7); they train with DDP over gloo here, in sync, each on its
    own rank, through a suspend/resume cycle."""
    from cron_operator_amd.bench.ddp_cycle import run_ddp_cycle

    res = await run_ddp_cycle(8, cpu=True, timeout=300, topology="replicas")
    assert [s for _, s in res["history"]] == ["Succeeded", "Succeeded"] and res["active"] == 0
    assert all(codes == [0] * 8 for codes in res["exit_codes"].values()), res["exit_codes"]
    for job, rep in res["ddp"].items():
        assert rep["world"] == 8 and rep["backend"] == "gloo", (job, rep)
        assert rep["devices"] == [f"cpu:{r}" for r in range(8)], rep


async def test_pod_template_busybox_config():
    # BASELINE config 1: a Cron spawning a no-op busybox Pod (core group; optimized mode only)
    env = TestEnv()
    pod = {"apiVersion": "v1", "kind": "Pod", "spec": {"containers": [{"name": "b", "image": "busybox",
                                                                       "command": ["true"]}]}}
    await env.create_cron(new_cron("pod", NS, "*/1 * * * *", pod, history_limit=1))
    await env.start_manager()
    await env.settle()
    await env.advance(60)
    pods = names(env.server, PODS, "pod")
    assert len(pods) == 1
    env.server.patch(PODS, NS, pods[0], {"status": {"phase": "Succeeded"}}, "merge", "status")
    await env.settle()
    hist = env.server.get(CRON_GVR, NS, "pod")["status"]["history"]
    assert hist[0]["status"] == "Succeeded"
    await env.advance(60)
    pods = names(env.server, PODS, "pod")
    assert len(pods) == 2  # one finished (kept by historyLimit=1) + the new active one
    env.server.patch(PODS, NS, pods[1], {"status": {"phase": "Failed"}}, "merge", "status")
    await env.settle()
    assert names(env.server, PODS, "pod") == [pods[1]]  # the older finished pod is GC'd
    hist = env.server.get(CRON_GVR, NS, "pod")["status"]["history"]
    assert [(h["object"]["name"], h["status"]) for h in hist] == [(pods[1], "Failed")]
    await env.stop()


@pytest.mark.parametrize("mode", MODES)
async def test_no_duplicate_creates_under_concurrency(mode):
    """Many workers, many Crons, event storms: exactly one job per Cron per tick."""
    env = TestEnv()
    n = 40
    for i in range(n):
        await env.create_cron(new_cron(f"c{i}", NS, "*/1 * * * *", PT_TMPL))
    await env.start_manager(MODES[mode], max_concurrent=32)
    await env.settle()
    for tick in range(1, 4):
        env.clock.advance(60)
        # storm: re-enqueue every cron repeatedly while the tick is being processed
        for _ in range(5):
            for i in range(n):
                env.controller.queue.add(env.controller.queue.__class__ and
                                         __import__("cron_operator_amd.runtime.controller",
                                                    fromlist=["Request"]).Request(NS, f"c{i}"))
            await asyncio.sleep(0)
        await env.settle()
        for i in range(n):
            assert len(names(env.server, PT, f"c{i}")) == tick, f"c{i} at tick {tick}"
    await env.stop()


async def test_failover_no_duplicates_with_deterministic_names():
    """Operator A creates the job and dies before writing status; B takes over and
    must not create a second job for the same tick (AlreadyExists == success)."""
    env = TestEnv()
    await env.create_cron(new_cron("f", NS, "*/1 * * * *", PT_TMPL))
    # A: the status patch always fails -> lastScheduleTime never advances
    env.server.faults.add(verb="patch", resource="crons", subresource="status", code=500)
    await env.start_manager()
    await env.settle()
    env.clock.advance(60)
    for _ in range(20):
        await asyncio.sleep(0.001)
    assert len(names(env.server, PT, "f")) == 1
    await env.stop()
    env.server.faults.clear()
    # B: a fresh manager on the same cluster, same virtual minute
    env2 = TestEnv.__new__(TestEnv)
    env2.__dict__.update(env.__dict__)
    env2.manager = env2.controller = env2.reconciler = env2._mgr_task = None
    await env2.start_manager()
    await env2.settle()
    assert len(names(env2.server, PT, "f")) == 1
    st = env2.server.get(CRON_GVR, NS, "f")["status"]
    assert st.get("lastScheduleTime")
    await env2.stop()


async def test_manager_leader_election_single_active():
    clock = FakeClock(1767268805 * 10**9)
    env = TestEnv(clock=clock)
    await env.create_cron(new_cron("le", NS, "*/1 * * * *", PT_TMPL))
    await env.start_manager(leader_election=True, leader_election_namespace=NS, leader_election_identity="a")
    from cron_operator_amd.controller.setup import setup_with_manager
    from cron_operator_amd.runtime.manager import Manager, ManagerOptions

    standby = Manager(env.new_client(), ManagerOptions(clock=clock, leader_election=True,
                                                       leader_election_namespace=NS,
                                                       leader_election_identity="b",
                                                       health_probe_bind_address="0"))
    await setup_with_manager(standby)
    t = asyncio.get_running_loop().create_task(standby.start())
    for _ in range(20):
        await asyncio.sleep(0.001)
    assert env.manager.elected.is_set() and not standby.elected.is_set()
    await env.advance(60)
    assert len(names(env.server, PT, "le")) == 1
    standby.stop()
    await asyncio.wait_for(t, 10)
    await env.stop()


@pytest.mark.parametrize("routing", ["hash", "labels"])
async def test_horizontal_sharding_splits_crons_and_leases(routing):
    """Two replicas with --shard-count 2: every Cron fires exactly once per tick, each shard only
    reconciles its own Crons, and each shard elects its own leader Lease.  With label routing
    each shard also caches only its own Crons and children, all labelled with their shard; with
    hash routing it stores only its own share of what it watches."""
    from cron_operator_amd.api.meta import GroupVersionResource as GVR
    from cron_operator_amd.controller.setup import setup_with_manager
    from cron_operator_amd.runtime.controller import shard_of
    from cron_operator_amd.runtime.manager import Manager, ManagerOptions

    clock = FakeClock(1767268805 * 10**9)
    env = TestEnv(clock=clock)
    n = 24
    for i in range(n):
        await env.create_cron(new_cron(f"s{i}", NS, "*/1 * * * *", PT_TMPL))
    owners = {0: set(), 1: set()}
    for i in range(n):
        owners[shard_of(NS, f"s{i}", 2)].add(f"s{i}")
    assert owners[0] and owners[1]  # the hash spreads the keys

    mgrs, ctrls, tasks = [], [], []
    for idx in (0, 1):
        m = Manager(env.new_client(), ManagerOptions(clock=clock, leader_election=True, leader_election_namespace=NS,
                                                     leader_election_identity=f"r{idx}", shard_index=idx,
                                                     shard_count=2, health_probe_bind_address="0",
                                                     metrics_bind_address="0", shard_routing=routing))
        ctrl, _ = await setup_with_manager(m)
        mgrs.append(m)
        ctrls.append(ctrl)
        tasks.append(asyncio.get_running_loop().create_task(m.start()))
    for m in mgrs:
        await asyncio.wait_for(m.started.wait(), 10)
    seen = {0: set(), 1: set()}
    for idx, c in enumerate(ctrls):
        orig = c.reconciler.reconcile

        async def spy(req, log, _orig=orig, _idx=idx):
            seen[_idx].add(req.name)
            return await _orig(req, log)
        c.reconciler.reconcile = spy
    for _ in range(2):
        for _ in range(60):
            clock.advance(1)
            await asyncio.sleep(0.001)
        await _quiesce(env, ctrls)
    for i in range(n):
        assert len(names(env.server, PT, f"s{i}")) == 2, f"s{i}"
    assert seen[0] <= owners[0] and seen[1] <= owners[1]
    leases = {o["metadata"]["name"] for o in env.server.list(GVR("coordination.k8s.io", "v1", "leases"), NS)["items"]}
    assert {"619a52b8.kubedl.io-shard-0", "619a52b8.kubedl.io-shard-1"} <= leases
    for idx, c in enumerate(ctrls):
        rec = c.reconciler
        assert {o["metadata"]["name"] for o in rec.cron_informer.store.values()} == owners[idx]
        assert {o["metadata"]["labels"][LABEL_CRON_NAME]
                for inf in rec.child_informers.values() for o in inf.store.values()} == owners[idx]
    if routing == "labels":
        from cron_operator_amd.controller.sharding import LABEL_SHARD

        for o in env.server.list(CRON_GVR, NS)["items"]:
            assert o["metadata"]["labels"][LABEL_SHARD] == f"{shard_of(NS, o['metadata']['name'], 2)}-of-2"
        for o in env.server.list(PT, NS)["items"]:
            cron = o["metadata"]["labels"][LABEL_CRON_NAME]
            assert o["metadata"]["labels"][LABEL_SHARD] == f"{shard_of(NS, cron, 2)}-of-2"
    for m in mgrs:
        m.stop()
    for t in tasks:
        try:
            await asyncio.wait_for(t, 10)
        except Exception:  # noqa: BLE001
            pass
    env.server.close_all_watches()


def test_shard_of_is_stable_and_balanced():
    from cron_operator_amd.runtime.controller import shard_of

    assert shard_of("default", "a", 1) == 0
    assert shard_of("default", "nightly", 4) == shard_of("default", "nightly", 4)
    counts = [0] * 4
    for i in range(4000):
        counts[shard_of("ns", f"cron-{i}", 4)] += 1
    assert min(counts) > 800


async def test_label_routing_reshard_relabels_crons_and_children():
    """Label routing, 2 shards then 3: the new shards relabel every Cron and every existing child
    (<i>-of-3) and keep firing each Cron exactly once per tick, with history intact."""
    from cron_operator_amd.controller.setup import setup_with_manager
    from cron_operator_amd.controller.sharding import LABEL_SHARD
    from cron_operator_amd.runtime.controller import shard_of
    from cron_operator_amd.runtime.manager import Manager, ManagerOptions

    clock = FakeClock(1767268805 * 10**9)
    env = TestEnv(clock=clock)
    trainer = FakeTrainingOperator(env.new_client(), clock, mode="timed", duration=30)
    await trainer.start()
    n = 12
    for i in range(n):
        await env.create_cron(new_cron(f"r{i}", NS, "*/1 * * * *", PT_TMPL, history_limit=5))

    async def run_shards(count, minutes):
        mgrs, tasks, ctrls = [], [], []
        for idx in range(count):
            m = Manager(env.new_client(), ManagerOptions(clock=clock, shard_index=idx, shard_count=count,
                                                         shard_routing="labels", health_probe_bind_address="0",
                                                         metrics_bind_address="0"))
            ctrls.append((await setup_with_manager(m))[0])
            mgrs.append(m)
            tasks.append(asyncio.get_running_loop().create_task(m.start()))
        for m in mgrs:
            await asyncio.wait_for(m.started.wait(), 10)
        await _quiesce(env, ctrls)
        for _ in range(minutes):
            for _ in range(60):
                clock.advance(1)
                await asyncio.sleep(0.001)
            await _quiesce(env, ctrls)
        for m in mgrs:
            m.stop()
        for t in tasks:
            await asyncio.wait_for(t, 10)

    await run_shards(2, 2)
    first = {}
    for i in range(n):
        first[i] = names(env.server, PT, f"r{i}")
        assert len(first[i]) == 2, f"r{i}"
    await run_shards(3, 2)
    for i in range(n):
        assert len(names(env.server, PT, f"r{i}")) == 4, f"r{i}"  # one per tick, none duplicated
        st = env.server.get(CRON_GVR, NS, f"r{i}")["status"]
        hist = {h["object"]["name"] for h in st.get("history") or []}
        assert set(first[i]) <= hist, f"r{i}"  # children made under 2 shards are still seen
    for o in env.server.list(CRON_GVR, NS)["items"]:
        assert o["metadata"]["labels"][LABEL_SHARD] == f"{shard_of(NS, o['metadata']['name'], 3)}-of-3"
    for o in env.server.list(PT, NS)["items"]:
        cron = o["metadata"]["labels"][LABEL_CRON_NAME]
        assert o["metadata"]["labels"][LABEL_SHARD] == f"{shard_of(NS, cron, 3)}-of-3"
    await trainer.stop()
    env.server.close_all_watches()


async def test_memos_dropped_when_crons_and_children_go_away():
    """Per-Cron memos (own writes, parsed status, expectations) and per-child memos are dropped
    when the Cron or the child is deleted, so a churning fleet does not grow them forever."""
    env = TestEnv()
    await env.create_cron(new_cron("m", NS, "*/1 * * * *", PT_TMPL))
    await env.start_manager()
    await env.settle()
    await env.advance(60)
    rec = env.reconciler
    job = names(env.server, PT, "m")[0]
    env.server.patch(PT, NS, job, {"status": {"conditions": [{"type": "Succeeded", "status": "True"}]}},
                     "merge", "status")
    await env.settle()
    uid = env.server.get(PT, NS, job)["metadata"]["uid"]
    # per-child memos live beside the cached object in the child informer (Informer.derive)
    inf = next(i for g, i in rec.child_informers.items() if g.kind == "PyTorchJob")
    assert inf.derived[f"{NS}/{job}"].uid == uid
    assert f"{NS}/m" in rec.own_writes and f"{NS}/m" in rec._parsed_status
    env.server.delete(PT, NS, job)
    await env.settle()
    assert f"{NS}/{job}" not in inf.derived and uid not in rec._class_cache
    env.server.delete(CRON_GVR, NS, "m")
    await env.settle()
    assert f"{NS}/m" not in rec.own_writes and f"{NS}/m" not in rec._parsed_status
    assert f"{NS}/m" not in rec.expect.created and f"{NS}/m" not in rec.expect.deleted
    await env.stop()


async def test_shard_assignment_watches_cache_metadata_only():
    """Before assignment the "unassigned" watch sees the whole fleet: it stores only this
    shard's share, and of that only names, labels, uid and resourceVersion, so a shard's
    memory follows its own share."""
    from cron_operator_amd.controller.sharding import ShardAssigner, shard_of

    env = TestEnv()
    for i in range(6):
        await env.create_cron(new_cron(f"u{i}", NS, "*/1 * * * *", PT_TMPL, history_limit=3))
    env.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "u0-1", "labels": {LABEL_CRON_NAME: "u0"}},
                               "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}})
    from cron_operator_amd.api.meta import GroupVersionKind
    from cron_operator_amd.runtime.informer import Cache

    cache = Cache(env.new_client(), NS)
    asg = ShardAssigner(env.new_client(), 0, 2)
    crons = await asg.watch(cache, GroupVersionKind("apps.kubedl.io", "v1alpha1", "Cron"), child=False)
    jobs = await asg.watch(cache, GroupVersionKind("kubeflow.org", "v1", "PyTorchJob"), child=True)
    cache.start()
    assert await cache.wait_for_sync(10)
    mine = {f"{NS}/u{i}" for i in range(6) if shard_of(NS, f"u{i}", 2) == 0}
    assert 0 < len(mine) < 6  # the names split over both shards
    assert set(crons.store) == mine
    assert len(jobs.store) == (f"{NS}/u0" in mine)  # a child follows its Cron's shard
    for o in list(crons.store.values()) + list(jobs.store.values()):
        assert set(o) == {"apiVersion", "kind", "metadata"}
        assert set(o["metadata"]) <= {"name", "namespace", "uid", "resourceVersion", "labels"}
    assert asg.pending() > 0  # and the shard's own objects are queued for labelling
    await cache.stop()


async def test_shard_assigner_holds_background_watch_tasks():
    """``watch_soon`` (used for child kinds discovered at run time) keeps its task alive until
    it finishes: the event loop only holds tasks weakly."""
    import gc

    from cron_operator_amd.api.meta import GroupVersionKind
    from cron_operator_amd.controller.sharding import ShardAssigner
    from cron_operator_amd.runtime.informer import Cache

    env = TestEnv()
    cache = Cache(env.new_client(), NS)
    asg = ShardAssigner(env.new_client(), 0, 2)
    gvk = GroupVersionKind("kubeflow.org", "v1", "PyTorchJob")
    asg.watch_soon(cache, gvk, child=True)  # result deliberately dropped
    assert len(asg._bg) == 1
    gc.collect()
    task = next(iter(asg._bg))
    inf = await task
    await asyncio.sleep(0)
    assert not asg._bg and asg.informers[gvk] is inf
    await cache.stop()


async def test_upgrade_from_hash_to_label_routing_keeps_running_children_in_view():
    """a hash-routed sharded fleet with running jobs restarts with label routing.
    Every object is unlabelled then; the child label PATCHes are slow (0.2 s each).  A Cron
    must not join its shard's informer before its running child does: under Forbid no second
    job may start while the first runs, and status.active never drops the running job."""
    from cron_operator_amd.controller.setup import setup_with_manager
    from cron_operator_amd.controller.sharding import LABEL_SHARD
    from cron_operator_amd.runtime.client import Client, InMemoryTransport
    from cron_operator_amd.runtime.manager import Manager, ManagerOptions

    clock = FakeClock(1767268805 * 10**9)
    env = TestEnv(clock=clock)
    n = 8
    for i in range(n):
        await env.create_cron(new_cron(f"u{i}", NS, "*/1 * * * *", PT_TMPL, concurrency_policy="Forbid"))

    class SlowChildLabels(InMemoryTransport):
        async def request(self, verb, gvr, namespace="", name="", subresource="", body=None, params=None):
            if verb == "patch" and gvr.resource == "pytorchjobs" and not subresource:
                await asyncio.sleep(0.2)  # the shard assigner's label PATCH of a child
            return await super().request(verb, gvr, namespace, name, subresource, body, params)

    async def run(routing, minutes, slow=False):
        mgrs, tasks, ctrls = [], [], []
        for idx in range(2):
            client = Client(SlowChildLabels(env.server) if slow else InMemoryTransport(env.server), qps=-1)
            m = Manager(client, ManagerOptions(clock=clock, shard_index=idx, shard_count=2, shard_routing=routing,
                                               health_probe_bind_address="0", metrics_bind_address="0"))
            ctrls.append((await setup_with_manager(m))[0])
            mgrs.append(m)
            tasks.append(asyncio.get_running_loop().create_task(m.start()))
        for m in mgrs:
            await asyncio.wait_for(m.started.wait(), 10)
        actives = []
        for _ in range(minutes):
            for _ in range(60):
                clock.advance(1)
                await asyncio.sleep(0.001)
                for i in range(n):
                    st = env.server.get(CRON_GVR, NS, f"u{i}").get("status") or {}
                    actives.append((i, len(st.get("active") or [])))
            await _quiesce(env, ctrls)
        for m in mgrs:
            m.stop()
        for t in tasks:
            await asyncio.wait_for(t, 10)
        return actives

    await run("hash", 1)  # the first tick: one running job per Cron (nothing completes them)
    first = {i: names(env.server, PT, f"u{i}") for i in range(n)}
    assert all(len(v) == 1 for v in first.values()), first
    actives = await run("labels", 2, slow=True)
    for i in range(n):
        assert names(env.server, PT, f"u{i}") == first[i], f"u{i}: Forbid violated after the routing change"
    # from the moment the job exists its Cron lists it as active, through the relabelling
    assert all(k == 1 for _, k in actives), [x for x in actives if x[1] != 1][:5]
    for o in env.server.list(PT, NS)["items"] + env.server.list(CRON_GVR, NS)["items"]:
        assert LABEL_SHARD in o["metadata"]["labels"]
    env.server.close_all_watches()


async def test_shard_assigner_shutdown_leaves_no_label_patch_in_flight():
    """Stopping the assigner (leader loss, shutdown) cancels its workers *and waits for them*:
    once ``run`` has returned, no label PATCH is still running or lands later."""
    from cron_operator_amd.api.v1alpha1 import CRON_GVK
    from cron_operator_amd.controller.sharding import LABEL_SHARD, ShardAssigner
    from cron_operator_amd.runtime.informer import Cache

    env = TestEnv()
    for i in range(6):
        await env.create_cron(new_cron(f"a{i}", NS, "*/1 * * * *", PT_TMPL))
    client = env.new_client()
    started, finished = [], []
    orig = client.patch

    async def slow_patch(gvk, ns, name, *a, **kw):
        started.append(name)
        await asyncio.sleep(0.3)  # a label PATCH the apiserver holds
        out = await orig(gvk, ns, name, *a, **kw)
        finished.append(name)
        return out

    client.patch = slow_patch  # type: ignore[assignment]
    cache = Cache(env.new_client(), NS)
    asg = ShardAssigner(client, 0, 1)
    await asg.watch(cache, CRON_GVK, child=False)
    cache.start()
    task = asyncio.get_running_loop().create_task(asg.run())
    for _ in range(200):
        if started:
            break
        await asyncio.sleep(0.005)
    assert started, "no label PATCH started"
    task.cancel()
    await asyncio.gather(task, return_exceptions=True)
    in_flight = [t for t in asyncio.all_tasks() if "_worker" in repr(t.get_coro()) and not t.done()]
    assert in_flight == []
    n = len(finished)
    await asyncio.sleep(0.5)  # nothing lands after run() returned
    assert len(finished) == n
    labelled = [o for o in env.server.list(CRON_GVR, NS)["items"] if LABEL_SHARD in (o["metadata"].get("labels") or {})]
    assert len(labelled) == n
    await cache.stop()


async def test_reference_mode_with_label_sharding_assigns_crons_without_waiting():
    """in live-list mode (``--compat-mode reference``) there are no child informers;
    a Cron with relabelled children must not wait ``observe_timeout`` for an informer that
    will never hold them."""
    import time

    from cron_operator_amd.controller.reconciler import ReconcilerOptions
    from cron_operator_amd.controller.setup import setup_with_manager
    from cron_operator_amd.controller.sharding import LABEL_SHARD
    from cron_operator_amd.runtime.manager import Manager, ManagerOptions

    env = TestEnv()
    n = 8
    for i in range(n):
        await env.create_cron(new_cron(f"l{i}", NS, "*/1 * * * *", PT_TMPL))
        env.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                   "metadata": {"name": f"l{i}-1", "labels": {LABEL_CRON_NAME: f"l{i}"}},
                                   "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}})
    mgrs, tasks = [], []
    t0 = time.monotonic()
    for idx in range(2):
        m = Manager(env.new_client(), ManagerOptions(clock=env.clock, shard_index=idx, shard_count=2,
                                                     shard_routing="labels", health_probe_bind_address="0",
                                                     metrics_bind_address="0"))
        await setup_with_manager(m, ReconcilerOptions.reference())
        mgrs.append(m)
        tasks.append(asyncio.get_running_loop().create_task(m.start()))
    try:
        while True:
            crons = env.server.list(CRON_GVR, NS)["items"]
            if all(LABEL_SHARD in (o["metadata"].get("labels") or {}) for o in crons):
                break
            assert time.monotonic() - t0 < 3.0, "Crons waited for child informers that live mode never starts"
            await asyncio.sleep(0.01)
    finally:
        for m in mgrs:
            m.stop()
        for t in tasks:
            await asyncio.wait_for(t, 10)
        env.server.close_all_watches()


async def test_shard_assigner_gives_up_a_child_it_may_not_label():
    """a child whose label PATCH keeps failing (403) is given up after
    ``max_child_attempts``: its Cron is assigned anyway instead of being parked forever."""
    from cron_operator_amd.api import errors as api_errors
    from cron_operator_amd.api.meta import GroupVersionKind
    from cron_operator_amd.api.v1alpha1 import CRON_GVK
    from cron_operator_amd.controller.sharding import LABEL_SHARD, ShardAssigner
    from cron_operator_amd.runtime.informer import Cache

    env = TestEnv()
    await env.create_cron(new_cron("f0", NS, "*/1 * * * *", PT_TMPL))
    env.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "f0-1", "labels": {LABEL_CRON_NAME: "f0"}},
                               "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}})
    client = env.new_client()
    orig = client.patch
    denied = []

    async def patch(gvk, ns, name, *a, **kw):
        if getattr(gvk, "kind", "") == "PyTorchJob" or getattr(gvk, "resource", "") == "pytorchjobs":
            denied.append(name)
            raise api_errors.ApiError(403, "Forbidden", f"pytorchjobs {name!r} is forbidden")
        return await orig(gvk, ns, name, *a, **kw)

    client.patch = patch  # type: ignore[assignment]
    cache = Cache(env.new_client(), NS)
    asg = ShardAssigner(client, 0, 1, retry_delay=0.01, max_child_attempts=3)
    await asg.watch(cache, CRON_GVK, child=False)
    await asg.watch(cache, GroupVersionKind("kubeflow.org", "v1", "PyTorchJob"), child=True)
    cache.start()
    task = asyncio.get_running_loop().create_task(asg.run())
    try:
        for _ in range(300):
            if LABEL_SHARD in (env.server.get(CRON_GVR, NS, "f0")["metadata"].get("labels") or {}):
                break
            await asyncio.sleep(0.01)
        assert LABEL_SHARD in (env.server.get(CRON_GVR, NS, "f0")["metadata"].get("labels") or {})
        assert len(denied) == 3 and asg.abandoned == 1
    finally:
        task.cancel()
        await asyncio.gather(task, return_exceptions=True)
        await cache.stop()


async def test_shard_assigner_keeps_retrying_a_child_through_transient_errors():
    """503s (and 429s) are transient -- a child whose label PATCH fails with them more
    than ``max_child_attempts`` times is NOT given up, so its Cron stays parked until the child is
    labelled (a given-up child is invisible to its shard's label-selected child informer)."""
    from cron_operator_amd.api import errors as api_errors
    from cron_operator_amd.api.meta import GroupVersionKind
    from cron_operator_amd.api.v1alpha1 import CRON_GVK
    from cron_operator_amd.controller.sharding import LABEL_SHARD, ShardAssigner, persistent_failure
    from cron_operator_amd.runtime.informer import Cache

    assert not persistent_failure(api_errors.ApiError(503, "ServiceUnavailable", "x"))
    assert not persistent_failure(api_errors.ApiError(429, "TooManyRequests", "x"))
    assert not persistent_failure(api_errors.ApiError(409, "Conflict", "x"))
    assert persistent_failure(api_errors.ApiError(403, "Forbidden", "x"))
    assert persistent_failure(api_errors.ApiError(422, "Invalid", "x"))

    env = TestEnv()
    await env.create_cron(new_cron("t0", NS, "*/1 * * * *", PT_TMPL))
    env.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                               "metadata": {"name": "t0-1", "labels": {LABEL_CRON_NAME: "t0"}},
                               "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}})
    client = env.new_client()
    orig = client.patch
    failed = []

    async def patch(gvk, ns, name, *a, **kw):
        if (getattr(gvk, "kind", "") == "PyTorchJob") and len(failed) < 8:
            failed.append(name)
            if len(failed) % 2:
                raise api_errors.ApiError(503, "ServiceUnavailable", "apiserver is shutting down")
            raise ConnectionResetError("connection reset by peer")
        return await orig(gvk, ns, name, *a, **kw)

    client.patch = patch  # type: ignore[assignment]
    cache = Cache(env.new_client(), NS)
    asg = ShardAssigner(client, 0, 1, retry_delay=0.001, max_child_attempts=3)
    asg._backoff = lambda key: 0.001  # no exponential wait in the test
    await asg.watch(cache, CRON_GVK, child=False)
    await asg.watch(cache, GroupVersionKind("kubeflow.org", "v1", "PyTorchJob"), child=True)
    cache.start()
    task = asyncio.get_running_loop().create_task(asg.run())
    try:
        for _ in range(500):
            if LABEL_SHARD in (env.server.get(CRON_GVR, NS, "t0")["metadata"].get("labels") or {}):
                break
            # parked while the child's PATCH keeps failing
            if len(failed) < 8:
                assert LABEL_SHARD not in (env.server.get(CRON_GVR, NS, "t0")["metadata"].get("labels") or {})
            await asyncio.sleep(0.01)
        assert len(failed) == 8 and asg.abandoned == 0
        assert LABEL_SHARD in (env.server.get(PT, NS, "t0-1")["metadata"].get("labels") or {})
        assert LABEL_SHARD in (env.server.get(CRON_GVR, NS, "t0")["metadata"].get("labels") or {})
    finally:
        task.cancel()
        await asyncio.gather(task, return_exceptions=True)
        await cache.stop()
