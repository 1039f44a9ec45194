"""Liveness under partial failure: one broken Cron (or a broken API path) must not stop
the others, and the operator must notice dead connections and lost leases in time.

Reference behaviour being matched:

* ``listWorkloads`` is a live LIST whose error is returned from ``Reconcile``, so the
  worker is freed and the Cron retried with the workqueue's rate-limited backoff
  (``/root/reference/internal/controller/cron_controller.go:129-133, 241-266``).
  Here children come from informers; a child informer that cannot LIST must surface
  that error the same way instead of holding the worker until it syncs.
"""
from __future__ import annotations

import asyncio
import io

from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.api.v1alpha1 import CRON_GVR, LABEL_CRON_NAME, new_cron
from cron_operator_amd.runtime.controller import Request
from cron_operator_amd.testing.env import TestEnv
from cron_operator_amd.utils.logging import get_logger, new_from_options, set_logger

PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
MPI = GroupVersionResource("kubeflow.org", "v1", "mpijobs")
NS = "default"
PT_TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}}
MPI_TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "MPIJob",
            "spec": {"mpiReplicaSpecs": {"Launcher": {"replicas": 1}, "Worker": {"replicas": 2}}}}


def jobs(env, gvr, cron):
    return sorted(o["metadata"]["name"] for o in
                  env.server.list(gvr, NS, label_selector=f"{LABEL_CRON_NAME}={cron}")["items"])


class _CapturedLog:
    """Route the root logger into a buffer for the duration of a test."""

    def __enter__(self) -> io.StringIO:
        self._prev = get_logger()
        self.buf = io.StringIO()
        set_logger(new_from_options(encoder="json", level="info", stream=self.buf))
        return self.buf

    def __exit__(self, *exc) -> None:
        set_logger(self._prev)


async def test_unlistable_kind_does_not_starve_workers():
    """Two Crons whose template kind the operator may not LIST (403) and one healthy Cron,
    with only two workers: the healthy Cron fires on every tick, the broken ones log
    ``Failed to list MPIJob`` and are retried with growing backoff (no worker is held)."""
    env = TestEnv()
    env.server.faults.add(verb="list", resource="mpijobs", code=403, reason="Forbidden",
                          message='mpijobs.kubeflow.org is forbidden: User "system:serviceaccount:cron-operator:'
                                  'cron-operator" cannot list resource "mpijobs" in API group "kubeflow.org"')
    for name in ("mpi-a", "mpi-b"):
        await env.create_cron(new_cron(name, NS, "*/1 * * * *", MPI_TMPL))
    await env.create_cron(new_cron("healthy", NS, "*/1 * * * *", PT_TMPL))
    with _CapturedLog() as buf:
        await env.start_manager(max_concurrent=2)
        await env.settle()
        for minute in range(1, 5):
            for _ in range(60):
                await env.advance(1)
            assert len(jobs(env, PT, "healthy")) == minute, f"healthy Cron missed a tick in minute {minute}"
            # nobody is parked inside a reconcile
            assert env.controller.queue.processing() == 0
        st = env.server.get(CRON_GVR, NS, "healthy").get("status") or {}
        assert st.get("lastScheduleTime")
        assert jobs(env, MPI, "mpi-a") == [] and jobs(env, MPI, "mpi-b") == []
        logged = buf.getvalue()
        await env.stop()
    assert "Failed to list MPIJob" in logged
    assert "forbidden" in logged
    # rate-limited retries: several, but backing off (far fewer than one per virtual second)
    q = env.controller.queue
    for name in ("mpi-a", "mpi-b"):
        n = q.num_requeues(Request(NS, name))
        assert n >= 3, (name, n)
    assert env.controller.errors >= 6
    assert env.controller.errors < 2 * 4 * 60 / 2


async def test_list_recovers_after_rbac_fixed():
    """Once the LIST is allowed again (RBAC fixed), the backed-off Cron fires."""
    env = TestEnv()
    fault = env.server.faults.add(verb="list", resource="mpijobs", code=403, reason="Forbidden")
    await env.create_cron(new_cron("mpi", NS, "*/1 * * * *", MPI_TMPL))
    await env.start_manager(max_concurrent=1)
    await env.settle()
    for _ in range(70):
        await env.advance(1)
    assert jobs(env, MPI, "mpi") == []
    env.server.faults.faults.remove(fault)
    # the informer retries with up to 30 s (real time) backoff; the test drives the
    # retry by waiting for the informer, then the Cron's own backoff by virtual time
    inf = next(i for g, i in env.reconciler.child_informers.items() if g.kind == "MPIJob")
    await asyncio.wait_for(inf.synced.wait(), 40)
    for _ in range(120):
        await env.advance(1)
        if jobs(env, MPI, "mpi"):
            break
    assert jobs(env, MPI, "mpi"), "Cron did not fire after the LIST became allowed"
    await env.stop()


async def test_slow_child_sync_falls_back_to_live_list():
    """A child informer whose first LIST hangs: after ``child_sync_timeout`` the reconcile
    LISTs the Cron's children live (the reference's path) and the tick still fires."""
    from cron_operator_amd.controller.reconciler import ReconcilerOptions

    env = TestEnv()
    orig_list_all = env.client.list_all
    gate = asyncio.Event()

    async def slow_list_all(target, *a, **kw):
        if "mpijobs" in str(target):
            await gate.wait()
        return await orig_list_all(target, *a, **kw)

    env.client.list_all = slow_list_all  # type: ignore[assignment]
    await env.create_cron(new_cron("mpi", NS, "*/1 * * * *", MPI_TMPL))
    opts = ReconcilerOptions(child_sync_timeout=0.05)
    await env.start_manager(opts, max_concurrent=1)
    for _ in range(60):
        await env.advance(1)
    assert len(jobs(env, MPI, "mpi")) == 1
    gate.set()
    await env.stop()


# ---------------------------------------------------------------- leader election (client-go semantics)


async def test_follower_clock_skew_cannot_steal_a_renewed_lease():
    """A follower whose clock runs 30 s ahead never takes a lease the leader keeps renewing
    (expiry is judged from *local* observation time, client-go ``observedTime``); once the
    leader stops, the follower takes over after one lease duration of its own time."""
    from cron_operator_amd.parallel.leaderelection import LEASES, LeaderElector
    from cron_operator_amd.utils.clock import FakeClock

    t0 = 1_800_000_000 * 10**9
    ca, cb = FakeClock(t0), FakeClock(t0 + 30 * 10**9)
    env = TestEnv(clock=ca)
    a = LeaderElector(env.new_client(), "619a52b8.kubedl.io", NS, "a", ca, 15, 10, 2)
    b = LeaderElector(env.new_client(), "619a52b8.kubedl.io", NS, "b", cb, 15, 10, 2)
    assert await a.try_acquire_or_renew()
    for _ in range(30):  # a minute of renewals every retryPeriod
        ca.advance(2)
        cb.advance(2)
        assert await a.try_acquire_or_renew()
        assert not await b.try_acquire_or_renew(), "skewed follower stole a live lease"
    assert env.server.get(LEASES, NS, "619a52b8.kubedl.io")["spec"]["holderIdentity"] == "a"
    # the leader dies; the follower keeps polling
    took = None
    for step in range(1, 15):
        ca.advance(2)
        cb.advance(2)
        if await b.try_acquire_or_renew():
            took = 2 * step
            break
    assert took is not None and 15 <= took <= 18, took
    spec = env.server.get(LEASES, NS, "619a52b8.kubedl.io")["spec"]
    assert spec["holderIdentity"] == "b" and spec["leaseTransitions"] == 1


async def test_leader_steps_down_within_renew_deadline_when_lease_updates_hang():
    """Lease PUTs hang (an apiserver that stopped answering): the leader must stop its
    controllers within ``renewDeadline`` of the renewal that hangs -- not after the
    transport's 60 s timeout -- so it never reconciles past its lease."""
    from cron_operator_amd.parallel.leaderelection import LEASES
    from cron_operator_amd.runtime.manager import LeaderElectionLost

    env = TestEnv()
    await env.create_cron(new_cron("pt", NS, "*/1 * * * *", PT_TMPL))
    await env.start_manager(leader_election=True, leader_election_namespace=NS, leader_election_identity="me",
                            lease_duration=15, renew_deadline=10, retry_period=2)
    await env.settle()
    assert env.manager.elector is not None and env.manager.elector.is_leader
    for _ in range(10):  # healthy renewals
        await env.advance(1)
    renew_time = env.server.get(LEASES, NS, "619a52b8.kubedl.io")["spec"]["renewTime"]
    hang = asyncio.Event()
    lease_client = env.manager.lease_client  # the elector's own client (Client.derive)
    assert lease_client is not None and lease_client is not env.client
    orig_update = lease_client.update

    async def hung_update(target, obj, *a, **kw):
        if target == LEASES:
            await hang.wait()
        return await orig_update(target, obj, *a, **kw)

    lease_client.update = hung_update  # type: ignore[assignment]
    stopped_after = None
    for sec in range(1, 30):
        env.clock.advance(1)
        # shutdown (workers, informers, broadcaster) waits for every cancelled task to end:
        # give it enough loop turns within one virtual second
        for _ in range(200):
            await asyncio.sleep(0)
        if env._mgr_task.done():
            stopped_after = sec
            break
    assert stopped_after is not None, "leader kept running with hung lease renewals"
    # next renewal starts within retryPeriod (2 s), its window closes renewDeadline (10 s) later
    assert stopped_after <= 2 + 10, stopped_after
    assert isinstance(env._mgr_task.exception(), LeaderElectionLost)
    assert not env.controller.started
    assert env.server.get(LEASES, NS, "619a52b8.kubedl.io")["spec"]["renewTime"] == renew_time
    hang.set()


# ---------------------------------------------------------------- watch liveness


async def test_silently_stalled_child_watch_is_reestablished_and_cron_converges():
    """The apiserver stops writing to the PyTorchJob watch without closing it (a half-open
    connection).  A Forbid Cron's running job then finishes: the operator cannot see it
    until the idle watchdog drops the silent stream and resumes the watch -- after which
    the job's completion arrives and the next tick fires."""
    from cron_operator_amd.trainingop.operator import finished_status
    from cron_operator_amd.utils.gotime import NANOS, UTC, GoTime

    env = TestEnv()
    await env.create_cron(new_cron("pt", NS, "*/1 * * * *", PT_TMPL, concurrency_policy="Forbid"))
    await env.start_manager(watch_idle_timeout=0.3)
    await env.settle()
    for _ in range(60):
        await env.advance(1)
    assert len(jobs(env, PT, "pt")) == 1
    inf = next(i for g, i in env.reconciler.child_informers.items() if g.kind == "PyTorchJob")
    assert env.server.stall_watches("pytorchjobs") >= 1
    job = jobs(env, PT, "pt")[0]
    ts = GoTime(env.clock.now_ns() // NANOS, 0, UTC).rfc3339()
    env.server.patch(PT, NS, job, {"status": finished_status("PyTorchJob", job, ts, True)}, "merge", "status")
    for _ in range(60):  # next tick: the operator still believes the job runs (Forbid)
        await env.advance(1)
    assert len(jobs(env, PT, "pt")) == 1
    # real time passes: the watchdog notices the silence and the watch resumes
    for _ in range(100):
        await asyncio.sleep(0.05)
        if inf.idle_timeouts:
            break
    assert inf.idle_timeouts >= 1
    await env.settle()
    for _ in range(60):
        await env.advance(1)
    assert len(jobs(env, PT, "pt")) == 2, "Cron did not converge after the watch was re-established"
    st = env.server.get(CRON_GVR, NS, "pt")["status"]
    assert [h["object"]["name"] for h in st.get("history") or []] == [job]
    await env.stop()


async def test_http_watch_carries_timeout_and_survives_a_silent_connection():
    """Over real HTTP: the informer's WATCH asks for ``timeoutSeconds`` in [300, 600), and a
    stream the server stops writing to (no FIN, no terminating chunk) is replaced; an
    object created meanwhile reaches the cache.  Connections have TCP keepalive on."""
    import socket

    from cron_operator_amd.apiserver.http import APIServerApp
    from cron_operator_amd.runtime.client import Client
    from cron_operator_amd.runtime.http import HttpTransport
    from cron_operator_amd.runtime.informer import Informer
    from cron_operator_amd.runtime.kubeconfig import RestConfig

    CM = GroupVersionResource("", "v1", "configmaps")
    env = TestEnv()
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)
    seen_params = []
    orig_watch = client.transport.watch

    async def spy_watch(gvr, namespace="", params=None):
        seen_params.append(dict(params or {}))
        return await orig_watch(gvr, namespace, params)

    client.transport.watch = spy_watch  # type: ignore[assignment]
    inf = Informer(client, CM, NS, watch_idle_timeout=0.4)
    try:
        inf.start()
        await asyncio.wait_for(inf.synced.wait(), 10)
        for _ in range(500):  # the WATCH was requested and its stream is established
            await asyncio.sleep(0.01)
            if seen_params and inf._watch is not None:
                break
        assert seen_params and 300 <= int(seen_params[0]["timeoutSeconds"]) < 600
        st = inf._watch._s  # the dedicated watch connection: native (_netconn) or asyncio protocol
        if hasattr(st, "_n"):
            import os

            with socket.socket(fileno=os.dup(st._n.fd)) as sock:
                assert sock.getsockopt(socket.SOL_SOCKET, socket.SO_KEEPALIVE) == 1
        else:
            sock = st._c.transport.get_extra_info("socket")
            assert sock.getsockopt(socket.SOL_SOCKET, socket.SO_KEEPALIVE) == 1
        assert env.server.stall_watches("configmaps") == 1
        env.server.create(CM, NS, {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "late"}})
        await asyncio.sleep(0.1)
        assert inf.get(NS, "late") is None  # the stalled stream delivered nothing
        for _ in range(200):
            await asyncio.sleep(0.02)
            if inf.get(NS, "late") is not None:
                break
        assert inf.get(NS, "late") is not None
        assert inf.idle_timeouts >= 1 and len(seen_params) >= 2
    finally:
        await inf.stop()
        await client.close()
        await app.stop()


async def test_failing_event_handler_closes_its_watch_and_the_informer_resumes():
    """A handler exception ends the watch loop's attempt: the stream it was reading is closed
    (not left registered with the loop buffering events nobody takes) and the next attempt
    resumes from the last applied resourceVersion, so no event is lost."""
    from cron_operator_amd.apiserver.http import APIServerApp
    from cron_operator_amd.runtime.client import Client
    from cron_operator_amd.runtime.http import HttpTransport
    from cron_operator_amd.runtime.informer import EventHandler, Informer
    from cron_operator_amd.runtime.kubeconfig import RestConfig

    CM = GroupVersionResource("", "v1", "configmaps")
    env = TestEnv()
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)
    streams = []
    orig_watch = client.transport.watch

    async def spy_watch(gvr, namespace="", params=None, **kw):
        s = await orig_watch(gvr, namespace, params, **kw)
        stops = []
        real_stop = s.stop
        s.stop = lambda: (stops.append(1), real_stop())  # type: ignore[assignment]
        streams.append(stops)
        return s

    client.transport.watch = spy_watch  # type: ignore[assignment]
    inf = Informer(client, CM, NS)
    boom = [True]
    added = []

    def on_add(o):
        name = o["metadata"]["name"]
        if name == "bad" and boom[0]:
            boom[0] = False
            raise RuntimeError("handler bug")
        added.append(name)

    inf.add_handler(EventHandler(on_add=on_add))
    try:
        inf.start()
        await asyncio.wait_for(inf.synced.wait(), 10)
        for _ in range(500):
            await asyncio.sleep(0.01)
            if streams:
                break
        for name in ("bad", "after"):
            env.server.create(CM, NS, {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name}})
        for _ in range(300):
            await asyncio.sleep(0.02)
            if len(streams) >= 2 and "after" in added:
                break
        assert streams[0], "the watch whose handler failed was not closed"
        assert len(streams) >= 2 and "after" in added
        assert inf.get(NS, "bad") is not None and inf.get(NS, "after") is not None
    finally:
        await inf.stop()
        await client.close()
        await app.stop()
