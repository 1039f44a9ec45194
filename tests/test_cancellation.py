"""Cancellation and expiry: a stopping operator must stop promptly, and in-memory bookkeeping
must age on the same clock as everything else.

Reference behaviour being matched: controller-runtime hands every reconcile a context that
is cancelled when the manager stops or loses its lease, and on leader loss it exits without
a graceful drain (manager wiring at ``/root/reference/cmd/operator/start.go:156-209``).  Here
a reconcile waiting on its history-GC DELETEs (``cron_controller.go:324-333``) must therefore
end with ``CancelledError`` at once instead of waiting for each DELETE's request timeout.
"""
from __future__ import annotations

import asyncio
import time

import pytest

from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.api.v1alpha1 import LABEL_CRON_NAME, new_cron
from cron_operator_amd.controller.reconciler import CronReconciler, ReconcilerOptions, child_info
from cron_operator_amd.cron.engine import NativeEngine
from cron_operator_amd.models.workload import WorkloadPolicy
from cron_operator_amd.runtime.controller import Request
from cron_operator_amd.runtime.events import FakeRecorder
from cron_operator_amd.testing.env import TestEnv
from cron_operator_amd.trainingop.operator import finished_status
from cron_operator_amd.utils import aio
from cron_operator_amd.utils.logging import get_logger

PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
NS = "default"
PT_TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}}
HOLD_S = 30.0  # every DELETE is held this long (real time) by the fake apiserver


def _finished_children(env: TestEnv, cron: str, n: int) -> None:
    for i in range(n):
        env.clock.advance(1)
        name = f"{cron}-{i}"
        env.server.create(PT, NS, {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                   "metadata": {"name": name, "labels": {LABEL_CRON_NAME: cron}}})
        env.server.patch(PT, NS, name, {"status": finished_status("PyTorchJob", name, "2026-01-01T11:00:00Z", True)},
                         "merge", "status")


def _count_deletes(env: TestEnv) -> list:
    """Record every DELETE the operator starts (the apiserver then holds it ``HOLD_S``)."""
    started: list = []
    orig = env.client.delete

    async def delete(*a, **kw):
        started.append(a)
        return await orig(*a, **kw)

    env.client.delete = delete  # type: ignore[assignment]
    return started


async def _spin_until(pred, turns: int = 5000) -> None:
    for _ in range(turns):
        if pred():
            return
        await asyncio.sleep(0)
    raise AssertionError("condition not reached")


@pytest.mark.parametrize("overlap", [True, False])
async def test_cancelled_reconcile_mid_gc_raises_promptly(overlap):
    env = TestEnv()
    await env.create_cron(new_cron("c", NS, "*/1 * * * *", PT_TMPL, history_limit=0))
    _finished_children(env, "c", 3)
    started = _count_deletes(env)
    env.server.faults.latency["delete"] = HOLD_S
    r = CronReconciler(env.client, None, FakeRecorder(), env.clock, NativeEngine(),
                       ReconcilerOptions(list_mode="live", overlap_gc_deletes=overlap))
    task = asyncio.get_running_loop().create_task(r.reconcile(Request(NS, "c"), get_logger()))
    await _spin_until(lambda: len(started) >= 1)
    before = set(asyncio.all_tasks())
    t0 = time.perf_counter()
    task.cancel()
    with pytest.raises(asyncio.CancelledError):
        await asyncio.wait_for(task, 1.0)
    assert time.perf_counter() - t0 < 0.1
    assert task.cancelled()
    # no DELETE is left running behind the cancelled reconcile
    for _ in range(5):
        await asyncio.sleep(0)
    leftover = [t for t in before if t is not task and not t.done() and "_gc_delete" in repr(t.get_coro())]
    assert leftover == []
    # the cancelled DELETEs no longer hide their children from the next reconcile
    assert r.expect.deleted == {}


async def test_controller_stop_does_not_wait_for_held_deletes():
    env = TestEnv()
    await env.create_cron(new_cron("c", NS, "*/1 * * * *", PT_TMPL, history_limit=0))
    _finished_children(env, "c", 3)
    started = _count_deletes(env)
    env.server.faults.latency["delete"] = HOLD_S
    await env.start_manager()
    await _spin_until(lambda: len(started) >= 3)
    # the reconcile's tail is parked on its GC DELETEs (the worker itself moved on)
    assert env.controller.in_flight() == 1 and env.controller.queue.processing() == 1
    t0 = time.perf_counter()
    await asyncio.wait_for(env.controller.stop(), 1.0)
    assert time.perf_counter() - t0 < 1.0
    assert env.controller.in_flight() == 0
    env.server.faults.clear()
    await env.stop()


async def test_leader_loss_ends_manager_within_renew_deadline_despite_held_deletes():
    """Another identity takes the Lease while a reconcile waits on DELETEs the apiserver holds
    for 30 s: the next renewal window fails, and the manager raises LeaderElectionLost within
    ``retryPeriod + renewDeadline`` of virtual time -- its shutdown takes well under a second
    of real time, instead of draining the held DELETEs."""
    from cron_operator_amd.parallel.leaderelection import LEASES
    from cron_operator_amd.runtime.manager import LeaderElectionLost

    env = TestEnv()
    await env.create_cron(new_cron("c", NS, "*/1 * * * *", PT_TMPL, history_limit=0))
    _finished_children(env, "c", 3)
    started = _count_deletes(env)
    env.server.faults.latency["delete"] = HOLD_S
    await env.start_manager(leader_election=True, leader_election_namespace=NS, leader_election_identity="me",
                            lease_duration=15, renew_deadline=10, retry_period=2)
    await _spin_until(lambda: len(started) >= 3)
    assert env.manager.elector.is_leader and env.controller.in_flight() == 1
    # a forced loss: another holder overwrites the lease record
    lease = env.server.get(LEASES, NS, "619a52b8.kubedl.io")
    lease["spec"]["holderIdentity"] = "usurper"
    env.server.update(LEASES, NS, "619a52b8.kubedl.io", lease)
    stopped_after = None
    lost_at = None
    for sec in range(1, 30):
        env.clock.advance(1)
        for _ in range(200):
            await asyncio.sleep(0)
            if lost_at is None and env.manager.elector.lost.is_set():
                lost_at = time.perf_counter()
            if env._mgr_task.done():
                break
        if env._mgr_task.done():
            stopped_after = sec
            break
        if lost_at is not None:  # shutting down: real time only from here
            await asyncio.wait({env._mgr_task}, timeout=1.0)
            assert env._mgr_task.done(), "manager shutdown waited on held DELETEs"
            stopped_after = sec
            break
    assert stopped_after is not None and stopped_after <= 2 + 10, stopped_after
    assert lost_at is not None and time.perf_counter() - lost_at < 1.0
    assert isinstance(env._mgr_task.exception(), LeaderElectionLost)
    assert not env.controller.started


async def test_expectation_of_unseen_create_expires_on_the_injected_clock():
    """The child informer never receives the events of the job a tick created (a watch that
    lost them).  Until ``expectation_ttl`` the reconciler keeps that job in view from its own
    CREATE, so a Forbid Cron does not run a second job beside it; once the TTL has passed *in
    virtual time* the expectation is dropped and the Cron schedules again, exactly one job per
    tick."""
    env = TestEnv()
    await env.create_cron(new_cron("c", NS, "*/1 * * * *", PT_TMPL, concurrency_policy="Forbid"))
    orig_emit = env.server._emit
    hidden = {"c-1767268920"}  # the job of the first tick, named <cron>-<unix(Next(tick))>

    def emit(ri, etype, obj, old, rv):
        if ri.resource == "pytorchjobs" and (obj.get("metadata") or {}).get("name") in hidden:
            return  # lost on the wire
        return orig_emit(ri, etype, obj, old, rv)

    env.server._emit = emit  # type: ignore[assignment]
    opts = ReconcilerOptions(expectation_ttl=300.0)
    await env.start_manager(opts)
    await env.settle()
    for _ in range(60):
        await env.advance(1)
    names = sorted(o["metadata"]["name"] for o in env.server.list(PT, NS)["items"])
    assert names == sorted(hidden), names
    assert env.reconciler.expect.created, "the CREATE is expected until its event arrives"
    # the job finishes, unseen; for the TTL the Cron still counts it as active (Forbid)
    env.server.patch(PT, NS, "c-1767268920",
                     {"status": finished_status("PyTorchJob", "c-1767268920", "2026-01-01T12:01:30Z", True)},
                     "merge", "status")
    for _ in range(4 * 60):
        await env.advance(1)
    assert env.server.count(PT, NS) == 1
    # past the TTL (virtual time): the expectation expires and scheduling resumes
    for _ in range(2 * 60):
        await env.advance(1)
    assert env.reconciler.expect.created == {}
    jobs = sorted(o["metadata"]["name"] for o in env.server.list(PT, NS)["items"])
    assert len(jobs) >= 2 and len(jobs) == len(set(jobs))
    n = len(jobs)
    for _ in range(60):
        await env.advance(1)
    # one more tick, one more job: no duplicate for any tick
    assert env.server.count(PT, NS) in (n, n + 1)
    await env.stop()


def test_child_info_never_raises_inside_the_informer():
    """A child the reconciler cannot read becomes a per-child error instead of an exception
    escaping into the informer's event handling (where it would stall the whole kind)."""
    from cron_operator_amd.api.meta import GroupVersionKind

    gvk = GroupVersionKind("kubeflow.org", "v1", "PyTorchJob")
    bad = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
           "metadata": {"name": "x", "uid": "u", "creationTimestamp": 12345},
           "status": {"conditions": "not-a-list"}}
    info = child_info(bad, gvk, WorkloadPolicy())
    assert info.err is not None and info.name == "x"
    odd = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob", "metadata": ["not", "a", "map"]}
    child_info(odd, gvk, WorkloadPolicy())  # must not raise
    # a readable, finished status but a malformed creationTimestamp: an error, never "finished"
    # (a finished child goes to history, whose entry needs the timestamp)
    done = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
            "metadata": {"name": "y", "uid": "v", "creationTimestamp": "yesterday"},
            "status": {"conditions": [{"type": "Succeeded", "status": "True"}]}}
    info = child_info(done, gvk, WorkloadPolicy())
    assert info.err is not None and info.cls is None and not info.finished


async def test_sequential_gc_survives_a_transport_error():
    """``overlap_gc_deletes=False``: a DELETE that fails below the API layer (connection
    reset) is only logged like any other Delete error, the remaining DELETEs still run, and
    no coroutine is left un-awaited."""
    import gc as pygc
    import warnings

    env = TestEnv()
    await env.create_cron(new_cron("c", NS, "*/1 * * * *", PT_TMPL, history_limit=0))
    _finished_children(env, "c", 3)
    orig = env.client.delete
    calls = []

    async def flaky(gvk, ns, name, *a, **kw):
        calls.append(name)
        if name == "c-0":
            raise ConnectionResetError("connection reset by peer")
        return await orig(gvk, ns, name, *a, **kw)

    env.client.delete = flaky  # type: ignore[assignment]
    r = CronReconciler(env.client, None, FakeRecorder(), env.clock, NativeEngine(),
                       ReconcilerOptions(list_mode="live", overlap_gc_deletes=False))
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        await r.reconcile(Request(NS, "c"), get_logger())
        pygc.collect()
    assert calls == ["c-0", "c-1", "c-2"]
    assert sorted(o["metadata"]["name"] for o in env.server.list(PT, NS)["items"]) == ["c-0"]
    assert not [x for x in w if "never awaited" in str(x.message)]


async def test_aio_helpers_keep_caller_cancellation():
    """``cancel_and_wait`` / ``wait_all`` propagate a cancellation aimed at the caller."""
    hold = asyncio.Event()

    async def child():
        try:
            await hold.wait()
        except asyncio.CancelledError:
            await asyncio.sleep(0.05)  # slow to stop
            raise

    async def caller():
        t = asyncio.get_running_loop().create_task(child())
        await asyncio.sleep(0)
        await aio.cancel_and_wait(t)
        return "finished"

    outer = asyncio.get_running_loop().create_task(caller())
    await asyncio.sleep(0.01)
    outer.cancel()
    with pytest.raises(asyncio.CancelledError):
        await outer
