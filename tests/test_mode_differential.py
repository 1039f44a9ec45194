"""Differential test: the optimized reconciler against the reference algorithm.

``ReconcilerOptions()`` adds caches, expectations, memos, overlapped DELETEs and event
filtering on top of the reference algorithm (``ReconcilerOptions.reference()``, a step
by step re-implementation of ``internal/controller/cron_controller.go:90-437``).  None of
that may change *what* happens to a cluster.  Hypothesis draws Crons (schedule,
concurrency policy, historyLimit) and a timeline (clock advances, jobs finishing with
success or failure, suspend toggles, spec edits of historyLimit and concurrencyPolicy, jobs
deleted by someone else); the same timeline runs
against two fake apiservers, one per mode, and after every step the two clusters must
agree on:

* which jobs exist for every Cron (so the same CREATEs, Replace DELETEs and history GC),
* ``status.lastScheduleTime``,
* ``status.active`` (names), and
* ``status.history`` (job names and their Succeeded/Failed status, in order).

``history[].finished`` is excluded: the reference stamps ``metav1.Now()`` on every
reconcile, the optimized mode keeps the job's completion time.
"""
from __future__ import annotations

import asyncio
from typing import Any, Dict, List, Optional, Tuple

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.api.v1alpha1 import CRON_GVR, LABEL_CRON_NAME, new_cron
from cron_operator_amd.controller.reconciler import ReconcilerOptions
from cron_operator_amd.testing.env import TestEnv
from cron_operator_amd.trainingop.operator import finished_status
from cron_operator_amd.utils.gotime import UTC, GoTime

PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
NS = "default"
PT_TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}}

cron_specs = st.lists(
    st.tuples(st.sampled_from(["*/1 * * * *", "*/2 * * * *", "*/3 * * * *"]),
              st.sampled_from(["Allow", "Forbid", "Replace"]),
              st.sampled_from([1, 2, 3, 5])),
    min_size=1, max_size=3)

step = st.tuples(
    st.integers(min_value=10, max_value=200),          # seconds to advance
    st.lists(st.tuples(st.integers(0, 9), st.booleans()), max_size=3),  # (active job pick, succeeded?)
    st.one_of(st.none(), st.integers(0, 2)),           # toggle suspend of Cron i
    st.one_of(st.none(), st.integers(0, 9)),           # delete one finished job (someone else)
    st.one_of(st.none(), st.tuples(st.integers(0, 2),  # edit Cron i's spec: historyLimit / policy
                                   st.sampled_from([1, 2, 4]),
                                   st.sampled_from(["Allow", "Forbid", "Replace"]))),
)


def _jobs(env: TestEnv, cron: str) -> List[Dict[str, Any]]:
    items = env.server.list(PT, NS, label_selector=f"{LABEL_CRON_NAME}={cron}")["items"]
    return sorted(items, key=lambda o: o["metadata"]["name"])


def _finished(o: Dict[str, Any]) -> bool:
    return bool((o.get("status") or {}).get("completionTime"))


def _observed(env: TestEnv, crons: List[str]) -> Dict[str, Tuple[Any, ...]]:
    out = {}
    for name in crons:
        stt = env.server.get(CRON_GVR, NS, name).get("status") or {}
        out[name] = (
            tuple(o["metadata"]["name"] for o in _jobs(env, name)),
            stt.get("lastScheduleTime"),
            tuple(a["name"] for a in stt.get("active") or []),
            tuple((h["object"]["name"], h["status"]) for h in stt.get("history") or []),
        )
    return out


class _HttpEnv(TestEnv):
    """The same fake apiserver, but the manager talks to it over HTTP: the keep-alive client
    pool, the streamed watch decoding and batched event application are all in the loop."""

    async def serve(self) -> None:
        from cron_operator_amd.apiserver.http import APIServerApp
        from cron_operator_amd.runtime.client import Client
        from cron_operator_amd.runtime.http import HttpTransport
        from cron_operator_amd.runtime.kubeconfig import RestConfig

        self.app = APIServerApp(self.server)
        port = await self.app.start("127.0.0.1", 0, bookmark_interval=0)
        self.client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)

    def _applied(self) -> int:
        assert self.manager is not None
        infs = list(self.manager.cache.informers())
        if self.reconciler is not None:
            infs += [i for i in self.reconciler.child_informers.values() if i not in infs]
        return sum(i.events for i in infs)

    async def settle(self, timeout: float = 30.0) -> None:
        # events travel through sockets: idle means no informer applied anything for a while
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout
        while loop.time() < deadline:
            await TestEnv.settle(self, timeout)
            before = self._applied()
            await asyncio.sleep(0.01)
            if self._applied() == before and self.controller is not None and self.controller.queue.idle():
                return
        raise TimeoutError("HTTP env did not settle")

    async def stop(self) -> None:
        await TestEnv.stop(self)
        await self.client.close()
        await self.app.stop()


def _opts(mode: str) -> ReconcilerOptions:
    return ReconcilerOptions() if mode == "optimized" else ReconcilerOptions.reference()


async def _scenario(mode: str, specs, steps, http: bool = False,
                    switch_at: Optional[int] = None) -> List[Dict[str, Tuple[Any, ...]]]:
    """``switch_at``: before that step, stop the operator and start one in the other mode on the
    same cluster (an upgrade or a rollback between the reference and this operator)."""
    env: TestEnv = _HttpEnv() if http else TestEnv()
    if http:
        await env.serve()  # type: ignore[attr-defined]
    names = [f"c{i}" for i in range(len(specs))]
    for name, (sched, policy, limit) in zip(names, specs):
        await env.create_cron(new_cron(name, NS, sched, PT_TMPL, concurrency_policy=policy, history_limit=limit))
    await env.start_manager(_opts(mode))
    await env.settle()
    seen = [_observed(env, names)]
    try:
        for idx, (secs, finishes, toggle, delete, edit) in enumerate(steps):
            if idx == switch_at:
                assert not http
                await env.stop()
                env.manager = env.controller = env.reconciler = env._mgr_task = None
                mode = "optimized" if mode == "reference" else "reference"
                await env.start_manager(_opts(mode))
                await env.settle()
            now = GoTime(env.clock.now_ns() // 1_000_000_000, 0, UTC).rfc3339()
            running = [o for n in names for o in _jobs(env, n) if not _finished(o)]
            for pick, ok in finishes:
                if running:
                    o = running.pop(pick % len(running))
                    env.server.patch(PT, NS, o["metadata"]["name"],
                                     {"status": finished_status("PyTorchJob", o["metadata"]["name"], now, ok)},
                                     "merge", "status")
            if toggle is not None and toggle < len(names):
                c = env.server.get(CRON_GVR, NS, names[toggle])
                env.server.patch(CRON_GVR, NS, names[toggle],
                                 {"spec": {"suspend": not (c["spec"].get("suspend") or False)}}, "merge")
            if edit is not None and edit[0] < len(names):
                env.server.patch(CRON_GVR, NS, names[edit[0]],
                                 {"spec": {"historyLimit": edit[1], "concurrencyPolicy": edit[2]}}, "merge")
            if delete is not None:
                done = [o for n in names for o in _jobs(env, n) if _finished(o)]
                if done:
                    env.server.delete(PT, NS, done[delete % len(done)]["metadata"]["name"])
            await env.settle()
            await env.advance(secs)
            seen.append(_observed(env, names))
    finally:
        await env.stop()
    return seen


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(cron_specs, st.lists(step, min_size=3, max_size=12))
def test_optimized_mode_matches_reference_algorithm(specs, steps):
    ref = asyncio.run(_scenario("reference", specs, steps))
    opt = asyncio.run(_scenario("optimized", specs, steps))
    for i, (r, o) in enumerate(zip(ref, opt)):
        assert o == r, f"step {i}: optimized {o} != reference {r}"


@settings(max_examples=15, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(cron_specs, st.lists(step, min_size=3, max_size=8))
def test_optimized_mode_over_http_matches_reference_algorithm(specs, steps):
    """The same, with the optimized operator talking HTTP + watch streams to the apiserver."""
    ref = asyncio.run(_scenario("reference", specs, steps))
    opt = asyncio.run(_scenario("optimized", specs, steps, http=True))
    for i, (r, o) in enumerate(zip(ref, opt)):
        assert o == r, f"step {i}: optimized/http {o} != reference {r}"


@settings(max_examples=30, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(cron_specs, st.lists(step, min_size=4, max_size=10), st.integers(1, 3), st.sampled_from(["reference",
                                                                                               "optimized"]))
def test_switching_operators_mid_timeline_leaves_the_same_cluster(specs, steps, switch_at, first):
    """Switching over: the cluster is run by one algorithm, which is stopped between two steps
    and replaced on the same cluster by the other (the reference → this operator, or a rollback).
    The new operator starts from the Crons' stored status and the jobs it finds -- including
    jobs the other one created and history it recorded -- and every step matches a cluster
    the reference algorithm ran throughout: no tick runs twice or is lost, no history entry
    is dropped."""
    ref = asyncio.run(_scenario("reference", specs, steps))
    cut = asyncio.run(_scenario(first, specs, steps, switch_at=switch_at))
    for i, (r, c) in enumerate(zip(ref, cut)):
        assert c == r, f"step {i} (switch before step {switch_at}, {first} first): {c} != reference {r}"
