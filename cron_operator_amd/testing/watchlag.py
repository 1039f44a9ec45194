"""Scheduling invariants under watch lag -- the condition a real informer cache goes stale under.

The operator reads Crons and their jobs from two informer caches fed by two watch streams.  A
real apiserver delivers those streams with independent delays (its watch cache, the network, a
busy client), so a reconcile can see a job's ADDED event before the Cron update that recorded
the tick it ran for -- the stale read behind the reference's Replace double-create
(``/root/reference/internal/controller/cron_controller.go:96-105`` reads the Cron from the cache,
``:210-237`` deletes the active jobs and creates the tick's job).

:func:`run` drives one seed: a fleet of Allow / Forbid / Replace Crons on ``*/1`` runs for a
few virtual minutes while :class:`~..apiserver.server.FaultInjector` lags the ``crons`` stream
and the ``pytorchjobs`` stream independently (5-200 ms per event); the clock moves in steps
the operator does not wait out, so it works with stale caches.  Checked: no tick's job is ever
created twice (from the apiserver's own event log, so a create-delete-create between two looks
still counts), and a Forbid Cron never has two unfinished jobs.  The lag then stops and every
Cron must converge.  ``tests/test_chaos.py`` runs a few seeds per mode; ``scripts/chaos_seeds.py``
sweeps hundreds.
"""
from __future__ import annotations

import asyncio
import random
from collections import Counter
from typing import Any, Dict, List, Tuple

from ..api.meta import GroupVersionResource
from ..api.v1alpha1 import CRON_GVR, LABEL_CRON_NAME, new_cron
from ..controller.reconciler import ReconcilerOptions
from ..trainingop.operator import finished_status
from ..utils.gotime import NANOS, UTC, GoTime
from .env import TestEnv

PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
NS = "default"
TMPL = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
        "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}}
POLICIES = ("Allow", "Forbid", "Replace")
LAG = (0.005, 0.2)  # seconds per event, per stream


def _finished(job: Dict[str, Any]) -> bool:
    return any(c.get("type") in ("Succeeded", "Failed") and c.get("status") == "True"
               for c in (job.get("status") or {}).get("conditions") or [])


def _complete_running(env: TestEnv) -> None:
    ts = GoTime(env.clock.now_ns() // NANOS, 0, UTC).rfc3339()
    for j in list(env.server.objects(PT, NS)):
        if not _finished(j):
            name = j["metadata"]["name"]
            env.server.patch(PT, NS, name, {"status": finished_status("PyTorchJob", name, ts, True)}, "merge",
                             "status")


def _double_creates(env: TestEnv) -> List[str]:
    """Job names the apiserver saw ADDED more than once (its event log holds every event)."""
    added = Counter(obj["metadata"]["name"] for (_, etype, obj, _) in env.server._log.get(("kubeflow.org",
                                                                                            "pytorchjobs"), ())
                    if etype == "ADDED")
    return sorted(n for n, k in added.items() if k > 1)


async def run(mode: str, seed: int, minutes: int = 3, per_policy: int = 3, step_s: int = 2,
              lag: Tuple[float, float] = LAG) -> Dict[str, Any]:
    """One seed.  ``mode``: ``optimized``, ``optimized-gated`` (a QPS bucket and an in-flight cap
    of 4 on the client, so released worker slots and request priorities run under the lag too) or
    ``reference`` (the control).  Returns the violations found and whether the fleet converged."""
    from ..runtime.ratelimit import InflightGate

    rng = random.Random(seed)
    opts = ReconcilerOptions.reference() if mode == "reference" else ReconcilerOptions()
    env = TestEnv(gc=True, qps=2000 if mode == "optimized-gated" else -1, burst=100)
    if mode == "optimized-gated":
        env.client.inflight = InflightGate(4)
    env.server.faults._rng = random.Random(seed)
    crons: Dict[str, str] = {}
    for i in range(per_policy * len(POLICIES)):
        policy = POLICIES[i % len(POLICIES)]
        name = f"lag-{policy.lower()}-{i}"
        crons[name] = policy
        await env.create_cron(new_cron(name, NS, "*/1 * * * *", TMPL, concurrency_policy=policy,
                                       history_limit=2))
    await env.start_manager(opts, max_concurrent=4)
    await env.settle()
    env.server.faults.watch_lag = {"crons": lag, "pytorchjobs": lag}
    forbid_violations: List[str] = []
    try:
        for _ in range(minutes):
            for sec in range(0, 60, step_s):
                env.clock.advance(step_s)
                if sec == 30:
                    _complete_running(env)
                # the operator runs on with lagging caches; the clock does not wait for it
                await asyncio.sleep(rng.uniform(0.0, 0.04))
                for name, policy in crons.items():
                    if policy == "Forbid":
                        running = [j for j in env.server.objects(PT, NS)
                                   if (j["metadata"].get("labels") or {}).get(LABEL_CRON_NAME) == name
                                   and not _finished(j)]
                        if len(running) > 1:
                            forbid_violations.append(f"{name}: {sorted(j['metadata']['name'] for j in running)}")
        # the lag stops: everything must converge
        env.server.faults.clear()
        await env.settle(timeout=60)
        for _ in range(90):
            env.clock.advance(1)
            await env.settle(timeout=60)
        _complete_running(env)
        for _ in range(30):
            env.clock.advance(1)
            await env.settle(timeout=60)
        tick_s = (env.clock.now_ns() // NANOS) // 60 * 60
        last_tick = GoTime(tick_s, 0, UTC).rfc3339()[:16]
        prev_tick = GoTime(tick_s - 60, 0, UTC).rfc3339()[:16]
        unconverged = []
        for name, policy in crons.items():
            st = env.server.get(CRON_GVR, NS, name).get("status") or {}
            jobs = [j for j in env.server.objects(PT, NS)
                    if (j["metadata"].get("labels") or {}).get(LABEL_CRON_NAME) == name]
            running = sorted(j["metadata"]["name"] for j in jobs if not _finished(j))
            done = sorted(j["metadata"]["name"] for j in jobs if _finished(j))
            # a Forbid Cron runs the tick it skipped when its job finishes, mid-minute, and then
            # skips the next tick while that job runs (cron_controller.go:204-207)
            ticks = (last_tick, prev_tick) if policy == "Forbid" else (last_tick,)
            if (st.get("lastScheduleTime") or "")[:16] not in ticks or \
                    sorted(a["name"] for a in st.get("active") or []) != running or \
                    sorted(h["object"]["name"] for h in st.get("history") or []) != done or len(done) > 2:
                unconverged.append(f"{name}: lastScheduleTime {st.get('lastScheduleTime')} (tick {last_tick}), "
                                   f"active {sorted(a['name'] for a in st.get('active') or [])} vs running {running}, "
                                   f"history {sorted(h['object']['name'] for h in st.get('history') or [])} vs "
                                   f"done {done}")
        return {"mode": mode, "seed": seed, "double_creates": _double_creates(env),
                "forbid_violations": forbid_violations, "unconverged": unconverged,
                "errors": env.controller.errors if env.controller is not None else 0}
    finally:
        await env.stop()
