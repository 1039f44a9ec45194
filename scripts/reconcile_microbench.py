#!/usr/bin/env python3
"""CPU cost of the reconcile logic alone, without I/O or the event loop's scheduling.

The headline bench measures the whole operator process (HTTP, watch decoding, asyncio,
informers, reconciles).  This isolates the part the reconciler itself owns: one Cron with a
full history (historyLimit=10) is driven through the bench's two phases -- its newest job
finishes (completion reconcile: history update, GC DELETE, status PATCH) and the next tick
fires (fire reconcile: CREATE, status PATCH) -- against a client whose verbs return at once
and informers fed directly (``Informer._apply``) with the objects the apiserver would echo.
Everything else runs as in production: the CronReconciler with its default options, the
wire codecs' memo, the child informer's derived memos and indexes.

    python scripts/reconcile_microbench.py --fires 20000 [--profile out.txt]

Prints microseconds of CPU per reconcile and per fire (two reconciles).  ``--profile`` adds a
cProfile of the same loop (sorted by own time).
"""
from __future__ import annotations

import argparse
import asyncio
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build():
    from cron_operator_amd.api.meta import GroupVersionKind, new_controller_ref
    from cron_operator_amd.api.v1alpha1 import CRON_GVK, LABEL_CRON_NAME, new_cron
    from cron_operator_amd.bench.harness import pytorchjob_template
    from cron_operator_amd.controller.reconciler import (CHILD_INDEX, CronReconciler, ReconcilerOptions, WireCodecs,
                                                         child_info, slim_child)
    from cron_operator_amd.runtime.events import FakeRecorder
    from cron_operator_amd.runtime.informer import Informer, label_index, strip_managed_fields
    from cron_operator_amd.trainingop.operator import finished_status
    from cron_operator_amd.utils import jsonutil
    from cron_operator_amd.utils.clock import FakeClock
    from cron_operator_amd.utils.gotime import NANOS, UTC, GoTime

    gvk = GroupVersionKind("kubeflow.org", "v1", "PyTorchJob")
    t0 = 1767268800 * NANOS
    clock = FakeClock(t0)
    opts = ReconcilerOptions()
    codecs = WireCodecs(opts.slim_child_cache)
    state = {"rv": 100, "uid": 0}

    def next_rv() -> str:
        state["rv"] += 1
        return str(state["rv"])

    def rfc(ns: int) -> str:
        return GoTime(ns // NANOS, 0, UTC).rfc3339()

    cron = new_cron("cron-00001", "bench", "* * * * *", pytorchjob_template(), history_limit=10).to_dict()
    cron["metadata"].update({"uid": "cron-uid-1", "resourceVersion": next_rv(), "generation": 1,
                             "creationTimestamp": rfc(t0 - 3600 * NANOS)})
    cron_inf = Informer(None, CRON_GVK, transform=strip_managed_fields, decoder=codecs.cron_event)
    child_inf = Informer(None, gvk, indexers={CHILD_INDEX: label_index(LABEL_CRON_NAME)}, transform=slim_child,
                         decoder=codecs.child_event)
    child_inf.set_derive(lambda o: child_info(o, gvk, opts.workload))
    child_inf.synced.set()

    def job(tick_ns: int, finished_ns: int = 0):
        state["uid"] += 1
        name = f"cron-00001-{tick_ns // NANOS}"
        j = jsonutil.deepcopy(pytorchjob_template())
        j["metadata"] = {"name": name, "namespace": "bench", "uid": f"job-uid-{state['uid']}",
                         "resourceVersion": next_rv(), "creationTimestamp": rfc(tick_ns),
                         "labels": {"app": "bench", LABEL_CRON_NAME: "cron-00001"},
                         "ownerReferences": [new_controller_ref(cron, CRON_GVK)]}
        if finished_ns:
            j["status"] = finished_status("PyTorchJob", name, rfc(finished_ns), True)
        return j

    # full history: ten finished jobs, one per past minute
    for i in range(10, 0, -1):
        child_inf._apply("ADDED", slim_child(job(t0 - i * 60 * NANOS, t0 - i * 60 * NANOS + 30 * NANOS)))

    class FakeClient:
        """Verbs complete at once; CREATE echoes the object with uid/resourceVersion."""

        def __init__(self):
            self.requests = 0

        def gate_saturated(self) -> bool:  # no in-flight cap: a reconcile may release its slot
            return False

        async def create(self, target, obj, namespace=None, dry_run=False, decoder=None, priority=None):
            self.requests += 1
            m = obj["metadata"]
            state["uid"] += 1
            m.update({"uid": f"job-uid-{state['uid']}", "resourceVersion": next_rv(),
                      "creationTimestamp": rfc(clock.now_ns())})
            return obj

        async def patch(self, *a, **kw):
            self.requests += 1

        async def delete(self, target, namespace, name, **kw):
            self.requests += 1
            gone = child_inf.store.get(f"{namespace}/{name}")
            if gone is not None:  # its watch event (DELETED)
                child_inf._apply("DELETED", gone)

    client = FakeClient()
    rec = CronReconciler(client, None, FakeRecorder(), clock, None, opts, cron_inf, codecs)
    rec.child_informers[gvk] = child_inf
    rec.cache = object()  # "an informer cache exists": the steady-state path reads child_informers
    # the child-event handlers setup_with_manager installs: expectations met, memos dropped
    from cron_operator_amd.runtime.informer import EventHandler

    def key_of(o):
        m = o.get("metadata") or {}
        return f"{m.get('namespace', '')}/{(m.get('labels') or {}).get(LABEL_CRON_NAME, '')}"

    exp = rec.expect
    child_inf.add_handler(EventHandler(
        on_add=lambda o: exp.created and exp.observe_add(key_of(o), o["metadata"]["uid"]),
        on_update=lambda old, o: exp.created and exp.observe_add(key_of(o), o["metadata"]["uid"]),
        on_delete=lambda o: ((exp.created or exp.deleted) and exp.observe_delete(key_of(o), o["metadata"]["uid"]),
                             rec.forget_child(o["metadata"]["uid"]))))

    def echo_cron_status():
        """The watch echo of our own status write: the stored Cron with the patched status."""
        key = "bench/cron-00001"
        status = rec.own_writes.get(key, (None, None))[1]
        cur = cron_inf.store.get(key) or cron
        obj = dict(cur)
        obj["spec"] = cron["spec"]  # the cache holds the template as its raw JSON text; the wire has JSON
        obj["metadata"] = dict(cur["metadata"], resourceVersion=next_rv())
        if status is not None:
            obj["status"] = status
        raw = codecs.status_patch.dumpb({"type": "MODIFIED", "object": obj})  # bytes as the server sends
        t, o = codecs.cron_event(raw)
        cron_inf._apply(t, o)

    cron_inf._apply("ADDED", codecs.cron_event(jsonutil.dumpb({"type": "ADDED", "object": cron}))[1])
    return clock, rec, cron_inf, child_inf, job, echo_cron_status, client, NANOS


async def run(fires: int, profile: str) -> None:
    from cron_operator_amd.runtime.controller import Request
    from cron_operator_amd.utils.logging import get_logger

    from cron_operator_amd.utils.logging import new_from_options, set_logger

    set_logger(new_from_options(encoder="json", level="error", stream=open(os.devnull, "w")))
    clock, rec, cron_inf, child_inf, job, echo, client, NANOS = build()
    log = get_logger()
    req = Request("bench", "cron-00001")
    t0 = clock.now_ns()
    clock.set(t0 + 60 * NANOS)  # tick 1: create the first job
    await rec.reconcile(req, log)
    echo()

    spent = {"completion": 0.0, "fire": 0.0, "echo": 0.0}
    pt = time.process_time

    async def one_fire(k: int) -> None:
        tick = t0 + (k + 1) * 60 * NANOS
        # completion: the current job finishes; its watch event reaches the child informer
        cur = sorted(child_inf.store.values(), key=lambda o: o["metadata"]["creationTimestamp"])[-1]
        fin = dict(cur, status=job(tick - 60 * NANOS, tick - 30 * NANOS)["status"])
        fin["metadata"] = dict(cur["metadata"], resourceVersion=str(int(cur["metadata"]["resourceVersion"]) + 1))
        child_inf._apply("MODIFIED", fin)
        clock.set(tick - 30 * NANOS)
        a = pt()
        await rec.reconcile(req, log)
        b = pt()
        echo()
        c = pt()
        # fire: the tick's CREATE (its ADDED event is applied inside, by the fake client), the echo
        clock.set(tick)
        d = pt()
        await rec.reconcile(req, log)
        e = pt()
        echo()
        f = pt()
        spent["completion"] += b - a
        spent["fire"] += e - d
        spent["echo"] += (c - b) + (f - e)

    # the created jobs must reach the child informer: wrap the client's create
    orig = client.create

    async def create(*a, **kw):
        obj = await orig(*a, **kw)
        from cron_operator_amd.controller.reconciler import slim_child
        from cron_operator_amd.utils import jsonutil

        child_inf._apply("ADDED", slim_child(jsonutil.deepcopy(obj)))
        return obj

    client.create = create
    for k in range(1, 200):  # warm up: memos, caches
        await one_fire(k)
    for v in spent:
        spent[v] = 0.0
    prof = cProfile.Profile() if profile else None
    c0 = time.process_time()
    if prof:
        prof.enable()
    chunk_cpu = []  # CPU per fire over each tenth of the run: whether a long run slows down
    c_chunk = c0
    step = max(1, fires // 10)
    for k in range(200, 200 + fires):
        await one_fire(k)
        if (k - 199) % step == 0:
            now = time.process_time()
            chunk_cpu.append(round((now - c_chunk) * 1e6 / step, 1))
            c_chunk = now
    if prof:
        prof.disable()
    cpu = time.process_time() - c0
    st = rec.stats
    print(f"{fires} fires: {cpu * 1e6 / fires:.1f} us CPU per fire (harness included), "
          f"creates {st['creates']}, deletes {st['deletes']}, patches {st['patches']}", flush=True)
    print("  completion reconcile {:.1f} us, fire reconcile {:.1f} us (incl. its CREATE's ADDED event), "
          "status-echo events {:.1f} us per fire".format(*(spent[k] * 1e6 / fires for k in
                                                          ("completion", "fire", "echo"))), flush=True)
    print(f"  us per fire by tenth of the run: {chunk_cpu}", flush=True)
    if prof:
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(40)
        with open(profile, "w") as fh:
            fh.write(buf.getvalue())


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fires", type=int, default=20000)
    ap.add_argument("--profile", default="")
    a = ap.parse_args()
    asyncio.run(run(a.fires, a.profile))
    return 0


if __name__ == "__main__":
    sys.exit(main())
