"""One operator shard as a child process of the benchmark harness.

The reference's controller runs its ``--max-concurrent-reconciles`` workers as
goroutines spread over every core of the pod.  This operator is an asyncio
process (one core); its horizontal-sharding feature (``--shard-count``) is how
it uses more than one.  With ``BenchConfig.shards > 1`` the harness starts one
of these workers per shard, all against the same fake apiserver, and drives them
over a line protocol on stdin/stdout:

``{"cmd": "time", "ns": <unix ns>, "phase": "completion"|"fire", "tick_ns": <ns>}``
    set this shard's (fake) clock and reply once every Cron it owns has settled
    for the phase: ``{"ok": true, "lat": [s, ...], "reconciles": n, "requests": n,
    "by_verb": {...}, "cpu": s, "maxrss_mib": peak RSS}`` (counters cumulative since start);
``{"cmd": "absorb", "rvs": {"<namespace>/<job>": resourceVersion, ...}}``
    reply ``{"ok": true}`` once this shard's job informer saw each of those writes (of the jobs
    it holds) and nothing is queued or in flight -- a lifecycle stage absorbed;
``{"cmd": "stop"}``
    shut the manager down and exit.

Latency is measured inside the shard from the moment it applied the tick to each
CREATE response, like the in-process harness does.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import resource
import sys
import time
from typing import List


def _trace_dump(tag: str) -> None:
    """``CRON_BENCH_TRACEMALLOC=<prefix>`` (set before start): the 25 biggest allocation sites,
    by traceback, appended to ``<prefix>.<pid>.txt`` at ``ready`` and at ``end``."""
    prefix = os.environ.get("CRON_BENCH_TRACEMALLOC")
    if not prefix:
        return
    import gc
    import tracemalloc

    gc.collect()
    snap = tracemalloc.take_snapshot()
    stats = snap.statistics("traceback")
    with open(f"{prefix}.{os.getpid()}.txt", "a") as fh:
        fh.write(f"== {tag}: traced {sum(x.size for x in stats) / 2**20:.1f} MiB, rss {_rss_mib():.1f} MiB\n")
        for x in stats[:25]:
            fh.write(f"{x.size / 2**20:8.2f} MiB {x.count:8d}  " +
                     " <- ".join(f"{f.filename.rsplit('/', 2)[-1]}:{f.lineno}" for f in x.traceback) + "\n")


_TRACE = {"fires": 0, "snap": None}


def _trace_diff(first: int, last: int) -> None:
    """With tracemalloc on: snapshot after fire ``first`` and, after fire ``last``, append the
    25 biggest growths between the two (by traceback) to ``<prefix>.<pid>.txt``."""
    import gc
    import tracemalloc

    _TRACE["fires"] += 1
    n = _TRACE["fires"]
    if n not in (first, last):
        return
    gc.collect()
    snap = tracemalloc.take_snapshot()
    if n == first:
        _TRACE["snap"] = snap
        return
    stats = snap.compare_to(_TRACE["snap"], "traceback")
    with open(f"{os.environ['CRON_BENCH_TRACEMALLOC']}.{os.getpid()}.txt", "a") as fh:
        fh.write(f"== growth fire {first} -> {last}: {sum(x.size_diff for x in stats) / 2**20:.2f} MiB, "
                 f"rss {_rss_mib():.1f}\n")
        for x in stats[:25]:
            fh.write(f"{x.size_diff / 2**20:8.2f} MiB {x.count_diff:8d}  " +
                     " <- ".join(f"{f.filename.rsplit('/', 2)[-1]}:{f.lineno}" for f in reversed(x.traceback))
                     + "\n")
    _TRACE["snap"] = None


def _mem_dump(tag: str, mgr, rec) -> None:
    """``CRON_BENCH_MEMDUMP=<prefix>``: per informer, the objects cached and their deep size
    (each object counted once, in the first place it is reached), the wire memo, the
    reconciler's memos, the derived child memos by slot, pymalloc's arena statistics, the live
    futures and container types, appended to ``<prefix>.<pid>.txt`` (plus the RSS after every
    phase and what the process held at the phase's highest RSS).  A diagnostic: the walk
    itself raises the peak RSS it reports."""
    prefix = os.environ.get("CRON_BENCH_MEMDUMP")
    if not prefix:
        return
    import gc
    from collections import Counter

    gc.collect()
    seen: set = set()

    def deep(o) -> int:
        stack, total = [o], 0
        while stack:
            x = stack.pop()
            i = id(x)
            if i in seen:
                continue
            seen.add(i)
            total += sys.getsizeof(x)
            if isinstance(x, dict):
                stack.extend(x.keys())
                stack.extend(x.values())
            elif isinstance(x, (list, tuple, set, frozenset)):
                stack.extend(x)
            elif hasattr(x, "__slots__"):
                stack.extend(getattr(x, s) for s in x.__slots__ if hasattr(x, s))
            elif hasattr(x, "__dict__") and not isinstance(x, type):
                stack.append(x.__dict__)
        return total

    with open(f"{prefix}.{os.getpid()}.txt", "a") as fh:
        fh.write(f"== {tag}: rss {_rss_mib():.1f} MiB\n")
        for name, inf in sorted(mgr.cache._informers.items(), key=lambda kv: str(kv[0])):
            st = deep(inf.store) / 2**20
            dv = deep(inf.derived) / 2**20
            stale = sum(1 for k, d in inf.derived.items() if getattr(d, "obj", None) is not None
                        and d.obj is not inf.store.get(k))
            fh.write(f"  informer {name}: {len(inf.store)} objects store {st:.2f} MiB derived {dv:.2f} MiB"
                     f" (derived of another version: {stale})\n")
        if rec.codecs is not None:
            fh.write(f"  wire memo: {rec.codecs.memo.stats()}\n")
        for attr, val in sorted(vars(rec).items()):
            if isinstance(val, (dict, list, set)) and len(val) > 100:
                fh.write(f"  rec.{attr}: {len(val)} entries {deep(val) / 2**20:.2f} MiB\n")
        for name, inf in sorted(mgr.cache._informers.items(), key=lambda kv: str(kv[0])):
            if not inf.store:
                continue
            keys = sorted(inf.store)
            for k in (keys[0], keys[-1]):
                o = inf.store[k]
                seen.clear()
                parts = {f: deep(v) for f, v in o.items()} if isinstance(o, dict) else {}
                seen.clear()
                d = inf.derived.get(k)
                fh.write(f"  sample {k}: {parts} derived {deep(d) if d is not None else 0} "
                         f"{type(d).__name__}\n    {json.dumps(o, default=str)[:1500]}\n")
                if d is not None:
                    kinds = [(s, type(getattr(d, s, None)).__name__) for s in getattr(d, "__slots__", ())]
                    fh.write(f"    derived: {kinds}\n")
        # the unique bytes of each derived slot, stores walked first: the oldest and the newest
        # finished child (LIST-decoded vs watch-decoded)
        seen.clear()
        for inf in mgr.cache._informers.values():
            deep(inf.store)
        for inf in mgr.cache._informers.values():
            fin = [(int((inf.store[k].get("metadata") or {}).get("resourceVersion") or 0), k)
                   for k, d in inf.derived.items() if getattr(d, "finished", False)]
            if not fin:
                continue
            fin.sort()
            groups: dict = {}
            for k, d in inf.derived.items():
                g = groups.setdefault(bool(getattr(d, "finished", False)), [0, 0, Counter()])
                g[0] += 1
                for s in d.__slots__:
                    n = deep(getattr(d, s, None))
                    g[1] += n
                    g[2][s] += n
            for f, (n, b, per) in groups.items():
                fh.write(f"  derived finished={f}: {n} memos, {b / max(1, n):.0f} B each: "
                         + str({s: round(v / max(1, n)) for s, v in per.items()}) + "\n")
            for _, k in (fin[0], fin[-1]):
                d = inf.derived[k]
                fh.write(f"  derived {k}: " + str({s: deep(getattr(d, s, None)) for s in d.__slots__}) + "\n")
                he = getattr(d, "history_entry", None)
                if he is not None:
                    fh.write(f"    history_entry: {he!r}\n")
        seen.clear()
        # pymalloc's own accounting (arenas vs allocated blocks: what fragmentation costs)
        r, w = os.pipe()
        saved = os.dup(2)
        os.dup2(w, 2)
        try:
            sys._debugmallocstats()
        finally:
            os.dup2(saved, 2)
            os.close(w)
            os.close(saved)
        txt = b""
        while True:
            chunk = os.read(r, 1 << 16)
            if not chunk:
                break
            txt += chunk
        os.close(r)
        tail = [ln for ln in txt.decode(errors="replace").splitlines() if ln.startswith(("#", "Total"))
                or "arenas" in ln or "bytes in" in ln]
        fh.write("  pymalloc: " + " | ".join(x.strip() for x in tail[-14:]) + "\n")
        futs = [o for o in gc.get_objects() if type(o).__name__ == "Future"]
        fh.write(f"  futures alive: {len(futs)} done {sum(1 for f in futs if f.done())}\n")
        for f in futs[:: max(1, len(futs) // 4)][:4]:
            refs = [r for r in gc.get_referrers(f) if r is not futs]
            names = [type(r).__name__ + ":" + str(getattr(r, "cr_code", getattr(r, "f_code", "")))[:60]
                     for r in refs][:4]
            fh.write(f"    future done={f.done()} referrers: {names}\n")
            for r in refs[:2]:
                rr = [type(x).__name__ for x in gc.get_referrers(r) if x is not refs][:5]
                fh.write(f"      {type(r).__name__} <- {rr}\n")
        cnt = Counter(type(o).__name__ for o in gc.get_objects())
        fh.write("  gc objects: " + ", ".join(f"{k} {v}" for k, v in cnt.most_common(12)) + "\n")


def _maxrss_mib() -> float:
    """Peak resident size: the kernel's high-water mark ``VmHWM`` (``/proc/self/status``), never
    below the resident size now.  ``ru_maxrss`` read below the same moment's ``statm`` RSS on the
    box (round-5 verdict: a "peak" under the end RSS), so it is only the fallback."""
    hwm = 0.0
    try:
        with open("/proc/self/status") as fh:
            for line in fh:
                if line.startswith("VmHWM:"):
                    hwm = int(line.split()[1]) / 1024  # kB
                    break
    except (OSError, ValueError, IndexError):
        hwm = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024
    return max(hwm, _rss_mib())


def _rss_mib() -> float:
    """Resident size now (``/proc/self/statm``), next to the peak."""
    try:
        with open("/proc/self/statm") as fh:
            return int(fh.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 2**20
    except (OSError, ValueError, IndexError):
        return 0.0


async def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", required=True)
    ap.add_argument("--namespace", required=True)
    ap.add_argument("--shard-index", type=int, required=True)
    ap.add_argument("--shard-count", type=int, required=True)
    ap.add_argument("--start-ns", type=int, required=True)
    ap.add_argument("--workers", type=int, default=10)
    ap.add_argument("--history-limit", type=int, default=10)
    ap.add_argument("--qps", type=float, default=-1.0)
    ap.add_argument("--burst", type=int, default=50)
    ap.add_argument("--max-inflight", type=int, default=128)
    ap.add_argument("--tick-reserve", type=int, default=-1, help="--tick-burst-reserve of the operator's client")
    ap.add_argument("--no-defer", action="store_true", help="ReconcilerOptions.defer_status_write=False (A/B)")
    ap.add_argument("--no-compact", action="store_true", help="ReconcilerOptions.compact_child_status=False (A/B)")
    ap.add_argument("--mode", default="optimized")
    ap.add_argument("--routing", default="hash", choices=["hash", "labels"])
    ap.add_argument("--ca-file", default="", help="https --url: verify the apiserver against this CA (as localhost)")
    a = ap.parse_args()

    from ..api.v1alpha1 import CRON_GVR
    from ..controller.reconciler import ReconcilerOptions
    from ..controller.setup import setup_with_manager
    from ..runtime.client import Client
    from ..runtime.controller import shard_of
    from ..runtime.http import HttpTransport
    from ..runtime.kubeconfig import RestConfig
    from ..runtime.manager import Manager, ManagerOptions
    from ..utils.clock import FakeClock
    from ..utils.logging import new_from_options, set_logger

    set_logger(new_from_options(encoder="json", level="error", stream=open(os.devnull, "w")))
    clock = FakeClock(a.start_ns)
    rc = RestConfig(host=a.url)
    if a.ca_file:
        with open(a.ca_file, "rb") as fh:
            rc = RestConfig(host=a.url, ca_data=fh.read(), tls_server_name="localhost")
    client = Client(HttpTransport(rc, pool_size=max(16, a.workers * 2, a.max_inflight)), qps=a.qps, burst=a.burst,
                    max_inflight=a.max_inflight, low_reserve=a.tick_reserve)
    opts = ReconcilerOptions.reference() if a.mode == "reference" else \
        ReconcilerOptions(defer_status_write=not a.no_defer, compact_child_status=not a.no_compact)
    mgr = Manager(client, ManagerOptions(clock=clock, max_concurrent_reconciles=a.workers,
                                         health_probe_bind_address="0", metrics_bind_address="0",
                                         namespace=a.namespace, shard_index=a.shard_index,
                                         shard_count=a.shard_count, shard_routing=a.routing))
    ctrl, rec = await setup_with_manager(mgr, opts)
    task = asyncio.get_running_loop().create_task(mgr.start())
    await asyncio.wait_for(mgr.started.wait(), 120)
    cron_inf = rec.cron_informer
    assert cron_inf is not None
    # the Crons this shard owns, paged (only names are kept: a whole-fleet LIST held at once
    # would set this process's peak memory)
    owned_keys: List[str] = []
    cont = None
    while True:
        page = await client.list(CRON_GVR, a.namespace, limit=500, continue_=cont)
        owned_keys += [f"{a.namespace}/{o['metadata']['name']}" for o in page.get("items") or []
                       if shard_of(a.namespace, o["metadata"]["name"], a.shard_count) == a.shard_index]
        cont = (page.get("metadata") or {}).get("continue")
        if not cont:
            break
    owned_keys.sort()
    # label routing: wait until the assigner has labelled every owned Cron and its children
    deadline = time.monotonic() + 300
    while any(k not in cron_inf.store for k in owned_keys) or (
            rec.shard_assigner is not None and rec.shard_assigner.pending()):
        if time.monotonic() > deadline:
            raise TimeoutError("shard assignment did not finish")
        await asyncio.sleep(0.05)
    await ctrl.wait_idle(timeout=120)

    from .harness import RvTracker, SettleTracker, completed_pred, fired_pred, job_informer

    tracker = SettleTracker(cron_inf, owned_keys)
    rv_tracker = RvTracker(job_informer(mgr, rec))
    n_owned = len(owned_keys)
    lat: List[float] = []
    tick_wall = [0.0]
    creates = [0]

    def on_create(key, missed, created) -> None:
        lat.append(time.perf_counter() - tick_wall[0])
        creates[0] += 1

    rec.latency_observer = on_create
    from ..utils.gctune import GcStats

    gcs = GcStats().start()
    out = sys.stdout
    _trace_dump("ready")
    _mem_dump("ready", mgr, rec)
    out.write(json.dumps({"ready": True, "owned": n_owned, "maxrss_mib": _maxrss_mib(), "rss_mib": _rss_mib()})
              + "\n")
    out.flush()

    loop = asyncio.get_running_loop()
    peak = [0.0, ""]
    if os.environ.get("CRON_BENCH_MEMDUMP"):
        async def sample() -> None:  # what the process held at its highest RSS
            while True:
                await asyncio.sleep(0.01)
                r = _rss_mib()
                if r > peak[0]:
                    pend = []
                    for inf in mgr.cache._informers.values():
                        w = getattr(getattr(inf, "_watch", None), "_s", None)
                        n = getattr(w, "_n", None)
                        pend.append(getattr(n, "pending", -1) if n is not None else -1)
                    lim, gate = client.limiter, client.inflight
                    peak[0], peak[1] = r, (
                        f"rss {r:.1f} active {ctrl.active} released {ctrl.released} queue {len(ctrl.queue)} "
                        f"tasks {len(asyncio.all_tasks())} limiter waiting {lim.waiting if lim else 0} "
                        f"inflight {gate.inflight if gate else 0} gate waiting {gate.waiting if gate else 0} "
                        f"watch pending {pend}")
        sampler = loop.create_task(sample())  # noqa: F841
    # an absorb command lists every owned job's resourceVersion: ~45 bytes a job, far past
    # StreamReader's 64 KiB line limit at 10,000 Crons
    reader = asyncio.StreamReader(limit=256 << 20)
    await loop.connect_read_pipe(lambda: asyncio.StreamReaderProtocol(reader), sys.stdin)

    async def settled(phase: str, tick_ns: int) -> None:
        tracker.begin(completed_pred(a.history_limit) if phase == "completion"
                      else fired_pred(tick_ns, a.history_limit))
        while True:
            if (phase == "completion" or creates[0] >= n_owned) and not tracker.pending and ctrl.queue.idle():
                return
            await tracker.wait_drained()

    prof = None
    while True:
        line = await reader.readline()
        if not line:
            break
        msg = json.loads(line)
        if msg.get("cmd") == "stop":
            break
        if msg.get("cmd") == "profile":  # cProfile of this shard over the harness's timed steps
            import cProfile

            if msg.get("action") == "start":
                prof = cProfile.Profile()
                prof.enable()
            elif prof is not None:
                prof.disable()
                prof.dump_stats(msg["path"])
                prof = None
            out.write(json.dumps({"ok": True}) + "\n")
            out.flush()
            continue
        if msg.get("cmd") == "absorb":  # a training-operator write reached every job: absorb it
            rv_tracker.begin(msg.get("rvs") or {})
            while rv_tracker.pending or not ctrl.queue.idle() or ctrl.in_flight():
                await asyncio.sleep(0.002)
            out.write(json.dumps({"ok": True}) + "\n")
            out.flush()
            continue
        if msg.get("cmd") == "time":
            lat.clear()
            creates[0] = 0
            tick_wall[0] = time.perf_counter()
            clock.set(int(msg["ns"]))
            await settled(msg.get("phase", "fire"), int(msg.get("tick_ns", msg["ns"])))
            if os.environ.get("CRON_BENCH_TRIM"):
                import ctypes
                ctypes.CDLL("libc.so.6").malloc_trim(0)
            if os.environ.get("CRON_BENCH_TRACEMALLOC") and msg.get("phase", "fire") == "fire":
                _trace_diff(int(os.environ.get("CRON_BENCH_TRACE_FROM", "3")),
                            int(os.environ.get("CRON_BENCH_TRACE_TO", "9")))
            if os.environ.get("CRON_BENCH_MEMDUMP"):
                with open(f"{os.environ['CRON_BENCH_MEMDUMP']}.{os.getpid()}.txt", "a") as fh:
                    fh.write(f"  {msg.get('phase', 'fire')} {msg['ns']}: rss {_rss_mib():.1f} "
                             f"maxrss {_maxrss_mib():.1f} | peak: {peak[1]}\n")
                peak[0] = 0.0
            # counters are cumulative: the harness differences them over its timed window
            ru = resource.getrusage(resource.RUSAGE_SELF)
            out.write(json.dumps({"ok": True, "lat": lat, "settle_s": time.perf_counter() - tick_wall[0],
                                  "reconciles": ctrl.reconciles,
                                  "requests": client.requests, "by_verb": dict(client.requests_by_verb),
                                  "cpu": time.process_time(), "gc_s": gcs.seconds,
                                  "gc_collections": list(gcs.collections), "gc_gen_s": list(gcs.gen_seconds),
                                  "maxrss_mib": _maxrss_mib(), "rss_mib": _rss_mib(),
                                  # context switches (voluntary: the loop slept on I/O; involuntary:
                                  # preempted by another runnable task on this CPU)
                                  "csw": [ru.ru_nvcsw, ru.ru_nivcsw]}) + "\n")
            out.flush()
    _trace_dump("end")
    _mem_dump("end", mgr, rec)
    mgr.stop()
    try:
        await asyncio.wait_for(task, 30)
    except Exception:  # noqa: BLE001
        pass
    await client.close()
    return 0


if __name__ == "__main__":
    if os.environ.get("CRON_BENCH_TRACEMALLOC"):
        import tracemalloc

        tracemalloc.start(6)
    from ..runtime import aioloop

    aioloop.install()  # an operator process: the native loop core, as `cron-operator start` uses
    _prof = os.environ.get("CRON_BENCH_SHARD_PROFILE")
    if _prof:  # cProfile of the whole worker (setup included): <prefix>.<pid>.pstats
        import cProfile

        cProfile.run("asyncio.run(main())", f"{_prof}.{os.getpid()}.pstats")
    else:
        sys.exit(asyncio.run(main()))
