"""Reconcile-throughput benchmark: N Crons on ``* * * * *`` with historyLimit=10.

This is the headline configuration of ``BASELINE.json``: "1000 Cron CRs at
``* * * * *``, historyLimit=10 -- reconcile-throughput + GC stress", measured as
reconciles/sec and the p50 schedule->create latency.

One **step** is one schedule tick across all Crons, in virtual time:

1. the timer starts; cluster side, the jobs of the previous tick run: with
   ``lifecycle="realistic"`` the training-operator's writes (Created, one
   ``replicaStatuses`` write per pod, Running) reach every job one stage at a time
   and the operator absorbs each before the next (the harness's write calls are
   excluded from the timed region -- another controller's requests -- the
   operator's absorption is not); then every job is marked Succeeded (apiserver
   work, not operator work, but kept inside the timed region -- conservative);
2. the operator's clock (and the apiserver's) jumps to the next minute
   boundary, which fires every Cron's ``RequeueAfter``;
3. the operator reconciles: moves finished jobs into ``status.history``,
   deletes the ones beyond ``historyLimit`` (GC), creates the tick's job,
   patches status, and absorbs the resulting watch events;
4. the timer stops once every Cron shows ``lastScheduleTime == tick`` with the
   new job active and the expected history, and the work queue is idle.

Nothing is skipped inside the timed region: every reconcile the operator
decides to run, every API request, every watch event.  Reported:

* ``cron_reconciles_per_s`` -- Crons fully reconciled for a tick per second
  (``n_crons * steps / elapsed``): the unit of useful work;
* ``raw_reconciles_per_s`` -- Reconcile() invocations per second (includes the
  event-driven follow-ups; a design that needs fewer of them scores lower here,
  which is why it is not the headline);
* ``p50/p99 tick->create latency`` -- from the clock jump to each CREATE response;
* API requests per fire (the request-count model of SURVEY section 3.2).

``transport="http"`` runs the fake apiserver in a separate process (the
operator talks HTTP/JSON + watch streams, like against kind/envtest);
``transport="memory"`` keeps everything in one event loop.
``mode="reference"`` runs the reference algorithm (ReconcilerOptions.reference():
live LIST per reconcile, ``finished=now``, no event filtering).
"""
from __future__ import annotations

import asyncio
import collections
import json
import os
import statistics
import subprocess
import sys
import threading
import time
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional

from ..api.meta import GroupVersionResource
from ..api.v1alpha1 import CRON_GVR, new_cron
from ..utils.gotime import NANOS

PYTORCHJOBS = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")

# 2026-01-01T12:00:00Z: crons are created here; step k ticks at +k minutes
T0_NS = 1767268800 * NANOS
# completion_writes="interleaved": completion PATCHes the fake apiserver applies per loop turn
COMPLETION_WRITES_PER_TURN = 32
# a settle wait's poll once no Cron is pending (the controller's queue draining its last items)
SETTLE_POLL_S = 0.0005


# Server-side latency models for the fake apiserver (seconds per verb, applied after setup).
# "etcd" is an ASSUMED model of a small kube-apiserver + etcd on SSD -- writes pay a quorum
# fsync, reads come from the watch cache / etcd range -- not a measurement; it turns the bench
# from CPU-bound into latency-bound, where request count per fire and worker count dominate.
# ``list_per_object``: a label-selected LIST is answered by scanning every object of the resource
# in the namespace (kube-apiserver filters the watch cache -- or an etcd range -- by label; there
# is no label index), charged per object scanned (ASSUMED 1 us: a watch-cache label filter; an
# etcd range read and decode costs several times that).  The fake apiserver itself answers from
# a label index, so that scan is latency here, not fixture CPU.
LATENCY_PROFILES: Dict[str, Dict[str, float]] = {
    "none": {},
    "etcd": {"create": 0.008, "update": 0.006, "patch": 0.006, "delete": 0.006, "get": 0.001, "list": 0.004,
             "list_per_object": 1e-6},
}


def pytorchjob_template() -> Dict[str, Any]:
    """A 1 master + 1 worker PyTorchJob (no-op container), like the reference example."""
    def replica(n: int) -> Dict[str, Any]:
        return {"replicas": n, "restartPolicy": "OnFailure", "template": {"spec": {"containers": [{
            "name": "pytorch", "image": "rocm/pytorch:latest",
            "command": ["python", "-c", "print('tick')"],
            "resources": {"limits": {"amd.com/gpu": 1}}}]}}}
    return {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
            "metadata": {"labels": {"app": "bench"}},
            "spec": {"pytorchReplicaSpecs": {"Master": replica(1), "Worker": replica(1)}}}


@dataclass
class BenchConfig:
    n_crons: int = 1000
    steps: int = 5
    warmup: int = 2
    history_limit: int = 10
    mode: str = "optimized"          # optimized | reference
    transport: str = "http"          # http | memory
    qps: float = -1.0                # client QPS (-1 = unthrottled)
    burst: int = 50
    max_inflight: int = 128          # client cap on concurrent requests (cmd/main.py DEFAULT_MAX_INFLIGHT)
    defer_writes: bool = True        # optimized mode: ReconcilerOptions.defer_status_write (A/B switch)
    workers: int = 10
    namespace: str = "bench"
    log_level: str = "error"
    step_timeout: float = 600.0
    seed_history: bool = True  # requires history_limit >= 1
    apiserver_profile: str = ""  # write a cProfile of the apiserver process over the timed steps here
    shard_profile: str = ""      # shards > 1: cProfile of each shard over the timed steps, <prefix>.<i>.pstats
    # operator shards (--shard-count): >1 runs one operator process per shard against the apiserver (or,
    # with apiserver_partitions, against its own partition)
    # (bench/shard_worker.py); 1 keeps the operator in this process
    shards: int = 1
    # how shards split the watch traffic: "hash" (every shard sees every event) or "labels"
    # (kubedl.io/shard labels + per-shard selectors, controller/sharding.py)
    shard_routing: str = "labels"
    # per-verb server-side latency (LATENCY_PROFILES name), applied after setup; needs transport="http"
    apiserver_latency: str = "none"
    # the fake apiserver process: "native" (apiserver/native.py, the C++ _apiserverd: the fixture
    # off the critical path) or "python" (apiserver/server.py + http.py; the A/B arm)
    apiserver_impl: str = "native"
    # fake apiserver processes: 1 (every shard against one server), or `shards` with label
    # routing -- a partitioned cluster, server i holding the Crons that hash to shard i (shard_of)
    # and their jobs, so no one single-threaded fixture bounds the shards (bench.py partitioned_*)
    apiserver_partitions: int = 1
    # instant lifecycle, native fixture: how the harness's "every job finishes" writes reach the
    # fake apiserver -- "interleaved" (queued, a few applied per server loop turn between the turns
    # serving the operator, as a training operator's writes interleave with everyone else's at a
    # real apiserver) or "batch" (rounds 1-5 and most of 6: all of them in one call that holds the
    # server and its watches for its length); the fixture's CPU for them is counted either way
    completion_writes: str = "interleaved"
    # events per resource the fake apiserver keeps for watch resume (a bounded watch cache: the
    # soak's fixture memory stays flat; 20,000 is ~5 ticks of 1000 Crons' job events)
    watch_window: int = 20_000
    # the fake apiserver serves HTTPS (self-signed CN=localhost) and every operator connection
    # verifies it against that CA, as against a real cluster's apiserver; needs transport="http"
    tls: bool = False
    # the operator's apiserver connections: native (_netconn) or asyncio's transports (A/B rows)
    native_http: bool = True
    # how the previous tick's jobs run before the tick: "realistic" -- the training-operator's
    # status sequence (Created, one replicaStatuses write per pod, Running, then Succeeded:
    # trainingop.operator.lifecycle_statuses), each write absorbed by the operator before the
    # next; "instant" -- a single Succeeded write (rounds 1-4)
    lifecycle: str = "realistic"
    # each Cron gets its own template (a per-Cron container command) instead of one shared by
    # all: nothing in the caches is then shared across Crons' specs (scripts/bench_scale.py)
    distinct_templates: bool = False
    # sample the first timed tick every 250 ms (BenchResult.tick_timeline; bench_configs rows)
    tick_timeline: bool = False
    # burst tokens deferrable (low-priority) writes may not spend (cmd/main.py --tick-burst-reserve)
    tick_reserve: int = -1
    # run even a single shard in its own process (bench/shard_worker.py): its peak RSS is then
    # the operator's alone (operator_maxrss_mib), not the harness's
    operator_process: bool = False
    # optimized mode: ReconcilerOptions.compact_child_status (A/B switch of the child-cache trim)
    compact_children: bool = True
    # one process: run leader election (the chart's default) on the operator's Lease; the result
    # reports whether it was ever lost and the longest renewal
    leader_elect: bool = False


@dataclass
class BenchResult:
    config: Dict[str, Any]
    steps: int
    elapsed_s: float
    ms_per_step: float
    cron_reconciles_per_s: float
    raw_reconciles_per_s: float
    p50_latency_ms: float
    p99_latency_ms: float
    max_latency_ms: float
    api_requests_per_fire: float
    api_requests_by_verb: Dict[str, int]
    reconciles_per_fire: float
    step_ms: List[float] = field(default_factory=list)
    phase_ms: Dict[str, List[float]] = field(default_factory=dict)
    engine: str = ""
    fastjson_native: bool = False
    # CPU seconds burnt in the timed region by the operator process and the apiserver process
    cpu_s_operator: float = 0.0
    cpu_s_apiserver: float = 0.0
    # peak RSS of each operator shard process (sharded runs; the in-process run shares the harness)
    operator_maxrss_mib: List[float] = field(default_factory=list)
    # shard processes: peak RSS once caches were synced and the first pass done (start-up's share
    # of the peak), and resident size at the end of the run
    operator_ready_maxrss_mib: List[float] = field(default_factory=list)
    operator_rss_mib: List[float] = field(default_factory=list)
    # cyclic-GC collections per generation and pause time in the operator process(es), timed region
    operator_gc: Dict[str, Any] = field(default_factory=dict)
    # one process: a starting (or newly elected) operator over the seeded cluster -- seconds from
    # Manager.start() to synced caches, and to the first pass over every Cron done (the queue idle)
    startup_sync_s: float = 0.0
    startup_first_pass_s: float = 0.0
    # one process, throttled: the client bucket's tokens and waiters (low/normal/high) at each
    # timed tick, and each tick's p50 tick->create
    tick_tokens: List[float] = field(default_factory=list)
    tick_waiting: List[List[int]] = field(default_factory=list)
    tick_p50_ms: List[float] = field(default_factory=list)
    tick_lat_q_ms: List[List[float]] = field(default_factory=list)
    tick_timeline: List[Dict[str, Any]] = field(default_factory=list)
    limiter_max_wait_s: List[float] = field(default_factory=list)  # per priority [low, normal, high]
    limiter_aged_grants: int = 0
    # leader_elect: the Lease was lost at some point / the longest successful renewal window (s)
    lease_lost: Optional[bool] = None
    lease_max_renew_s: Optional[float] = None
    # sharded runs, per timed step: the operator shards' CPU s (summed) and the apiserver's CPU s
    # (the harness's own lifecycle writes taken out) -- the soak's per-window split
    step_cpu_operator_s: List[float] = field(default_factory=list)
    step_cpu_apiserver_s: List[float] = field(default_factory=list)
    # apiserver_partitions > 1: each fake apiserver's CPU s over the timed steps (writes taken out)
    cpu_s_apiserver_parts: List[float] = field(default_factory=list)
    # sharded runs: the shard processes' context switches over the timed steps, summed
    # [voluntary (waits for I/O), involuntary (preempted)]
    operator_ctx_switches: List[int] = field(default_factory=list)

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)


def _pct(xs: List[float], p: float) -> float:
    if not xs:
        return float("nan")
    s = sorted(xs)
    k = min(len(s) - 1, max(0, int(round(p / 100.0 * (len(s) - 1)))))
    return s[k]


class _RemoteServer:
    """The fake apiserver in a child process, driven over HTTP."""

    def __init__(self, tls: bool = False, impl: str = "native", watch_window: int = 20_000):
        self.impl = impl
        self.watch_window = watch_window
        self.proc: Optional[subprocess.Popen] = None
        self.url = ""
        self.tls_dir = ""
        self.ca_file = ""
        if tls:
            import tempfile

            self.tls_dir = tempfile.mkdtemp(prefix="bench-tls-")
            self.ca_file = os.path.join(self.tls_dir, "tls.crt")

    def rest_config(self):
        """The operator's RestConfig for this server (CA-verified against host name localhost under TLS)."""
        from ..runtime.kubeconfig import RestConfig

        if not self.tls_dir:
            return RestConfig(host=self.url)
        with open(self.ca_file, "rb") as fh:
            return RestConfig(host=self.url, ca_data=fh.read(), tls_server_name="localhost")

    def ssl_context(self):
        """The harness's own admin connection: the CA, without the host-name check (it dials the IP)."""
        import ssl

        if not self.tls_dir:
            return None
        ctx = ssl.create_default_context(cafile=self.ca_file)
        ctx.check_hostname = False
        return ctx

    def start(self) -> str:
        env = dict(os.environ)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        extra = ["--tls-dir", self.tls_dir] if self.tls_dir else []
        self.proc = subprocess.Popen([sys.executable, "-m", "cron_operator_amd.bench.apiserver_proc",
                                      "--start-ns", str(T0_NS), "--impl", self.impl,
                                      "--watch-window", str(self.watch_window)] + extra,
                                     stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, text=True)
        assert self.proc.stdout is not None
        line = self.proc.stdout.readline()
        if not line.startswith("LISTENING "):
            rest = self.proc.stdout.read() if self.proc.poll() is not None else ""
            raise RuntimeError(f"fake apiserver failed to start: {line}{rest}")
        self.url = line.split()[1].strip()
        # keep draining the pipe: a child blocked on a full stdout pipe would stall the bench
        self.tail: "collections.deque[str]" = collections.deque(maxlen=50)
        threading.Thread(target=self._drain, daemon=True, name="apiserver-stdout").start()
        return self.url

    def _drain(self) -> None:
        assert self.proc is not None and self.proc.stdout is not None
        for ln in self.proc.stdout:
            self.tail.append(ln)

    def stop(self) -> None:
        if self.proc is not None and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        if self.tls_dir:
            import shutil

            shutil.rmtree(self.tls_dir, ignore_errors=True)


class SettleTracker:
    """The owned Crons whose status has not reached the current phase's target yet.

    An informer handler re-evaluates one Cron per event (O(1)), so waiting for a
    step to settle is a counter check instead of a scan of every Cron on each poll --
    a scan that ran inside the operator's process and event loop every 2 ms and made
    the harness itself cost O(N) per poll."""

    def __init__(self, informer, keys: Optional[List[str]] = None):
        from ..runtime.informer import EventHandler

        self.inf = informer
        self.keys = set(keys) if keys is not None else None
        self.pred = None
        self.pending: set = set()
        self.drained: Optional[asyncio.Event] = None  # set while nothing is pending
        informer.add_handler(EventHandler(on_add=self._on, on_update=lambda old, new: self._on(new)))

    def _on(self, obj: Dict[str, Any]) -> None:
        if self.pred is None:
            return
        from ..runtime.informer import obj_key

        k = obj_key(obj)
        if self.keys is not None and k not in self.keys:
            return
        if self.pred(obj):
            self.pending.discard(k)
            if not self.pending and self.drained is not None:
                self.drained.set()
        else:
            self.pending.add(k)
            if self.drained is not None:
                self.drained.clear()

    def begin(self, pred) -> None:
        self.pred = pred
        self.pending = {k for k, o in self.inf.store.items()
                        if (self.keys is None or k in self.keys) and not pred(o)}
        if self.keys is not None:
            self.pending |= {k for k in self.keys if k not in self.inf.store}
        if self.drained is None:
            self.drained = asyncio.Event()
        if self.pending:
            self.drained.clear()
        else:
            self.drained.set()

    async def wait_drained(self, timeout: float = 0.05) -> None:
        """Until nothing is pending (an event wakes the waiter: no polling while the phase's
        events arrive), or ``timeout`` -- then the caller checks its full condition again."""
        if self.pending and self.drained is not None:
            try:
                await asyncio.wait_for(self.drained.wait(), timeout)
            except asyncio.TimeoutError:
                pass
        else:
            await asyncio.sleep(SETTLE_POLL_S)


class RvTracker:
    """The children whose latest write (a training-operator status write) the operator's job
    informer has not seen yet: ``begin`` takes ``{namespace/name: resourceVersion}`` of the
    writes, an event handler drops a key once its object reaches that version (O(1) per
    event).  Keys the informer does not hold (another shard's jobs) are not waited for."""

    def __init__(self, informer):
        from ..runtime.informer import EventHandler

        self.inf = informer
        self.want: Dict[str, int] = {}
        self.pending: set = set()
        informer.add_handler(EventHandler(on_add=self._on, on_update=lambda old, new: self._on(new)))

    @staticmethod
    def _rv(obj: Dict[str, Any]) -> int:
        try:
            return int((obj.get("metadata") or {}).get("resourceVersion") or 0)
        except ValueError:
            return 0

    def _on(self, obj: Dict[str, Any]) -> None:
        if not self.pending:
            return
        from ..runtime.informer import obj_key

        k = obj_key(obj)
        w = self.want.get(k)
        if w is not None and self._rv(obj) >= w:
            self.pending.discard(k)

    def begin(self, rvs: Dict[str, Any]) -> None:
        self.want = {k: int(v) for k, v in rvs.items()}
        store = self.inf.store
        self.pending = {k for k, w in self.want.items() if k in store and self._rv(store[k]) < w}


def job_informer(mgr, rec, gvr: GroupVersionResource = None):
    """The operator's own informer of the bench's job kind (cache mode: the label-indexed child
    informer; live mode: the owned-kind watch) -- not a shard assigner's "unassigned" watch."""
    gvr = gvr or PYTORCHJOBS
    for inf in list(rec.child_informers.values()) + mgr.cache.informers():
        if inf.target == gvr and "notin" not in (inf.label_selector or ""):
            return inf
    raise RuntimeError(f"no informer for {gvr}")


def lifecycle_stages(cfg: "BenchConfig") -> int:
    """Training-operator status writes per job before the final Succeeded one (0: instant)."""
    if cfg.lifecycle != "realistic":
        return 0
    from ..trainingop.operator import lifecycle_statuses

    return len(lifecycle_statuses(pytorchjob_template(), "", "")) - 1


def fired_pred(tick_ns: int, want_hist: int):
    """Status of a Cron that ran tick ``tick_ns``: one active job, ``want_hist`` in history."""
    from ..utils.gotime import UTC, GoTime

    want_ts = GoTime(tick_ns // NANOS, 0, UTC).rfc3339()

    def pred(obj: Dict[str, Any]) -> bool:
        st = obj.get("status") or {}
        return st.get("lastScheduleTime") == want_ts and len(st.get("active") or ()) == 1 and \
            len(st.get("history") or ()) == want_hist
    return pred


def completed_pred(want_hist: int):
    """Status of a Cron whose job finished: nothing active, ``want_hist`` in history (GC done)."""
    def pred(obj: Dict[str, Any]) -> bool:
        st = obj.get("status") or {}
        return not st.get("active") and len(st.get("history") or ()) == want_hist
    return pred


def _proc_cpu(remote: "_RemoteServer") -> float:
    """CPU s (user + system) of a fake apiserver process so far."""
    if remote.proc is None:
        return 0.0
    try:
        with open(f"/proc/{remote.proc.pid}/stat") as fh:
            f = fh.read().rsplit(")", 1)[1].split()
        return (int(f[11]) + int(f[12])) / os.sysconf("SC_CLK_TCK")
    except (OSError, IndexError, ValueError):
        return float("nan")


def _cpu_times(remote) -> "tuple[float, float]":
    """(operator process CPU s, apiserver CPU s) -- the apiserver shares our process in memory
    mode; ``remote`` may be a list of partitions (their CPU summed)."""
    me = time.process_time()
    if remote is None:
        return me, 0.0
    parts = remote if isinstance(remote, list) else [remote]
    return me, sum(_proc_cpu(r) for r in parts)


async def run(cfg: BenchConfig, on_step=None) -> BenchResult:
    from ..utils.logging import new_from_options, set_logger

    set_logger(new_from_options(encoder="json", level=cfg.log_level, stream=open(os.devnull, "w")))
    if cfg.tls and cfg.transport != "http":
        raise ValueError("tls needs transport='http'")
    from ..runtime import fasthttp

    saved_native = fasthttp.DEFAULT_NATIVE
    if not cfg.native_http:
        fasthttp.DEFAULT_NATIVE = False
    try:
        return await _run(cfg, on_step)
    finally:
        fasthttp.DEFAULT_NATIVE = saved_native


async def _run(cfg: BenchConfig, on_step=None) -> BenchResult:
    from ..controller.reconciler import ReconcilerOptions
    from ..controller.setup import setup_with_manager
    from ..cron.engine import default_engine
    from ..runtime.client import Client, InMemoryTransport
    from ..runtime.manager import Manager, ManagerOptions
    from ..utils import gctune, jsonutil
    from ..utils.clock import FakeClock, RealClock

    clock = FakeClock(T0_NS)
    remote: Optional[_RemoteServer] = None
    remotes: List[_RemoteServer] = []
    ssl_of: Dict[str, Any] = {}
    transports: List[Any] = []
    server = None
    admin = None
    parts = max(1, cfg.apiserver_partitions)
    if parts > 1 and (cfg.transport != "http" or parts != cfg.shards or cfg.shard_routing != "labels"):
        raise ValueError("apiserver_partitions > 1 needs transport='http', label routing and one partition per shard")
    if cfg.transport == "memory":
        from ..api.v1alpha1.crd import crd
        from ..apiserver.server import APIServer
        from ..trainingop.crds import kubeflow_crds

        server = APIServer(clock, gc=False)
        server.install_crd(crd())
        for c in kubeflow_crds():
            server.install_crd(c)
        transport = InMemoryTransport(server)
    else:
        import aiohttp

        from ..runtime.http import HttpTransport

        for _ in range(parts):
            remotes.append(_RemoteServer(tls=cfg.tls, impl=cfg.apiserver_impl, watch_window=cfg.watch_window))
            remotes[-1].start()
            transports.append(HttpTransport(remotes[-1].rest_config(),
                                            pool_size=max(16, cfg.workers * 2, cfg.max_inflight)))
        remote, transport = remotes[0], transports[0]
        ssl_of = {r.url: r.ssl_context() for r in remotes}
        sslctx = ssl_of[remote.url]
        admin = aiohttp.ClientSession(connector=aiohttp.TCPConnector(ssl=sslctx) if sslctx else None)

    async def admin_post(path: str, payload: Dict[str, Any]) -> List[Any]:
        """POST a /debug/fake control to every fake apiserver (partition); their JSON answers."""
        async def one(r: _RemoteServer) -> Any:
            # each partition has its own self-signed CA under TLS
            kw = {"ssl": ssl_of[r.url]} if ssl_of.get(r.url) is not None else {}
            async with admin.post(r.url + path, json=payload, **kw) as resp:
                body = await resp.read()
                return json.loads(body) if body else None
        return list(await asyncio.gather(*(one(r) for r in remotes)))

    async def set_time(ns: int) -> None:
        clock.set(ns)
        if admin is not None:
            await admin_post("/debug/fake/clock", {"nowNs": ns})

    def _ts(ns: int) -> str:
        from ..utils.gotime import UTC, GoTime

        return GoTime(ns // NANOS, 0, UTC).rfc3339()

    async def job_stage(stage: int, start_ns: int, end_ns: int) -> Dict[str, Any]:
        """Write lifecycle stage ``stage`` (-1: Succeeded) to every unfinished job; returns
        ``{namespace/name: resourceVersion}`` of the writes."""
        start, end = _ts(start_ns), _ts(end_ns)
        if server is not None:
            from ..trainingop.operator import lifecycle_status

            rvs: Dict[str, Any] = {}
            for obj in list(server.objects(PYTORCHJOBS, cfg.namespace)):
                if (obj.get("status") or {}).get("completionTime"):
                    continue
                m = obj["metadata"]
                out = server.patch(PYTORCHJOBS, cfg.namespace, m["name"],
                                   {"status": lifecycle_status(obj, stage, start, end)}, "merge", "status")
                rvs[f"{cfg.namespace}/{m['name']}"] = out["metadata"]["resourceVersion"]
            return rvs
        rvs = {}
        for ans in await admin_post("/debug/fake/lifecycle",
                                    {"namespace": cfg.namespace, "stage": stage, "start": start, "end": end}):
            rvs.update(ans["resourceVersions"])
        return rvs

    async def complete_jobs(tick_ns: int) -> None:
        ts = _ts(tick_ns)
        if cfg.lifecycle == "realistic":
            # the jobs of the previous tick were admitted a second after it
            await job_stage(-1, tick_ns - 29 * NANOS, tick_ns)
            return
        if server is not None:
            from ..trainingop.operator import finished_status

            for obj in list(server.objects(PYTORCHJOBS, cfg.namespace)):
                if not (obj.get("status") or {}).get("completionTime"):
                    m = obj["metadata"]
                    server.patch(PYTORCHJOBS, cfg.namespace, m["name"],
                                 {"status": finished_status("PyTorchJob", m["name"], ts, True)}, "merge", "status")
        else:
            req = {"namespace": cfg.namespace, "time": ts}
            if cfg.completion_writes == "interleaved":
                req["perTurn"] = COMPLETION_WRITES_PER_TURN
            await admin_post("/debug/fake/complete", req)


    try:
        # ---------------------------------------------------------------- setup (untimed)
        # one setup client per fake apiserver: a Cron (and its jobs) goes to the partition of the
        # shard it hashes to
        setup_clients = [Client(t, qps=-1) for t in (transports or [transport])]
        setup_client = setup_clients[0]

        def part_of(name: str) -> int:
            if parts == 1:
                return 0
            from ..runtime.controller import shard_of

            return shard_of(cfg.namespace, name, parts)

        for sc in setup_clients:
            try:
                await sc.create(GroupVersionResource("", "v1", "namespaces"),
                                {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": cfg.namespace}}, "")
            except Exception:
                pass
        tmpl = pytorchjob_template()
        crons = []
        for i in range(cfg.n_crons):
            t = jsonutil.deepcopy(tmpl)
            if cfg.distinct_templates:  # every Cron's template differs (its own container command)
                for rs in t["spec"]["pytorchReplicaSpecs"].values():
                    rs["template"]["spec"]["containers"][0]["command"] = ["python", "-c", f"print('tick {i}')"]
            c = new_cron(f"cron-{i:05d}", cfg.namespace, "* * * * *", t, history_limit=cfg.history_limit)
            crons.append(await setup_clients[part_of(c.name)].create(CRON_GVR, c.to_dict(), cfg.namespace))
        # Seed each Cron with a full history (historyLimit finished jobs from the past hour) so
        # every timed tick exercises history GC, as in a long-running deployment.
        if cfg.seed_history:
            from ..api.meta import new_controller_ref
            from ..api.v1alpha1 import CRON_GVK, LABEL_CRON_NAME
            from ..trainingop.operator import finished_status
            from ..utils.gotime import UTC, GoTime

            for j in range(cfg.history_limit):
                t_ns = T0_NS - (cfg.history_limit - j) * 60 * NANOS
                await set_time(t_ns)
                ts = GoTime(t_ns // NANOS, 0, UTC).rfc3339()
                for cobj in crons:
                    name = f"{cobj['metadata']['name']}-{t_ns // NANOS + 60}"
                    job = jsonutil.deepcopy(tmpl)
                    job["metadata"] = {"name": name, "namespace": cfg.namespace,
                                       "labels": {"app": "bench", LABEL_CRON_NAME: cobj["metadata"]["name"]},
                                       "ownerReferences": [new_controller_ref(cobj, CRON_GVK)]}
                    sc = setup_clients[part_of(cobj["metadata"]["name"])]
                    await sc.create(PYTORCHJOBS, job, cfg.namespace)
                    await sc.patch(PYTORCHJOBS, cfg.namespace, name,
                                   {"status": finished_status("PyTorchJob", name, ts, True)}, "merge", "status")
        await set_time(T0_NS + NANOS // 2)
        if admin is not None:  # the apiserver process holds the seeded store for the whole run
            await admin_post("/debug/fake/gc", {})
        latency = LATENCY_PROFILES[cfg.apiserver_latency]
        if latency:
            if admin is None:
                raise ValueError("apiserver_latency needs transport='http'")
            await admin_post("/debug/fake/faults", {"latency": latency})

        if cfg.shards > 1 or cfg.operator_process:
            if remote is None:
                raise ValueError("shards > 1 / operator_process need transport='http'")
            for sc in setup_clients:
                await sc.close()
            return await _run_sharded(cfg, remotes, admin, set_time, complete_jobs, on_step, job_stage)

        client = Client(transport, qps=cfg.qps, burst=cfg.burst, max_inflight=cfg.max_inflight,
                        low_reserve=cfg.tick_reserve)
        opts = ReconcilerOptions.reference() if cfg.mode == "reference" else \
            ReconcilerOptions(defer_status_write=cfg.defer_writes, compact_child_status=cfg.compact_children)
        mgr = Manager(client, ManagerOptions(clock=clock, max_concurrent_reconciles=cfg.workers,
                                             health_probe_bind_address="0", metrics_bind_address="0",
                                             namespace=cfg.namespace, leader_election=cfg.leader_elect,
                                             leader_election_namespace=cfg.namespace,
                                             leader_election_identity="bench-operator",
                                             leader_election_clock=RealClock()))
        ctrl, rec = await setup_with_manager(mgr, opts)
        t_start0 = time.perf_counter()
        mgr_task = asyncio.get_running_loop().create_task(mgr.start())
        await asyncio.wait_for(mgr.started.wait(), 120)
        startup_sync_s = time.perf_counter() - t_start0
        cron_inf = rec.cron_informer
        assert cron_inf is not None

        lat: List[float] = []
        tick_wall = [0.0]
        creates_this_tick = [0]

        def on_create(key, missed, created) -> None:
            lat.append(time.perf_counter() - tick_wall[0])
            creates_this_tick[0] += 1

        rec.latency_observer = on_create

        tracker = SettleTracker(cron_inf)

        async def wait_settled(tick_ns: int, k: int, deadline: float) -> None:
            """Every Cron reflects tick k and the queue is idle."""
            want_hist = cfg.history_limit if cfg.seed_history else min(k - 1, cfg.history_limit)
            tracker.begin(fired_pred(tick_ns, want_hist))
            while True:
                if time.monotonic() > deadline:
                    raise TimeoutError(f"step {k} did not settle (creates={creates_this_tick[0]})")
                if creates_this_tick[0] >= cfg.n_crons and not tracker.pending and ctrl.queue.idle():
                    return
                await tracker.wait_drained()

        want_hist = cfg.history_limit

        async def wait_completed(deadline: float) -> None:
            """Every Cron moved its finished job into history (and GC'd the overflow)."""
            tracker.begin(completed_pred(want_hist))
            while True:
                if time.monotonic() > deadline:
                    raise TimeoutError("completion phase did not settle")
                if not tracker.pending and ctrl.queue.idle():
                    return
                await tracker.wait_drained()

        n_pre = lifecycle_stages(cfg)
        rv_tracker = RvTracker(job_informer(mgr, rec)) if n_pre else None
        write_cpu = [0.0]  # apiserver CPU s inside the harness's lifecycle write calls

        async def run_lifecycle(tick_ns: int, deadline: float) -> float:
            """The previous tick's jobs start: each training-operator write reaches every job,
            then the operator absorbs it (its informer saw every write, nothing queued).
            Returns the seconds spent inside the harness's write calls."""
            writes = 0.0
            for s in range(n_pre):
                w0 = time.perf_counter()
                c0 = _cpu_times(remote)[1]
                rvs = await job_stage(s, tick_ns - 59 * NANOS, tick_ns - 30 * NANOS)
                writes += time.perf_counter() - w0
                write_cpu[0] += _cpu_times(remote)[1] - c0
                rv_tracker.begin(rvs)
                while rv_tracker.pending or not ctrl.queue.idle() or ctrl.in_flight():
                    if time.monotonic() > deadline:
                        raise TimeoutError(f"lifecycle stage {s} was not absorbed")
                    await asyncio.sleep(0.002)
            return writes

        await ctrl.wait_idle(timeout=600)
        startup_first_pass_s = time.perf_counter() - t_start0

        # ---------------------------------------------------------------- steps
        total = cfg.warmup + cfg.steps
        step_ms: List[float] = []
        timed_lat: List[float] = []
        rec0 = req0 = 0
        reqv0: Dict[str, int] = {}
        t_start = 0.0
        excluded = 0.0  # timed steps: seconds inside the harness's lifecycle write calls
        tick_tokens: List[float] = []
        tick_waiting: List[List[int]] = []
        tick_p50_ms: List[float] = []
        tick_lat_q_ms: List[List[float]] = []  # per tick: tick->create at 0/10/30/50/90/100 %
        tick_timeline: List[Dict[str, Any]] = []  # the first timed tick, sampled every 250 ms
        gc_in_tick = [0, 0.0]

        async def sample_tick(t1: float) -> None:
            """Creates done, limiter and gate state, controller state and the event loop's
            lateness, every 250 ms for the first 4 s of a tick (where a tick's time goes)."""
            import gc as _gc

            def cb(phase: str, info: Dict[str, Any]) -> None:
                if phase == "start":
                    gc_in_tick[1] -= time.perf_counter()
                else:
                    gc_in_tick[0] += 1
                    gc_in_tick[1] += time.perf_counter()

            _gc.callbacks.append(cb)
            try:
                lim, gate = client.limiter, client.inflight
                nxt = t1 + 0.25
                lag = 0.0
                while time.perf_counter() - t1 < 4.0:
                    w0 = time.perf_counter()
                    await asyncio.sleep(0.005)
                    lag = max(lag, time.perf_counter() - w0 - 0.005)
                    now = time.perf_counter()
                    if now < nxt:
                        continue
                    nxt += 0.25
                    if lim is not None:
                        lim._refill(time.monotonic())
                    tick_timeline.append({
                        "t_ms": round((now - t1) * 1000), "creates": creates_this_tick[0],
                        "tokens": round(lim._tokens, 1) if lim is not None else None,
                        "waiting": [lim.waiting_at(p) for p in (0, 1, 2)] if lim is not None else None,
                        "inflight": gate.inflight if gate is not None else None,
                        "gate_waiting": gate.waiting if gate is not None else None,
                        "active": ctrl.active, "released": ctrl.released, "queue": len(ctrl.queue),
                        "max_loop_lag_ms": round(lag * 1000, 1), "gc": list(gc_in_tick)})
                    lag = 0.0
            finally:
                _gc.callbacks.remove(cb)
        phase_ms: Dict[str, List[float]] = {"completion": [], "fire": []}
        if n_pre:
            phase_ms["lifecycle_writes"] = []
        for k in range(1, total + 1):
            tick_ns = T0_NS + k * 60 * NANOS
            if k == cfg.warmup + 1:
                if cfg.apiserver_profile and admin is not None:
                    async with admin.post(remote.url + "/debug/fake/profile", json={"action": "start"}) as r:
                        await r.read()
                cpu0 = _cpu_times(remote)
                gcs = gctune.GcStats().start()
                rec0 = ctrl.reconciles
                req0 = client.requests
                reqv0 = dict(client.requests_by_verb)
                write_cpu[0] = 0.0
                t_start = time.perf_counter()
            deadline = time.monotonic() + cfg.step_timeout
            t0 = time.perf_counter()
            writes = 0.0
            if k > 1:
                # the previous tick's jobs run (realistic lifecycle: the operator's absorption of
                # each write is timed, the harness's write calls themselves are not -- they are
                # another controller's requests) and finish half a minute before this tick
                # (cluster side; the apiserver work of that last write is inside the timed
                # region -- conservative)
                if n_pre:
                    writes = await run_lifecycle(tick_ns, deadline)
                await complete_jobs(tick_ns - 30 * NANOS)
                await set_time(tick_ns - 30 * NANOS)
                await wait_completed(deadline)
            t1 = time.perf_counter()
            lat.clear()
            creates_this_tick[0] = 0
            tick_wall[0] = t1
            lim = client.limiter
            if lim is not None and k > cfg.warmup:  # the bucket the tick's CREATEs find
                lim._refill(time.monotonic())
                tick_tokens.append(round(lim._tokens, 1))
                tick_waiting.append([lim.waiting_at(p) for p in (0, 1, 2)])
            sampler = None
            if cfg.tick_timeline and k == cfg.warmup + 1:  # the first timed tick, every 250 ms
                sampler = asyncio.get_running_loop().create_task(sample_tick(t1))
            await set_time(tick_ns)
            await wait_settled(tick_ns, k, deadline)
            t2 = time.perf_counter()
            if sampler is not None:
                sampler.cancel()
            if k > cfg.warmup and lat:
                tick_p50_ms.append(round(_pct(lat, 50) * 1000, 1))
                tick_lat_q_ms.append([round(_pct(lat, q) * 1000, 1) for q in (0, 10, 30, 50, 90, 100)])
            dt = t2 - t0 - writes
            if k > cfg.warmup:
                step_ms.append(dt * 1000)
                phase_ms["completion"].append((t1 - t0 - writes) * 1000)
                phase_ms["fire"].append((t2 - t1) * 1000)
                if n_pre:
                    phase_ms["lifecycle_writes"].append(writes * 1000)
                excluded += writes
                timed_lat.extend(lat)
            if on_step is not None:
                on_step(k, dt, k > cfg.warmup)
        elapsed = time.perf_counter() - t_start - excluded
        cpu1 = _cpu_times(remote)
        gc_stats = gcs.stop().to_dict() if cfg.warmup < total else {}
        if cfg.apiserver_profile and admin is not None:
            async with admin.post(remote.url + "/debug/fake/profile",
                                  json={"action": "stop", "path": os.path.abspath(cfg.apiserver_profile)}) as r:
                await r.read()
        reconciles = ctrl.reconciles - rec0
        requests = client.requests - req0
        by_verb = {v: n - reqv0.get(v, 0) for v, n in client.requests_by_verb.items()}
        fires = cfg.n_crons * cfg.steps
        res = BenchResult(
            config=asdict(cfg), steps=cfg.steps, elapsed_s=elapsed,
            ms_per_step=elapsed * 1000 / max(1, cfg.steps),
            cron_reconciles_per_s=fires / elapsed, raw_reconciles_per_s=reconciles / elapsed,
            p50_latency_ms=_pct(timed_lat, 50) * 1000, p99_latency_ms=_pct(timed_lat, 99) * 1000,
            max_latency_ms=max(timed_lat) * 1000 if timed_lat else float("nan"),
            api_requests_per_fire=requests / fires, api_requests_by_verb=by_verb,
            reconciles_per_fire=reconciles / fires, step_ms=step_ms, phase_ms=phase_ms,
            engine=default_engine().name, fastjson_native=jsonutil.NATIVE,
            cpu_s_operator=cpu1[0] - cpu0[0], cpu_s_apiserver=cpu1[1] - cpu0[1] - write_cpu[0], operator_gc=gc_stats,
            startup_sync_s=startup_sync_s, startup_first_pass_s=startup_first_pass_s)
        res.tick_tokens, res.tick_waiting, res.tick_p50_ms = tick_tokens, tick_waiting, tick_p50_ms
        res.tick_lat_q_ms = tick_lat_q_ms
        if client.limiter is not None:  # the longest waits of the run, warm-up included
            res.limiter_max_wait_s = [round(x, 3) for x in client.limiter.max_wait_by_priority]
            res.limiter_aged_grants = client.limiter.aged_grants
        res.tick_timeline = tick_timeline
        if mgr.elector is not None:
            res.lease_lost = mgr.elector.lost.is_set() or not mgr.elector.is_leader
            res.lease_max_renew_s = mgr.elector.max_renew_s
        mgr.stop()
        try:
            await asyncio.wait_for(mgr_task, 30)
        except Exception:
            pass
        await client.close()
        return res
    finally:
        if admin is not None:
            await admin.close()
        for r in remotes:
            r.stop()


class _Shard:
    """A shard_worker child process and its JSON-lines pipe."""

    def __init__(self, proc: "asyncio.subprocess.Process"):
        self.proc = proc

    async def send(self, msg: Dict[str, Any]) -> None:
        assert self.proc.stdin is not None
        self.proc.stdin.write((json.dumps(msg) + "\n").encode())
        await self.proc.stdin.drain()

    async def recv(self, timeout: float) -> Dict[str, Any]:
        assert self.proc.stdout is not None
        line = await asyncio.wait_for(self.proc.stdout.readline(), timeout)
        if not line:
            err = (await self.proc.stderr.read()).decode()[-3000:] if self.proc.stderr else ""
            raise RuntimeError(f"shard worker exited rc={self.proc.returncode}: {err}")
        return json.loads(line)


async def _run_sharded(cfg: BenchConfig, remotes: List["_RemoteServer"], admin, set_time, complete_jobs,
                       on_step, job_stage=None) -> BenchResult:
    """The step loop of :func:`run` with the operator split over ``cfg.shards`` processes (shard
    i against ``remotes[i % len(remotes)]``: one fake apiserver, or one partition per shard)."""
    from ..cron.engine import default_engine
    from ..utils import jsonutil

    env = dict(os.environ)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    if not cfg.native_http:
        env["CRON_OPERATOR_NATIVE_HTTP"] = "python"
    shards: List[_Shard] = []
    try:
        for i in range(cfg.shards):
            remote = remotes[i % len(remotes)]
            p = await asyncio.create_subprocess_exec(
                sys.executable, "-m", "cron_operator_amd.bench.shard_worker", "--url", remote.url,
                "--namespace", cfg.namespace, "--shard-index", str(i), "--shard-count", str(cfg.shards),
                "--start-ns", str(T0_NS + NANOS // 2), "--workers", str(cfg.workers),
                "--history-limit", str(cfg.history_limit), "--qps", str(cfg.qps), "--burst", str(cfg.burst),
                "--max-inflight", str(cfg.max_inflight), "--tick-reserve", str(cfg.tick_reserve),
                *([] if cfg.defer_writes else ["--no-defer"]),
                *([] if cfg.compact_children else ["--no-compact"]),
                "--mode", cfg.mode, "--routing", cfg.shard_routing,
                *(["--ca-file", remote.ca_file] if remote.ca_file else []),
                env=env, stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
                stderr=asyncio.subprocess.PIPE, limit=1 << 24)
            shards.append(_Shard(p))
        remote = remotes[0]
        # what _cpu_times reads: the one server (scripts wrap _cpu_times and read its url), or the list
        cpu_of = remotes[0] if len(remotes) == 1 else remotes
        ready = await asyncio.gather(*(s.recv(300) for s in shards))
        assert sum(r["owned"] for r in ready) == cfg.n_crons, ready

        async def phase(ns: int, name: str, tick_ns: int) -> List[Dict[str, Any]]:
            await asyncio.gather(*(s.send({"cmd": "time", "ns": ns, "phase": name, "tick_ns": tick_ns})
                                   for s in shards))
            return list(await asyncio.gather(*(s.recv(cfg.step_timeout) for s in shards)))

        n_pre = lifecycle_stages(cfg)
        total = cfg.warmup + cfg.steps
        step_ms: List[float] = []
        phase_ms: Dict[str, List[float]] = {"completion": [], "fire": [], "completion_calls": [],
                                            "completion_settle_max": [], "fire_settle_max": []}
        comp: List[Dict[str, Any]] = []
        timed_lat: List[float] = []
        base: Optional[List[Dict[str, Any]]] = None
        tc = 0.0
        last: List[Dict[str, Any]] = []
        api0 = api1 = 0.0
        t_start = 0.0
        excluded = 0.0
        write_cpu = 0.0
        if n_pre:
            phase_ms["lifecycle_writes"] = []
        step_cpu_op: List[float] = []
        step_cpu_api: List[float] = []
        prev_op_cpu = 0.0
        parts0 = [0.0] * len(remotes)
        parts_write = [0.0] * len(remotes)
        for k in range(1, total + 1):
            tick_ns = T0_NS + k * 60 * NANOS
            if k == cfg.warmup + 1:
                if cfg.shard_profile:
                    await asyncio.gather(*(s.send({"cmd": "profile", "action": "start"}) for s in shards))
                    await asyncio.gather(*(s.recv(60) for s in shards))
                if cfg.apiserver_profile:
                    async with admin.post(remote.url + "/debug/fake/profile", json={"action": "start"}) as r:
                        await r.read()
                api0 = _cpu_times(cpu_of)[1]
                parts0 = [_proc_cpu(r) for r in remotes]
                t_start = time.perf_counter()
            t0 = time.perf_counter()
            writes = 0.0
            step_api0 = _cpu_times(cpu_of)[1]
            step_write_cpu = 0.0
            if k > 1:
                for st in range(n_pre):  # the previous tick's jobs start (realistic lifecycle)
                    w0 = time.perf_counter()
                    c0 = [_proc_cpu(r) for r in remotes]
                    rvs = await job_stage(st, tick_ns - 59 * NANOS, tick_ns - 30 * NANOS)
                    writes += time.perf_counter() - w0  # the harness's write call: not timed
                    if k > cfg.warmup:
                        dw = [_proc_cpu(r) - c for r, c in zip(remotes, c0)]
                        step_write_cpu += sum(dw)
                        write_cpu += sum(dw)
                        parts_write = [a + b for a, b in zip(parts_write, dw)]
                    await asyncio.gather(*(s.send({"cmd": "absorb", "rvs": rvs}) for s in shards))
                    await asyncio.gather(*(s.recv(cfg.step_timeout) for s in shards))
                tc = time.perf_counter()
                await complete_jobs(tick_ns - 30 * NANOS)
                await set_time(tick_ns - 30 * NANOS)
                tc = time.perf_counter() - tc
                comp = await phase(tick_ns - 30 * NANOS, "completion", tick_ns)
            t1 = time.perf_counter()
            await set_time(tick_ns)
            last = await phase(tick_ns, "fire", tick_ns)
            t2 = time.perf_counter()
            if k == cfg.warmup:
                base = last
            if k > cfg.warmup:
                step_ms.append((t2 - t0 - writes) * 1000)
                op_cpu = sum(r["cpu"] for r in last)
                step_cpu_op.append(op_cpu - prev_op_cpu)
                step_cpu_api.append(_cpu_times(cpu_of)[1] - step_api0 - step_write_cpu)
                phase_ms["completion"].append((t1 - t0 - writes) * 1000)
                phase_ms["fire"].append((t2 - t1) * 1000)
                # inside the completion phase: the harness's completion write and clock calls
                phase_ms["completion_calls"].append(tc * 1000 if k > 1 else 0.0)
                # ... and the slowest shard's own wait for its Crons to settle after the clock moved
                phase_ms["completion_settle_max"].append(
                    max(r.get("settle_s", 0.0) for r in comp) * 1000 if k > 1 else 0.0)
                phase_ms["fire_settle_max"].append(max(r.get("settle_s", 0.0) for r in last) * 1000)
                if n_pre:
                    phase_ms["lifecycle_writes"].append(writes * 1000)
                excluded += writes
                for r in last:
                    timed_lat.extend(r["lat"])
            prev_op_cpu = sum(r["cpu"] for r in last)
            if on_step is not None:
                on_step(k, t2 - t0 - writes, k > cfg.warmup)
        elapsed = time.perf_counter() - t_start - excluded
        api1 = _cpu_times(cpu_of)[1]
        parts1 = [_proc_cpu(r) for r in remotes]
        if cfg.shard_profile:
            await asyncio.gather(*(s.send({"cmd": "profile", "action": "stop",
                                           "path": os.path.abspath(f"{cfg.shard_profile}.{i}.pstats")})
                                   for i, s in enumerate(shards)))
            await asyncio.gather(*(s.recv(60) for s in shards))
        if cfg.apiserver_profile:
            async with admin.post(remote.url + "/debug/fake/profile",
                                  json={"action": "stop", "path": os.path.abspath(cfg.apiserver_profile)}) as r:
                await r.read()
        if base is None:  # warmup == 0: counters since process start
            base = [{"reconciles": 0, "requests": 0, "by_verb": {}, "cpu": 0.0} for _ in shards]
        reconciles = sum(r["reconciles"] - b["reconciles"] for r, b in zip(last, base))
        requests = sum(r["requests"] - b["requests"] for r, b in zip(last, base))
        by_verb: Dict[str, int] = {}
        for r, b in zip(last, base):
            for v, n in r["by_verb"].items():
                by_verb[v] = by_verb.get(v, 0) + n - b["by_verb"].get(v, 0)
        fires = cfg.n_crons * cfg.steps
        return BenchResult(
            config=asdict(cfg), steps=cfg.steps, elapsed_s=elapsed, ms_per_step=elapsed * 1000 / max(1, cfg.steps),
            cron_reconciles_per_s=fires / elapsed, raw_reconciles_per_s=reconciles / elapsed,
            p50_latency_ms=_pct(timed_lat, 50) * 1000, p99_latency_ms=_pct(timed_lat, 99) * 1000,
            max_latency_ms=max(timed_lat) * 1000 if timed_lat else float("nan"),
            api_requests_per_fire=requests / fires, api_requests_by_verb=by_verb,
            reconciles_per_fire=reconciles / fires, step_ms=step_ms, phase_ms=phase_ms,
            engine=default_engine().name, fastjson_native=jsonutil.NATIVE,
            cpu_s_operator=sum(r["cpu"] - b["cpu"] for r, b in zip(last, base)),
            cpu_s_apiserver=api1 - api0 - write_cpu,
            step_cpu_operator_s=step_cpu_op, step_cpu_apiserver_s=step_cpu_api,
            cpu_s_apiserver_parts=[b - a - w for a, b, w in zip(parts0, parts1, parts_write)]
            if len(remotes) > 1 else [],
            operator_ctx_switches=[sum(r.get("csw", [0, 0])[i] - b.get("csw", [0, 0])[i] for r, b in zip(last, base))
                                   for i in range(2)],
            operator_maxrss_mib=[round(r.get("maxrss_mib", 0.0), 1) for r in last],
            operator_ready_maxrss_mib=[round(r.get("maxrss_mib", 0.0), 1) for r in ready],
            operator_rss_mib=[round(r.get("rss_mib", 0.0), 1) for r in last],
            operator_gc={"collections": [sum(r.get("gc_collections", [0, 0, 0])[g] - b.get("gc_collections",
                                                                                            [0, 0, 0])[g]
                                             for r, b in zip(last, base)) for g in range(3)],
                         "ms": round(sum(r.get("gc_s", 0.0) - b.get("gc_s", 0.0) for r, b in zip(last, base))
                                     * 1000, 2),
                         "ms_by_generation": [
                             round(sum(r.get("gc_gen_s", [0.0] * 3)[g] - b.get("gc_gen_s", [0.0] * 3)[g]
                                       for r, b in zip(last, base)) * 1000, 2) for g in range(3)]})
    finally:
        for s in shards:
            try:
                await s.send({"cmd": "stop"})
            except Exception:  # noqa: BLE001
                pass
        for s in shards:
            try:
                await asyncio.wait_for(s.proc.wait(), 30)
            except Exception:  # noqa: BLE001
                s.proc.kill()


def run_sync(cfg: BenchConfig, on_step=None) -> BenchResult:
    if cfg.transport == "http":
        # the operator (in this process with one shard, else in shard_worker processes) runs on the
        # native loop core like `cron-operator start`; the fake apiserver process keeps asyncio's
        # stock loop (an in-memory transport would put the fixture on this loop: left stock)
        from ..runtime import aioloop

        aioloop.install()
    return asyncio.run(run(cfg, on_step))


def summarize(r: BenchResult) -> str:
    return (f"{r.config['mode']}/{r.config['transport']} n={r.config['n_crons']}: "
            f"{r.cron_reconciles_per_s:,.0f} cron-reconciles/s, {r.raw_reconciles_per_s:,.0f} raw reconciles/s, "
            f"p50 {r.p50_latency_ms:.1f} ms p99 {r.p99_latency_ms:.1f} ms, {r.ms_per_step:.0f} ms/step, "
            f"{r.api_requests_per_fire:.2f} req/fire, {r.reconciles_per_fire:.2f} reconciles/fire "
            f"(median step {statistics.median(r.step_ms):.0f} ms; CPU operator {r.cpu_s_operator:.2f} s, "
            f"apiserver {r.cpu_s_apiserver:.2f} s)")
