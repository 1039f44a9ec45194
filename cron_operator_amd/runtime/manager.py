"""Manager: owns the client, cache, controllers, servers and leader election.

Counterpart of ``ctrl.NewManager(cfg, ctrl.Options{...})`` + ``mgr.Start``
(``cmd/operator/start.go:156-209``) [ext controller-runtime]:

1. probe and metrics servers start first (they answer while not leader);
2. the event broadcaster starts;
3. with leader election, the manager campaigns for the Lease
   (ID ``619a52b8.kubedl.io``) and only the leader starts informers and
   controllers; losing the lease raises :class:`LeaderElectionLost` (the CLI
   exits non-zero, as controller-runtime does);
4. informers sync, then controller workers start.
"""
from __future__ import annotations

import asyncio
import os
from dataclasses import dataclass, field
from typing import Any, Awaitable, Callable, Dict, List, Optional

from ..parallel.leaderelection import LeaderElector, in_cluster_namespace
from ..utils import aio, gctune
from ..utils.clock import Clock, RealClock
from ..utils.logging import get_logger
from .client import Client
from .controller import Controller
from .events import Broadcaster, Recorder
from .informer import WATCH_IDLE_TIMEOUT, Cache
from .servers import Check, MetricsServer, ProbeServer, ping

DEFAULT_LEADER_ELECTION_ID = "619a52b8.kubedl.io"


class LeaderElectionLost(RuntimeError):
    pass


@dataclass
class ManagerOptions:
    clock: Clock = field(default_factory=RealClock)
    namespace: str = ""  # restrict the cache to one namespace ("" = all)
    leader_election: bool = False
    leader_election_id: str = DEFAULT_LEADER_ELECTION_ID
    leader_election_namespace: str = ""
    leader_election_identity: Optional[str] = None
    lease_duration: float = 15.0
    renew_deadline: float = 10.0
    retry_period: float = 2.0
    leader_election_release_on_cancel: bool = False
    # the elector's clock (default: ``clock``): a harness that jumps the schedule clock over
    # virtual minutes keeps lease timing on real time
    leader_election_clock: Optional[Clock] = None
    metrics_bind_address: str = "0"
    secure_metrics: bool = True
    metrics_cert_path: str = ""
    metrics_cert_name: str = "tls.crt"
    metrics_cert_key: str = "tls.key"
    health_probe_bind_address: str = ":8081"
    # which clients the probe port's /debug views answer: local (loopback only), all, off
    debug_views: str = "local"
    enable_http2: bool = False
    max_concurrent_reconciles: int = 10
    cache_sync_timeout: float = 120.0
    # controller-runtime's cache SyncPeriod: every object is re-reconciled at least this often
    sync_period: float = 10 * 3600.0
    # horizontal sharding: this replica reconciles the Crons with shard_of(key) == shard_index; each
    # shard elects its own leader (Lease "<leader_election_id>-shard-<index>")
    shard_index: int = 0
    shard_count: int = 1
    # "hash": every shard watches everything and drops other shards' keys; "labels": objects carry
    # kubedl.io/shard and each shard's informers select on it (controller/sharding.py)
    shard_routing: str = "labels"  # only used when shard_count > 1
    # informer watch liveness (runtime/informer.py): seconds without an event or bookmark
    # before a watch is presumed dead and re-established
    watch_idle_timeout: float = WATCH_IDLE_TIMEOUT


class Manager:
    def __init__(self, client: Client, options: Optional[ManagerOptions] = None,
                 lease_client: Optional[Client] = None):
        """``lease_client``: the client the leader elector uses.  Default: derived from
        ``client`` when the election starts (:meth:`Client.derive`) -- same connections and
        credentials, its own QPS bucket, no in-flight cap -- as controller-runtime gives the
        resource lock a client of its own (``/root/reference/cmd/operator/start.go:156-177``
        [ext]).  Passing ``client`` itself shares the reconciler's budget (a test control)."""
        self.client = client
        self.lease_client = lease_client
        self.opts = options or ManagerOptions()
        self.clock = self.opts.clock
        self.cache = Cache(client, self.opts.namespace, self.opts.sync_period, self.clock,
                           watch_idle_timeout=self.opts.watch_idle_timeout)
        self.broadcaster = Broadcaster(client, self.clock)
        self.controllers: List[Controller] = []
        self.runnables: List[Callable[[], Awaitable[None]]] = []
        self.probes = ProbeServer(self.opts.health_probe_bind_address, self.opts.debug_views)
        self.probes.debug["caches"] = self.cache_view
        self.metrics_server = MetricsServer(self.opts.metrics_bind_address, self.opts.secure_metrics,
                                            self.opts.metrics_cert_path, self.opts.metrics_cert_name,
                                            self.opts.metrics_cert_key, client=client,
                                            enable_http2=self.opts.enable_http2)
        self.elector: Optional[LeaderElector] = None
        self.elected = asyncio.Event()
        self.started = asyncio.Event()
        self._stop = asyncio.Event()
        self._tasks: List[asyncio.Task] = []
        self.log = get_logger("manager")

    # -- wiring
    def get_client(self) -> Client:
        return self.client

    def get_cache(self) -> Cache:
        return self.cache

    def get_event_recorder_for(self, name: str) -> Recorder:
        return self.broadcaster.recorder_for(name)

    def add_controller(self, c: Controller) -> None:
        self.controllers.append(c)

    def add(self, runnable: Callable[[], Awaitable[None]]) -> None:
        """A leader-only runnable started after the caches sync."""
        self.runnables.append(runnable)

    def add_healthz_check(self, name: str, check: Check = ping) -> None:
        self.probes.healthz[name] = check

    def add_readyz_check(self, name: str, check: Check = ping) -> None:
        self.probes.readyz[name] = check

    def add_debug_view(self, name: str, fn: Callable[[], Any]) -> None:
        """``GET /debug/<name>`` on the probe port answers ``fn()`` as JSON."""
        self.probes.debug[name] = fn

    def cache_view(self) -> Dict[str, Any]:
        """``/debug/caches``: what each informer holds, and the process's resident memory."""
        infs = []
        for inf in self.cache.informers():
            infs.append({"informer": inf.name, "objects": len(inf.store),
                         "derived": len(inf.derived) if inf.derive is not None else None,
                         "synced": inf.synced.is_set(), "relists": inf.relists, "events": inf.events})
        rss = None
        try:
            with open("/proc/self/statm") as fh:
                rss = round(int(fh.read().split()[1]) * os.sysconf("SC_PAGE_SIZE") / 2**20, 1)
        except (OSError, ValueError, IndexError):
            pass
        return {"informers": infs, "rss_mib": rss}

    # -- lifecycle
    async def _start_leading(self) -> None:
        self.elected.set()
        self.cache.start()
        ok = await self.cache.wait_for_sync(self.opts.cache_sync_timeout)
        if not ok:
            raise TimeoutError("timed out waiting for cache to be synced")
        gctune.tune()
        gctune.freeze()  # the synced caches are long-lived: keep them out of GC scans
        for c in self.controllers:
            c.start()
        loop = asyncio.get_running_loop()
        for r in self.runnables:
            self._tasks.append(loop.create_task(r()))
        self.started.set()
        self.log.info("Starting workers", controllers=[c.name for c in self.controllers])

    async def start(self) -> None:
        """Run until :meth:`stop` (or leadership loss, which raises)."""
        await self.probes.start()
        await self.metrics_server.start()
        from .supervisor import report_ports

        report_ports(self.metrics_server.port, self.probes.port)
        self.broadcaster.start()
        lost = False
        try:
            if self.opts.leader_election:
                ns = self.opts.leader_election_namespace or in_cluster_namespace()
                lease = self.opts.leader_election_id if self.opts.shard_count <= 1 else \
                    f"{self.opts.leader_election_id}-shard-{self.opts.shard_index}"
                if self.lease_client is None:
                    self.lease_client = self.client.derive()
                self.elector = LeaderElector(self.lease_client, lease, ns,
                                             self.opts.leader_election_identity,
                                             self.opts.leader_election_clock or self.clock,
                                             self.opts.lease_duration, self.opts.renew_deadline,
                                             self.opts.retry_period,
                                             self.opts.leader_election_release_on_cancel)
                le_task = asyncio.get_running_loop().create_task(
                    self.elector.run(self._start_leading, lambda: None))
                stop_task = asyncio.get_running_loop().create_task(self._stop.wait())
                done, _ = await asyncio.wait({le_task, stop_task}, return_when=asyncio.FIRST_COMPLETED)
                if le_task in done:
                    exc = le_task.exception()
                    if exc is not None:
                        raise exc
                    lost = True
                else:
                    await aio.cancel_and_wait(le_task)
                stop_task.cancel()
            else:
                await self._start_leading()
                await self._stop.wait()
        finally:
            await self.shutdown()
        if lost:
            self.log.info("leader election lost")
            raise LeaderElectionLost("leader election lost")

    def stop(self) -> None:
        self._stop.set()

    async def shutdown(self) -> None:
        for c in self.controllers:
            await c.stop()
        tasks, self._tasks = self._tasks, []
        await aio.cancel_and_wait(*tasks)
        await self.cache.stop()
        await self.broadcaster.stop()
        await self.metrics_server.stop()
        await self.probes.stop()
