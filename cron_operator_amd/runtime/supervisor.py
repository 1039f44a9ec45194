"""``start --shard-processes N``: one pod, N operator processes, one shard each.

The reference's manager runs its reconcile workers as goroutines, so a single pod
uses every core it is given (``cmd/operator/start.go:174-176``).  This operator is
an asyncio process, so it uses cores by sharding (``controller/sharding.py``).
Without this module that means one Deployment per shard; with it the pod's main
process becomes a supervisor:

* it starts ``N`` children, ``start ... --shard-count C*N --shard-index I*N+i``
  (``C``/``I`` are the pod-level ``--shard-count``/``--shard-index``, so pods of
  processes compose), each with its own shard Lease, informers and workers;
* children serve plain metrics and probes on loopback ports they bind themselves
  (port 0, reported back over a pipe on every start); the supervisor serves
  the configured ``--metrics-bind-address`` (with the same TokenReview /
  SubjectAccessReview filter when secure) as the merge of the children's
  expositions, every series labelled ``shard="<index>"``;
* ``/healthz`` is ok while every child runs; ``/readyz`` asks every child's
  ``/readyz``;
* a child that exits is restarted with exponential backoff (1 s doubling to
  30 s); SIGTERM/SIGINT are forwarded and the supervisor exits once the children have.
"""
from __future__ import annotations

import asyncio
import math
import os
import signal
import sys
import time
from typing import TYPE_CHECKING, Dict, List, Optional, Tuple

from ..utils.logging import get_logger
from . import miniweb as web
from .servers import MetricsServer, ProbeServer

if TYPE_CHECKING:  # the scraping client is imported by the supervisor only (Supervisor.run)
    import aiohttp

RESTART_BACKOFF = (1.0, 30.0)


def available_cpus(cgroup_root: str = "/sys/fs/cgroup") -> int:
    """CPUs this container may use: the cgroup CPU quota rounded up (v2 ``cpu.max``, v1
    ``cpu.cfs_quota_us``/``cpu.cfs_period_us``), else the scheduler affinity mask; at least 1."""
    quota = None
    try:
        with open(os.path.join(cgroup_root, "cpu.max")) as fh:
            q, period = (fh.read().split() + ["100000"])[:2]  # "max 100000" or "<quota> <period>"
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        try:
            with open(os.path.join(cgroup_root, "cpu", "cpu.cfs_quota_us")) as fh:
                q1 = int(fh.read())
            with open(os.path.join(cgroup_root, "cpu", "cpu.cfs_period_us")) as fh:
                p1 = int(fh.read())
            if q1 > 0 and p1 > 0:
                quota = q1 / p1
        except (OSError, ValueError):
            pass
    try:
        cpus = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        cpus = os.cpu_count() or 1
    if quota is not None:
        cpus = min(cpus, math.ceil(quota))
    return max(1, cpus)


def merge_expositions(parts: List[Tuple[str, str]]) -> str:
    """Merge Prometheus text expositions ``[(shard, text)]`` into one: each family's
    ``# HELP``/``# TYPE`` once, then its samples from every part with ``shard`` added."""
    families: Dict[str, Tuple[List[str], List[str]]] = {}
    order: List[str] = []

    def fam(name: str) -> Tuple[List[str], List[str]]:
        f = families.get(name)
        if f is None:
            f = families[name] = ([], [])
            order.append(name)
        return f

    for shard, text in parts:
        current = ""
        label = f'shard="{shard}"'
        for line in text.splitlines():
            if not line.strip():
                continue
            if line.startswith("#"):
                bits = line.split(" ", 3)
                if len(bits) >= 3 and bits[1] in ("HELP", "TYPE"):
                    current = bits[2]
                    meta = fam(current)[0]
                    if not any(m.split(" ", 2)[1] == bits[1] for m in meta):
                        meta.append(line)
                continue
            brace, space = line.find("{"), line.find(" ")
            if brace >= 0 and (space < 0 or brace < space):
                name = line[:brace]
                rest = line[brace + 1:]
                sample = f"{name}{{{label}{'' if rest.startswith('}') else ','}{rest}"
            else:
                name = line[:space]
                sample = f"{name}{{{label}}}{line[space:]}"
            if not current or not (name == current or name.startswith(current + "_")):
                current = name
            fam(current)[1].append(sample)
    out: List[str] = []
    for name in order:
        meta, samples = families[name]
        out.extend(meta)
        out.extend(samples)
    return "\n".join(out) + "\n"


REPORT_FD_ENV = "CRON_OPERATOR_REPORT_FD"


def report_ports(metrics_port: Optional[int], probe_port: Optional[int]) -> None:
    """In a supervised child: tell the supervisor which loopback ports the servers bound
    (one JSON line on the inherited pipe named by ``$CRON_OPERATOR_REPORT_FD``)."""
    fd = os.environ.pop(REPORT_FD_ENV, None)
    if not fd:
        return
    import json

    try:
        with os.fdopen(int(fd), "w") as fh:
            fh.write(json.dumps({"metrics": metrics_port, "probes": probe_port}) + "\n")
    except (OSError, ValueError):
        pass


class _Child:
    """One shard process.  Its metrics and probe servers bind loopback port 0 -- the kernel
    picks a free port at bind time, on every (re)start -- and the child reports the ports
    back over a pipe, so nothing can take a port between choosing and binding it."""

    def __init__(self, index: int, argv: List[str]):
        self.index = index
        self.argv = argv
        self.metrics_port: Optional[int] = None
        self.probe_port: Optional[int] = None
        self.proc: Optional[asyncio.subprocess.Process] = None
        self.restarts = 0
        self._reader: Optional[asyncio.Future] = None  # held: the loop only weakly references tasks

    async def spawn(self) -> None:
        self.metrics_port = self.probe_port = None
        r, w = os.pipe()
        try:
            env = dict(os.environ, **{REPORT_FD_ENV: str(w)})
            self.proc = await asyncio.create_subprocess_exec(
                sys.executable, "-m", "cron_operator_amd", *self.argv,
                "--metrics-bind-address=127.0.0.1:0", "--metrics-secure=false",
                "--health-probe-bind-address=127.0.0.1:0", env=env, pass_fds=(w,))
        except BaseException:
            os.close(r)
            raise
        finally:
            os.close(w)
        self._reader = asyncio.ensure_future(self._read_ports(r, self.proc))

    async def _read_ports(self, r: int, proc: asyncio.subprocess.Process) -> None:
        import json

        def read() -> bytes:
            with os.fdopen(r, "rb") as fh:
                return fh.readline()

        line = await asyncio.get_running_loop().run_in_executor(None, read)
        if self.proc is not proc or not line:
            return
        try:
            ports = json.loads(line)
        except ValueError:
            return
        self.metrics_port, self.probe_port = ports.get("metrics"), ports.get("probes")

    @property
    def running(self) -> bool:
        return self.proc is not None and self.proc.returncode is None


class Supervisor:
    def __init__(self, argv: List[str], processes: int, shard_count: int, shard_index: int,
                 metrics: Optional[MetricsServer], probe_bind: str, debug_views: str = "local"):
        self.log = get_logger("supervisor")
        total = shard_count * processes
        self.children = [
            _Child(shard_index * processes + i,
                   [*argv, "--shard-processes=1", f"--shard-count={total}",
                    f"--shard-index={shard_index * processes + i}"])
            for i in range(processes)]
        self.metrics = metrics
        self.probes = ProbeServer(probe_bind, debug_views)
        self.probes.healthz["children"] = self._alive
        self._ready: Dict[int, bool] = {}
        self.probes.readyz["children"] = self._all_ready
        self._stopping = asyncio.Event()
        self._session: Optional[aiohttp.ClientSession] = None

    def _sess(self) -> aiohttp.ClientSession:
        assert self._session is not None
        return self._session

    def _alive(self) -> Optional[str]:
        dead = [c.index for c in self.children if not c.running]
        return f"shard processes not running: {dead}" if dead else None

    def _all_ready(self) -> Optional[str]:
        bad = [c.index for c in self.children if not self._ready.get(c.index)]
        return f"shard processes not ready: {bad}" if bad else None

    async def _poll_ready(self) -> None:
        import aiohttp

        while not self._stopping.is_set():
            for c in self.children:
                ok = False
                if c.running and c.probe_port:
                    try:
                        async with self._sess().get(f"http://127.0.0.1:{c.probe_port}/readyz") as r:
                            ok = r.status == 200
                    except (aiohttp.ClientError, asyncio.TimeoutError, OSError):
                        ok = False
                self._ready[c.index] = ok
            try:
                await asyncio.wait_for(self._stopping.wait(), 1.0)
            except asyncio.TimeoutError:
                pass

    async def scrape(self) -> str:
        import aiohttp

        async def one(c: _Child) -> Tuple[str, str]:
            if not c.running or not c.metrics_port:
                return str(c.index), ""
            try:
                async with self._sess().get(f"http://127.0.0.1:{c.metrics_port}/metrics") as r:
                    return str(c.index), (await r.text()) if r.status == 200 else ""
            except (aiohttp.ClientError, asyncio.TimeoutError, OSError):
                return str(c.index), ""

        return merge_expositions(list(await asyncio.gather(*(one(c) for c in self.children))))

    async def _keep(self, c: _Child) -> None:
        backoff = RESTART_BACKOFF[0]
        while not self._stopping.is_set():
            started = time.monotonic()
            await c.spawn()
            proc = c.proc
            assert proc is not None
            if self._stopping.is_set():  # stop() ran while this child was being spawned
                proc.send_signal(signal.SIGTERM)
            self.log.info("started shard process", shard=c.index, pid=proc.pid)
            rc = await proc.wait()
            if self._stopping.is_set():
                return
            if time.monotonic() - started > 2 * RESTART_BACKOFF[1]:
                backoff = RESTART_BACKOFF[0]
            c.restarts += 1
            self.log.info("shard process exited; restarting", shard=c.index, exitCode=rc, backoff=backoff)
            try:
                await asyncio.wait_for(self._stopping.wait(), backoff)
            except asyncio.TimeoutError:
                pass
            backoff = min(backoff * 2, RESTART_BACKOFF[1])

    def stop(self) -> None:
        if self._stopping.is_set():
            return
        self._stopping.set()
        for c in self.children:
            if c.running:
                try:
                    c.proc.send_signal(signal.SIGTERM)  # type: ignore[union-attr]
                except ProcessLookupError:
                    pass

    async def run(self) -> int:
        import aiohttp

        self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=5))
        if self.metrics is not None:
            async def handle(req: web.Request) -> web.Response:
                denied = await self.metrics._authorize(req)
                if denied is not None:
                    return denied
                return web.Response(body=(await self.scrape()).encode(),
                                    headers={"Content-Type": "text/plain; version=0.0.4; charset=utf-8"})
            self.metrics.handler = handle
            await self.metrics.start()
        await self.probes.start()
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGINT, signal.SIGTERM):
            try:
                loop.add_signal_handler(sig, self.stop)
            except (NotImplementedError, RuntimeError):
                pass
        keepers = [asyncio.ensure_future(self._keep(c)) for c in self.children]
        poller = asyncio.ensure_future(self._poll_ready())
        try:
            await self._stopping.wait()
            for c in self.children:
                if c.proc is not None:
                    try:
                        await asyncio.wait_for(c.proc.wait(), 30)
                    except asyncio.TimeoutError:
                        c.proc.kill()
                        await c.proc.wait()
        finally:
            for t in (*keepers, poller):
                t.cancel()
            await asyncio.gather(*keepers, poller, return_exceptions=True)
            await self.probes.stop()
            if self.metrics is not None:
                await self.metrics.stop()
            await self._session.close()
        codes = [c.proc.returncode for c in self.children if c.proc is not None]
        return 0 if all(rc in (0, -signal.SIGTERM) for rc in codes) else 1

