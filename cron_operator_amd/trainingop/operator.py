"""Fake training-operator: drives Kubeflow job ``.status`` for tests, bench and smoke runs.

In a real cluster the Kubeflow training-operator turns a PyTorchJob into pods
and writes ``.status.conditions`` (Created -> Running -> Succeeded/Failed); the
Cron operator only reads those conditions (SURVEY 3.4,
``internal/controller/cron_util.go:92-114``).  envtest has no such controller, so
the reference tests cannot observe a job finishing.  This component fills
that gap in three modes:

* ``manual`` -- the test/bench calls :meth:`complete` / :meth:`complete_all`;
* ``timed``  -- jobs go through the training-operator's status sequence (Created, one
  ``replicaStatuses`` write per pod, Running: :func:`lifecycle_statuses`) and become
  Succeeded ``duration`` seconds of (possibly virtual) clock time after admission;
* ``real``   -- each replica's container ``command``/``args`` runs as a local
  subprocess with the env the training-operator injects for PyTorchJob
  (``MASTER_ADDR``/``MASTER_PORT``/``WORLD_SIZE``/``RANK``); the job succeeds or
  fails with the processes' exit codes.  This is how a scheduled PyTorchJob
  runs PyTorch-ROCm on an MI355X box (``examples/mi355x``, ``smoke()``).

It talks to the apiserver through a normal :class:`~cron_operator_amd.runtime.client.Client`
(its own QPS budget), so the operator under test sees ordinary watch events.
"""
from __future__ import annotations

import asyncio
import os
import sys
from typing import Any, Dict, List, Optional, Tuple

from ..api import errors
from ..api.meta import GroupVersionResource
from ..runtime.client import Client
from ..runtime.informer import EventHandler, Informer
from ..utils import aio
from ..utils.clock import Clock, RealClock
from ..utils.gotime import GoTime, UTC
from ..utils.logging import get_logger

JOB_GVRS = [GroupVersionResource("kubeflow.org", "v1", r) for r in
            ("pytorchjobs", "tfjobs", "xgboostjobs", "paddlejobs", "jaxjobs", "mpijobs")] + \
    [GroupVersionResource("kubeflow.org", "v1alpha1", "mpijobs")]  # the reference's MPI example (cron-mpi.yaml)


def _mpi_v1alpha1(gvr: GroupVersionResource) -> bool:
    """MPIJob v1alpha1: no conditions, the launcher's phase in ``status.launcherStatus``."""
    return gvr.version == "v1alpha1" and gvr.resource == "mpijobs"

# replica-type order used to pick the "master" process in real mode
_MASTER_TYPES = ("Master", "Chief", "Launcher", "Worker", "PS", "Evaluator")


def _free_port() -> int:
    """A loopback port free at this moment (the rendezvous port of one job's replicas).  The
    real training-operator uses a fixed port in each pod's own network namespace; here every
    replica shares the host, so concurrent jobs must not collide."""
    from ..utils.ports import free_port

    return free_port()


def _now_str(clock: Clock) -> str:
    return GoTime(clock.now_ns() // 1_000_000_000, 0, UTC).rfc3339()


def _cond(ctype: str, reason: str, msg: str, ts: str) -> Dict[str, Any]:
    return {"type": ctype, "status": "True", "reason": reason, "message": msg, "lastUpdateTime": ts,
            "lastTransitionTime": ts}


def running_status(kind: str, name: str, ts: str) -> Dict[str, Any]:
    return {"conditions": [_cond("Created", f"{kind}Created", f"{kind} {name} is created.", ts),
                           _cond("Running", f"{kind}Running", f"{kind} {name} is running.", ts)],
            "startTime": ts, "replicaStatuses": {}}


def finished_status(kind: str, name: str, ts: str, succeeded: bool, start: Optional[str] = None) -> Dict[str, Any]:
    st = running_status(kind, name, start or ts)
    st["conditions"][-1]["status"] = "False"
    ctype = "Succeeded" if succeeded else "Failed"
    st["conditions"].append(_cond(ctype, f"{kind}{ctype}",
                                  f"{kind} {name} successfully completed." if succeeded else f"{kind} {name} failed.",
                                  ts))
    st["completionTime"] = ts
    return st


def replica_counts(obj: Dict[str, Any]) -> List[Tuple[str, int]]:
    """``[(replica type, replicas)]`` of a Kubeflow job, master-like types first."""
    spec = obj.get("spec") or {}
    specs = next((v for k, v in spec.items() if k.endswith("ReplicaSpecs") and isinstance(v, dict)), None) \
        if isinstance(spec, dict) else None
    if not specs:
        return []
    order = sorted(specs, key=lambda t: _MASTER_TYPES.index(t) if t in _MASTER_TYPES else 99)
    return [(t, int((specs[t] or {}).get("replicas", 1) or 1)) for t in order]


def lifecycle_statuses(obj: Dict[str, Any], start: str, end: str, succeeded: bool = True) -> List[Dict[str, Any]]:
    """The status writes the Kubeflow training-operator makes over one job's life, in order.

    ``Created`` on admission (with ``startTime`` and an empty ``replicaStatuses`` entry per
    replica type); one write per pod as it starts (``replicaStatuses[type].active`` counting up);
    ``Running``; then ``Succeeded`` / ``Failed`` with ``completionTime`` (the ``JobStatus``
    schema of ``/root/reference/test/crds/kubeflow.org_pytorchjobs.yaml:4739-4828``).  Every
    write changes the job's resourceVersion: an operator that folds it into ``status.active``
    pays a Cron status PATCH per write (reference ``cron_controller.go:284-304``)."""
    kind, name = obj.get("kind", ""), (obj.get("metadata") or {}).get("name", "")
    created = _cond("Created", f"{kind}Created", f"{kind} {name} is created.", start)
    reps = replica_counts(obj)
    rs: Dict[str, Dict[str, Any]] = {t: {} for t, _ in reps}

    def snap(conds: List[Dict[str, Any]]) -> Dict[str, Any]:
        return {"conditions": [dict(c) for c in conds], "startTime": start,
                "replicaStatuses": {t: dict(v) for t, v in rs.items()}}

    out = [snap([created])]
    for t, n in reps:
        for i in range(n):
            rs[t]["active"] = i + 1
            out.append(snap([created]))
    running = _cond("Running", f"{kind}Running", f"{kind} {name} is running.", start)
    out.append(snap([created, running]))
    for t, n in reps:
        rs[t] = {"succeeded": n} if succeeded else {"failed": n}
    fin = finished_status(kind, name, end, succeeded, start)
    fin["replicaStatuses"] = {t: dict(v) for t, v in rs.items()}
    out.append(fin)
    return out


def lifecycle_status(obj: Dict[str, Any], stage: int, start: str, end: str,
                     reps: Optional[List[Tuple[str, int]]] = None) -> Dict[str, Any]:
    """Stage ``stage`` of :func:`lifecycle_statuses` (negative: from the end) without building the
    others -- the bench writes one stage to every job at a time.  ``reps``: the job's
    :func:`replica_counts`, when the caller knows them already."""
    reps = replica_counts(obj) if reps is None else reps
    n = 3 + sum(k for _, k in reps)
    if stage < 0:
        stage += n
    if not 0 <= stage < n:
        raise IndexError(stage)
    if stage == n - 1:
        return lifecycle_statuses(obj, start, end)[-1]
    kind, name = obj.get("kind", ""), (obj.get("metadata") or {}).get("name", "")
    conds = [_cond("Created", f"{kind}Created", f"{kind} {name} is created.", start)]
    if stage == n - 2:
        conds.append(_cond("Running", f"{kind}Running", f"{kind} {name} is running.", start))
    left = stage if stage < n - 2 else n
    rs: Dict[str, Dict[str, Any]] = {}
    for t, k in reps:
        take = min(k, left)
        left -= take
        rs[t] = {"active": take} if take else {}
    return {"conditions": conds, "startTime": start, "replicaStatuses": rs}


class FakeTrainingOperator:
    def __init__(self, client: Client, clock: Optional[Clock] = None, mode: str = "manual", duration: float = 30.0,
                 namespace: str = "", kinds: Optional[List[GroupVersionResource]] = None,
                 workdir: Optional[str] = None, env: Optional[Dict[str, str]] = None, timeout: float = 900.0,
                 lifecycle: str = "realistic"):
        """``lifecycle`` (timed mode): ``realistic`` writes the training-operator's status
        sequence (:func:`lifecycle_statuses`); ``instant`` only Running, then Succeeded."""
        if mode not in ("manual", "timed", "real"):
            raise ValueError(f"unknown mode {mode}")
        if lifecycle not in ("realistic", "instant"):
            raise ValueError(f"unknown lifecycle {lifecycle}")
        self.lifecycle = lifecycle
        self.client = client
        self.clock = clock or RealClock()
        self.mode = mode
        self.duration = duration
        self.namespace = namespace
        self.kinds = kinds or JOB_GVRS
        self.workdir = workdir
        self.extra_env = env or {}
        self.timeout = timeout
        self.informers: List[Informer] = []
        self._tasks: List[asyncio.Task] = []
        self._handled: set = set()
        self.results: Dict[str, Tuple[bool, List[int], float]] = {}
        self.outputs: Dict[str, str] = {}  # real mode: "ns/name" -> the first replica's (rank 0's) output
        self.log = get_logger("training-operator")

    # ------------------------------------------------------------------ status writes
    async def _write_status(self, gvr: GroupVersionResource, ns: str, name: str, status: Dict[str, Any]) -> None:
        try:
            await self.client.patch(gvr, ns, name, {"status": status}, "merge", "status")
        except errors.ApiError as e:
            if not errors.is_not_found(e):
                raise

    async def mark_running(self, gvr: GroupVersionResource, obj: Dict[str, Any]) -> None:
        m = obj["metadata"]
        st = {"launcherStatus": "Active"} if _mpi_v1alpha1(gvr) else \
            running_status(obj.get("kind", ""), m["name"], _now_str(self.clock))
        await self._write_status(gvr, m["namespace"], m["name"], st)

    async def complete(self, gvr: GroupVersionResource, ns: str, name: str, succeeded: bool = True) -> None:
        kind = gvr.resource
        try:
            obj = await self.client.get(gvr, ns, name)
            kind = obj.get("kind", kind)
            start = (obj.get("status") or {}).get("startTime")
        except errors.ApiError:
            start = None
        if _mpi_v1alpha1(gvr):
            st = {"launcherStatus": "Succeeded" if succeeded else "Failed", "completionTime": _now_str(self.clock)}
        else:
            st = finished_status(kind, name, _now_str(self.clock), succeeded, start)
        await self._write_status(gvr, ns, name, st)

    # ------------------------------------------------------------------ watch loop
    async def start(self) -> None:
        for gvr in self.kinds:
            try:
                await self.client.mapper.kind_for(gvr)
            except errors.ApiError:
                continue
            inf = Informer(self.client, gvr, self.namespace, name=f"trainingop:{gvr.resource}")
            inf.add_handler(EventHandler(on_add=lambda o, g=gvr: self._on_job(g, o)))
            self.informers.append(inf)
            inf.start()
        await asyncio.gather(*(i.synced.wait() for i in self.informers))

    def _on_job(self, gvr: GroupVersionResource, obj: Dict[str, Any]) -> None:
        if self.mode == "manual":
            return
        m = obj.get("metadata") or {}
        key = (gvr.resource, m.get("namespace"), m.get("name"), m.get("uid"))
        if key in self._handled or (obj.get("status") or {}).get("completionTime"):
            return
        self._handled.add(key)
        coro = self._drive_timed(gvr, obj) if self.mode == "timed" else self._drive_real(gvr, obj)
        self._tasks.append(asyncio.get_running_loop().create_task(coro))

    async def _drive_timed(self, gvr: GroupVersionResource, obj: Dict[str, Any]) -> None:
        m = obj["metadata"]
        if self.lifecycle == "instant" or _mpi_v1alpha1(gvr):
            await self.mark_running(gvr, obj)
            await self.clock.sleep(self.duration)
            await self.complete(gvr, m["namespace"], m["name"], True)
            return
        # the training-operator's write sequence as the pods start (each its own write and
        # resourceVersion, awaited in turn; no clock time passes, so a test's virtual clock
        # sees Running at once as before), then Succeeded ``duration`` seconds after admission
        start_ns = self.clock.now_ns()
        start = _now_str(self.clock)
        end = GoTime((start_ns + int(self.duration * 1e9)) // 1_000_000_000, 0, UTC).rfc3339()
        stages = lifecycle_statuses(obj, start, end, True)
        for st in stages[:-1]:
            await self._write_status(gvr, m["namespace"], m["name"], st)
        await self.clock.sleep(self.duration)
        await self._write_status(gvr, m["namespace"], m["name"], stages[-1])

    # ------------------------------------------------------------------ real mode
    def _replica_processes(self, obj: Dict[str, Any]) -> List[Tuple[str, int, Dict[str, Any]]]:
        spec = obj.get("spec") or {}
        specs = None
        for k, v in spec.items():
            if k.endswith("ReplicaSpecs") and isinstance(v, dict):
                specs = v
                break
        if not specs:
            return []
        out = []
        order = sorted(specs.keys(), key=lambda t: _MASTER_TYPES.index(t) if t in _MASTER_TYPES else 99)
        for rtype in order:
            rs = specs[rtype] or {}
            n = int(rs.get("replicas", 1) or 1)
            containers = (((rs.get("template") or {}).get("spec") or {}).get("containers")) or []
            if not containers:
                continue
            for i in range(n):
                out.append((rtype, i, containers[0]))
        return out

    async def _drive_real(self, gvr: GroupVersionResource, obj: Dict[str, Any]) -> None:
        m = obj["metadata"]
        ns, name = m["namespace"], m["name"]
        procs_spec = self._replica_processes(obj)
        await self.mark_running(gvr, obj)
        if not procs_spec:
            await self.complete(gvr, ns, name, False)
            return
        world = len(procs_spec)
        port = _free_port()  # one host for every replica: a port nothing else holds right now
        procs = []
        t0 = self.clock.monotonic()
        for rank, (rtype, idx, c) in enumerate(procs_spec):
            cmd = list(c.get("command") or []) + list(c.get("args") or [])
            if not cmd:
                continue
            if cmd[0] in ("python", "python3"):
                cmd[0] = sys.executable
            env = dict(os.environ)
            for e in c.get("env") or []:
                if isinstance(e, dict) and "name" in e and "value" in e:
                    env[e["name"]] = str(e["value"])
            env.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(world),
                        "RANK": str(rank), "LOCAL_RANK": str(rank), "PYTHONUNBUFFERED": "1",
                        "KUBEFLOW_JOB_NAME": name, "KUBEFLOW_REPLICA_TYPE": rtype.lower(),
                        "KUBEFLOW_REPLICA_INDEX": str(idx)})
            env.update(self.extra_env)
            self.log.info("starting replica", job=f"{ns}/{name}", replica=f"{rtype}-{idx}", cmd=" ".join(cmd))
            procs.append(await asyncio.create_subprocess_exec(*cmd, env=env, cwd=self.workdir or c.get("workingDir"),
                                                              stdout=asyncio.subprocess.PIPE,
                                                              stderr=asyncio.subprocess.STDOUT))
        codes: List[int] = []
        for i, p in enumerate(procs):
            try:
                out, _ = await asyncio.wait_for(p.communicate(), self.timeout)
            except asyncio.TimeoutError:
                p.kill()
                out, _ = await p.communicate()
            codes.append(p.returncode if p.returncode is not None else -9)
            text = (out or b"").decode(errors="replace")
            if i == 0:
                self.outputs[f"{ns}/{name}"] = text[-20000:]
            if text:
                self.log.info("replica output", job=f"{ns}/{name}", output=text[-4000:])
        ok = bool(codes) and all(c == 0 for c in codes)
        self.results[f"{ns}/{name}"] = (ok, codes, self.clock.monotonic() - t0)
        await self.complete(gvr, ns, name, ok)

    async def wait_all(self, timeout: float = 600.0) -> None:
        if self._tasks:
            await asyncio.wait_for(asyncio.gather(*self._tasks, return_exceptions=True), timeout)

    async def stop(self) -> None:
        for inf in self.informers:
            await inf.stop()
        await aio.cancel_and_wait(*self._tasks)
