"""Test environment -- the envtest suite analog.

Reference: ``internal/controller/suite_test.go:53-124`` starts a kube-apiserver,
installs ``charts/cron-operator/crds`` and ``test/crds``, and hands tests a client.
:class:`TestEnv` does the same in-process: a fake :class:`APIServer` (optionally
with a :class:`FakeClock`), the Cron CRD, the Kubeflow job CRDs, an in-memory
client, and helpers to run a manager + controller against it.
"""
from __future__ import annotations

import asyncio
from typing import Any, Dict, Optional

from ..api.v1alpha1 import CRON_GVR, Cron
from ..api.v1alpha1.crd import crd as cron_crd
from ..apiserver.server import APIServer
from ..controller.reconciler import CronReconciler, ReconcilerOptions
from ..controller.setup import setup_with_manager
from ..runtime.client import Client, InMemoryTransport
from ..runtime.controller import Controller
from ..runtime.manager import Manager, ManagerOptions
from ..trainingop.crds import kubeflow_crds
from ..utils.clock import Clock, FakeClock
from ..utils.gotime import NANOS


def aligned_start(minute_offset_s: float = 5.0) -> int:
    """A fake-clock start 5s past a fixed UTC minute (2026-01-01T12:00:05Z)."""
    return (1767268800 + int(minute_offset_s)) * NANOS


class TestEnv:
    __test__ = False  # not a pytest class

    def __init__(self, clock: Optional[Clock] = None, gc: bool = False, qps: float = -1, burst: int = 50,
                 install_kubeflow: bool = True):
        self.clock = clock if clock is not None else FakeClock(aligned_start())
        self.server = APIServer(self.clock, gc=gc)
        self.server.install_crd(cron_crd())
        if install_kubeflow:
            for c in kubeflow_crds():
                self.server.install_crd(c)
        self.transport = InMemoryTransport(self.server)
        self.client = Client(self.transport, qps=qps, burst=burst)
        self.manager: Optional[Manager] = None
        self.controller: Optional[Controller] = None
        self.reconciler: Optional[CronReconciler] = None
        self._mgr_task: Optional[asyncio.Task] = None

    def new_client(self, qps: float = -1, burst: int = 50) -> Client:
        return Client(InMemoryTransport(self.server), qps=qps, burst=burst)

    async def create_cron(self, cron: Cron) -> Dict[str, Any]:
        return await self.client.create(CRON_GVR, cron.to_dict(), cron.namespace)

    async def start_manager(self, options: Optional[ReconcilerOptions] = None, max_concurrent: int = 10,
                            **mgr_kw: Any) -> Manager:
        mopts = ManagerOptions(clock=self.clock, max_concurrent_reconciles=max_concurrent,
                               health_probe_bind_address=mgr_kw.pop("health_probe_bind_address", "0"),
                               metrics_bind_address=mgr_kw.pop("metrics_bind_address", "0"), **mgr_kw)
        self.manager = Manager(self.client, mopts)
        self.controller, self.reconciler = await setup_with_manager(self.manager, options)
        self._mgr_task = asyncio.get_running_loop().create_task(self.manager.start())
        await asyncio.wait_for(self.manager.started.wait(), 30)
        return self.manager

    async def settle(self, timeout: float = 30.0) -> None:
        """Let informers deliver pending events and the controller drain its queue."""
        assert self.controller is not None
        for _ in range(3):
            await asyncio.sleep(0)
        loop_deadline = asyncio.get_running_loop().time() + timeout
        idle_rounds = 0
        while asyncio.get_running_loop().time() < loop_deadline:
            await asyncio.sleep(0)
            if self.controller.queue.idle() and self._watches_drained():
                idle_rounds += 1
                if idle_rounds >= 3:
                    return
            else:
                idle_rounds = 0
                await asyncio.sleep(0.0005)
        raise TimeoutError("controller did not settle")

    def _watches_drained(self) -> bool:
        for lst in self.server._watchers.values():
            for w in lst:
                if not w.queue.empty() or w.lagged:
                    return False
        return True

    async def advance(self, seconds: float) -> None:
        """Advance the fake clock (firing due requeues) and settle."""
        assert isinstance(self.clock, FakeClock)
        self.clock.advance(seconds)
        await self.settle()

    async def stop(self) -> None:
        if self.manager is not None:
            self.manager.stop()
        if self._mgr_task is not None:
            try:
                await asyncio.wait_for(self._mgr_task, 10)
            except Exception:
                pass
        self.server.close_all_watches()
