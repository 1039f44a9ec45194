"""BASELINE.json config 5: "Cron -> PyTorchJob 8-worker DDP template targeting one
8xMI355X ROCm node, suspend/resume cycle".

Two topologies, each an example Cron read from the repo:

* ``torchrun`` -- ``examples/mi355x/cron-pytorch-ddp-mi355x.yaml``: one Master
  replica running ``torchrun --nproc-per-node 8``;
* ``replicas`` -- ``examples/mi355x/cron-pytorch-ddp-8worker-mi355x.yaml``: Master
  + 7 Worker replicas, one process each, ranked by the training-operator's env
  (the reference examples' replica topology, ``examples/v1alpha1/cron/cron-pytorch.yaml``);
  the Worker count is ``nproc - 1``.

The torchrun Cron gets three environment-sized substitutions: the schedule becomes
``*/1 * * * *`` (the scenario runs on a virtual clock), ``torchrun`` gets one
worker per available device (``--nproc-per-node``; 8 on a full MI355X node, 1 on
the single-GPU box, 2 CPU ranks over gloo in the CPU tier) and a loopback
rendezvous, and the model is shrunk so one job takes seconds.  Everything else
-- Forbid, historyLimit, the RCCL env, the DDP payload and its bucket size -- is
the example's.

Cycle (reference semantics: ``cron_controller.go:169-173`` suspend returns
without requeue; on resume the missed ticks collapse into the most recent one,
``:408-436``; Forbid delays while a job is active, ``:204-207``):

1. tick -> the PyTorchJob is created, the fake training-operator (real mode) runs
   the replica's ``torchrun`` command, DDP trains over RCCL (or gloo), the job
   becomes ``Succeeded`` and moves to ``status.history``;
2. ``spec.suspend=true`` -> three more ticks pass with no job;
3. ``spec.suspend=false`` -> exactly one job, named for the latest tick, runs
   and succeeds.
"""
from __future__ import annotations

import asyncio
import os
import sys
import time
from typing import Any, Dict, List

import yaml

from ..api.meta import GroupVersionResource
from ..api.v1alpha1 import CRON_GVR

PYTORCHJOBS = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
EXAMPLE = os.path.join(ROOT, "examples", "mi355x", "cron-pytorch-ddp-mi355x.yaml")
# Master + 7 Worker replicas, one process (and one GPU) each -- BASELINE config 5 as written
EXAMPLE_REPLICAS = os.path.join(ROOT, "examples", "mi355x", "cron-pytorch-ddp-8worker-mi355x.yaml")


def _free_port() -> int:
    from ..utils.ports import free_port

    return free_port()


def _shrink(ctr: Dict[str, Any], cpu: bool, steps: int, hidden: int) -> None:
    args: List[str] = list(ctr["args"])
    for flag, val in (("--steps", steps), ("--hidden", hidden), ("--layers", 2), ("--batch", 8)):
        args[args.index(flag) + 1] = str(val)
    if cpu:
        args.append("--cpu")
    ctr["args"] = args


def ddp_cron(nproc: int, cpu: bool, steps: int = 5, hidden: int = 256, topology: str = "torchrun") -> Dict[str, Any]:
    """The example Cron, sized for this environment (see the module docstring).

    ``topology="torchrun"``: one Master replica running ``torchrun --nproc-per-node``;
    ``"replicas"``: the Master + Worker example with ``nproc - 1`` Workers, one process per
    replica, ranks from the training-operator's env (``WORLD_SIZE``/``RANK``)."""
    with open(EXAMPLE if topology == "torchrun" else EXAMPLE_REPLICAS) as fh:
        cron = yaml.safe_load(fh)
    cron["metadata"]["namespace"] = "default"
    cron["spec"]["schedule"] = "*/1 * * * *"
    specs = cron["spec"]["template"]["workload"]["spec"]["pytorchReplicaSpecs"]
    if topology == "replicas":
        assert specs["Master"]["replicas"] == 1 and specs["Worker"]["replicas"] == 7, specs
        if nproc > 1:
            specs["Worker"]["replicas"] = nproc - 1
        else:
            del specs["Worker"]
        for rs in specs.values():
            rs["template"] = yaml.safe_load(yaml.safe_dump(rs["template"]))  # unshare the YAML anchor
            ctr = rs["template"]["spec"]["containers"][0]
            assert ctr["command"][-1] == "cron_operator_amd.models.payloads.ddp_train", ctr["command"]
            _shrink(ctr, cpu, steps, hidden)
        return cron
    ctr = specs["Master"]["template"]["spec"]["containers"][0]
    assert ctr["command"][0] == "torchrun" and "--nproc-per-node" in ctr["command"], ctr["command"]
    ctr["command"] = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
                      str(nproc), "--master-addr", "127.0.0.1", "--master-port", str(_free_port())]
    _shrink(ctr, cpu, steps, hidden)
    return cron


def _ddp_report(trainer, job: str) -> Dict[str, Any]:
    """The payload's ``DDP_OK {...}`` line of ``job`` (rank 0's output), parsed."""
    import json

    for line in trainer.outputs.get(job, "").splitlines():
        if line.startswith("DDP_OK "):
            return json.loads(line.split(" ", 1)[1])
    return {}


async def run_ddp_cycle(nproc: int = 1, cpu: bool = False, timeout: float = 600.0,
                        topology: str = "torchrun") -> Dict[str, Any]:
    from ..testing.env import TestEnv
    from ..trainingop.operator import FakeTrainingOperator

    env = TestEnv()
    pp = os.environ.get("PYTHONPATH", "")
    extra = {"PYTHONPATH": ROOT + (os.pathsep + pp if pp else "")}
    if cpu:
        extra["CUDA_VISIBLE_DEVICES"] = ""
        extra["HIP_VISIBLE_DEVICES"] = ""
    trainer = FakeTrainingOperator(env.new_client(), env.clock, mode="real", workdir=ROOT, timeout=timeout, env=extra)
    cron = ddp_cron(nproc, cpu, topology=topology)
    name = cron["metadata"]["name"]
    t0 = time.perf_counter()

    def jobs() -> List[str]:
        return sorted(j["metadata"]["name"] for j in env.server.list(PYTORCHJOBS, "default")["items"])

    def status() -> Dict[str, Any]:
        return env.server.get(CRON_GVR, "default", name).get("status") or {}

    async def finish_running() -> None:
        await trainer.wait_all(timeout)
        await env.settle()

    try:
        await env.client.create(CRON_GVR, cron, "default")
        await trainer.start()
        await env.start_manager()
        await env.settle()
        # 1. a tick runs the DDP job to completion
        await env.advance(60)
        first = jobs()
        if len(first) != 1:
            raise AssertionError(f"expected one PyTorchJob after the first tick, found {first}")
        await finish_running()
        # 2. suspended: ticks pass, nothing is created
        obj = env.server.get(CRON_GVR, "default", name)
        obj["spec"]["suspend"] = True
        env.server.update(CRON_GVR, "default", name, obj)
        await env.settle()
        for _ in range(3):
            await env.advance(60)
        suspended = jobs()
        if suspended != first:
            raise AssertionError(f"a suspended Cron created jobs: {suspended}")
        # 3. resumed: the missed ticks collapse into one run, named for the latest tick
        obj = env.server.get(CRON_GVR, "default", name)
        obj["spec"]["suspend"] = False
        env.server.update(CRON_GVR, "default", name, obj)
        await env.settle()
        resumed = jobs()
        new = [j for j in resumed if j not in first]
        if len(new) != 1:
            raise AssertionError(f"resume should run exactly one job, found {new}")
        await finish_running()
        # the job's completion reaches the Cron through a watch event and one more reconcile:
        # on a loaded machine that can trail the settle, so wait for it (bounded)
        want = [(first[0], "Succeeded"), (new[0], "Succeeded")]
        deadline = time.perf_counter() + 60.0
        while True:
            st = status()
            hist = [(h["object"]["name"], h["status"]) for h in st.get("history") or []]
            if (hist == want and not st.get("active")) or time.perf_counter() > deadline:
                break
            await asyncio.sleep(0.05)
            await env.settle()
        results = {k.split("/", 1)[1]: v for k, v in trainer.results.items()}
        out = {"jobs": resumed, "history": hist, "active": len(st.get("active") or []),
               "exit_codes": {j: results.get(j, (False, [], 0))[1] for j in resumed},
               "payload_s": {j: round(results.get(j, (False, [], 0.0))[2], 2) for j in resumed},
               "nproc": nproc, "device": "cpu" if cpu else "gpu", "topology": topology,
               "ddp": {j: _ddp_report(trainer, f"default/{j}") for j in resumed},
               "total_s": round(time.perf_counter() - t0, 2)}
        if hist != [(first[0], "Succeeded"), (new[0], "Succeeded")] or out["active"]:
            raise AssertionError(f"suspend/resume cycle did not end with two succeeded runs: {out}")
        return out
    finally:
        await trainer.stop()
        await env.stop()


def main() -> int:
    import argparse

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--nproc", type=int, default=0, help="DDP workers (default: visible GPUs, or 2 on CPU)")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--topology", choices=["torchrun", "replicas"], default="torchrun")
    a = ap.parse_args()
    nproc = a.nproc
    if nproc <= 0:
        if a.cpu:
            nproc = 2
        else:
            import torch

            nproc = max(1, torch.cuda.device_count())
    print(asyncio.run(run_ddp_cycle(nproc, a.cpu, topology=a.topology)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
