"""End-to-end smoke scenario: a Cron schedules a PyTorchJob that trains on the GPU.

SURVEY.md section 7.3's minimum slice: one ``Cron`` on ``*/1 * * * *`` whose
PyTorchJob Master runs :mod:`cron_operator_amd.models.payloads.train_smoke`
(one bf16 forward/backward/optimizer step on ``cuda:0``).  The operator runs
in-process against the fake apiserver with a virtual schedule clock; the fake
training-operator in *real* mode launches the replica as a subprocess (the
operator process itself never touches the GPU).  The scenario advances the
clock to the next tick, waits for the job to finish, and checks that the Cron
recorded it in ``status.history`` as ``Succeeded`` with no active children.
"""
from __future__ import annotations

import asyncio
import os
import sys
import time
from typing import Any, Dict

from ..api.meta import GroupVersionResource
from ..api.v1alpha1 import CRON_GVR, new_cron

PYTORCHJOBS = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")


def smoke_template(device: str) -> Dict[str, Any]:
    return {
        "apiVersion": "kubeflow.org/v1",
        "kind": "PyTorchJob",
        "metadata": {"labels": {"app": "mi355x-smoke"}},
        "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1, "restartPolicy": "Never", "template": {
            "spec": {"containers": [{
                "name": "pytorch", "image": "rocm/pytorch:latest",
                "command": ["python", "-m", "cron_operator_amd.models.payloads.train_smoke"],
                "args": ["--device", device],
                "resources": {"limits": {"amd.com/gpu": 1}}}]}}}}},
    }


async def run_smoke(device: str = "cuda:0", timeout: float = 900.0) -> Dict[str, Any]:
    from ..testing.env import TestEnv
    from ..trainingop.operator import FakeTrainingOperator

    env = TestEnv()
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    pp = os.environ.get("PYTHONPATH", "")
    trainer = FakeTrainingOperator(env.new_client(), env.clock, mode="real", workdir=root, timeout=timeout,
                                   env={"PYTHONPATH": root + (os.pathsep + pp if pp else "")})
    t0 = time.perf_counter()
    try:
        await env.create_cron(new_cron("mi355x-smoke", "default", "*/1 * * * *", smoke_template(device),
                                       history_limit=1, concurrency_policy="Forbid"))
        await trainer.start()
        await env.start_manager()
        await env.settle()
        await env.advance(60)  # next minute: the Cron fires
        jobs = env.server.list(PYTORCHJOBS, "default")["items"]
        if len(jobs) != 1:
            raise AssertionError(f"expected one PyTorchJob after the tick, found {len(jobs)}")
        await trainer.wait_all(timeout)
        await env.settle()
        cron = env.server.get(CRON_GVR, "default", "mi355x-smoke")
        st = cron.get("status") or {}
        hist = st.get("history") or []
        name = jobs[0]["metadata"]["name"]
        ok, codes, secs = trainer.results.get(f"default/{name}", (False, [], 0.0))
        result = {"job": name, "exit_codes": codes, "payload_s": round(secs, 2),
                  "history": [(h["object"]["name"], h["status"]) for h in hist], "active": len(st.get("active") or []),
                  "total_s": round(time.perf_counter() - t0, 2)}
        if not ok or not hist or hist[-1]["status"] != "Succeeded" or st.get("active"):
            raise AssertionError(f"scheduled training job did not succeed: {result}")
        return result
    finally:
        await trainer.stop()
        await env.stop()


def main() -> int:
    dev = sys.argv[1] if len(sys.argv) > 1 else "cuda:0"
    print(asyncio.run(run_smoke(dev)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
