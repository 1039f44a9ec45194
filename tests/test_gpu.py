"""GPU tier: runs on a real MI355X (``pytest -m gpu``).

The operator is CPU control plane; what touches the GPU is the *scheduled
workload*.  These tests check that path end to end on the box and that the
operator process ran on its native components:

* the smoke payload itself on ``cuda:0`` (bf16 step vs fp32 CPU reference);
* the full scheduled-training scenario (Cron -> PyTorchJob -> payload on the
  GPU -> history ``Succeeded``);
* a 1-rank RCCL DDP payload run (``backend=nccl`` is RCCL on ROCm);
* a short headline-bench run on the box (native engine loaded, its payload probe over RCCL).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpu_available() -> bool:
    try:
        out = subprocess.run([sys.executable, "-c", "import torch;print(torch.cuda.is_available())"],
                             capture_output=True, text=True, timeout=600)
        return out.stdout.strip().endswith("True")
    except Exception:
        return False


pytestmark = pytest.mark.gpu


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    return env


@pytest.fixture(scope="module")
def gpu():
    if not _gpu_available():
        pytest.fail("no GPU visible to PyTorch on a gpu-marked run")
    return True


def test_native_components_loaded():
    from cron_operator_amd.cron.engine import NativeEngine
    from cron_operator_amd.ops import cron_native
    from cron_operator_amd.utils import jsonutil

    from cron_operator_amd.apiserver import http as srvhttp
    from cron_operator_amd.runtime import fasthttp

    NativeEngine()
    assert os.path.realpath(cron_native.engine_path()).startswith(os.path.realpath(ROOT))
    assert jsonutil.NATIVE
    assert fasthttp._codec is not None and srvhttp._codec is not None
    assert os.path.realpath(fasthttp._codec.__file__).startswith(os.path.realpath(ROOT))
    # the benchmark's fake apiserver: the in-tree C++ server, not the Python one
    from cron_operator_amd.apiserver.native import load

    mod = load()
    assert mod is not None and os.path.realpath(mod.__file__).startswith(os.path.realpath(ROOT))


def test_train_smoke_payload_on_gpu(gpu):
    out = subprocess.run([sys.executable, "-m", "cron_operator_amd.models.payloads.train_smoke", "--device",
                          "cuda:0"], capture_output=True, text=True, timeout=900, env=_env(), cwd=ROOT)
    assert out.returncode == 0, out.stdout + out.stderr
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("SMOKE_OK")][0]
    info = json.loads(line.split(" ", 1)[1])
    assert info["hip"], "expected a ROCm build of PyTorch"
    assert info["grad_rel_err"] < 0.05


def test_scheduled_training_on_gpu(gpu):
    import asyncio

    os.environ["CRON_OPERATOR_ENGINE"] = "native"
    from cron_operator_amd.bench.smoke import run_smoke

    res = asyncio.run(run_smoke("cuda:0"))
    assert res["exit_codes"] == [0]
    assert res["history"][-1][1] == "Succeeded"


def test_ddp_payload_rccl_single_rank(gpu):
    env = _env()
    env.update({"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": "29611"})
    out = subprocess.run([sys.executable, "-m", "cron_operator_amd.models.payloads.ddp_train", "--steps", "5"],
                         capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "DDP_OK" in out.stdout and '"backend": "nccl"' in out.stdout


def test_ddp_cron_suspend_resume_cycle_on_gpu(gpu):
    """BASELINE config 5 on the box: the examples/mi355x DDP Cron (torchrun, RCCL) through a
    suspend/resume cycle (cron_operator_amd/bench/ddp_cycle.py)."""
    import asyncio

    import torch

    from cron_operator_amd.bench.ddp_cycle import run_ddp_cycle

    n = torch.cuda.device_count()
    res = asyncio.run(run_ddp_cycle(max(1, n), cpu=False))
    assert [s for _, s in res["history"]] == ["Succeeded", "Succeeded"]
    assert all(codes == [0] for codes in res["exit_codes"].values())
    for rep in res["ddp"].values():
        # one rank per visible GPU, each on its own device (PCI address), over RCCL
        assert rep["world"] == n and rep["backend"] == "nccl", rep
        assert len(set(rep["devices"])) == rep["world"], rep


def test_ddp_8_replica_cron_cycle_on_gpu(gpu):
    """The Master + Worker example (one process per replica, ranks from the PyTorchJob env):
    Workers = visible GPUs - 1, so world == device_count (8 on a full node, 1 here), each
    rank on a distinct GPU."""
    import asyncio

    import torch

    from cron_operator_amd.bench.ddp_cycle import run_ddp_cycle

    n = torch.cuda.device_count()
    res = asyncio.run(run_ddp_cycle(max(1, n), cpu=False, topology="replicas"))
    assert [s for _, s in res["history"]] == ["Succeeded", "Succeeded"]
    for job, rep in res["ddp"].items():
        assert rep["world"] == n and rep["backend"] == "nccl", (job, rep)
        assert len(set(rep["devices"])) == n, rep


def test_headline_bench_short_run():
    out = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--crons", "300",
                          "--baseline-steps", "1"],
                         capture_output=True, text=True, timeout=900, env=_env(), cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["value"] > 0 and res["cron_engine"] == "native"
    assert res["config"]["apiserver_impl"] == "native"  # served by the in-tree _apiserverd
    assert res["baseline_source"].startswith("measured") and res["vs_baseline"] > 1
    # the untimed payload probe ran the scheduled DDP payload over RCCL on this box's GPU
    probe = res["payload_ddp"]
    assert probe.get("ok") is True and probe["backend"] == "nccl" and probe["world"] == 1, probe
