"""bench.py driver contract: one JSON line with the required keys, 1 rank and 2 ranks (gloo)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env["MASTER_ADDR"] = "127.0.0.1"
    return env


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def test_single_rank_line():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--crons", "20"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and d["config"]["global_batch"] == 20 and d["scaling"] == "weak"
    assert d["config"]["operator_shards"] == 3 and d["config"]["shard_routing"] == "labels"
    assert abs(d["value"] - 20 * 2 / (d["ms_per_step"] * 2 / 1000)) / d["value"] < 0.01


def test_two_ranks_aggregate():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--crons", "20"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)  # rank 0 only
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 40 and d["config"]["parallelism"] == "ranks2x3shards"
