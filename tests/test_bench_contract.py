"""bench.py driver contract: one JSON line with the required keys, 1 rank and 2 ranks (gloo),
launched by torch.distributed.run or spawned by bench.py itself; operator-cost keys; a
vs_baseline denominator measured in the same invocation."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

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
    # operator cost, separated from the fake apiserver fixture
    assert d["operator_cpu_ms_per_fire"] > 0
    assert 0 <= d["apiserver_busy_frac"] < 2  # /proc CPU ticks are 10 ms: a 40-fire run may read 0
    assert 10 < d["operator_shard_peak_rss_mib"] < 1024  # the largest shard process's peak (VmHWM)
    # round-5 verdict: the "peak" (ru_maxrss) read below the end RSS; a high-water mark cannot
    assert 10 < d["operator_shard_end_rss_mib"] <= d["operator_shard_peak_rss_mib"]
    # the denominator is the reference algorithm measured by this same invocation
    assert d["baseline_source"].startswith("measured")
    assert d["baseline_value"] > 0 and d["baseline_p50_schedule_to_create_ms"] > 0
    assert d["baseline_api_requests_per_fire"] > d["api_requests_per_fire"]
    assert abs(d["vs_baseline"] - d["value"] / d["baseline_value"]) < 0.01 * d["vs_baseline"] + 0.002
    # the shipped default (one operator process), measured in the same invocation
    assert d["single_process_value"] > 0 and d["single_process_p50_ms"] > 0
    assert d["single_process_p99_ms"] >= d["single_process_p50_ms"]
    assert d["single_process_operator_cpu_ms_per_fire"] > 0 and 0 <= d["single_process_apiserver_busy_frac"] < 2
    # the headline's shards each have a fake apiserver process of their own (a partitioned
    # cluster: 8 CPUs here); the same shards against one shared fake apiserver run alongside
    assert d["config"]["fixture"] == "partitioned" and d["config"]["apiserver_partitions"] == 3
    assert "per shard" in d["data"]
    assert d["shared_fixture_value"] > 0 and d["shared_fixture_p50_ms"] > 0
    assert d["shared_fixture_operator_cpu_ms_per_fire"] > 0 and 0 <= d["shared_fixture_apiserver_busy_frac"] < 2
    # the deployment-shaped pair (TLS + etcd latency, one process, both algorithms), same invocation
    assert d["deployment_config"]["tls"] is True and d["deployment_config"]["apiserver_latency"] == "etcd"
    assert d["deployment_value"] > 0 and d["deployment_baseline_value"] > 0
    assert abs(d["vs_baseline_deployment"] - d["deployment_value"] / d["deployment_baseline_value"]) \
        < 0.01 * d["vs_baseline_deployment"] + 0.002
    assert d["deployment_baseline_api_requests_per_fire"] > d["deployment_api_requests_per_fire"]
    assert d["deployment_p50_ms"] > 0 and d["deployment_baseline_p50_ms"] > 0
    # the scheduled payload's RCCL probe runs only where every rank has a GPU (not in this container)
    assert "payload_ddp" in d and ("skipped" in d["payload_ddp"] or d["payload_ddp"].get("ok") is True)


def test_recorded_baseline_option():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "1", "--crons", "10", "--shards", "1",
                        "--baseline", "recorded"], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["baseline_value"] == 80.72 and d["baseline_source"].startswith("recorded")


def test_tls_apiserver_option():
    """``--tls``: the fake apiserver serves HTTPS and every operator connection -- one process and
    the shard processes -- verifies it against its CA; the run completes with the same request model."""
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "1", "--crons", "12", "--shards", "2",
                        "--tls", "--baseline", "none"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["config"]["tls"] is True and d["value"] > 0 and d["single_process_value"] > 0
    assert d["config"]["fixture"] == "partitioned"  # each partition with its own CA
    assert d["shared_fixture_value"] > 0
    assert d["api_requests_per_fire"] == 4.0


def test_gpus_without_launcher_spawns_ranks():
    """``--gpus 2`` with no WORLD_SIZE: bench.py starts both ranks itself; one line, 2 ranks' work."""
    env = _env()
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--crons", "20",
                        "--baseline", "none"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 40 and d["config"]["parallelism"] == "ranks2x3shards"
    assert d["vs_baseline"] is None


def test_gpus_mismatching_world_size_is_refused():
    env = _env()
    env["WORLD_SIZE"] = "1"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--crons", "5"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "refusing" in r.stderr


def test_two_ranks_aggregate():
    """The driver's launcher, 2 ranks; the payload probe rehearsed over gloo (``--payload-probe
    cpu``): rank 0 runs a 2-process DDP child job while rank 1 waits at the barrier, and both
    tear down together after the line is printed."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                        "--steps", "2", "--warmup", "1", "--crons", "20", "--payload-probe", "cpu"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)  # rank 0 only
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 40 and d["config"]["parallelism"] == "ranks2x3shards"
    # 8 CPUs cannot give 2 ranks a core per shard and per fake apiserver partition: one shared
    # fake apiserver per rank, and no other-fixture arm
    from cron_operator_amd.runtime.supervisor import available_cpus

    if available_cpus() // 2 < 7:
        assert d["config"]["fixture"] == "shared" and "partitioned_value" not in d
    probe = d["payload_ddp"]
    assert probe.get("ok") is True and probe["world"] == 2 and probe["backend"] == "gloo", probe


def test_payload_probe_runs_the_ddp_payload_as_a_clean_child_job(monkeypatch):
    """The probe a rank-0 of a launched bench starts: a child ``torch.distributed.run`` of the DDP
    payload that must not inherit the bench's own rendezvous (RANK/WORLD_SIZE/MASTER_PORT/
    TORCHELASTIC_* of the outer launcher).  On CPU (``cpu=True``: gloo) it trains in sync on 2
    ranks and reports the all-reduce bus bandwidth; a time limit is reported, not raised."""
    sys.path.insert(0, ROOT)
    import bench

    for k, v in {"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "8", "MASTER_PORT": "1", "MASTER_ADDR": "10.9.9.9",
                 "TORCHELASTIC_RUN_ID": "outer", "PYTHONPATH": _env()["PYTHONPATH"]}.items():
        monkeypatch.setenv(k, v)
    r = bench._payload_probe(2, 150, cpu=True, allreduce_mb=1, steps=2)
    assert r.get("ok") is True, r
    assert r["world"] == 2 and r["backend"] == "gloo" and r["distinct_devices"] == 2
    assert r["allreduce"]["mb"] == 1 and r["allreduce"]["busbw_gbs"] > 0
    slow = bench._payload_probe(2, 0.5, cpu=True, allreduce_mb=1, steps=2)
    assert slow.get("error", "").startswith("timed out"), slow


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.slow
def test_eight_ranks_the_drivers_line_shape():
    """Round-5 verdict #7: the driver's N=8 invocation shape on the CPU (gloo), before any 8-GPU
    node runs it: 8 ranks under ``torch.distributed.run``, each its own 200-Cron deployment; the
    shards per rank are chosen from the CPUs the job may use (never oversubscribed); rank 0 prints
    one line with the whole-job aggregate; the payload probe (``--payload-probe cpu``) runs the
    8-process DDP child job over gloo while the other ranks wait at the barrier."""
    from cron_operator_amd.runtime.supervisor import available_cpus

    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "8",
                        "--steps", "2", "--warmup", "1", "--crons", "200", "--payload-probe", "cpu"], cwd=ROOT,
                       env=_env(), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)  # rank 0 only
    shards = max(1, min(3, available_cpus() // 8 - 1))
    assert d["n_gpus"] == 8 and d["config"]["global_batch"] == 1600
    assert d["config"]["operator_shards"] == shards and d["config"]["parallelism"] == f"ranks8x{shards}shards"
    # aggregate: 8 ranks' fires over the slowest rank's timed window
    assert abs(d["value"] - 1600 * 2 / (d["ms_per_step"] * 2 / 1000)) / d["value"] < 0.01
    assert d["api_requests_per_fire"] == 4.0 and d["baseline_value"] > 0
    assert d["deployment_value"] > 0 and d["deployment_baseline_value"] > 0
    probe = d["payload_ddp"]
    assert probe.get("ok") is True and probe["world"] == 8 and probe["backend"] == "gloo", probe
    assert probe["distinct_devices"] == 8 and probe["allreduce"]["busbw_gbs"] > 0, probe


@pytest.mark.slow
def test_a_killed_rank_fails_the_eight_rank_job_without_a_hang():
    """One rank of the 8 dies mid-run (SIGKILL, as an OOM kill would): the launcher tears the
    others down and the job exits non-zero well inside the limit -- no rank waits forever at a
    barrier for the dead one."""
    import signal
    import time

    import psutil

    p = subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "8",
                          "--steps", "400", "--warmup", "1", "--crons", "100", "--baseline", "none",
                          "--deployment", "none", "--payload-probe", "none"], cwd=ROOT, env=_env(),
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        victim = None
        t0 = time.monotonic()
        while victim is None and time.monotonic() - t0 < 120:
            ranks = [c for c in psutil.Process(p.pid).children()
                     if "bench.py" in " ".join(c.cmdline()) and c.environ().get("RANK") == "5"]
            if ranks:
                victim = ranks[0]
            time.sleep(0.5)
        assert victim is not None, "rank 5 never started"
        time.sleep(8)  # past setup: the ranks are stepping, at or between barriers
        assert p.poll() is None, "the job ended before the kill"
        victim.send_signal(signal.SIGKILL)
        t_kill = time.monotonic()
        out, err = p.communicate(timeout=240)
        assert p.returncode != 0, err[-2000:]
        took = time.monotonic() - t_kill
        assert took < 240
        print(f"job ended {took:.1f} s after the kill, rc={p.returncode}")
        assert not [ln for ln in out.splitlines() if ln.startswith("{")]  # no partial line reported
    finally:
        if p.poll() is None:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()


def test_five_cpus_per_rank_run_two_partitioned_shards():
    """With 5-6 CPUs per rank the headline keeps a fake apiserver partition per shard and runs
    2 shards (a core each, a core per partition, one for the harness) rather than 3 shards
    against one shared fixture."""
    import shutil

    if shutil.which("taskset") is None or (os.cpu_count() or 1) < 5:
        pytest.skip("needs taskset and 5 CPUs")
    r = subprocess.run(["taskset", "-c", "0-4", sys.executable, "bench.py", "--steps", "1", "--warmup", "1",
                        "--crons", "12", "--baseline", "none", "--deployment", "none", "--single-process", "none",
                        "--payload-probe", "none"], cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["config"]["cpus_per_rank"] == 5 and d["config"]["parallelism"] == "ranks1x2shards"
    assert d["config"]["fixture"] == "partitioned" and d["config"]["apiserver_partitions"] == 2
