#!/usr/bin/env python3
"""Idle cost of a running operator: CPU it burns while nothing is due.

Starts the fake apiserver and ``cron-operator start`` (leader election on, metrics and
probes served) as separate processes on the real clock, creates N Crons whose schedule
does not fire during the window (``0 0 1 1 *``) plus their history jobs, waits for the
operator to sync, then samples the operator process's CPU over ``--seconds``.  What runs
then is only background machinery: lease renewals (every 2 s), work-queue metric refreshes
(every 500 ms), watch liveness timers and BOOKMARK events.

    python scripts/idle_cpu.py --crons 1000 --seconds 30
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _post(base: str, path: str, body: dict) -> None:
    req = urllib.request.Request(base + path, data=json.dumps(body).encode(), method="POST",
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=30) as r:
        r.read()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--crons", type=int, default=1000)
    ap.add_argument("--history", type=int, default=10, help="finished jobs per Cron")
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--settle", type=float, default=40.0, help="seconds between readiness and sampling")
    a = ap.parse_args()
    import psutil

    env = dict(os.environ, PYTHONPATH=ROOT)
    port = _port()
    base = f"http://127.0.0.1:{port}"
    with tempfile.TemporaryDirectory() as d:
        kc = os.path.join(d, "kc")
        api = subprocess.Popen([sys.executable, "-m", "cron_operator_amd", "fake-apiserver", "--port", str(port),
                                "--kubeconfig-out", kc], env=env, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL)
        op = None
        try:
            for _ in range(600):
                try:
                    urllib.request.urlopen(base + "/api/v1/namespaces", timeout=1).read()
                    break
                except OSError:
                    time.sleep(0.1)
            _post(base, "/api/v1/namespaces", {"apiVersion": "v1", "kind": "Namespace",
                                               "metadata": {"name": "idle"}})
            for i in range(a.crons):
                name = f"idle-{i:05d}"
                cron = {"apiVersion": "apps.kubedl.io/v1alpha1", "kind": "Cron",
                        "metadata": {"name": name, "namespace": "idle"},
                        "spec": {"schedule": "0 0 1 1 *", "historyLimit": a.history,
                                 "template": {"workload": {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                                           "spec": {"pytorchReplicaSpecs": {
                                                               "Master": {"replicas": 1}}}}}}}
                _post(base, "/apis/apps.kubedl.io/v1alpha1/namespaces/idle/crons", cron)
                for j in range(a.history):
                    job = {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                           "metadata": {"name": f"{name}-{j}", "namespace": "idle",
                                        "labels": {"kubedl.io/cron-name": name}},
                           "spec": {"pytorchReplicaSpecs": {"Master": {"replicas": 1}}}}
                    _post(base, "/apis/kubeflow.org/v1/namespaces/idle/pytorchjobs", job)
            mport, pport = _port(), _port()
            op = subprocess.Popen([sys.executable, "-m", "cron_operator_amd", "start", "--kubeconfig", kc,
                                   "--leader-elect", f"--metrics-bind-address=127.0.0.1:{mport}",
                                   "--metrics-secure=false", f"--health-probe-bind-address=127.0.0.1:{pport}",
                                   "--zap-log-level=error"], env=env, stdout=subprocess.DEVNULL,
                                  stderr=subprocess.DEVNULL)
            for _ in range(1200):
                try:
                    if urllib.request.urlopen(f"http://127.0.0.1:{pport}/readyz", timeout=1).status == 200:
                        break
                except OSError:
                    pass
                time.sleep(0.1)
            time.sleep(a.settle)  # initial reconciles of every Cron, then quiet
            p = psutil.Process(op.pid)
            c0, t0 = p.cpu_times(), time.monotonic()
            time.sleep(a.seconds)
            c1, t1 = p.cpu_times(), time.monotonic()
            cpu = (c1.user + c1.system) - (c0.user + c0.system)
            rss = p.memory_info().rss / 2**20
            print(json.dumps({"crons": a.crons, "jobs": a.crons * a.history, "window_s": round(t1 - t0, 1),
                              "operator_cpu_s": round(cpu, 3), "operator_cpu_pct": round(100 * cpu / (t1 - t0), 3),
                              "operator_rss_mib": round(rss, 1)}))
        finally:
            for proc in (op, api):
                if proc is not None and proc.poll() is None:
                    proc.terminate()
                    try:
                        proc.wait(10)
                    except subprocess.TimeoutExpired:
                        proc.kill()
    return 0


if __name__ == "__main__":
    sys.exit(main())
