#!/usr/bin/env python3
"""The soak: a long run of the headline harness, split into 20-tick windows.

Round-5 verdict #2: the 80-tick soak's step time grew ~10% from its first 20-tick window to its
last.  This runs the 3-shard headline configuration (1000 Crons, ``* * * * *``, historyLimit 10,
label-routed shards, the native fake apiserver) for ``--steps`` ticks and reports, per window:
the mean step time, the operator shards' CPU per fire, the fake apiserver's CPU per fire, and
each window's step time relative to the first.  It ends with what the fixture holds (watch-log
events per resource, objects) and the shards' resident size, so a window that drifts points at
the structure that grew.

    python scripts/soak_windows.py --steps 200 --out soak.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def windows(series, size):
    return [series[i:i + size] for i in range(0, len(series) - size + 1, size)]


def _fixture_windows(snaps, fires):
    """Per window: the fixture's requests, sends and phase kcycles per fire, and its RSS."""
    out = []
    for a, b in zip(snaps, snaps[1:]):
        if not a.get("io") or not b.get("io"):
            continue
        row = {"requests_per_fire": round((b["requests"] - a["requests"]) / fires, 3),
               "rss_mib": b.get("rss_mib")}
        row.update({k + "_per_fire": round((b["io"][k] - a["io"][k]) / fires, 3) for k in b["io"]})
        row["phase_kcycles_per_fire"] = {k: round((b["phase_cycles"][k] - a["phase_cycles"][k]) / fires / 1000, 1)
                                         for k in b["phase_cycles"]}
        row["thread_cpu_us_per_fire"] = {k: round((b["server_thread_cpu_s"][k] - a["server_thread_cpu_s"][k]) * 1e6
                                                  / fires, 1) for k in b["server_thread_cpu_s"]}
        out.append(row)
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--crons", type=int, default=1000)
    ap.add_argument("--shards", type=int, default=3)
    ap.add_argument("--window", type=int, default=20)
    ap.add_argument("--partitions", type=int, default=1,
                    help="fake apiserver processes (1: shared by the shards; --shards: one per shard, the "
                         "headline's layout -- the fixture counters then come from the first partition)")
    ap.add_argument("--impl", default="native", choices=["native", "python"])
    ap.add_argument("--watch-window", type=int, default=20_000)
    ap.add_argument("--lifecycle", default="instant", choices=["instant", "realistic"],
                    help="the jobs' status sequence (the headline's, bench.py --lifecycle: instant)")
    ap.add_argument("--tolerance", type=float, default=0.05, help="allowed |window / first window - 1|")
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    from cron_operator_amd.bench import harness

    fixture = {}
    orig = harness._cpu_times
    done = [False]
    url = [""]
    pid = [0]
    per_window = []  # the fixture's counters (and resident size) at each window boundary

    def fixture_snapshot():
        row = {}
        try:
            with urllib.request.urlopen(url[0] + "/debug/fake/stats", timeout=10) as f:
                st = json.loads(f.read())
            row = {"requests": st.get("total"), "io": st.get("io"), "phase_cycles": st.get("phase_cycles"),
                   "server_thread_cpu_s": st.get("server_thread_cpu_s")}
            with open(f"/proc/{pid[0]}/status") as fh:
                for line in fh:
                    if line.startswith("VmRSS"):
                        row["rss_mib"] = round(int(line.split()[1]) / 1024, 1)
        except (OSError, ValueError):
            pass
        return row

    # at each window boundary: ms for a fixed CPU-bound loop (the core's speed) and for a walk
    # over 64 MiB (what the memory system gives under the neighbours' load) -- the box is shared
    calib = []
    import numpy as np

    walk = np.random.default_rng(0).permutation(1 << 23).astype(np.int64)  # 64 MiB of indices

    def calibrate():
        t0 = time.perf_counter()
        x = 0
        for i in range(300_000):
            x += i * i
        t1 = time.perf_counter()
        int(walk[walk[::16]].sum())  # a gather over the whole array: cache-missing loads
        t2 = time.perf_counter()
        return [round((t1 - t0) * 1000, 2), round((t2 - t1) * 1000, 2)]

    def progress(k, dt, timed):
        if k % 20 == 0:
            print(f"tick {k}: {dt * 1000:.0f} ms", flush=True)
        if url[0] and k >= a.warmup and (k - a.warmup) % a.window == 0:
            per_window.append(fixture_snapshot())
            calib.append(calibrate())
        done[0] = k == a.warmup + a.steps

    # the fixture's holdings at the end of the run: read once, after the timed region closed
    def cpu(remote):
        r = orig(remote)
        if isinstance(remote, list):  # partitions: the first one's counters and holdings
            remote = remote[0] if remote else None
        if remote is not None and remote.url and remote.proc is not None:
            url[0], pid[0] = remote.url, remote.proc.pid
        if done[0] and not fixture and remote is not None and remote.url:
            try:
                with urllib.request.urlopen(remote.url + "/debug/fake/watch-log", timeout=10) as f:
                    fixture["watch_log"] = json.loads(f.read())
                with urllib.request.urlopen(remote.url + "/debug/fake/count?group=kubeflow.org&version=v1"
                                            "&resource=pytorchjobs", timeout=10) as f:
                    fixture["pytorchjobs"] = json.loads(f.read())["count"]
                with open(f"/proc/{remote.proc.pid}/status") as fh:
                    for line in fh:
                        if line.startswith(("VmRSS", "VmHWM")):
                            k, v = line.split(":")
                            fixture[k] = round(int(v.split()[0]) / 1024, 1)
            except (OSError, ValueError, KeyError):
                pass
        return r

    harness._cpu_times = cpu
    try:
        res = harness.run_sync(harness.BenchConfig(n_crons=a.crons, steps=a.steps, warmup=a.warmup,
                                                   shards=a.shards, apiserver_impl=a.impl, lifecycle=a.lifecycle,
                                                   watch_window=a.watch_window,
                                                   apiserver_partitions=a.partitions), on_step=progress)
    finally:
        harness._cpu_times = orig
    n = a.crons * a.window
    step_w = [statistics.mean(w) for w in windows(res.step_ms, a.window)]
    op_w = [sum(w) * 1000 / n for w in windows(res.step_cpu_operator_s, a.window)]
    api_w = [sum(w) * 1e6 / n for w in windows(res.step_cpu_apiserver_s, a.window)]
    rel = [round(x / step_w[0] - 1, 4) for x in step_w]
    out = {"config": {"crons": a.crons, "steps": a.steps, "warmup": a.warmup, "shards": a.shards,
                      "partitions": a.partitions,
                      "impl": a.impl, "watch_window": a.watch_window, "window": a.window, "lifecycle": a.lifecycle},
           "value": round(res.cron_reconciles_per_s, 1),
           "ms_per_step_by_window": [round(x, 1) for x in step_w],
           "step_vs_first_window": rel,
           "operator_cpu_ms_per_fire_by_window": [round(x, 4) for x in op_w],
           "apiserver_cpu_us_per_fire_by_window": [round(x, 1) for x in api_w],
           "within_tolerance": all(abs(x) <= a.tolerance for x in rel),
           "shard_peak_rss_mib": res.operator_maxrss_mib, "shard_end_rss_mib": res.operator_rss_mib,
           "fixture_end": fixture, "operator_gc": res.operator_gc,
           "fixture_by_window": _fixture_windows(per_window, n),
           "calibration_ms_at_window_starts": {"cpu_loop": [c[0] for c in calib],
                                               "memory_walk_64mib": [c[1] for c in calib]}}
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
