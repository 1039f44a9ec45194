#!/usr/bin/env python3
"""Where the benchmark's time goes, fixture side: the fake apiserver's CPU over the timed steps.

Runs the headline harness (1000 Crons, `* * * * *`, historyLimit 10) and reports, per run, the
apiserver process's CPU and busy fraction and the operator's CPU per fire -- and, for the native
fake apiserver (``--impl native``), its server thread's CPU by phase (socket reads + request
parsing, verbs, the Python fallback that runs the harness's job writes, framing + socket writes)
and per verb.  ``--impl python`` measures the rounds 1-5 fixture the same way (process CPU only).

    python scripts/fixture_split.py --shards 3 1 --impl native python --reps 2 --out split.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(shards: int, impl: str, steps: int, warmup: int, crons: int, lifecycle: str,
        watch_window: int = 20_000, profile: str = "") -> dict:
    from cron_operator_amd.bench import harness

    # the native server's counters when the timed region opens (after the last warmup step) and
    # once it closed (the first CPU read after the last step)
    snaps = []
    orig = harness._cpu_times
    url = [""]
    at = [0]

    def snap():
        with urllib.request.urlopen(url[0] + "/debug/fake/stats") as f:
            snaps.append(json.loads(f.read()))

    def cpu(remote):
        r = orig(remote)
        if remote is not None and remote.url:
            url[0] = remote.url
            if impl == "native" and at[0] == warmup + steps and len(snaps) == 1:
                snap()
        return r

    def on_step(k, dt, timed):
        at[0] = k
        if k == warmup and impl == "native" and url[0]:
            snap()

    harness._cpu_times = cpu
    try:
        res = harness.run_sync(harness.BenchConfig(n_crons=crons, steps=steps, warmup=warmup, shards=shards,
                                                   lifecycle=lifecycle, apiserver_impl=impl,
                                                   watch_window=watch_window, apiserver_profile=profile),
                               on_step=on_step)
    finally:
        harness._cpu_times = orig
    fires = crons * steps
    out = {"shards": shards, "impl": impl, "value": round(res.cron_reconciles_per_s, 1),
           "p50_ms": round(res.p50_latency_ms, 2), "elapsed_s": round(res.elapsed_s, 3),
           "apiserver_busy_frac": round(res.cpu_s_apiserver / res.elapsed_s, 3),
           "apiserver_cpu_us_per_fire": round(res.cpu_s_apiserver * 1e6 / fires, 1),
           "operator_cpu_ms_per_fire": round(res.cpu_s_operator * 1000 / fires, 4),
           "step_ms": [round(x, 1) for x in res.step_ms]}
    if len(snaps) >= 2:
        a, b = snaps[0], snaps[-1]
        out["server_thread_cpu_us_per_fire"] = {
            k: round((b["server_thread_cpu_s"][k] - a["server_thread_cpu_s"][k]) * 1e6 / fires, 1)
            for k in b["server_thread_cpu_s"]}
        per_verb = {}
        for k, (s1, n1) in b["verb_cpu"].items():
            s0, n0 = a["verb_cpu"].get(k, (0.0, 0))
            if n1 > n0:
                per_verb[k] = {"calls_per_fire": round((n1 - n0) / fires, 3),
                               "us_per_call": round((s1 - s0) * 1e6 / (n1 - n0), 1)}
        out["per_verb"] = per_verb
        # the verbs' phases (TSC cycles per fire; `finish` includes `emit`)
        out["io_per_fire"] = {k: round((b["io"][k] - a["io"][k]) / fires, 2) for k in b.get("io", {})}
        out["phase_kcycles_per_fire"] = {k: round((b["phase_cycles"][k] - a["phase_cycles"][k]) / fires / 1000, 1)
                                         for k in b["phase_cycles"]}
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--shards", type=int, nargs="+", default=[3, 1])
    ap.add_argument("--impl", nargs="+", default=["native", "python"], choices=["native", "python"])
    ap.add_argument("--reps", type=int, default=1, help="alternating repetitions of every (impl, shards) arm")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--crons", type=int, default=1000)
    ap.add_argument("--lifecycle", default="instant", choices=["instant", "realistic"])
    ap.add_argument("--watch-window", type=int, default=20_000)
    ap.add_argument("--profile-dir", default="",
                    help="also sample the native fake apiserver's stacks per run: <dir>/<impl>_<shards>_<rep>.txt")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    for rep in range(a.reps):
        for impl in a.impl:
            for shards in a.shards:
                prof = os.path.join(a.profile_dir, f"{impl}_{shards}_{rep}.txt") if a.profile_dir and impl == "native" \
                    else ""
                r = run(shards, impl, a.steps, a.warmup, a.crons, a.lifecycle, a.watch_window, prof)
                r["rep"] = rep
                rows.append(r)
                print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rows, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
