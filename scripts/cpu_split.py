#!/usr/bin/env python3
"""User vs kernel CPU of one operator process and of the fake apiserver over the bench's
timed steps (1000 Crons, one process): how much of each side's cost is system calls.

    python scripts/cpu_split.py [--crons 1000 --steps 10 --warmup 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--crons", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--tls", action="store_true")
    a = ap.parse_args()
    from cron_operator_amd.bench import harness

    tck = os.sysconf("SC_CLK_TCK")
    marks = []

    def split(remote):
        t = os.times()
        api = (float("nan"), float("nan"))
        if remote is not None and remote.proc is not None:
            with open(f"/proc/{remote.proc.pid}/stat") as fh:
                f = fh.read().rsplit(")", 1)[1].split()
            api = (int(f[11]) / tck, int(f[12]) / tck)
        marks.append((t.user, t.system) + api)
        return orig(remote)

    orig = harness._cpu_times
    harness._cpu_times = split
    cfg = harness.BenchConfig(n_crons=a.crons, steps=a.steps, warmup=a.warmup, history_limit=10, transport="http",
                              shards=1, tls=a.tls)
    res = harness.run_sync(cfg)
    (u0, s0, au0, as0), (u1, s1, au1, as1) = marks[0], marks[-1]
    fires = a.crons * a.steps
    out = {"value": round(a.crons * a.steps / res.elapsed_s, 1), "fires": fires,
           "operator_user_us_per_fire": round((u1 - u0) * 1e6 / fires, 1),
           "operator_sys_us_per_fire": round((s1 - s0) * 1e6 / fires, 1),
           "apiserver_user_us_per_fire": round((au1 - au0) * 1e6 / fires, 1),
           "apiserver_sys_us_per_fire": round((as1 - as0) * 1e6 / fires, 1)}
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
