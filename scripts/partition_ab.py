#!/usr/bin/env python3
"""Shared fixture vs partitioned fixture, arms alternating on one box.

The headline runs 3 label-routed operator shards against ONE fake apiserver process; bench.py's
``partitioned_*`` arm runs the same shards each against a fake apiserver of its own (the Crons
that hash to that shard and their jobs).  This alternates the two ``--reps`` times and reports,
per run, throughput, operator CPU per fire, the fixture's busy fraction (the one server; the
busiest partition), and the shards' context switches per fire -- voluntary ones count the event
loop's sleeps on I/O (how many wake-ups a fire costs), involuntary ones preemptions by another
runnable task.

    python scripts/partition_ab.py --reps 3 --out gpurun_out/partition_ab.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(parts: int, crons: int, steps: int, warmup: int, shards: int, completion: str = "batch") -> dict:
    from cron_operator_amd.bench.harness import BenchConfig, run_sync

    t = time.perf_counter()
    r = run_sync(BenchConfig(n_crons=crons, steps=steps, warmup=warmup, shards=shards, lifecycle="instant",
                             apiserver_partitions=parts, namespace=f"ab-p{parts}", completion_writes=completion))
    fires = crons * steps
    busy = [c / r.elapsed_s for c in r.cpu_s_apiserver_parts] if parts > 1 else [r.cpu_s_apiserver / r.elapsed_s]
    vol, invol = (r.operator_ctx_switches + [0, 0])[:2]
    return {"partitions": parts, "completion_writes": completion, "value": round(fires / r.elapsed_s, 1),
            "ms_per_step_median": round(statistics.median(r.step_ms), 2),
            "operator_cpu_ms_per_fire": round(r.cpu_s_operator * 1000 / fires, 4),
            "fixture_busy_max": round(max(busy), 3), "fixture_busy": [round(b, 3) for b in busy],
            "fixture_cpu_us_per_fire": round(r.cpu_s_apiserver * 1e6 / fires, 1),
            "voluntary_csw_per_fire": round(vol / fires, 3), "involuntary_csw_per_fire": round(invol / fires, 3),
            "p50_ms": round(r.p50_latency_ms, 2), "wall_s": round(time.perf_counter() - t, 1),
            "phase_ms_median": {k: round(statistics.median(v), 1) for k, v in r.phase_ms.items() if v}}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--crons", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--shards", type=int, default=3)
    ap.add_argument("--arms", default="",
                    help="comma-separated partitions:completion_writes arms, e.g. 1:batch,1:interleaved "
                         "(default: 1:batch,<shards>:batch)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    arms = [(int(x.split(":")[0]), x.split(":")[1]) for x in a.arms.split(",")] if a.arms else \
        [(1, "batch"), (a.shards, "batch")]
    rows = []
    for rep in range(a.reps):
        for parts, completion in arms:
            row = one(parts, a.crons, a.steps, a.warmup, a.shards, completion)
            row["rep"] = rep
            rows.append(row)
            print(json.dumps(row), flush=True)
    out = {"config": vars(a), "cpus": os.cpu_count(),
           "affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None, "runs": rows}
    for parts, completion in arms:
        rs = [r for r in rows if r["partitions"] == parts and r["completion_writes"] == completion]
        tag = f"median_partitions_{parts}" + ("" if completion == "batch" else f"_{completion}")
        out[tag] = {k: statistics.median(r[k] for r in rs)
                    for k in ("value", "operator_cpu_ms_per_fire", "fixture_busy_max", "voluntary_csw_per_fire",
                              "involuntary_csw_per_fire")}
    print(json.dumps({k: v for k, v in out.items() if k.startswith("median")}), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
