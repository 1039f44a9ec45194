#!/usr/bin/env python3
"""Scaling curve: the headline bench at 1 / 10 / 100 / 1000 Cron CRs (``--sizes``; 10000 for
the large-fleet row).

BASELINE.json asks for reconciles/sec and tick->create latency "at 1, 10, 100
and 1000 concurrent Cron CRs with the scaling curve reported".  This runs
``cron_operator_amd.bench.harness`` for each size, in both modes
(``optimized`` = this operator, ``reference`` = the reference algorithm), and
prints a Markdown table plus one JSON document (``--out``).
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,10,100,1000")
    ap.add_argument("--modes", default="optimized,reference")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--transport", default="http")
    ap.add_argument("--shards", type=int, default=1, help="operator shard processes")
    ap.add_argument("--shard-routing", choices=["labels", "hash"], default="labels",
                    help="how the shards split the watch traffic (controller/sharding.py)")
    ap.add_argument("--operator-process", action="store_true",
                    help="run a single shard in its own process too (its peak RSS is the operator's alone)")
    ap.add_argument("--lifecycle", choices=["realistic", "instant"], default="instant")
    ap.add_argument("--no-compact", action="store_true", help="A/B: ReconcilerOptions.compact_child_status=False")
    ap.add_argument("--distinct-templates", action="store_true",
                    help="every Cron its own template (a per-Cron container command), nothing shared across specs")
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    from cron_operator_amd.bench.harness import BenchConfig, run_sync

    rows = []
    for mode in a.modes.split(","):
        for n in (int(x) for x in a.sizes.split(",")):
            t0 = time.perf_counter()
            # small fleets get more ticks so percentiles rest on >= ~30 samples
            steps = max(a.steps, min(30, -(-30 // n)))
            r = run_sync(BenchConfig(n_crons=n, steps=steps, warmup=a.warmup, mode=mode, transport=a.transport,
                                     shards=a.shards if a.transport == "http" else 1,
                                     shard_routing=a.shard_routing,
                                     operator_process=a.operator_process, lifecycle=a.lifecycle,
                                     compact_children=not a.no_compact,
                                     distinct_templates=a.distinct_templates))
            rows.append({"mode": mode, "n_crons": n, "steps": steps, "shards": a.shards,
                         "shard_routing": a.shard_routing, "cron_reconciles_per_s": r.cron_reconciles_per_s,
                         "raw_reconciles_per_s": r.raw_reconciles_per_s, "p50_ms": r.p50_latency_ms,
                         "p99_ms": r.p99_latency_ms, "ms_per_step": r.ms_per_step,
                         "api_requests_per_fire": r.api_requests_per_fire,
                         "reconciles_per_fire": r.reconciles_per_fire, "wall_s": time.perf_counter() - t0,
                         "operator_cpu_ms_per_fire": r.cpu_s_operator * 1000 / (n * steps),
                         "apiserver_cpu_ms_per_fire": r.cpu_s_apiserver * 1000 / (n * steps),
                         "operator_gc": r.operator_gc, "phase_ms": r.phase_ms,
                         # peak RSS of each operator shard process (sharded runs only)
                         "operator_maxrss_mib": r.operator_maxrss_mib,
                         "operator_ready_maxrss_mib": r.operator_ready_maxrss_mib,
                         "operator_rss_mib": r.operator_rss_mib,
                         # one process: start (or fail-over) over the seeded cluster
                         "startup_sync_s": r.startup_sync_s, "startup_first_pass_s": r.startup_first_pass_s,
                         # one process: the operator runs in this process (with the harness's own
                         # bookkeeping; the apiserver is another process): an upper bound, cumulative
                         "this_process_peak_rss_mib": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
                                                            / 1024, 1)})
            print(f"{mode:>9} n={n:>5}: {r.cron_reconciles_per_s:9.1f} cron-reconciles/s  "
                  f"p50 {r.p50_latency_ms:8.1f} ms  p99 {r.p99_latency_ms:8.1f} ms  "
                  f"{r.api_requests_per_fire:.1f} req/fire  operator {r.cpu_s_operator * 1000 / (n * steps):.3f} "
                  f"ms CPU/fire, apiserver {r.cpu_s_apiserver * 1000 / (n * steps):.3f}, GC {r.operator_gc}"
                  + (f", shard peak RSS {r.operator_maxrss_mib} MiB" if r.operator_maxrss_mib else
                     f", process peak RSS {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024:.0f} MiB, "
                     f"start: caches synced {r.startup_sync_s:.2f} s, first pass {r.startup_first_pass_s:.2f} s"),
                  flush=True)
    print()
    print("| mode | Crons | cron-reconciles/s | p50 tick→create ms | p99 ms | ms/tick | API req/fire "
          "| reconciles/fire |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|")
    for x in rows:
        print(f"| {x['mode']} | {x['n_crons']} | {x['cron_reconciles_per_s']:.1f} | {x['p50_ms']:.1f} | "
              f"{x['p99_ms']:.1f} | {x['ms_per_step']:.0f} | {x['api_requests_per_fire']:.1f} | "
              f"{x['reconciles_per_fire']:.1f} |")
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"transport": a.transport, "steps": a.steps, "warmup": a.warmup, "rows": rows}, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
