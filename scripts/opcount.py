#!/usr/bin/env python3
"""Deterministic cost proxy for the reconcile microbench: Python bytecodes executed and
C functions called per fire (sys.settrace with opcode events), for comparing hot-path
changes on a machine too noisy for wall/CPU timing.

    python scripts/opcount.py [--fires 200]
"""
from __future__ import annotations

import argparse
import asyncio
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def lifecycle_kw(a) -> dict:
    """``lifecycle`` for BenchConfig when this tree's harness has the field (older trees: none)."""
    from cron_operator_amd.bench import harness

    return {"lifecycle": a.lifecycle} if "lifecycle" in harness.BenchConfig.__dataclass_fields__ else {}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fires", type=int, default=200)
    ap.add_argument("--top", type=int, default=0, help="also list the functions executing the most bytecodes")
    ap.add_argument("--bench", type=int, default=0, metavar="CRONS",
                    help="count the whole operator process of the headline bench instead (one process, CRONS "
                         "Crons, 3 timed steps; the fake apiserver's own process is not counted)")
    ap.add_argument("--lifecycle", default="instant", choices=["instant", "realistic"],
                    help="--bench: the jobs' status sequence (the headline's is instant)")
    a = ap.parse_args()
    import cProfile

    import reconcile_microbench as rm

    import collections

    counts = {"op": 0, "ccall": 0}
    by_code: "collections.Counter[object]" = collections.Counter()

    def tracer(frame, event, arg):
        frame.f_trace_opcodes = True
        if event == "opcode":
            counts["op"] += 1
            by_code[frame.f_code] += 1
        return tracer

    def prof(frame, event, arg):
        if event == "c_call":
            counts["ccall"] += 1

    class P:  # the microbench's profiler hook, reused as the measurement window
        def enable(self):
            sys.settrace(tracer)
            sys.setprofile(prof)
            # settrace only applies to frames entered from now on: count the running ones too
            f = sys._getframe(1)
            while f is not None:
                f.f_trace = tracer
                f.f_trace_opcodes = True
                f = f.f_back

        def disable(self):
            sys.settrace(None)
            sys.setprofile(None)

    if a.bench:
        from cron_operator_amd.bench import harness

        steps, warmup = 3, 2
        win = P()

        def on_step(k: int, dt: float, timed: bool) -> None:
            if k == warmup:
                win.enable()
            elif k == warmup + steps:
                win.disable()

        harness.run_sync(harness.BenchConfig(n_crons=a.bench, steps=steps, warmup=warmup, history_limit=10,
                                             transport="http", shards=1, **lifecycle_kw(a)), on_step=on_step)
        fires = a.bench * steps
        print(f"per fire: {counts['op'] / fires:.0f} bytecodes, {counts['ccall'] / fires:.0f} C calls", flush=True)
        for co, n in by_code.most_common(a.top):
            fn = co.co_filename.replace(ROOT + "/", "")
            print(f"{n / fires:8.0f}  {fn}:{co.co_firstlineno}({co.co_name})")
        by_file: "collections.Counter[str]" = collections.Counter()
        for co, n in by_code.items():
            by_file[co.co_filename.replace(ROOT + "/", "")] += n
        print("\n## by source file (share of all bytecodes)")
        for fn, n in by_file.most_common(a.top and 25):
            print(f"{n / fires:8.0f}  {100.0 * n / max(1, counts['op']):5.1f}%  {fn}")
        return 0

    cProfile.Profile = P  # type: ignore[misc]

    import pstats

    class _S:
        def __init__(self, *a, **k):
            pass

        def sort_stats(self, *a):
            return self

        def print_stats(self, *a):
            pass

    pstats.Stats = _S  # type: ignore[misc]
    asyncio.run(rm.run(a.fires, os.devnull))
    print(f"per fire: {counts['op'] / a.fires:.0f} bytecodes, {counts['ccall'] / a.fires:.0f} C calls", flush=True)
    for co, n in by_code.most_common(a.top):
        fn = co.co_filename.replace(ROOT + "/", "")
        print(f"{n / a.fires:8.0f}  {fn}:{co.co_firstlineno}({co.co_name})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
