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


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fires", type=int, default=200)
    ap.add_argument("--top", type=int, default=0, help="also list the functions executing the most bytecodes")
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
