#!/usr/bin/env python3
"""Host-side profile of the operator process during the headline bench.

The operator is CPU control plane, so its "kernel trace" is a cProfile of the
reconcile hot path (the fake apiserver runs in its own process and is not
included).  Writes the top functions by self time and by cumulative time.
"""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Sampler:
    """Statistical profiler of the main thread: a SIGPROF timer (process CPU time) records
    the interrupted Python stack; ``report`` ranks functions by self and inclusive samples."""

    def __init__(self, interval: float = 0.0005):
        import collections
        import signal

        self.interval = interval
        self.self_counts: "collections.Counter[str]" = collections.Counter()
        self.incl_counts: "collections.Counter[str]" = collections.Counter()
        self.samples = 0
        self.cpu_s = 0.0
        self._signal = signal
        self.line_counts: "collections.Counter[str]" = collections.Counter()

    def _on(self, signum, frame) -> None:
        self.samples += 1
        seen = set()
        first = True
        while frame is not None:
            co = frame.f_code
            key = f"{co.co_filename.replace(ROOT + '/', '')}:{co.co_firstlineno}({co.co_name})"
            if first:
                self.self_counts[key] += 1
                self.line_counts[f"{key} line {frame.f_lineno}"] += 1
                first = False
            if key not in seen:
                seen.add(key)
                self.incl_counts[key] += 1
            frame = frame.f_back

    def enable(self) -> None:
        self._c0 = time.process_time()
        self._signal.signal(self._signal.SIGPROF, self._on)
        self._signal.setitimer(self._signal.ITIMER_PROF, self.interval, self.interval)

    def disable(self) -> None:
        self._signal.setitimer(self._signal.ITIMER_PROF, 0, 0)
        self.cpu_s += time.process_time() - self._c0

    def report(self, top: int) -> str:
        n = max(1, self.samples)
        # the kernel delivers SIGPROF at its tick (often 4 ms) and Python runs the handler between
        # bytecodes, so the real rate is lower than requested: report what was collected
        out = [f"# {self.samples} samples over {self.cpu_s:.2f} s of process CPU (requested every "
               f"{self.interval * 1e3:.1f} ms); a C function's time is charged to its Python caller\n",
               "\n## by self samples\n"]
        for k, c in self.self_counts.most_common(top):
            out.append(f"{100.0 * c / n:6.2f}%  {k}\n")
        out.append("\n## by self samples, per source line (the line executing when sampled)\n")
        for k, c in self.line_counts.most_common(top):
            out.append(f"{100.0 * c / n:6.2f}%  {k}\n")
        out.append("\n## by inclusive samples\n")
        for k, c in self.incl_counts.most_common(top):
            out.append(f"{100.0 * c / n:6.2f}%  {k}\n")
        return "".join(out)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--crons", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--transport", default="http")
    ap.add_argument("--mode", default="optimized")
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--shards", type=int, default=1,
                    help="operator shard processes (then only the apiserver profile is meaningful)")
    ap.add_argument("--lifecycle", default="instant", choices=["instant", "realistic"],
                    help="the jobs' status sequence before each tick (the headline's: instant)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--sampler", action="store_true",
                    help="statistical profile (SIGPROF every 0.5 ms of CPU) instead of cProfile: no per-call "
                         "hook overhead, so coroutine-heavy code is not over-weighted")
    a = ap.parse_args()

    from cron_operator_amd.bench.harness import BenchConfig, run_sync, summarize

    api_prof = a.out + ".apiserver.pstats" if a.transport == "http" else ""
    shard_prof = a.out + ".shard" if a.shards > 1 else ""
    cfg = BenchConfig(n_crons=a.crons, steps=a.steps, warmup=a.warmup, transport=a.transport, mode=a.mode,
                      apiserver_profile=api_prof, shards=a.shards, shard_profile=shard_prof, lifecycle=a.lifecycle)
    prof = Sampler() if a.sampler else cProfile.Profile()
    t0, c0 = time.perf_counter(), time.process_time()

    def on_step(k: int, dt: float, timed: bool) -> None:
        # profile only the timed steps (setup and warmup excluded)
        if k == cfg.warmup:
            prof.enable()
        if k == cfg.warmup + cfg.steps:
            prof.disable()

    if cfg.warmup == 0:
        prof.enable()
    res = run_sync(cfg, on_step)
    prof.disable()
    wall, cpu = time.perf_counter() - t0, time.process_time() - c0
    buf = io.StringIO()
    buf.write(f"# operator-process cProfile of the {a.steps} timed steps ({a.mode}/{a.transport}, {a.crons} Crons, "
              f"{a.warmup} warmup steps excluded; profiler overhead inflates absolute times)\n")
    buf.write(f"# {summarize(res)}\n# wall {wall:.2f} s, operator CPU {cpu:.2f} s\n\n")
    if a.sampler:
        buf.write(prof.report(a.top))
    else:
        prof.dump_stats(a.out + ".operator.pstats")
        st = pstats.Stats(prof, stream=buf)
        st.sort_stats("tottime").print_stats(a.top)
        st.sort_stats("cumulative").print_stats(a.top)
    if shard_prof and os.path.exists(shard_prof + ".0.pstats"):
        buf.write("\n\n# ===== operator shard 0 process, same timed steps =====\n")
        sst = pstats.Stats(shard_prof + ".0.pstats", stream=buf)
        sst.sort_stats("tottime").print_stats(a.top)
        sst.sort_stats("cumulative").print_stats(a.top)
    if api_prof and os.path.exists(api_prof):
        buf.write("\n\n# ===== fake apiserver process, same timed steps =====\n")
        try:
            ast = pstats.Stats(api_prof, stream=buf)
            ast.sort_stats("tottime").print_stats(a.top)
        except ValueError:  # the native fake apiserver's sampler writes a text report
            with open(api_prof) as fh:
                buf.write(fh.read())
    with open(a.out, "w") as fh:
        fh.write(buf.getvalue())
    print(summarize(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
