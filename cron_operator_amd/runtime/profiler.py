"""In-process diagnostics of a running operator, served on the probe port.

The reference exposes none (pprof is only an indirect dependency); a Go operator
would reach for ``net/http/pprof``'s goroutine dump and CPU profile.  This process runs its
reconcilers, informers and clients as asyncio tasks on one loop, so the two equivalents are:

* ``GET /debug/tasks`` -- every live task grouped by where it is suspended (the innermost
  frame of its await chain outside asyncio itself), the analogue of ``/debug/pprof/goroutine?debug=1``:
  thousands of tasks parked on one line name the queue a stalled operator is waiting in.
  ``?stacks=1`` adds one sample await chain per location.  Always on: it only reads.
* ``GET /debug/profile?seconds=N`` -- a statistical CPU profile of the event-loop thread over
  N seconds (a ``SIGPROF`` interval timer on process CPU time records the interrupted Python
  stack; no per-call hook, so the loop runs at nearly full speed), ranked by self and inclusive
  samples per function and by line.  Opt-in (``cron-operator start --enable-profiling``), one
  at a time, and only where the loop runs on the main thread (signal handlers run there).
"""
from __future__ import annotations

import asyncio
import collections
import math
import os
import signal
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))) + os.sep
MAX_SECONDS = 120.0

_allowed = False
_running: Optional["Sampler"] = None


def allow(on: bool = True) -> None:
    """Serve ``/debug/profile`` (``--enable-profiling``)."""
    global _allowed
    _allowed = on


def allowed() -> bool:
    return _allowed


def _where(code: Any, lineno: int) -> str:
    fn = code.co_filename
    if fn.startswith(_PKG_ROOT):
        fn = fn[len(_PKG_ROOT):]
    return f"{fn}:{lineno}({code.co_name})"


class Sampler:
    """Statistical profiler of the main thread: every ``interval`` seconds of process CPU the
    kernel sends ``SIGPROF`` and the handler (run by the interpreter between bytecodes) counts
    the interrupted stack -- self samples for the innermost Python frame, inclusive samples for
    every function on it.  A C function's time is charged to its Python caller."""

    def __init__(self, interval: float = 0.001):
        self.interval = interval
        self.self_counts: "collections.Counter[str]" = collections.Counter()
        self.incl_counts: "collections.Counter[str]" = collections.Counter()
        self.line_counts: "collections.Counter[str]" = collections.Counter()
        self.samples = 0
        self.cpu_s = 0.0
        self._c0 = 0.0
        self._prev: Any = None

    def _on(self, signum: int, frame: Any) -> None:
        self.samples += 1
        first = True
        seen = set()
        while frame is not None:
            co = frame.f_code
            key = _where(co, co.co_firstlineno)
            if first:
                self.self_counts[key] += 1
                self.line_counts[f"{key} line {frame.f_lineno}"] += 1
                first = False
            if key not in seen:
                seen.add(key)
                self.incl_counts[key] += 1
            frame = frame.f_back

    def enable(self) -> None:
        if threading.current_thread() is not threading.main_thread():
            raise RuntimeError("the CPU profiler needs the event loop on the main thread")
        self._c0 = time.process_time()
        self._prev = signal.signal(signal.SIGPROF, self._on)
        signal.setitimer(signal.ITIMER_PROF, self.interval, self.interval)

    def disable(self) -> None:
        signal.setitimer(signal.ITIMER_PROF, 0, 0)
        signal.signal(signal.SIGPROF, self._prev if self._prev is not None else signal.SIG_DFL)
        self.cpu_s += time.process_time() - self._c0

    def report(self, top: int = 40, wall_s: Optional[float] = None) -> str:
        n = max(1, self.samples)
        # the kernel delivers SIGPROF at its tick and Python runs the handler between bytecodes,
        # so the real rate is lower than requested: report what was collected
        head = f"# {self.samples} samples over {self.cpu_s:.2f} s of process CPU"
        if wall_s is not None:
            head += f" in {wall_s:.1f} s of wall time ({100.0 * self.cpu_s / max(wall_s, 1e-9):.1f}% of one core)"
        out = [head + f"; requested every {self.interval * 1e3:.1f} ms of CPU; a C function's time is "
                      "charged to its Python caller\n", "\n## by self samples\n"]
        for k, c in self.self_counts.most_common(top):
            out.append(f"{100.0 * c / n:6.2f}%  {k}\n")
        out.append("\n## by self samples, per source line\n")
        for k, c in self.line_counts.most_common(top):
            out.append(f"{100.0 * c / n:6.2f}%  {k}\n")
        out.append("\n## by inclusive samples\n")
        for k, c in self.incl_counts.most_common(top):
            out.append(f"{100.0 * c / n:6.2f}%  {k}\n")
        return "".join(out)


async def cpu_profile(seconds: float, interval: float = 0.001, top: int = 40) -> str:
    """Profile this process's loop thread for ``seconds`` (at most :data:`MAX_SECONDS`) and
    return the text report.  Raises ``RuntimeError`` when a profile is already running or the
    loop is not on the main thread."""
    global _running
    if _running is not None:
        raise RuntimeError("a profile is already running")
    if not math.isfinite(seconds):
        raise ValueError(f"seconds must be finite, not {seconds!r}")
    seconds = min(max(seconds, 0.1), MAX_SECONDS)
    s = Sampler(interval)
    s.enable()
    _running = s
    t0 = time.perf_counter()
    try:
        await asyncio.sleep(seconds)
    finally:
        s.disable()
        _running = None
    return s.report(top, wall_s=time.perf_counter() - t0)


def _await_chain(task: "asyncio.Task[Any]") -> List[Tuple[Any, int]]:
    """(code, line) of every coroutine frame from the task's coroutine down the ``await`` chain
    to the innermost suspended one (``Task.get_stack`` stops at the outermost)."""
    out: List[Tuple[Any, int]] = []
    c: Any = task.get_coro()
    for _ in range(64):
        frame = getattr(c, "cr_frame", None) or getattr(c, "gi_frame", None) or getattr(c, "ag_frame", None)
        if frame is None:
            break
        out.append((frame.f_code, frame.f_lineno))
        c = getattr(c, "cr_await", None) or getattr(c, "gi_yieldfrom", None) or getattr(c, "ag_await", None)
        if c is None:
            break
    return out


_ASYNCIO_DIR = os.path.dirname(asyncio.__file__) + os.sep


def _suspended_at(chain: List[Tuple[Any, int]]) -> str:
    """The innermost frame of the chain that is not asyncio's own (``Event.wait``,
    ``Queue.get``, ``sleep``): the line of this program that is waiting."""
    for co, ln in reversed(chain):
        if not co.co_filename.startswith(_ASYNCIO_DIR):
            return _where(co, ln)
    return _where(*chain[-1])


def task_dump(stacks: bool = False, top: int = 50, loop: Optional[asyncio.AbstractEventLoop] = None) -> Dict[str, Any]:
    """Live tasks of the loop grouped by where they are suspended: the innermost frame of their
    await chain outside asyncio itself."""
    tasks = asyncio.all_tasks(loop)
    groups: "collections.Counter[str]" = collections.Counter()
    sample: Dict[str, List[str]] = {}
    for t in tasks:
        chain = _await_chain(t)
        where = _suspended_at(chain) if chain else "<running or not started>"
        groups[where] += 1
        if stacks and where not in sample:
            sample[where] = [_where(co, ln) for co, ln in chain]
    out: Dict[str, Any] = {"tasks": len(tasks), "locations": len(groups),
                           "by_location": [{"where": w, "tasks": n, **({"await_chain": sample[w]} if stacks else {})}
                                           for w, n in groups.most_common(top)]}
    return out
