"""The fake apiserver's native implementation (``ops/csrc/apiserverd.cpp``) and its test controls.

:class:`~.server.APIServer` + :mod:`.http` is the envtest analog the test suite drives in
process.  In the benchmark it runs in a process of its own and used to be the bottleneck: one
Python core answering ~20,000 requests a second sat 86-94% busy, so the headline measured the
fixture (round-5 verdict #1).  ``_apiserverd`` serves the same REST contract from a C++ store on
one epoll thread -- merge-patch and ``/status`` semantics, resourceVersions, label-selected LIST
and WATCH (resume, synthetic ADDED, scope transitions), CRD structural-schema admission, the
per-verb latency model, TLS -- without the GIL.

What it does not serve natively comes here, to :class:`NativeAPIServer.fallback` on the server
thread: the ``/debug/fake/*`` test controls the bench drives (clock, latency faults, bulk job
completion and lifecycle writes, request stats, counts).  Server-side Table printing and JSON
patch answer 501 -- use :mod:`.http` for those, as for authn/RBAC and ownerReference GC.

``tests/test_apiserverd.py`` replays one request stream against both implementations and
compares the answers.
"""
from __future__ import annotations

import json
from typing import Any, Dict, Optional, Tuple
from urllib.parse import parse_qsl

from ..ops import build as _build
from ..utils import jsonutil


def load():
    """The ``_apiserverd`` module, building it if its source is newer (None if it cannot load)."""
    try:
        if _build.needs_build("_apiserverd"):
            _build.build_extension("_apiserverd")
        from ..ops import _apiserverd  # type: ignore[attr-defined]

        return _apiserverd
    except Exception:  # noqa: BLE001 - a missing toolchain leaves the Python server
        return None


PYTORCHJOBS = ("kubeflow.org", "v1", "pytorchjobs")
_NAME = "@@name@@"  # stands for each job's name in a bulk status body (never a valid object name)
_KINDS = {"pytorchjobs": "PyTorchJob", "tfjobs": "TFJob", "mpijobs": "MPIJob"}


def _status_body(code: int, reason: str, message: str) -> bytes:
    return json.dumps({"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
                       "message": message, "reason": reason, "code": code}).encode()


def profile_report(stacks, dropped: int = 0, top: int = 40) -> str:
    """Rank the sampled stacks' functions (addr2line resolves the frames; frames outside a file
    addr2line can read keep their module's name)."""
    import collections
    import os
    import subprocess

    names: Dict[Tuple[str, int], str] = {}
    by_mod: Dict[str, set] = collections.defaultdict(set)
    for st in stacks:
        for mod, off in st:
            by_mod[mod].add(off)
    for mod, offs in by_mod.items():
        offs = sorted(offs)
        resolved = ["?"] * len(offs)
        if os.path.exists(mod):
            try:
                out = subprocess.run(["addr2line", "-f", "-C", "-e", mod] + [hex(o) for o in offs],
                                     capture_output=True, text=True, timeout=60).stdout.splitlines()
                resolved = [out[2 * i] if 2 * i < len(out) else "?" for i in range(len(offs))]
            except (OSError, subprocess.SubprocessError):
                pass
        base = os.path.basename(mod)
        for o, fn in zip(offs, resolved):
            names[(mod, o)] = f"{fn} [{base}]" if fn != "??" else f"?? [{base}+{o:#x}]"
    # samples of the server thread waiting in epoll_wait: idle time, not CPU
    idle = sum(1 for st in stacks if st and "epoll_wait" in names[st[0]])
    stacks = [st for st in stacks if st and "epoll_wait" not in names[st[0]]]
    self_c: collections.Counter = collections.Counter()
    incl_c: collections.Counter = collections.Counter()
    for st in stacks:
        if not st:
            continue
        self_c[names[st[0]]] += 1
        for f in {names[x] for x in st}:
            incl_c[f] += 1
    # which of the server's own functions the time outside it (malloc, memcpy, syscalls) is spent for
    via: collections.Counter = collections.Counter()
    for st in stacks:
        if not st or "_apiserverd" in names[st[0]]:
            continue
        own = next((names[x] for x in st if "_apiserverd" in names[x]), None)
        if own is not None:
            via[f"{names[st[0]]}  <-  {own}"] += 1
    n = max(1, len(stacks))
    out = [f"# {len(stacks)} busy samples of the fake apiserver's server thread ({idle} more idle in "
           f"epoll_wait, {dropped} dropped)\n",
           "\n## by self samples\n"]
    out += [f"{100.0 * c / n:6.2f}%  {k}\n" for k, c in self_c.most_common(top)]
    out.append("\n## by inclusive samples\n")
    out += [f"{100.0 * c / n:6.2f}%  {k}\n" for k, c in incl_c.most_common(top)]
    out.append("\n## time outside the extension, by the extension function it ran for\n")
    out += [f"{100.0 * c / n:6.2f}%  {k}\n" for k, c in via.most_common(top)]
    return "".join(out)


class NativeAPIServer:
    """A ``_apiserverd.Server`` with the CRDs installed and the ``/debug/fake`` controls."""

    def __init__(self, start_ns: int = 0, watch_window: int = 200_000, bookmark_interval: float = 60.0):
        mod = load()
        if mod is None:
            raise RuntimeError("the native fake apiserver (_apiserverd) did not build or load")
        self.srv = mod.Server(now_ns=start_ns, watch_window=watch_window, bookmark_interval=bookmark_interval)
        self.srv.set_fallback(self.fallback)
        self._faults = 0
        self._serving = False

    # ------------------------------------------------------------------ setup
    def install_crd(self, crd: Dict[str, Any]) -> None:
        st, body = self.srv.request("POST", "/apis/apiextensions.k8s.io/v1/customresourcedefinitions",
                                    body=jsonutil.dumpb(crd), content_type="application/json")
        if st not in (200, 201):
            raise RuntimeError(f"installing CRD {crd.get('metadata', {}).get('name')}: {st} {body[:300]!r}")

    def start(self, host: str = "127.0.0.1", port: int = 0, certfile: str = "", keyfile: str = "") -> int:
        port = self.srv.start(host, port, certfile, keyfile)
        self._serving = True
        return port

    def stop(self) -> None:
        self.srv.stop()
        self._serving = False

    def _kind_of(self, group: str, version: str, resource: str) -> str:
        st, raw = self.srv.request("GET", f"/apis/{group}/{version}" if group else f"/api/{version}")
        for e in (jsonutil.loads(raw).get("resources") or []) if st == 200 else []:
            if e.get("name") == resource:
                return e.get("kind", "")
        raise KeyError(f"unknown resource {group}/{version}/{resource}")

    # ------------------------------------------------------------------ /debug/fake
    def fallback(self, method: str, path: str, query: str, headers: Dict[str, str],
                 body: bytes) -> Optional[Tuple[Any, ...]]:
        if not path.startswith("/debug/fake/"):
            if path.startswith(("/api/", "/apis/")):
                return 501, _status_body(501, "NotImplemented", "not served by the native fake apiserver "
                                                                "(server-side Table, JSON patch): use --impl python")
            return None
        try:
            out = self._debug(method, path[len("/debug/fake/"):], dict(parse_qsl(query)), body)
        except Exception as e:  # noqa: BLE001 - a broken control answers 500, never kills the server
            return 500, _status_body(500, "InternalError", f"{type(e).__name__}: {e}")
        if out is None:
            return 404, _status_body(404, "NotFound", f"unknown debug endpoint {path}")
        if isinstance(out, tuple):
            return out
        return 200, jsonutil.dumpb(out)

    def _debug(self, method: str, what: str, q: Dict[str, str], raw: bytes) -> Any:
        srv = self.srv
        body = jsonutil.loads(raw) if raw else {}
        if what == "stats":
            st = srv.stats()
            return {"total": st["total"], "by_verb": st["by_verb"], "by_resource_verb": st["by_resource_verb"],
                    "resourceVersion": st["resourceVersion"], "native": True,
                    "server_thread_cpu_s": st["server_thread_cpu_s"], "verb_cpu": st["verb_cpu"],
                    "phase_cycles": st["phase_cycles"], "io": st["io"]}
        if what == "clock":
            if method == "POST":
                srv.set_clock(int(body["nowNs"]))
            return {"nowNs": srv.now_ns()}
        if what == "faults" and method == "POST":
            if body.get("clear"):
                srv.clear_latency()
                self._faults = 0
            if body.get("faults") or body.get("watchLag"):
                return 501, _status_body(501, "NotImplemented", "error faults and watch lag are injected by the "
                                                                "Python fake apiserver (--impl python); the "
                                                                "native one models latency only")
            lat = {str(k): float(v) for k, v in (body.get("latency") or {}).items()}
            if lat:
                srv.set_latency(lat)
            return {"faults": self._faults}
        if what == "complete" and method == "POST":
            from ..trainingop.operator import finished_status

            g, v, r = body.get("group", PYTORCHJOBS[0]), body.get("version", PYTORCHJOBS[1]), \
                body.get("resource", PYTORCHJOBS[2])
            ts = body.get("time") or ""
            # one body for every job of the kind, the name filled in natively per job
            kind = _KINDS.get(r) or self._kind_of(g, v, r)
            tmpl = jsonutil.dumpb({"status": finished_status(kind, _NAME, ts, True)})
            # perTurn > 0: queued, the server applies that many per loop turn between the turns
            # serving the other clients (the response comes back before they are all applied)
            per_turn = int(body.get("perTurn") or 0)
            n = srv.patch_unfinished(g, v, r, body.get("namespace") or "", tmpl, _NAME, "status", per_turn)
            return {"completed": n, "queued": per_turn > 0 and self._serving}
        if what == "lifecycle" and method == "POST":
            from ..trainingop.operator import lifecycle_status, replica_counts

            g, v, r = body.get("group", PYTORCHJOBS[0]), body.get("version", PYTORCHJOBS[1]), \
                body.get("resource", PYTORCHJOBS[2])
            ns = body.get("namespace") or ""
            stage = int(body.get("stage", -1))
            start, end = body.get("start") or "", body.get("end") or ""
            items, keys = [], []
            reps_memo: Dict[bytes, Any] = {}
            for name, kind, enc in srv.unfinished(g, v, r, ns):
                obj = jsonutil.loads(enc)
                spec_key = jsonutil.dumpb(obj.get("spec") or {})
                reps = reps_memo.get(spec_key)
                if reps is None:
                    reps = reps_memo[spec_key] = replica_counts(obj)
                items.append((name, jsonutil.dumpb({"status": lifecycle_status(obj, stage, start, end, reps)})))
                keys.append(f"{(obj.get('metadata') or {}).get('namespace', ns)}/{name}")
            rvs = srv.patch_many(g, v, r, ns, items, "status")
            return {"resourceVersions": {k: rv for k, rv in zip(keys, rvs) if rv is not None}}
        if what == "profile" and method == "POST":
            # a SIGPROF stack sampler inside the extension (the boxes have no perf): start, then
            # stop with a path -- the report ranks functions by self and inclusive samples
            if body.get("action") == "start":
                srv.profile_start(float(body.get("interval", 0.0005)))
                return {"profiling": True, "native": True}
            stacks, dropped = srv.profile_stop()
            report = profile_report(stacks, dropped)
            if body.get("path"):
                with open(body["path"], "w") as fh:
                    fh.write(report)
            return {"profiling": False, "native": True, "samples": len(stacks), "path": body.get("path", "")}
        if what == "gc" and method == "POST":
            from ..utils import gctune

            gctune.tune()
            gctune.freeze()
            return {"frozen": True}
        if what == "count":
            return {"count": srv.count(q.get("group", ""), q.get("version", "v1"), q["resource"],
                                       q.get("namespace"))}
        if what == "watch-log":  # events kept per resource for watch resume (the soak's memory bound)
            return {"log": srv.log_sizes(), "watchers": srv.watchers()}
        return None
