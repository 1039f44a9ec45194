"""Serve the fake :class:`APIServer` over the Kubernetes REST protocol (aiohttp).

Paths follow kube-apiserver: ``/api/v1/...`` for the core group and
``/apis/<group>/<version>/...`` otherwise, with ``namespaces/<ns>/`` scoping,
``/<name>/<subresource>``, discovery (``/api``, ``/apis``, ``/api/v1``,
``/apis/<g>/<v>``), ``/version`` and ``/healthz``.  LIST/WATCH take
``labelSelector``, ``fieldSelector``, ``resourceVersion``, ``limit``,
``continue``, ``allowWatchBookmarks`` and ``timeoutSeconds``; watches stream
newline-delimited JSON events.  PATCH honours the content type
(merge / json / strategic); DELETE reads ``DeleteOptions`` from the body or
``propagationPolicy`` from the query.  Errors are ``metav1.Status`` bodies.

Optional bearer-token authentication (``tokens``) mirrors what the metrics
authn/authz filter needs.  ``/debug/fake/*`` endpoints expose test controls
(clock, request stats, faults, bulk job completion) to out-of-process drivers
such as the benchmark.
"""
from __future__ import annotations

import asyncio
import json
import time
from typing import Any, Dict, List, Optional, Tuple

from aiohttp import web

from ..api import errors
from ..api.meta import GroupVersionResource
from ..utils import jsonutil
from ..utils.clock import FakeClock
from .server import APIServer

PATCH_TYPES = {
    "application/merge-patch+json": "merge",
    "application/json-patch+json": "json",
    "application/strategic-merge-patch+json": "strategic",
    "application/apply-patch+yaml": "apply",
}


class _EncodeCache:
    """Serialised bytes of stored objects.  A write's response and its watch events
    carry the same (immutable) stored object, so it is encoded once."""

    def __init__(self, size: int = 8192):
        self._d: Dict[int, Tuple[Any, bytes]] = {}
        self._size = size

    def encode(self, obj: Any) -> bytes:
        hit = self._d.get(id(obj))
        if hit is not None and hit[0] is obj:
            return hit[1]
        b = jsonutil.dumpb(obj)
        if len(self._d) >= self._size:
            self._d.clear()
        self._d[id(obj)] = (obj, b)
        return b


_ENC = _EncodeCache()


def _json(data: Any, status: int = 200) -> web.Response:
    return web.Response(body=_ENC.encode(data) if status < 300 else jsonutil.dumpb(data), status=status,
                        content_type="application/json")


def _event_line(etype: str, obj: Any) -> bytes:
    return b'{"type":"' + etype.encode() + b'","object":' + _ENC.encode(obj) + b"}"


_USER = web.RequestKey("user", dict) if hasattr(web, "RequestKey") else "user"


def _err(e: errors.ApiError) -> web.Response:
    return _json(e.status(), e.code)


class APIServerApp:
    def __init__(self, server: APIServer, request_log: bool = False):
        self.server = server
        self.request_log = request_log
        self._runner: Optional[web.AppRunner] = None
        self.port: Optional[int] = None
        self._streams: List[Any] = []

    # ------------------------------------------------------------------ discovery
    def _core_list(self) -> Dict[str, Any]:
        return {"kind": "APIResourceList", "apiVersion": "v1", "groupVersion": "v1",
                "resources": [ri.discovery_entry() for ri in self.server.resources() if ri.group == ""]}

    def _groups(self) -> Dict[str, Any]:
        groups: Dict[str, List[str]] = {}
        for ri in self.server.resources():
            if ri.group:
                vs = groups.setdefault(ri.group, [])
                if ri.version not in vs:
                    vs.append(ri.version)
        out = []
        for g, vs in sorted(groups.items()):
            versions = [{"groupVersion": f"{g}/{v}", "version": v} for v in vs]
            out.append({"name": g, "versions": versions, "preferredVersion": versions[-1]})
        return {"kind": "APIGroupList", "apiVersion": "v1", "groups": out}

    def _group_version(self, group: str, version: str) -> Optional[Dict[str, Any]]:
        res = [ri.discovery_entry() for ri in self.server.resources() if ri.group == group and ri.version == version]
        if not res:
            return None
        return {"kind": "APIResourceList", "apiVersion": "v1", "groupVersion": f"{group}/{version}",
                "resources": res}

    # ------------------------------------------------------------------ auth
    def _authenticate(self, req: web.Request) -> Optional[web.Response]:
        if self.server.tokens is None:
            return None
        auth = req.headers.get("Authorization", "")
        token = auth[7:].strip() if auth.startswith("Bearer ") else ""
        user = self.server.tokens.get(token)
        if user is None:
            return _json(errors.ApiError(401, "Unauthorized", "Unauthorized").status(), 401)
        req[_USER] = user
        return None

    def _authorize(self, req: web.Request, attrs: Dict[str, Any]) -> None:
        rbac = self.server.rbac
        user = req.get(_USER)
        if rbac is None or user is None:
            return
        if not rbac.authorize(user.get("username", ""), user.get("groups") or [], attrs):
            from .rbac import forbidden_message

            raise errors.ApiError(403, "Forbidden", forbidden_message(user.get("username", ""), attrs))

    # ------------------------------------------------------------------ routing
    @staticmethod
    def _parse(path: str) -> Optional[Tuple[GroupVersionResource, str, str, str, bool]]:
        """-> (gvr, namespace, name, subresource, namespaced_path) or None."""
        parts = [p for p in path.split("/") if p]
        if not parts:
            return None
        if parts[0] == "api":
            if len(parts) < 3:
                return None
            group, version, rest = "", parts[1], parts[2:]
        elif parts[0] == "apis":
            if len(parts) < 4:
                return None
            group, version, rest = parts[1], parts[2], parts[3:]
        else:
            return None
        ns = ""
        namespaced = False
        if rest[0] == "namespaces" and len(rest) >= 3:
            ns = rest[1]
            rest = rest[2:]
            namespaced = True
        resource = rest[0]
        name = rest[1] if len(rest) > 1 else ""
        sub = rest[2] if len(rest) > 2 else ""
        if len(rest) > 3:
            return None
        return GroupVersionResource(group, version, resource), ns, name, sub, namespaced

    async def handle(self, req: web.Request) -> web.StreamResponse:
        denied = self._authenticate(req)
        if denied is not None:
            return denied
        path = req.path
        if path in ("/healthz", "/readyz", "/livez"):
            return web.Response(text="ok")
        if path == "/version":
            return _json({"major": "1", "minor": "34", "gitVersion": "v1.34.0-cron-operator-amd-fake",
                          "platform": "linux/amd64"})
        if path == "/api":
            return _json({"kind": "APIVersions", "versions": ["v1"]})
        if path == "/api/v1":
            return _json(self._core_list())
        if path == "/apis":
            return _json(self._groups())
        if path.startswith("/debug/fake/"):
            return await self._debug(req)
        if self.server.rbac is not None and req.get(_USER) is not None and not path.startswith(("/api/", "/apis/")):
            try:
                self._authorize(req, {"verb": req.method.lower(), "path": path})
            except errors.ApiError as e:
                return _err(e)
        parts = [p for p in path.split("/") if p]
        if len(parts) == 3 and parts[0] == "apis":
            gv = self._group_version(parts[1], parts[2])
            if gv is None:
                return _err(errors.ApiError(404, "NotFound", "the server could not find the requested resource"))
            return _json(gv)
        parsed = self._parse(path)
        if parsed is None:
            return _err(errors.ApiError(404, "NotFound", "the server could not find the requested resource"))
        gvr, ns, name, sub, _ = parsed
        try:
            return await self._resource(req, gvr, ns, name, sub)
        except errors.ApiError as e:
            return _err(e)
        except (ValueError, KeyError, TypeError) as e:
            return _err(errors.bad_request(str(e)))

    async def _body(self, req: web.Request) -> Any:
        raw = await req.read()
        if not raw:
            return None
        try:
            return json.loads(raw)
        except ValueError as e:
            raise errors.bad_request(f"invalid JSON body: {e}") from None

    async def _delay(self, verb: str) -> None:
        d = self.server.faults.delay_for(verb) if self.server.faults.latency else 0.0
        if d > 0:
            await asyncio.sleep(d)

    async def _resource(self, req: web.Request, gvr: GroupVersionResource, ns: str, name: str,
                        sub: str) -> web.StreamResponse:
        s = self.server
        q = req.query
        m = req.method
        ri = s.resource(gvr)
        if not ri.namespaced and ns:
            raise errors.ApiError(404, "NotFound", "the server could not find the requested resource")
        verb = {"GET": "get" if name else ("watch" if q.get("watch") in ("true", "1") else "list"),
                "POST": "create", "PUT": "update", "PATCH": "patch",
                "DELETE": "delete" if name else "deletecollection"}.get(m)
        if verb is None:
            raise errors.ApiError(405, "MethodNotAllowed", f"method {m} not allowed")
        if s.rbac is not None:
            self._authorize(req, {"verb": verb, "group": gvr.group, "resource": gvr.resource, "subresource": sub,
                                  "namespace": ns, "name": name})
        await self._delay(verb)
        if s.faults.faults:
            s.faults.check(verb, gvr.resource, sub or None, name or None)
        if verb == "watch":
            return await self._watch(req, gvr, ns)
        body: Any = None
        ptype = "merge"
        if verb in ("create", "update", "patch", "delete"):
            if verb == "patch":
                ptype = PATCH_TYPES.get(req.content_type)
                if ptype is None or ptype == "apply":
                    accepted = ", ".join(k for k in PATCH_TYPES if k != "application/apply-patch+yaml")
                    raise errors.ApiError(415, "UnsupportedMediaType", "the body of the request was in an unknown "
                                                                       f"format - accepted media types include: "
                                                                       f"{accepted}")
            body = await self._body(req)
            if verb in ("create", "update") and not isinstance(body, dict):
                raise errors.bad_request("request body must be a JSON object")
        # The verb runs synchronously and its result is serialised right here, so the
        # stored object can be returned without a defensive copy.
        s.copy_responses = False
        try:
            resp = self._apply(verb, gvr, ns, name, sub, body, ptype, q)
        finally:
            s.copy_responses = True
        if s.faults.faults:  # "lost response" faults fire after the verb was applied
            s.faults.check(verb, gvr.resource, sub or None, name or None, after=True)
        return resp

    def _apply(self, verb: str, gvr: GroupVersionResource, ns: str, name: str, sub: str, body: Any, ptype: Any,
               q: Any) -> web.Response:
        s = self.server
        if verb == "list":
            return _json(s.list(gvr, ns or None, q.get("labelSelector"), q.get("fieldSelector"),
                                int(q.get("limit") or 0), q.get("continue"), copy=False))
        if verb == "get":
            return _json(s.get(gvr, ns, name))
        if verb == "create":
            return _json(s.create(gvr, ns, body, dry_run=q.get("dryRun") == "All"), 201)
        if verb == "update":
            return _json(s.update(gvr, ns, name, body, sub or None))
        if verb == "patch":
            return _json(s.patch(gvr, ns, name, body, ptype, sub or None))
        if verb == "delete":
            opts = body or {}
            policy = opts.get("propagationPolicy") or q.get("propagationPolicy")
            return _json(s.delete(gvr, ns, name, policy, opts.get("preconditions")))
        n = s.delete_collection(gvr, ns or None, q.get("labelSelector"))
        return _json({"kind": "Status", "apiVersion": "v1", "status": "Success", "details": {"deleted": n}})

    async def _watch(self, req: web.Request, gvr: GroupVersionResource, ns: str) -> web.StreamResponse:
        q = req.query
        w = self.server.watch(gvr, ns or None, q.get("resourceVersion", ""), q.get("labelSelector"),
                              q.get("fieldSelector"), q.get("allowWatchBookmarks") in ("true", "1"),
                              copy_events=False)
        resp = web.StreamResponse(status=200, headers={"Content-Type": "application/json",
                                                       "Transfer-Encoding": "chunked"})
        await resp.prepare(req)
        timeout = float(q.get("timeoutSeconds") or 1800)
        deadline = time.monotonic() + timeout
        self._streams.append(w)
        try:
            while True:
                remaining = deadline - time.monotonic()
                if remaining <= 0:
                    break
                try:
                    ev = await asyncio.wait_for(w.queue.get(), remaining)
                except asyncio.TimeoutError:
                    break
                if ev is None:
                    break
                buf = [_event_line(ev[0], ev[1])]
                # coalesce whatever is already queued into one write
                while not w.queue.empty() and len(buf) < 512:
                    nxt = w.queue.get_nowait()
                    if nxt is None:
                        w.closed = True
                        break
                    buf.append(_event_line(nxt[0], nxt[1]))
                await resp.write(b"\n".join(buf) + b"\n")
                if w.closed:
                    break
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            w.stop()
            if w in self._streams:
                self._streams.remove(w)
        return resp

    # ------------------------------------------------------------------ debug / test controls
    async def _debug(self, req: web.Request) -> web.Response:
        s = self.server
        what = req.path[len("/debug/fake/"):]
        if what == "stats":
            snap = s.stats.snapshot()
            snap["resourceVersion"] = s.current_rv()
            return _json(snap)
        if what == "clock":
            if req.method == "POST":
                body = await self._body(req) or {}
                if not isinstance(s.clock, FakeClock):
                    raise errors.bad_request("server clock is not settable")
                s.clock.set(int(body["nowNs"]))
            return _json({"nowNs": s.clock.now_ns()})
        if what == "faults" and req.method == "POST":
            body = await self._body(req) or {}
            if body.get("clear"):
                s.faults.clear()
            for f in body.get("faults") or []:
                s.faults.add(**f)
            for verb, lat in (body.get("latency") or {}).items():
                s.faults.latency[verb] = float(lat)
            return _json({"faults": len(s.faults.faults)})
        if what == "complete" and req.method == "POST":
            # bench helper: mark every job (of the given resource) without completionTime as finished
            body = await self._body(req) or {}
            from ..trainingop.operator import finished_status

            gvr = GroupVersionResource(body.get("group", "kubeflow.org"), body.get("version", "v1"),
                                       body.get("resource", "pytorchjobs"))
            ts = body.get("time") or ""
            n = 0
            for obj in list(s.objects(gvr, body.get("namespace"))):
                st = obj.get("status") or {}
                if st.get("completionTime"):
                    continue
                m = obj["metadata"]
                s.patch(gvr, m["namespace"], m["name"],
                        {"status": finished_status(obj.get("kind", ""), m["name"], ts, True)}, "merge", "status")
                n += 1
            return _json({"completed": n})
        if what == "count":
            gvr = GroupVersionResource(req.query.get("group", ""), req.query.get("version", "v1"),
                                       req.query["resource"])
            return _json({"count": s.count(gvr, req.query.get("namespace"))})
        return _err(errors.ApiError(404, "NotFound", f"unknown debug endpoint {what}"))

    # ------------------------------------------------------------------ lifecycle
    def app(self) -> web.Application:
        app = web.Application(client_max_size=64 * 1024 * 1024)
        app.router.add_route("*", "/{tail:.*}", self.handle)
        return app

    async def start(self, host: str = "127.0.0.1", port: int = 0, ssl_context=None) -> int:
        self._runner = web.AppRunner(self.app(), access_log=None, handle_signals=False)
        await self._runner.setup()
        site = web.TCPSite(self._runner, host, port, ssl_context=ssl_context, backlog=1024)
        await site.start()
        server = getattr(site, "_server", None)
        self.port = server.sockets[0].getsockname()[1] if server is not None else port
        return self.port

    async def stop(self) -> None:
        for w in list(self._streams):
            w.stop()
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None
