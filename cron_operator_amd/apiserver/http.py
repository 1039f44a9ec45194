"""Serve the fake :class:`APIServer` over the Kubernetes REST protocol.

Paths follow kube-apiserver: ``/api/v1/...`` for the core group and
``/apis/<group>/<version>/...`` otherwise, with ``namespaces/<ns>/`` scoping,
``/<name>/<subresource>``, discovery (``/api``, ``/apis``, ``/api/v1``,
``/apis/<g>/<v>``), ``/version`` and ``/healthz``.  LIST/WATCH take
``labelSelector``, ``fieldSelector``, ``resourceVersion``, ``limit``,
``continue``, ``allowWatchBookmarks`` and ``timeoutSeconds``; watches stream
newline-delimited JSON events (chunked).  PATCH honours the content type
(merge / json / strategic); DELETE reads ``DeleteOptions`` from the body or
``propagationPolicy`` from the query.  Errors are ``metav1.Status`` bodies.

Optional bearer-token authentication (``tokens``) and RBAC authorization
(``APIServer(authorization="RBAC")``).  ``/debug/fake/*`` endpoints expose test
controls (clock, request stats, faults, bulk job completion) to out-of-process
drivers such as the benchmark.

The HTTP/1.1 front end is a small ``asyncio.Protocol`` server (keep-alive,
pipelining, ``Content-Length`` and chunked request bodies, ``Expect:
100-continue``, optional TLS).  It replaced aiohttp's web stack because in the
1000-Cron benchmark the apiserver process sits on the critical path and
aiohttp's per-request machinery was a third of its CPU; request handling is
synchronous except for watches and injected latency.
"""
from __future__ import annotations

import asyncio
import json
import time
from typing import Any, Dict, List, Optional, Tuple, Union
from urllib.parse import parse_qsl, unquote

from ..api import errors
from ..api.meta import GroupVersionResource
from ..ops import httpcodec_native
from ..utils import jsonutil
from ..utils.clock import FakeClock
from .server import APIServer, Watcher

PATCH_TYPES = {
    "application/merge-patch+json": "merge",
    "application/json-patch+json": "json",
    "application/strategic-merge-patch+json": "strategic",
    "application/apply-patch+yaml": "apply",
}
_REASONS = {200: "OK", 201: "Created", 202: "Accepted", 204: "No Content", 400: "Bad Request",
            401: "Unauthorized", 403: "Forbidden", 404: "Not Found", 405: "Method Not Allowed", 409: "Conflict",
            410: "Gone", 413: "Payload Too Large", 415: "Unsupported Media Type", 422: "Unprocessable Entity",
            429: "Too Many Requests", 431: "Request Header Fields Too Large", 500: "Internal Server Error",
            503: "Service Unavailable", 504: "Gateway Timeout"}
MAX_BODY = 64 * 1024 * 1024
_codec = httpcodec_native.load()  # native request framing (ops/csrc/httpcodec.cpp), else None
_CODEC_ERRORS = {400: b"bad request", 413: b"request body too large", 431: b"request header too large"}


_VOLATILE = ("metadata",)  # rewritten by every write (resourceVersion): never worth caching


class _EncodeCache:
    """Serialised bytes of stored objects.  A write's response and its watch events
    carry the same (immutable) stored object, so it is encoded once.

    With ``shared=True`` (stored objects only: they are never mutated) the top-level
    values of the object (but ``metadata``) are cached by identity too: a status write
    shares the stored object's ``spec``, a tombstone everything but its metadata, so
    only the changed parts are serialised again (``_fastjson.dumpb_shared``)."""

    def __init__(self, size: int = 8192, sub_size: int = 16384):
        self._d: Dict[int, Tuple[Any, bytes]] = {}
        self._size = size
        self._sub: Dict[int, Tuple[Any, bytes]] = {}
        self._sub_size = sub_size
        self._shared_enc = getattr(jsonutil, "dumpb_shared", None)

    def encode(self, obj: Any, shared: bool = False) -> bytes:
        hit = self._d.get(id(obj))
        if hit is not None and hit[0] is obj:
            return hit[1]
        if shared and self._shared_enc is not None:
            if len(self._sub) >= self._sub_size:
                self._sub.clear()
            b = self._shared_enc(obj, self._sub, _VOLATILE)
        else:
            b = jsonutil.dumpb(obj)
        if len(self._d) >= self._size:
            self._d.clear()
        self._d[id(obj)] = (obj, b)
        return b


_ENC = _EncodeCache()


class Request:
    """What a handler sees: method, decoded path, query (first value per key),
    lower-cased headers, the raw body and the authenticated user."""

    __slots__ = ("method", "path", "query", "headers", "body", "user")

    def __init__(self, method: str, path: str, query: Dict[str, str], headers: Dict[str, str], body: bytes):
        self.method = method
        self.path = path
        self.query = query
        self.headers = headers
        self.body = body
        self.user: Optional[Dict[str, Any]] = None

    @property
    def content_type(self) -> str:
        return self.headers.get("content-type", "").split(";", 1)[0].strip().lower()


class Response:
    __slots__ = ("status", "body", "content_type", "headers")

    def __init__(self, status: int, body: bytes, content_type: str = "application/json",
                 headers: Optional[Dict[str, str]] = None):
        self.status = status
        self.body = body
        self.content_type = content_type
        self.headers = headers


class WatchResponse:
    """A streaming response: newline-delimited watch events until timeout/stop."""

    __slots__ = ("watcher", "timeout")

    def __init__(self, watcher: Watcher, timeout: float):
        self.watcher = watcher
        self.timeout = timeout


Reply = Union[Response, WatchResponse]


def _json(data: Any, status: int = 200, stored: bool = False) -> Response:
    """``stored``: ``data`` is a stored object (immutable), see :class:`_EncodeCache`."""
    return Response(status, _ENC.encode(data, stored) if status < 300 else jsonutil.dumpb(data))


def _event_line(etype: str, obj: Any) -> bytes:
    return b'{"type":"' + etype.encode() + b'","object":' + _ENC.encode(obj, True) + b"}"


def _err(e: errors.ApiError) -> Response:
    r = _json(e.status(), e.code)
    if e.retry_after is not None:
        r.headers = {"Retry-After": str(e.retry_after)}
    return r


class APIServerApp:
    def __init__(self, server: APIServer, request_log: bool = False):
        self.server = server
        self.request_log = request_log
        self.port: Optional[int] = None
        self._srv: Optional[asyncio.AbstractServer] = None
        self._conns: "set[_ServerConn]" = set()
        self._streams: List[Watcher] = []
        self._bookmarks: Optional[asyncio.Task] = None
        self.requests = 0

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
    def _authenticate(self, req: Request) -> Optional[Response]:
        if self.server.tokens is None:
            return None
        auth = req.headers.get("authorization", "")
        token = auth[7:].strip() if auth.startswith("Bearer ") else ""
        user = self.server.tokens.get(token)
        if user is None:
            return _json(errors.ApiError(401, "Unauthorized", "Unauthorized").status(), 401)
        req.user = user
        return None

    def _authorize(self, req: Request, attrs: Dict[str, Any]) -> None:
        rbac = self.server.rbac
        user = req.user
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

    def dispatch(self, req: Request) -> Union[Reply, "asyncio.Future[Reply]"]:
        """Handle one request: a reply, or an awaitable one when the verb must wait
        (injected latency)."""
        self.requests += 1
        denied = self._authenticate(req)
        if denied is not None:
            return denied
        path = req.path
        if path in ("/healthz", "/readyz", "/livez"):
            return Response(200, b"ok", "text/plain")
        if path == "/version":
            return _json({"major": "1", "minor": "34", "gitVersion": "v1.34.0-cron-operator-amd-fake",
                          "platform": "linux/amd64"})
        if path == "/api":
            return _json({"kind": "APIVersions", "versions": ["v1"]})
        if path == "/api/v1":
            return _json(self._core_list())
        if path == "/apis":
            return _json(self._groups())
        try:
            if path.startswith("/debug/fake/"):
                return self._debug(req)
            if self.server.rbac is not None and req.user is not None and not path.startswith(("/api/", "/apis/")):
                self._authorize(req, {"verb": req.method.lower(), "path": path})
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
            return self._resource(req, gvr, ns, name, sub)
        except errors.ApiError as e:
            return _err(e)
        except (ValueError, KeyError, TypeError) as e:
            return _err(errors.bad_request(str(e)))

    @staticmethod
    def _body(req: Request) -> Any:
        raw = req.body
        if not raw:
            return None
        try:
            return jsonutil.loads(raw)
        except ValueError as e:
            raise errors.bad_request(f"invalid JSON body: {e}") from None

    def _resource(self, req: Request, gvr: GroupVersionResource, ns: str, name: str,
                  sub: str) -> Union[Reply, "asyncio.Future[Reply]"]:
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
        delay = s.faults.delay_for(verb) if s.faults.latency else 0.0
        if verb == "list" and delay:
            # a real apiserver filters a label-selected LIST by scanning every object of the
            # resource in the namespace (watch cache or etcd range): charged per object scanned,
            # as latency, while this fixture answers it from a label index
            per = s.faults.latency.get("list_per_object", 0.0)
            if per:
                delay += per * s.count(gvr, ns or None)
        if delay > 0:
            return asyncio.ensure_future(self._delayed(delay, req, gvr, ns, name, sub, verb))
        return self._verb(req, gvr, ns, name, sub, verb)

    async def _delayed(self, delay: float, req: Request, gvr: GroupVersionResource, ns: str, name: str, sub: str,
                       verb: str) -> Reply:
        await asyncio.sleep(delay)
        try:
            return self._verb(req, gvr, ns, name, sub, verb)
        except errors.ApiError as e:
            return _err(e)
        except (ValueError, KeyError, TypeError) as e:
            return _err(errors.bad_request(str(e)))

    def _verb(self, req: Request, gvr: GroupVersionResource, ns: str, name: str, sub: str, verb: str) -> Reply:
        s = self.server
        q = req.query
        if s.faults.faults:
            s.faults.check(verb, gvr.resource, sub or None, name or None)
        if verb == "watch":
            w = s.watch(gvr, ns or None, q.get("resourceVersion", ""), q.get("labelSelector"), q.get("fieldSelector"),
                        q.get("allowWatchBookmarks") in ("true", "1"), copy_events=False)
            return WatchResponse(w, float(q.get("timeoutSeconds") or 1800))
        if verb in ("get", "list") and "as=Table" in req.headers.get("accept", ""):
            from .table import wants_table

            if wants_table(req.headers["accept"]):
                return self._table(req, gvr, ns, name)
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
            body = self._body(req)
            if verb in ("create", "update") and not isinstance(body, dict):
                raise errors.bad_request("request body must be a JSON object")
        # The verb runs synchronously and its result is serialised right here, so the
        # stored object can be returned without a defensive copy.
        s.copy_responses = False
        s.copy_inputs = False  # `body` was decoded for this request alone
        try:
            resp = self._apply(verb, gvr, ns, name, sub, body, ptype, q)
        finally:
            s.copy_responses = True
            s.copy_inputs = True
        if s.faults.faults:  # "lost response" faults fire after the verb was applied
            s.faults.check(verb, gvr.resource, sub or None, name or None, after=True)
        return resp

    def _table(self, req: Request, gvr: GroupVersionResource, ns: str, name: str) -> Response:
        """``kubectl get``'s server-side printing (see :mod:`.table`)."""
        from .table import printer_columns_of, to_table

        s = self.server
        q = req.query
        ri = s.resource(gvr)
        if name:
            objs = [s.get(gvr, ns, name)]
            rv = objs[0]["metadata"].get("resourceVersion", "")
        else:
            lst = s.list(gvr, ns or None, q.get("labelSelector"), q.get("fieldSelector"), copy=False)
            objs = lst["items"]
            rv = lst["metadata"].get("resourceVersion", "")
        return Response(200, jsonutil.dumpb(to_table(printer_columns_of(ri), objs, s.clock.now_ns(), rv,
                                                      q.get("includeObject", "Metadata"))))

    def _apply(self, verb: str, gvr: GroupVersionResource, ns: str, name: str, sub: str, body: Any, ptype: Any,
               q: Dict[str, str]) -> Response:
        s = self.server
        if verb == "list":
            return _json(s.list(gvr, ns or None, q.get("labelSelector"), q.get("fieldSelector"),
                                int(q.get("limit") or 0), q.get("continue"), copy=False))
        if verb == "get":
            return _json(s.get(gvr, ns, name), stored=True)
        if verb == "create":
            return _json(s.create(gvr, ns, body, dry_run=q.get("dryRun") == "All"), 201, stored=True)
        if verb == "update":
            return _json(s.update(gvr, ns, name, body, sub or None), stored=True)
        if verb == "patch":
            return _json(s.patch(gvr, ns, name, body, ptype, sub or None), stored=True)
        if verb == "delete":
            opts = body or {}
            policy = opts.get("propagationPolicy") or q.get("propagationPolicy")
            return _json(s.delete(gvr, ns, name, policy, opts.get("preconditions")), stored=True)
        n = s.delete_collection(gvr, ns or None, q.get("labelSelector"))
        return _json({"kind": "Status", "apiVersion": "v1", "status": "Success", "details": {"deleted": n}})

    # ------------------------------------------------------------------ debug / test controls
    def _debug(self, req: Request) -> Response:
        s = self.server
        what = req.path[len("/debug/fake/"):]
        if what == "stats":
            snap = s.stats.snapshot()
            snap["resourceVersion"] = s.current_rv()
            return _json(snap)
        if what == "clock":
            if req.method == "POST":
                body = self._body(req) or {}
                if not isinstance(s.clock, FakeClock):
                    raise errors.bad_request("server clock is not settable")
                s.clock.set(int(body["nowNs"]))
            return _json({"nowNs": s.clock.now_ns()})
        if what == "faults" and req.method == "POST":
            body = self._body(req) or {}
            if body.get("clear"):
                s.faults.clear()
            for f in body.get("faults") or []:
                s.faults.add(**f)
            for verb, lat in (body.get("latency") or {}).items():
                s.faults.latency[verb] = float(lat)
            # per-resource watch delivery lag, [min s, max s] per event, each stream on its own
            for resource, (lo, hi) in (body.get("watchLag") or {}).items():
                s.faults.watch_lag[resource] = (float(lo), float(hi))
            return _json({"faults": len(s.faults.faults), "watchLag": sorted(s.faults.watch_lag)})
        if what == "complete" and req.method == "POST":
            # bench helper: mark every job (of the given resource) without completionTime as finished
            body = self._body(req) or {}
            from ..trainingop.operator import finished_status

            gvr = GroupVersionResource(body.get("group", "kubeflow.org"), body.get("version", "v1"),
                                       body.get("resource", "pytorchjobs"))
            ts = body.get("time") or ""
            n = 0
            # each patch body is built here and its result discarded: no defensive copies (as in _verb)
            s.copy_responses = s.copy_inputs = False
            try:
                for obj in list(s.objects(gvr, body.get("namespace"))):
                    st = obj.get("status") or {}
                    if st.get("completionTime"):
                        continue
                    m = obj["metadata"]
                    s.patch(gvr, m["namespace"], m["name"],
                            {"status": finished_status(obj.get("kind", ""), m["name"], ts, True)}, "merge", "status")
                    n += 1
            finally:
                s.copy_responses = s.copy_inputs = True
            return _json({"completed": n})
        if what == "lifecycle" and req.method == "POST":
            # bench helper: write stage ``stage`` of the training-operator's status sequence
            # (trainingop.operator.lifecycle_statuses; -1 = the final Succeeded write) to every
            # job without completionTime; returns each written job's new resourceVersion
            body = self._body(req) or {}
            from ..trainingop.operator import lifecycle_status

            gvr = GroupVersionResource(body.get("group", "kubeflow.org"), body.get("version", "v1"),
                                       body.get("resource", "pytorchjobs"))
            stage = int(body.get("stage", -1))
            rvs: Dict[str, str] = {}
            s.copy_responses = s.copy_inputs = False
            try:
                for obj in list(s.objects(gvr, body.get("namespace"))):
                    if (obj.get("status") or {}).get("completionTime"):
                        continue
                    m = obj["metadata"]
                    st = lifecycle_status(obj, stage, body.get("start") or "", body.get("end") or "")
                    out = s.patch(gvr, m["namespace"], m["name"], {"status": st}, "merge", "status")
                    rvs[f"{m['namespace']}/{m['name']}"] = out["metadata"]["resourceVersion"]
            finally:
                s.copy_responses = s.copy_inputs = True
            return _json({"resourceVersions": rvs})
        if what == "profile" and req.method == "POST":
            # cProfile of this process between "start" and "stop" (the bench profiles its timed steps)
            import cProfile

            body = self._body(req) or {}
            if body.get("action") == "start":
                self._prof = cProfile.Profile()
                self._prof.enable()
                return _json({"profiling": True})
            prof = getattr(self, "_prof", None)
            if prof is None:
                raise errors.bad_request("profiling was not started")
            prof.disable()
            self._prof = None
            if body.get("path"):
                prof.dump_stats(body["path"])
            return _json({"profiling": False, "path": body.get("path", "")})
        if what == "gc" and req.method == "POST":
            from ..utils import gctune

            gctune.tune()
            gctune.freeze()
            return _json({"frozen": True})
        if what == "count":
            gvr = GroupVersionResource(req.query.get("group", ""), req.query.get("version", "v1"),
                                       req.query["resource"])
            return _json({"count": s.count(gvr, req.query.get("namespace"))})
        return _err(errors.ApiError(404, "NotFound", f"unknown debug endpoint {what}"))

    # ------------------------------------------------------------------ lifecycle
    async def start(self, host: str = "127.0.0.1", port: int = 0, ssl_context=None,
                    bookmark_interval: float = 60.0) -> int:
        """``bookmark_interval``: seconds between BOOKMARK events on watches that allow them
        (kube-apiserver sends one about every minute, so a resumed watch starts from a fresh
        resourceVersion instead of hitting "too old" and relisting); 0 disables."""
        loop = asyncio.get_running_loop()
        self._srv = await loop.create_server(lambda: _ServerConn(self), host, port, ssl=ssl_context, backlog=1024)
        self.port = self._srv.sockets[0].getsockname()[1]
        if bookmark_interval > 0:
            self._bookmarks = loop.create_task(self._bookmark_loop(bookmark_interval))
        return self.port

    async def _bookmark_loop(self, interval: float) -> None:
        while True:
            await asyncio.sleep(interval)
            self.server.send_bookmarks()

    async def stop(self) -> None:
        if self._bookmarks is not None:
            self._bookmarks.cancel()
            self._bookmarks = None
        for w in list(self._streams):
            w.stop()
        if self._srv is not None:
            self._srv.close()
            for c in list(self._conns):
                c.close()
            try:
                await asyncio.wait_for(self._srv.wait_closed(), 5)
            except asyncio.TimeoutError:
                pass
            self._srv = None


def _origin_form(target: str) -> str:
    """RFC 9112 3.2.2: a server accepts the absolute form (``http://host:port/path?q``) that
    clients use through a proxy; routing only needs the path and query."""
    scheme, sep, rest = target.partition("://")
    if not sep or scheme.lower() not in ("http", "https"):
        return target
    slash = rest.find("/")
    q = rest.find("?")
    if slash < 0 or (0 <= q < slash):
        return "/" + (rest[q:] if q >= 0 else "")
    return rest[slash:]


class _ServerConn(asyncio.Protocol):
    """One client connection: parse requests, dispatch in order, write replies."""

    def __init__(self, app: APIServerApp):
        self.app = app
        self.transport: Optional[asyncio.Transport] = None
        self.buf = bytearray()
        self.busy = False               # a reply (watch / delayed) is pending; later requests wait
        self.closed = False
        self._continued = False         # "100 Continue" already sent for the pending request
        self._watch: Optional["_WatchStream"] = None

    def connection_made(self, transport: asyncio.BaseTransport) -> None:
        self.transport = transport  # type: ignore[assignment]
        self.app._conns.add(self)

    def connection_lost(self, exc: Optional[BaseException]) -> None:
        self.closed = True
        self.app._conns.discard(self)
        if self._watch is not None:
            self._watch.end()

    def close(self) -> None:
        if self.transport is not None and not self.closed:
            self.transport.close()

    def data_received(self, data: bytes) -> None:
        self.buf += data
        if not self.busy:
            self._drain()

    # --------------------------------------------------------------- parsing
    def _next_request(self) -> Optional[Tuple[Request, bool]]:
        if _codec is None:
            return self._next_request_py()
        r = _codec.parse_request(self.buf, MAX_BODY)
        if r is None:
            return None
        if r.__class__ is int:
            if r == 100:
                if not self._continued:
                    self._continued = True
                    assert self.transport is not None
                    self.transport.write(b"HTTP/1.1 100 Continue\r\n\r\n")
                return None
            self._reply_raw(r, _CODEC_ERRORS.get(r, b"bad request"), "text/plain", close=True)
            return None
        method, target, headers, raw, consumed, keep = r
        del self.buf[:consumed]
        self._continued = False
        if target[:1] != "/":
            target = _origin_form(target)
        path, _, qs = target.partition("?")
        query: Dict[str, str] = {}
        if qs:
            for k, v in parse_qsl(qs, keep_blank_values=True):
                query.setdefault(k, v)
        return Request(method.upper(), unquote(path) if "%" in path else path, query, headers, raw), keep

    def _next_request_py(self) -> Optional[Tuple[Request, bool]]:
        """Pure-Python framing: the fallback, and the oracle of tests/test_httpcodec.py."""
        buf = self.buf
        end = buf.find(b"\r\n\r\n")
        if end < 0:
            if len(buf) > 1 << 20:
                self._reply_raw(431, b"request header too large", "text/plain", close=True)
            return None
        head = bytes(buf[:end]).decode("latin-1")
        lines = head.split("\r\n")
        try:
            method, target, version = lines[0].split(" ", 2)
        except ValueError:
            self._reply_raw(400, b"bad request line", "text/plain", close=True)
            return None
        headers: Dict[str, str] = {}
        for line in lines[1:]:
            k, _, v = line.partition(":")
            headers[k.strip().lower()] = v.strip()
        pos = end + 4
        te = headers.get("transfer-encoding", "").lower()
        if "chunked" in te:
            body = bytearray()
            while True:
                nl = buf.find(b"\r\n", pos)
                if nl < 0:
                    return None
                size = int(bytes(buf[pos:nl]).split(b";", 1)[0], 16)
                if size == 0:
                    tend = buf.find(b"\r\n\r\n", nl)
                    if tend < 0:
                        return None
                    pos = tend + 4
                    break
                if len(buf) < nl + 2 + size + 2:
                    return None
                body += buf[nl + 2:nl + 2 + size]
                pos = nl + 2 + size + 2
            raw = bytes(body)
        else:
            clen = int(headers.get("content-length") or 0)
            if clen > MAX_BODY:
                self._reply_raw(413, b"request body too large", "text/plain", close=True)
                return None
            if len(buf) < pos + clen:
                if headers.get("expect", "").lower() == "100-continue" and not self._continued:
                    self._continued = True
                    assert self.transport is not None
                    self.transport.write(b"HTTP/1.1 100 Continue\r\n\r\n")
                return None
            raw = bytes(buf[pos:pos + clen])
            pos += clen
        del buf[:pos]
        self._continued = False
        if target[:1] != "/":
            target = _origin_form(target)
        path, _, qs = target.partition("?")
        query: Dict[str, str] = {}
        if qs:
            for k, v in parse_qsl(qs, keep_blank_values=True):
                query.setdefault(k, v)
        conn_hdr = headers.get("connection", "").lower()
        keep = (conn_hdr != "close") if version == "HTTP/1.1" else (conn_hdr == "keep-alive")
        return Request(method.upper(), unquote(path), query, headers, raw), keep

    def _drain(self) -> None:
        while not self.busy and not self.closed:
            nxt = self._next_request()
            if nxt is None:
                return
            req, keep = nxt
            try:
                reply = self.app.dispatch(req)
            except Exception as e:  # noqa: BLE001 - never kill the connection on a handler bug
                reply = _err(errors.ApiError(500, "InternalError", f"{type(e).__name__}: {e}"))
            if isinstance(reply, Response):
                self._reply(reply, keep)
                continue
            self.busy = True
            if isinstance(reply, WatchResponse):
                self._start_watch(reply, keep)
            else:
                reply.add_done_callback(lambda f, keep=keep: self._delayed_done(f, keep))

    def _delayed_done(self, fut: "asyncio.Future[Reply]", keep: bool) -> None:
        self.busy = False
        if self.closed:
            return
        try:
            reply = fut.result()
        except Exception as e:  # noqa: BLE001
            reply = _err(errors.ApiError(500, "InternalError", str(e)))
        if isinstance(reply, WatchResponse):
            self.busy = True
            self._start_watch(reply, keep)
            return
        self._reply(reply, keep)
        self._drain()

    # --------------------------------------------------------------- replies
    def _reply(self, r: Response, keep: bool) -> None:
        self._reply_raw(r.status, r.body, r.content_type, close=not keep, headers=r.headers)

    def _reply_raw(self, status: int, body: bytes, ctype: str, close: bool = False,
                   headers: Optional[Dict[str, str]] = None) -> None:
        if self.transport is None or self.closed:
            return
        extra = "".join(f"{k}: {v}\r\n" for k, v in headers.items()) if headers else ""
        head = (f"HTTP/1.1 {status} {_REASONS.get(status, 'Unknown')}\r\nContent-Type: {ctype}\r\n"
                f"Content-Length: {len(body)}\r\n{extra}" + ("Connection: close\r\n" if close else "") + "\r\n")
        self.transport.write(head.encode("latin-1") + body)
        if close:
            self.transport.close()
            self.closed = True

    def _start_watch(self, wr: WatchResponse, keep: bool) -> None:
        ws = _WatchStream(self, wr, keep)
        if not ws.ended:  # a watcher stopped before it started has already finished the reply
            self._watch = ws

    def _after_watch(self) -> None:
        """The watch response ended on a kept-alive connection: serve what queued up."""
        if self.closed:
            return
        self.busy = False
        self._drain()


_WATCH_HEAD = b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n"


class _WatchStream:
    """One watch response, fed synchronously by its :class:`Watcher` (``Watcher.sink``).

    Each event is encoded when it happens; everything that arrives within one turn of
    the event loop goes out as one chunk (``call_soon`` flush).  Compared with a
    consumer coroutine per stream this saves a queue hand-off, a task wake-up and a
    ``wait_for`` timer per batch.  ``timeoutSeconds`` is one ``call_later``.
    """

    __slots__ = ("conn", "watcher", "keep", "lines", "loop", "flush_h", "timer", "ended")

    def __init__(self, conn: "_ServerConn", wr: WatchResponse, keep: bool):
        self.conn = conn
        self.watcher = w = wr.watcher
        self.keep = keep
        self.lines: List[bytes] = []
        self.loop = asyncio.get_running_loop()
        self.flush_h: Optional[asyncio.Handle] = None
        self.ended = False
        conn.app._streams.append(w)
        assert conn.transport is not None
        conn.transport.write(_WATCH_HEAD)
        # events queued before the sink attached: the initial state or the resumed backlog
        stopped = False
        while not w.queue.empty():
            ev = w.queue.get_nowait()
            if ev is None:
                stopped = True
                break
            self.lines.append(_event_line(ev[0], ev[1]))
        w.sink = self.on_event
        self.timer = self.loop.call_later(wr.timeout, self.end)
        if stopped or w.closed:
            self.end()
        elif self.lines:
            self.flush_h = self.loop.call_soon(self.flush)

    def on_event(self, ev: Optional[Tuple[str, Dict[str, Any]]]) -> None:
        if self.ended:
            return
        if ev is None:
            self.end()
            return
        self.lines.append(_event_line(ev[0], ev[1]))
        if self.flush_h is None:
            self.flush_h = self.loop.call_soon(self.flush)

    def flush(self) -> None:
        self.flush_h = None
        if not self.lines:
            return
        conn = self.conn
        if conn.closed or conn.transport is None:
            self.lines.clear()
            return
        chunk = b"\n".join(self.lines) + b"\n"
        self.lines.clear()
        conn.transport.write(b"%x\r\n" % len(chunk) + chunk + b"\r\n")

    def end(self) -> None:
        if self.ended:
            return
        self.ended = True
        self.timer.cancel()
        if self.watcher.stalled:  # a dead connection: nothing more reaches the client, not even the end
            self.watcher.sink = None
            self.watcher.stop()
            if self.watcher in self.conn.app._streams:
                self.conn.app._streams.remove(self.watcher)
            return
        if self.flush_h is not None:
            self.flush_h.cancel()
        self.flush()  # what is pending goes out before the terminating chunk
        w = self.watcher
        w.sink = None
        w.stop()
        streams = self.conn.app._streams
        if w in streams:
            streams.remove(w)
        conn = self.conn
        conn._watch = None
        if conn.closed or conn.transport is None:
            return
        conn.transport.write(b"0\r\n\r\n")
        if not self.keep:
            conn.transport.close()
            conn.closed = True
            return
        # not from inside whatever stopped the watcher (a handler, a timer): next turn
        self.loop.call_soon(conn._after_watch)
