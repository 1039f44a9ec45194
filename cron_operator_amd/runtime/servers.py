"""Health-probe and metrics HTTP servers.

* Probes: ``/healthz`` and ``/readyz`` (plus ``/healthz/<check>``), answered from
  registered checks like controller-runtime's ``healthz.Ping``
  (``cmd/operator/start.go:195-203``; probed on :8081 by the chart,
  ``charts/cron-operator/templates/deployment.yaml:74-83``).  The same port serves
  ``/debug/traces`` (Chrome trace JSON of recent reconciles) when tracing is on, and
  ``/debug/<name>`` views registered by the manager and the controller (``/debug/caches``: the
  objects each informer holds and the process's memory; ``/debug/wire-memo``), ``/debug/tasks``
  (live asyncio tasks by where they wait) and, with ``--enable-profiling``, ``/debug/profile``
  (a CPU profile of the loop thread; :mod:`.profiler`).  The ``/debug`` views expose internals
  (object keys, await chains with source lines), unlike the probes: by default
  (``--debug-views=local``) they answer only clients on the loopback interface (``kubectl
  port-forward``, ``kubectl exec ... curl localhost``) and 403 everyone else; ``all`` serves
  any client (put the probe port behind a NetworkPolicy), ``off`` none.
* Metrics: ``/metrics`` in Prometheus text format.  ``--metrics-secure`` (default
  true, ``start.go:226``) serves HTTPS and guards the endpoint with the
  authn/authz filter: the bearer token is checked with a TokenReview and the
  caller must be allowed ``get`` on the ``/metrics`` non-resource URL by a
  SubjectAccessReview (``start.go:127-133``).  Without ``--metrics-cert-path`` a
  self-signed certificate is generated (openssl), as controller-runtime does.
  ``--metrics-bind-address=0`` disables the server.

Both run on :mod:`.miniweb` (asyncio, HTTP/1.1), not a web framework.
"""
from __future__ import annotations

import asyncio
import math
import os
import ssl
import subprocess
import tempfile
from typing import Any, Awaitable, Callable, Dict, Optional, Tuple

from ..api import errors
from ..api.meta import GroupVersionResource
from ..utils.logging import get_logger
from . import metrics
from . import miniweb as web

Check = Callable[[], Optional[str]]  # returns None when healthy, else a reason

TOKENREVIEWS = GroupVersionResource("authentication.k8s.io", "v1", "tokenreviews")
SUBJECTACCESSREVIEWS = GroupVersionResource("authorization.k8s.io", "v1", "subjectaccessreviews")


def ping() -> Optional[str]:
    return None


def parse_bind_address(addr: str) -> Optional[Tuple[str, int]]:
    """":8080" -> ("0.0.0.0", 8080); "0" -> None (disabled)."""
    if addr in ("", "0"):
        return None
    host, _, port = addr.rpartition(":")
    if not port:
        raise ValueError(f"invalid bind address {addr!r}")
    return (host or "0.0.0.0", int(port))


def _render(checks: Dict[str, Check], kind: str, verbose: bool) -> Tuple[int, str]:
    lines = []
    failed = False
    for name, fn in sorted(checks.items()):
        try:
            reason = fn()
        except Exception as e:  # noqa: BLE001
            reason = str(e)
        if reason is None:
            lines.append(f"[+]{name} ok")
        else:
            failed = True
            lines.append(f"[-]{name} failed: {reason}")
    if failed:
        return 500, "\n".join(lines) + f"\n{kind} check failed\n"
    if verbose:
        return 200, "\n".join(lines) + f"\n{kind} check passed\n"
    return 200, "ok"


DEBUG_VIEWS = ("local", "all", "off")


def is_loopback(addr: str) -> bool:
    import ipaddress

    try:
        ip = ipaddress.ip_address(addr.split("%", 1)[0])
    except ValueError:
        return False
    mapped = getattr(ip, "ipv4_mapped", None)
    return (mapped or ip).is_loopback


class ProbeServer:
    def __init__(self, bind: str, debug_views: str = "local"):
        if debug_views not in DEBUG_VIEWS:
            raise ValueError(f"debug_views must be one of {DEBUG_VIEWS}, not {debug_views!r}")
        self.debug_views = debug_views
        self.bind = bind
        self.healthz: Dict[str, Check] = {}
        self.readyz: Dict[str, Check] = {}
        # /debug/<name>: JSON of what the callable returns (cache sizes, the wire memo, memory)
        self.debug: Dict[str, Callable[[], Any]] = {}
        self._server: Optional[web.Server] = None
        self.port: Optional[int] = None

    def app(self) -> web.Router:
        app = web.Router()

        def handler(checks: Dict[str, Check], kind: str):
            async def h(req: web.Request) -> web.Response:
                sub = req.match_info.get("check")
                if sub:
                    if sub not in checks:
                        return web.Response(status=404, text=f"no such check {sub}\n")
                    code, body = _render({sub: checks[sub]}, kind, False)
                    return web.Response(status=code, text=body)
                code, body = _render(checks, kind, "verbose" in req.query)
                return web.Response(status=code, text=body)
            return h

        def guarded(h):
            """A /debug view: served to the clients ``debug_views`` allows, 403 to the others."""
            async def g(req: web.Request) -> web.Response:
                if self.debug_views == "off":
                    return web.Response(status=404, text="debug views disabled (--debug-views=off)\n")
                if self.debug_views == "local" and not is_loopback(req.peer):
                    return web.Response(status=403, text="debug views are served to loopback clients only "
                                                         "(--debug-views=local); use kubectl port-forward\n")
                return await h(req)
            return g

        app.add_get("/healthz", handler(self.healthz, "healthz"))
        app.add_get("/healthz/{check}", handler(self.healthz, "healthz"))
        app.add_get("/readyz", handler(self.readyz, "readyz"))
        app.add_get("/readyz/{check}", handler(self.readyz, "readyz"))

        async def traces(req: web.Request) -> web.Response:
            from . import tracing

            t = tracing.get_tracer()
            if not t.enabled:
                return web.Response(status=404, text="tracing disabled (start with --enable-tracing)\n")
            if req.query.get("format") == "spans":
                return web.json_response({"spans": t.spans()})
            return web.json_response(t.chrome_trace())

        app.add_get("/debug/traces", guarded(traces))

        async def tasks(req: web.Request) -> web.Response:
            from . import profiler

            return web.json_response(profiler.task_dump(stacks=req.query.get("stacks") in ("1", "true")))

        async def profile(req: web.Request) -> web.Response:
            from . import profiler

            if not profiler.allowed():
                return web.Response(status=404, text="profiling disabled (start with --enable-profiling)\n")
            try:
                seconds = float(req.query.get("seconds", "10"))
            except ValueError:
                seconds = math.nan
            if not math.isfinite(seconds):  # nan/inf would corrupt the loop's timer heap
                return web.Response(status=400, text="seconds: a finite number\n")
            try:
                return web.Response(text=await profiler.cpu_profile(seconds))
            except RuntimeError as e:
                return web.Response(status=409, text=f"{e}\n")

        app.add_get("/debug/tasks", guarded(tasks))
        app.add_get("/debug/profile", guarded(profile))

        async def debug(req: web.Request) -> web.Response:
            fn = self.debug.get(req.match_info["name"])
            if fn is None:
                return web.Response(status=404, text=f"no such debug view; have: {', '.join(sorted(self.debug))}\n")
            return web.json_response(fn())

        app.add_get("/debug/{name}", guarded(debug))
        return app

    async def start(self) -> None:
        addr = parse_bind_address(self.bind)
        if addr is None:
            return
        self._server = web.Server(self.app())
        await self._server.start(addr[0], addr[1])
        self.port = self._server.port

    async def stop(self) -> None:
        if self._server is not None:
            await self._server.stop()
            self._server = None


def self_signed_cert(directory: str, host: str = "localhost") -> Tuple[str, str]:
    crt = os.path.join(directory, "tls.crt")
    key = os.path.join(directory, "tls.key")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "365",
                    "-subj", f"/CN={host}", "-keyout", key, "-out", crt],
                   check=True, capture_output=True)
    return crt, key


# certwatcher's polling interval (it also reacts to fsnotify events; polling alone is
# enough for a certificate that cert-manager renews well before expiry)
CERT_POLL_INTERVAL = 10.0


class MetricsServer:
    def __init__(self, bind: str, secure: bool = True, cert_dir: str = "", cert_name: str = "tls.crt",
                 key_name: str = "tls.key", client=None, enable_http2: bool = False,
                 cert_poll_interval: float = CERT_POLL_INTERVAL):
        self.bind = bind
        # a certificate from --metrics-cert-path is watched and reloaded when its files change
        # (controller-runtime's certwatcher), so a cert-manager rotation needs no restart
        self.cert_poll_interval = cert_poll_interval
        self._ctx: Optional[ssl.SSLContext] = None
        self._cert_watch: Optional[asyncio.Task] = None
        self.cert_reloads = 0
        self.secure = secure
        self.cert_dir = cert_dir
        self.cert_name = cert_name
        self.key_name = key_name
        self.client = client  # for TokenReview / SubjectAccessReview
        self.enable_http2 = enable_http2
        self._server: Optional[web.Server] = None
        self._tmp: Optional[tempfile.TemporaryDirectory] = None
        self.port: Optional[int] = None
        self.extra_handlers: Dict[str, Callable[[web.Request], Awaitable[web.Response]]] = {}
        # replaces the /metrics handler (the shard-process supervisor serves merged expositions)
        self.handler: Optional[Callable[[web.Request], Awaitable[web.Response]]] = None
        self.log = get_logger("controller-runtime.metrics")

    async def _authorize(self, req: web.Request) -> Optional[web.Response]:
        if not self.secure or self.client is None:
            return None
        auth = req.headers.get("Authorization", "")
        if not auth.startswith("Bearer "):
            return web.Response(status=401, text="Unauthorized\n")
        token = auth[len("Bearer "):].strip()
        try:
            tr = await self.client.create(TOKENREVIEWS, {"apiVersion": "authentication.k8s.io/v1",
                                                         "kind": "TokenReview", "spec": {"token": token}}, "")
        except errors.ApiError as e:
            return web.Response(status=500, text=f"authentication failed: {e}\n")
        st = tr.get("status") or {}
        if not st.get("authenticated"):
            return web.Response(status=401, text="Unauthorized\n")
        user = st.get("user") or {}
        sar = {"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview",
               "spec": {"user": user.get("username", ""), "groups": user.get("groups") or [],
                        "nonResourceAttributes": {"path": req.path, "verb": "get"}}}
        try:
            res = await self.client.create(SUBJECTACCESSREVIEWS, sar, "")
        except errors.ApiError as e:
            return web.Response(status=500, text=f"authorization failed: {e}\n")
        if not (res.get("status") or {}).get("allowed"):
            return web.Response(status=403, text=f'Authorization denied for user {user.get("username", "")}\n')
        return None

    def app(self) -> web.Router:
        app = web.Router()

        async def handle(req: web.Request) -> web.Response:
            denied = await self._authorize(req)
            if denied is not None:
                return denied
            body = metrics.exposition()
            return web.Response(body=body, headers={"Content-Type": "text/plain; version=0.0.4; charset=utf-8"})

        app.add_get("/metrics", self.handler or handle)
        for path, h in self.extra_handlers.items():
            app.add_get(path, h)
        return app

    def _ssl(self) -> Optional[ssl.SSLContext]:
        if not self.secure:
            return None
        if self.cert_dir:
            crt = os.path.join(self.cert_dir, self.cert_name)
            key = os.path.join(self.cert_dir, self.key_name)
        else:
            self._tmp = tempfile.TemporaryDirectory(prefix="cron-operator-metrics-")
            crt, key = self_signed_cert(self._tmp.name)
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        if self.cert_dir:
            metrics.CERT_READS.inc()
        ctx.load_cert_chain(crt, key)
        # HTTP/2 is off unless --enable-http2 (start.go:83-98); this server speaks HTTP/1.1 only
        ctx.set_alpn_protocols(["http/1.1"])
        self._ctx = ctx
        return ctx

    @staticmethod
    def _stamp(*paths: str) -> Tuple[Any, ...]:
        """What identifies a certificate's current content: the files' identity, size and
        mtime after symlinks (a Secret volume swaps its ``..data`` link on update)."""
        out = []
        for p in paths:
            try:
                st = os.stat(p)
                out.append((st.st_ino, st.st_size, st.st_mtime_ns))
            except OSError:
                out.append(None)
        return tuple(out)

    def _reload_pair(self, crt: str, key: str) -> None:
        """Load a rotated pair into the live SSLContext only once it is known to load.

        ``SSLContext.load_cert_chain`` installs the certificate *before* it checks the key,
        so loading a new certificate with a stale or mismatched key straight into the live
        context would leave it unusable (every handshake then fails).  The pair is therefore
        snapshotted into private files (so it cannot change between the checks), loaded into
        a scratch context first, and only then into the live one."""
        with open(crt, "rb") as fh:
            crt_pem = fh.read()
        with open(key, "rb") as fh:
            key_pem = fh.read()
        with tempfile.TemporaryDirectory(prefix="cron-operator-cert-") as d:
            scrt, skey = os.path.join(d, "tls.crt"), os.path.join(d, "tls.key")
            for path, data in ((scrt, crt_pem), (skey, key_pem)):
                fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
                with os.fdopen(fd, "wb") as fh:
                    fh.write(data)
            ssl.create_default_context(ssl.Purpose.CLIENT_AUTH).load_cert_chain(scrt, skey)
            assert self._ctx is not None
            self._ctx.load_cert_chain(scrt, skey)

    async def _watch_certs(self, crt: str, key: str) -> None:
        """certwatcher: poll the certificate and key; load a changed pair into the live
        SSLContext (new handshakes use it).  A pair that does not load -- caught mid
        rotation, or a new certificate next to the old key -- keeps the previous certificate
        serving and is retried on the next poll."""
        last = self._stamp(crt, key)
        while True:
            await asyncio.sleep(self.cert_poll_interval)
            cur = self._stamp(crt, key)
            if cur == last or self._ctx is None:
                continue
            metrics.CERT_READS.inc()
            try:
                self._reload_pair(crt, key)
            except (OSError, ssl.SSLError) as e:
                metrics.CERT_READ_ERRORS.inc()
                self.log.error(e, "error loading the rotated certificate, keeping the current one",
                               certPath=crt, keyPath=key)
                continue
            last = cur
            self.cert_reloads += 1
            self.log.info("Updated current TLS certificate", certPath=crt, keyPath=key)

    async def start(self) -> None:
        addr = parse_bind_address(self.bind)
        if addr is None:
            return
        if self.enable_http2:
            self.log.info("HTTP/2 requested but the metrics server only serves HTTP/1.1")
        self._server = web.Server(self.app())
        await self._server.start(addr[0], addr[1], ssl_context=self._ssl())
        self.port = self._server.port
        if self.secure and self.cert_dir and self.cert_poll_interval > 0:
            self._cert_watch = asyncio.get_running_loop().create_task(self._watch_certs(
                os.path.join(self.cert_dir, self.cert_name), os.path.join(self.cert_dir, self.key_name)))
        self.log.info("Serving metrics server", bindAddress=self.bind, secure=self.secure)

    async def stop(self) -> None:
        if self._cert_watch is not None:
            self._cert_watch.cancel()
            self._cert_watch = None
        if self._server is not None:
            await self._server.stop()
            self._server = None
        if self._tmp is not None:
            self._tmp.cleanup()
            self._tmp = None

