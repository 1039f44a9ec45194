"""A minimal HTTP/1.1 server for the operator's own endpoints.

The probe port (``/healthz``, ``/readyz``, ``/debug/traces``) and the metrics port
(``/metrics``) answer a handful of GETs from the kubelet and Prometheus
(controller-runtime's ``healthz`` and metrics servers, reference
``cmd/operator/start.go:195-203``, ``:226``).  A web framework for that costs more than
the endpoints: importing aiohttp adds ~13 MiB of resident memory to every operator
process and ~0.2 s to its start, so these servers run on asyncio directly -- request
line and headers parsed per connection, keep-alive, optional TLS (the metrics port),
GET and HEAD only.
"""
from __future__ import annotations

import asyncio
import json
import ssl
from typing import Any, Awaitable, Callable, Dict, List, Optional, Tuple
from urllib.parse import parse_qsl, unquote

MAX_HEAD = 16 * 1024  # request line + headers
MAX_BODY = 1 << 20    # a GET with a body is read and ignored up to this size
IDLE_TIMEOUT = 75.0   # a keep-alive connection with no request in flight is closed after this
REQUEST_TIMEOUT = 30.0  # a request must be complete (head and body) this long after its first byte
_REASONS = {200: "OK", 400: "Bad Request", 401: "Unauthorized", 403: "Forbidden", 404: "Not Found",
            405: "Method Not Allowed", 409: "Conflict", 413: "Payload Too Large",
            431: "Request Header Fields Too Large", 500: "Internal Server Error", 503: "Service Unavailable"}


class Request:
    """What a handler reads: method, path, query, headers (lower-case names) and the values
    of a ``{name}`` route segment (``match_info``)."""

    __slots__ = ("method", "path", "query", "headers", "match_info", "peer")

    def __init__(self, method: str, path: str, query: Dict[str, str], headers: Dict[str, str],
                 peer: str = ""):
        self.method = method
        self.path = path
        self.query = query
        self.headers = _Headers(headers)
        self.match_info: Dict[str, str] = {}
        self.peer = peer  # the client's IP address ("" when unknown)


class _Headers(dict):
    """Header map with case-insensitive ``get`` (names are stored lower-case)."""

    def get(self, key: str, default: Any = None) -> Any:  # type: ignore[override]
        return dict.get(self, key.lower(), default)

    def __getitem__(self, key: str) -> str:
        return dict.__getitem__(self, key.lower())

    def __contains__(self, key: object) -> bool:
        return dict.__contains__(self, key.lower() if isinstance(key, str) else key)


class Response:
    __slots__ = ("status", "body", "headers")

    def __init__(self, status: int = 200, text: Optional[str] = None, body: Optional[bytes] = None,
                 headers: Optional[Dict[str, str]] = None, content_type: str = "text/plain; charset=utf-8"):
        self.status = status
        self.body = body if body is not None else (text or "").encode()
        self.headers = {"Content-Type": content_type}
        if headers:
            self.headers.update(headers)


def json_response(obj: Any, status: int = 200) -> Response:
    return Response(status=status, body=json.dumps(obj).encode(), content_type="application/json; charset=utf-8")


Handler = Callable[[Request], Awaitable[Response]]


class Router:
    """Exact paths, plus ``/prefix/{name}`` routes that bind one trailing segment."""

    def __init__(self) -> None:
        self._exact: Dict[str, Handler] = {}
        self._param: List[Tuple[str, str, Handler]] = []

    def add_get(self, path: str, handler: Handler) -> None:
        if path.endswith("}") and "/{" in path:
            prefix, _, name = path.rpartition("/{")
            self._param.append((prefix + "/", name[:-1], handler))
        else:
            self._exact[path] = handler

    def match(self, path: str) -> Tuple[Optional[Handler], Dict[str, str]]:
        h = self._exact.get(path)
        if h is not None:
            return h, {}
        for prefix, name, handler in self._param:
            if path.startswith(prefix):
                seg = path[len(prefix):]
                if seg and "/" not in seg:
                    return handler, {name: unquote(seg)}
        return None, {}


class _Conn(asyncio.Protocol):
    def __init__(self, server: "Server"):
        self.s = server
        self.t: Optional[asyncio.Transport] = None
        self.buf = bytearray()
        self.busy = False
        self.closing = False
        self.task: Optional[asyncio.Task] = None
        self.timer: Optional[asyncio.TimerHandle] = None
        self.reading = False  # a request's first bytes arrived, the rest not yet

    def _arm(self, seconds: float) -> None:
        """(Re)start the connection's deadline: an idle keep-alive connection, or a request that
        trickles in (a slow client holding the port), is closed when it passes."""
        if self.timer is not None:
            self.timer.cancel()
        self.timer = asyncio.get_running_loop().call_later(seconds, self._expire)

    def _expire(self) -> None:
        self.timer = None
        if not self.busy and self.t is not None:
            self.t.close()

    def connection_made(self, transport: asyncio.BaseTransport) -> None:
        self.t = transport  # type: ignore[assignment]
        self.s._conns.add(self)
        self._arm(IDLE_TIMEOUT)

    def connection_lost(self, exc: Optional[BaseException]) -> None:
        self.s._conns.discard(self)
        self.closing = True
        if self.timer is not None:
            self.timer.cancel()
            self.timer = None
        if self.task is not None and not self.task.done():
            self.task.cancel()

    def data_received(self, data: bytes) -> None:
        self.buf += data
        if len(self.buf) > MAX_HEAD + MAX_BODY:
            self._fail(413)
            return
        if not self.busy:
            if not self.reading:
                self.reading = True
                self._arm(REQUEST_TIMEOUT)
            self._next()

    def _fail(self, status: int) -> None:
        if self.t is not None and not self.t.is_closing():
            self.t.write(_head(status, {"Content-Type": "text/plain; charset=utf-8", "Connection": "close"},
                               len(_REASONS.get(status, "")) + 1) + (_REASONS.get(status, "") + "\n").encode())
            self.t.close()
        self.closing = True

    def _next(self) -> None:
        end = self.buf.find(b"\r\n\r\n")
        if end < 0:
            if len(self.buf) > MAX_HEAD:
                self._fail(431)
            return
        try:
            head = bytes(self.buf[:end]).decode("latin-1")
            lines = head.split("\r\n")
            method, target, version = lines[0].split(" ", 2)
            headers: Dict[str, str] = {}
            for ln in lines[1:]:
                k, sep, v = ln.partition(":")
                if not sep:
                    raise ValueError(ln)
                headers[k.strip().lower()] = v.strip()
            n = int(headers.get("content-length", "0") or "0")
        except (ValueError, UnicodeDecodeError):
            self._fail(400)
            return
        if n < 0 or n > MAX_BODY or "chunked" in headers.get("transfer-encoding", ""):
            self._fail(400)
            return
        if len(self.buf) < end + 4 + n:
            return  # the (ignored) body is still arriving
        del self.buf[:end + 4 + n]
        self.reading = False
        if self.timer is not None:
            self.timer.cancel()
            self.timer = None
        keep = version == "HTTP/1.1" and headers.get("connection", "").lower() != "close"
        path, _, qs = target.partition("?")
        peer = self.t.get_extra_info("peername") if self.t is not None else None
        req = Request(method, unquote(path), dict(parse_qsl(qs, keep_blank_values=True)), headers,
                      peer[0] if isinstance(peer, tuple) and peer else "")
        self.busy = True
        self.task = asyncio.get_running_loop().create_task(self._serve(req, keep))

    async def _serve(self, req: Request, keep: bool) -> None:
        try:
            if req.method not in ("GET", "HEAD"):
                resp = Response(405, "Method Not Allowed\n", headers={"Allow": "GET, HEAD"})
            else:
                handler, info = self.s.router.match(req.path)
                if handler is None:
                    resp = Response(404, "404: Not Found")
                else:
                    req.match_info = info
                    try:
                        resp = await handler(req)
                    except asyncio.CancelledError:
                        raise
                    except Exception as e:  # noqa: BLE001 - a failing endpoint answers 500
                        resp = Response(500, f"500 Internal Server Error: {e}\n")
        except asyncio.CancelledError:
            return
        t = self.t
        if t is None or t.is_closing():
            return
        hdrs = dict(resp.headers)
        if not keep:
            hdrs["Connection"] = "close"
        t.write(_head(resp.status, hdrs, len(resp.body)) + (b"" if req.method == "HEAD" else resp.body))
        if not keep:
            t.close()
            return
        self.busy = False
        self.task = None
        if self.closing:
            return
        if self.buf:
            self.reading = True
            self._arm(REQUEST_TIMEOUT)
            self._next()
        else:
            self._arm(IDLE_TIMEOUT)


def _head(status: int, headers: Dict[str, str], length: int) -> bytes:
    out = [f"HTTP/1.1 {status} {_REASONS.get(status, 'Status')}"]
    out += [f"{k}: {v}" for k, v in headers.items()]
    out.append(f"Content-Length: {length}")
    return ("\r\n".join(out) + "\r\n\r\n").encode("latin-1")


class Server:
    """``router`` served on ``host:port`` (port 0: any free one, see :attr:`port`)."""

    def __init__(self, router: Router):
        self.router = router
        self._srv: Optional[asyncio.base_events.Server] = None
        self._conns: "set[_Conn]" = set()
        self.port: Optional[int] = None

    async def start(self, host: str, port: int, ssl_context: Optional[ssl.SSLContext] = None) -> None:
        loop = asyncio.get_running_loop()
        self._srv = await loop.create_server(lambda: _Conn(self), host, port, ssl=ssl_context, backlog=128,
                                             reuse_address=True)
        socks = self._srv.sockets or ()
        self.port = socks[0].getsockname()[1] if socks else None

    async def stop(self) -> None:
        if self._srv is not None:
            self._srv.close()
            for c in list(self._conns):
                if c.t is not None:
                    c.t.close()
            await self._srv.wait_closed()
            self._srv = None
