"""Lean HTTP/1.1 keep-alive client for the request/response verbs.

Profiling the operator during the 1000-Cron bench (round 1)
put aiohttp's client machinery (request/response objects, header multidicts,
timers, stream readers) at roughly a third of the operator's CPU per API call.
A Kubernetes client needs far less: one request in flight per connection, a
fixed header set, ``Content-Length`` or ``chunked`` responses, keep-alive.
This module is exactly that, on ``asyncio.Protocol``:

* a pool of persistent connections per host (TLS via the kubeconfig's
  ``ssl.SSLContext``; plain TCP for ``http://``), optionally through an http
  proxy (absolute-form requests, or a ``CONNECT`` tunnel under TLS);
* request bytes built once per call (method, path, fixed auth headers,
  ``Content-Length``);
* an incremental response parser (status line, headers, ``Content-Length`` /
  ``chunked`` / read-to-close bodies) that completes a future with
  ``(status, body bytes)``;
* a request that dies on a *reused* connection before any response byte
  arrived (the server closed an idle keep-alive socket) is retried once on a
  fresh connection, as Go's ``net/http`` does; the operator's writes are
  idempotent anyway (deterministic names, merge patches).

Watch streams (:meth:`HttpPool.open_stream`) get a dedicated connection whose
protocol de-chunks the body, splits it into lines and decodes each line as it
arrives, so an informer receives ready-made events in batches (no per-line
stream-reader round trips).

With the ``_netconn`` extension (``ops/csrc/netconn.cpp``) the connections
themselves are native: the pool dials the socket and hands it over, and the
loop calls the native connection straight from its selector -- receive,
framing, de-chunking, line splitting and TLS (OpenSSL, configured by the same
``ssl.SSLContext``) run in C++; through an http proxy the pool dials the proxy
(a ``CONNECT`` tunnel first for TLS servers) and hands that socket over.  The
asyncio protocols below remain for builds without the extension
(``CRON_OPERATOR_NATIVE_HTTP=python``) and as the behavioural oracle of the native
path's tests.
"""
from __future__ import annotations

import asyncio
import base64
import socket as _socket
import ssl as _ssl
from collections import deque
from typing import Any, Deque, Dict, List, Optional, Tuple
from urllib.parse import unquote, urlsplit

from ..ops import httpcodec_native

_codec = httpcodec_native.load()  # native response framing (ops/csrc/httpcodec.cpp), else None


class ConnectionFailed(Exception):
    """The connection broke; ``no_response`` + ``reused`` tell whether a retry is safe."""

    def __init__(self, msg: str, no_response: bool, reused: bool):
        super().__init__(msg)
        self.no_response = no_response
        self.reused = reused


class _Conn(asyncio.Protocol):
    __slots__ = ("transport", "buf", "fut", "alive", "used", "_state", "_status", "_clen", "_chunked",
                 "_close_after", "_body", "_got_any", "retry_after", "ssl_gen", "deadline")

    def __init__(self) -> None:
        self.transport: Optional[asyncio.Transport] = None
        self.buf = bytearray()
        self.fut: Optional[asyncio.Future] = None
        self.alive = True
        self.used = 0
        self.ssl_gen = 0         # HttpPool TLS-context generation this connection was made with
        self.deadline = 0.0      # loop time by which the in-flight response must have arrived
        self._reset()

    def _reset(self) -> None:
        self.retry_after: Optional[int] = None   # Retry-After of the last response (seconds)
        self._state = 0          # 0 headers, 1 body by length, 2 chunked, 3 until close
        self._status = 0
        self._clen = -1
        self._chunked = False
        self._close_after = False
        self._body = bytearray()
        self._got_any = False

    # --------------------------------------------------------------- protocol
    def connection_made(self, transport: asyncio.BaseTransport) -> None:
        self.transport = transport  # type: ignore[assignment]

    def connection_lost(self, exc: Optional[BaseException]) -> None:
        self.alive = False
        fut = self.fut
        if fut is not None and not fut.done():
            if self._state == 3:
                self._finish()
                return
            fut.set_exception(ConnectionFailed(f"connection lost: {exc or 'closed by peer'}",
                                               not self._got_any, self.used > 1))

    def eof_received(self) -> Optional[bool]:
        return False

    def data_received(self, data: bytes) -> None:
        self._got_any = True
        self.buf += data
        try:
            self._parse()
        except Exception as e:  # noqa: BLE001 - malformed response
            self.alive = False
            if self.fut is not None and not self.fut.done():
                self.fut.set_exception(ConnectionFailed(f"bad HTTP response: {e}", False, False))
            if self.transport is not None:
                self.transport.close()

    def _parse(self) -> None:
        if _codec is not None and self._state == 0:
            r = _codec.parse_response(self.buf)
            if r is None:
                return
            if r.__class__ is tuple:
                self._status, self._body, consumed, self._close_after, self.retry_after = r
                del self.buf[:consumed]
                self._finish()
                return
            # -1: an interim 1xx or a read-until-close body: the incremental parser below
        self._parse_py()

    def _parse_py(self) -> None:
        buf = self.buf
        while True:
            if self._state == 0:
                end = buf.find(b"\r\n\r\n")
                if end < 0:
                    return
                head = bytes(buf[:end]).decode("latin-1")
                del buf[:end + 4]
                lines = head.split("\r\n")
                parts = lines[0].split(" ", 2)
                self._status = int(parts[1])
                clen = -1
                chunked = False
                retry_after: Optional[int] = None
                close = parts[0] == "HTTP/1.0"
                for line in lines[1:]:
                    k, _, v = line.partition(":")
                    k = k.strip().lower()
                    if k == "content-length":
                        clen = int(v.strip())
                    elif k == "transfer-encoding":
                        chunked = "chunked" in v.lower()
                    elif k == "connection":
                        lv = v.strip().lower()
                        close = lv == "close" if lv in ("close", "keep-alive") else close
                    elif k == "retry-after":
                        try:
                            retry_after = int(v.strip())
                        except ValueError:
                            retry_after = None
                self._close_after = close
                self.retry_after = retry_after if self._status >= 400 else None
                if self._status in (204, 304) or 100 <= self._status < 200:
                    if 100 <= self._status < 200:  # interim response: parse the next head
                        continue
                    self._finish()
                    return
                if chunked:
                    self._state = 2
                elif clen >= 0:
                    self._clen = clen
                    self._state = 1
                else:
                    self._state = 3
                    self._close_after = True
            if self._state == 1:
                if len(buf) < self._clen:
                    return
                self._body = buf[:self._clen]
                del buf[:self._clen]
                self._finish()
                return
            if self._state == 2:
                while True:
                    nl = buf.find(b"\r\n")
                    if nl < 0:
                        return
                    size = int(bytes(buf[:nl]).split(b";", 1)[0], 16)
                    if size == 0:
                        # trailers end with an empty line
                        end = buf.find(b"\r\n\r\n", nl)
                        if end < 0:
                            if len(buf) >= nl + 4 and buf[nl:nl + 4] == b"\r\n\r\n":
                                end = nl
                            else:
                                return
                        del buf[:end + 4]
                        self._finish()
                        return
                    if len(buf) < nl + 2 + size + 2:
                        return
                    self._body += buf[nl + 2:nl + 2 + size]
                    del buf[:nl + 2 + size + 2]
            if self._state == 3:
                self._body += buf
                buf.clear()
                return

    def _finish(self) -> None:
        fut = self.fut
        status, body, ra = self._status, bytes(self._body), self.retry_after
        if self._close_after:
            self.alive = False
            if self.transport is not None:
                self.transport.close()
        self._reset()
        self.fut = None
        if fut is not None and not fut.done():
            fut.set_result((status, body, ra))

    # --------------------------------------------------------------- client side
    def send(self, data: bytes) -> asyncio.Future:
        loop = asyncio.get_running_loop()
        self.fut = loop.create_future()
        self.used += 1
        self._got_any = False
        assert self.transport is not None
        self.transport.write(data)
        return self.fut

    def close(self) -> None:
        if self.transport is not None:
            self.transport.close()

    def closing(self) -> bool:
        return self.transport is None or self.transport.is_closing()


class HttpStatusError(Exception):
    """A streaming request was answered with an error status."""

    def __init__(self, status: int, body: bytes):
        super().__init__(f"HTTP {status}")
        self.status = status
        self.body = body


class _StreamConn(asyncio.Protocol):
    """One streaming response (chunked or read-to-close), split into decoded lines."""

    def __init__(self, decode):
        self.decode = decode
        self.transport: Optional[asyncio.Transport] = None
        self.buf = bytearray()
        self.lines = bytearray()
        self.items: Deque = deque()
        self.ready = asyncio.Event()
        self.head: Optional[asyncio.Future] = None
        self.status = 0
        self.chunked = False
        self.done = False
        self.error: Optional[BaseException] = None
        self._err_body = bytearray()
        self._clen = -1

    def connection_made(self, transport: asyncio.BaseTransport) -> None:
        self.transport = transport  # type: ignore[assignment]

    def connection_lost(self, exc: Optional[BaseException]) -> None:
        self.done = True
        if self.head is not None and not self.head.done():
            if self.status >= 400:
                self.head.set_exception(HttpStatusError(self.status, bytes(self._err_body)))
            else:
                self.head.set_exception(ConnectionFailed(f"stream closed: {exc or 'by peer'}", True, False))
        self.ready.set()

    def data_received(self, data: bytes) -> None:
        self.buf += data
        try:
            self._parse()
        except Exception as e:  # noqa: BLE001 - malformed stream: end it
            self.error = e
            self.done = True
            self.ready.set()
            if self.transport is not None:
                self.transport.close()

    def _parse(self) -> None:
        buf = self.buf
        if self.status == 0:
            end = buf.find(b"\r\n\r\n")
            if end < 0:
                return
            lines = bytes(buf[:end]).decode("latin-1").split("\r\n")
            del buf[:end + 4]
            self.status = int(lines[0].split(" ", 2)[1])
            for line in lines[1:]:
                k, _, v = line.partition(":")
                k = k.strip().lower()
                if k == "transfer-encoding" and "chunked" in v.lower():
                    self.chunked = True
                elif k == "content-length":
                    self._clen = int(v.strip())
            if self.status < 400 and self.head is not None and not self.head.done():
                self.head.set_result(self.status)
        if self.status >= 400:  # collect the error body, then fail the open
            self._err_body += self._dechunk() if self.chunked else bytes(buf)
            if not self.chunked:
                buf.clear()
            if (self._clen >= 0 and len(self._err_body) >= self._clen) or self.done:
                if self.head is not None and not self.head.done():
                    self.head.set_exception(HttpStatusError(self.status, bytes(self._err_body)))
            return
        self.lines += self._dechunk() if self.chunked else bytes(buf)
        if not self.chunked:
            buf.clear()
        got = False
        while True:
            nl = self.lines.find(b"\n")
            if nl < 0:
                break
            line = bytes(self.lines[:nl]).strip()
            del self.lines[:nl + 1]
            if line:
                self.items.append(self.decode(line))
                got = True
        if got:
            self.ready.set()

    def _dechunk(self) -> bytes:
        buf = self.buf
        out = bytearray()
        while True:
            nl = buf.find(b"\r\n")
            if nl < 0:
                break
            size = int(bytes(buf[:nl]).split(b";", 1)[0], 16)
            if size == 0:
                self.done = True
                del buf[:]
                break
            if len(buf) < nl + 2 + size + 2:
                break
            out += buf[nl + 2:nl + 2 + size]
            del buf[:nl + 2 + size + 2]
        return bytes(out)

    def close(self) -> None:
        self.done = True
        self.ready.set()
        if self.transport is not None:
            self.transport.close()


class Stream:
    """Async iterator over a streaming response's decoded lines."""

    def __init__(self, conn: _StreamConn):
        self._c = conn

    def __aiter__(self) -> "Stream":
        return self

    async def __anext__(self):
        c = self._c
        while not c.items:
            if c.done:
                raise StopAsyncIteration
            c.ready.clear()
            if c.items or c.done:
                continue
            await c.ready.wait()
        if c.error is not None and not c.items:
            raise StopAsyncIteration
        return c.items.popleft()

    def take_ready(self) -> list:
        """Every item decoded so far, without waiting (an informer applies a whole batch per
        wake-up instead of one coroutine round trip per event)."""
        items = self._c.items
        if not items:
            return []
        out = list(items)
        items.clear()
        return out

    async def wait_ready(self) -> bool:
        """Wait until items are ready (True) or the stream ended (False)."""
        c = self._c
        while not c.items:
            if c.done:
                return False
            c.ready.clear()
            if c.items or c.done:
                continue
            await c.ready.wait()
        return True

    def close(self) -> None:
        self._c.close()


class NativeStream(Stream):
    """:class:`Stream` over a native connection in stream mode (``_netconn.Conn``)."""

    def __init__(self, conn) -> None:  # noqa: D107 - no _StreamConn here
        self._n = conn

    async def __anext__(self):
        n = self._n
        while not n.pending:
            if n.done:
                raise StopAsyncIteration
            w = n.wait()
            if w is not None:
                await w
        return n.take_one()

    def take_ready(self) -> list:
        return self._n.take()

    async def wait_ready(self) -> bool:
        n = self._n
        while not n.pending:
            if n.done:
                return False
            w = n.wait()
            if w is not None:
                await w
        return True

    def close(self) -> None:
        self._n.close()


# TCP keepalive on every connection (Go's net.Dialer probes after 30 s idle): a peer that
# vanished without a FIN -- node loss, a dropped NAT entry -- is detected in about a minute
# instead of never on a long-lived watch connection
KEEPALIVE_IDLE = 30
KEEPALIVE_INTERVAL = 10
KEEPALIVE_COUNT = 3


def enable_keepalive(transport: Optional[asyncio.BaseTransport]) -> bool:
    sock = transport.get_extra_info("socket") if transport is not None else None
    if sock is None:
        return False
    return keepalive_socket(sock)


def keepalive_socket(sock) -> bool:
    try:
        sock.setsockopt(_socket.SOL_SOCKET, _socket.SO_KEEPALIVE, 1)
        for opt, val in (("TCP_KEEPIDLE", KEEPALIVE_IDLE), ("TCP_KEEPINTVL", KEEPALIVE_INTERVAL),
                         ("TCP_KEEPCNT", KEEPALIVE_COUNT)):
            if hasattr(_socket, opt):
                sock.setsockopt(_socket.IPPROTO_TCP, getattr(_socket, opt), val)
    except OSError:
        return False
    return True


def _expire(fut: asyncio.Future) -> None:
    if not fut.done():
        fut.set_exception(asyncio.TimeoutError())


# default of HttpPool(native=None): None picks the native connections whenever they can serve
# the pool; False keeps the asyncio protocols (tests run the pool both ways)
DEFAULT_NATIVE: Optional[bool] = None

# request deadlines are checked by one sweep timer per pool instead of a timer per request
# (a TimerHandle, a heap push and a cancel on every call); the sweep runs at most this often,
# and at least four times per timeout
SWEEP_INTERVAL = 1.0


class _Tunnel(asyncio.Protocol):
    """Reads a proxy's answer to ``CONNECT``; ``done`` resolves to its status code."""

    def __init__(self) -> None:
        self.done: asyncio.Future = asyncio.get_running_loop().create_future()
        self.buf = bytearray()

    def data_received(self, data: bytes) -> None:
        self.buf += data
        end = self.buf.find(b"\r\n\r\n")
        if end >= 0 and not self.done.done():
            line = bytes(self.buf[:self.buf.find(b"\r\n")]).split(b" ", 2)
            try:
                self.done.set_result(int(line[1]))
            except (IndexError, ValueError):
                self.done.set_exception(ConnectionFailed("bad proxy response", True, False))

    def connection_lost(self, exc: Optional[BaseException]) -> None:
        if not self.done.done():
            self.done.set_exception(ConnectionFailed(f"proxy closed the connection: {exc}", True, False))


class HttpPool:
    """Keep-alive connection pool to one ``scheme://host:port``."""

    def __init__(self, base_url: str, ssl_context: Optional[_ssl.SSLContext] = None,
                 headers: Optional[Dict[str, str]] = None, max_idle: int = 64, timeout: float = 60.0,
                 server_hostname: Optional[str] = None, proxy: str = "", native: Optional[bool] = None,
                 tls_material: Optional[Dict[str, Any]] = None):
        """``native``: use ``_netconn`` connections (None: whenever the extension is built and it
        can drive the TLS context; True: required).  ``tls_material``: the PEM material behind
        ``ssl_context`` (``RestConfig.tls_material``): native TLS then runs on an ``SSL_CTX`` the
        extension builds itself (``_netconn.TlsContext``) instead of the ``ssl.SSLContext``'s."""
        u = urlsplit(base_url)
        self.scheme = u.scheme or "http"
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or (443 if self.scheme == "https" else 80)
        self.base_path = (u.path or "").rstrip("/")
        self.ssl = ssl_context if self.scheme == "https" else None
        if self.scheme == "https" and self.ssl is None:
            self.ssl = _ssl.create_default_context()
        self.server_hostname = server_hostname
        self._hosthdr = self.host if (self.port in (80, 443)) else f"{self.host}:{self.port}"
        self._proxy: Optional[Tuple[str, int]] = None
        self._proxy_auth = ""
        self._target = self.base_path  # request-target prefix: absolute form through an http proxy
        if proxy:
            pu = urlsplit(proxy if "://" in proxy else "http://" + proxy)
            if pu.scheme != "http":
                raise ValueError(f"proxy {proxy!r}: only http:// proxies are supported")
            self._proxy = (pu.hostname or "127.0.0.1", pu.port or 80)
            if pu.username is not None:
                cred = f"{unquote(pu.username)}:{unquote(pu.password or '')}".encode()
                self._proxy_auth = f"Proxy-Authorization: Basic {base64.b64encode(cred).decode()}\r\n"
            if self.scheme == "http":
                self._target = f"http://{self._hosthdr}{self.base_path}"
        self._np = None  # the native pool (request path in C++) when the native connections serve
        self._tls_material = tls_material if self.scheme == "https" else None
        self._native_tls: Any = None  # _netconn.TlsContext built from _tls_material
        self.set_headers(headers)
        self._pidle: Deque[_Conn] = deque()
        self.max_idle = max_idle
        self.timeout = timeout
        self.connects = 0
        self._closed = False
        self._ssl_gen = 0
        self._busy: set = set()   # connections with a request in flight (deadline sweep)
        self._sweeper: Optional[asyncio.TimerHandle] = None
        self._sweep_every = min(SWEEP_INTERVAL, max(0.01, timeout / 4))
        self._want_native = native if native is not None else DEFAULT_NATIVE
        self.native = False
        self._pick_native()

    @property
    def _idle(self) -> List[Any]:
        """The idle keep-alive connections (the native pool's, or the asyncio protocols')."""
        return self._np.idle() if self._np is not None else self._pidle  # type: ignore[return-value]

    def _pick_native(self) -> None:
        from ..ops import netconn_native

        want = self._want_native
        mod = netconn_native.load() if want is not False else None
        self._native_tls = None
        if mod is not None and self.ssl is not None and self._tls_material is not None:
            self._native_tls = netconn_native.tls_context(self._tls_material)
        ok = mod is not None and (self.ssl is None or self._native_tls is not None
                                  or mod.ssl_context_supported(self.ssl))
        if want and not ok:
            raise RuntimeError("native HTTP connections unavailable for this pool "
                               f"(extension {'missing' if mod is None else 'loaded'})")
        self._netconn = mod if ok else None
        self.native = ok
        if ok and self._np is None:
            self._np = mod.Pool(self.max_idle, self.timeout)
            self._np.set_fixed(self._target, self._fixed)
        if self._np is not None:
            self._np.ssl_gen = self._ssl_gen
            if not ok:  # the new TLS context needs the asyncio protocols: retire the native pool
                self._np.close()
                self._np = None

    def set_headers(self, headers: Optional[Dict[str, str]]) -> None:
        """Replace the headers sent with every request (e.g. a rotated ``Authorization``)."""
        hdrs = {"User-Agent": "cron-operator-amd"}
        hdrs.update({k: v for k, v in (headers or {}).items() if k.lower() != "accept"})
        extra = "".join(f"{k}: {v}\r\n" for k, v in hdrs.items())
        if self._proxy is not None and self.scheme == "http":
            extra += self._proxy_auth  # plain requests go to the proxy itself
        self._fixed = f"Host: {self._hosthdr}\r\n{extra}"
        if self._np is not None:
            self._np.set_fixed(self._target, self._fixed)

    def set_ssl(self, ctx: _ssl.SSLContext, tls_material: Optional[Dict[str, Any]] = None) -> None:
        """New connections handshake with ``ctx`` (a rotated client certificate); idle
        connections made with the old one are closed, busy ones when they are given back."""
        self.ssl = ctx
        self._tls_material = tls_material
        self._ssl_gen += 1
        self._pick_native()
        if self._np is not None:
            self._np.close_idle()
        while self._pidle:
            self._pidle.pop().close()

    async def _open(self, factory):
        """A connected protocol from ``factory``: direct, to an http proxy (plain servers), or
        through a ``CONNECT`` tunnel to the server with TLS on top (https servers)."""
        loop = asyncio.get_running_loop()
        if self._proxy is None or self.ssl is None:
            kw = {}
            if self.ssl is not None:
                kw["ssl"] = self.ssl
                kw["server_hostname"] = self.server_hostname or self.host
            host, port = self._proxy or (self.host, self.port)
            tr, proto = await asyncio.wait_for(loop.create_connection(factory, host, port, **kw), self.timeout)
            enable_keepalive(tr)
            return proto
        transport, tun = await asyncio.wait_for(loop.create_connection(_Tunnel, *self._proxy), self.timeout)
        enable_keepalive(transport)
        authority = f"{self.host}:{self.port}" if ":" not in self.host else f"[{self.host}]:{self.port}"
        transport.write(f"CONNECT {authority} HTTP/1.1\r\nHost: {authority}\r\n{self._proxy_auth}\r\n"
                        .encode("latin-1"))
        try:
            status = await asyncio.wait_for(tun.done, self.timeout)
            if status != 200:
                raise ConnectionFailed(f"proxy CONNECT {authority}: HTTP {status}", True, False)
            proto = factory()
            tls = await asyncio.wait_for(loop.start_tls(transport, proto, self.ssl,
                                                        server_hostname=self.server_hostname or self.host),
                                         self.timeout)
        except BaseException:
            transport.close()
            raise
        proto.connection_made(tls)
        return proto

    async def _connect(self) -> _Conn:
        gen = self._ssl_gen
        if self._netconn is not None:
            proto = await asyncio.wait_for(self._open_native(), self.timeout)
        else:
            proto = await self._open(_Conn)
        proto.ssl_gen = gen
        self.connects += 1
        return proto

    async def _dial(self) -> _socket.socket:
        """A connected non-blocking TCP socket to the server -- or, through an http proxy, to the
        proxy (a TLS server behind it gets a ``CONNECT`` tunnel first) -- with addresses tried in
        order like Go's dialer without a fallback delay; TCP_NODELAY and keepalive probes on."""
        host, port = self._proxy or (self.host, self.port)
        sock = await self._dial_addr(host, port)
        if self._proxy is not None and self.ssl is not None:
            try:
                await self._connect_tunnel(sock)
            except BaseException:
                sock.close()
                raise
        return sock

    async def _connect_tunnel(self, sock: _socket.socket) -> None:
        """``CONNECT host:port`` on a fresh proxy connection; returns once the proxy answered 200
        (the socket then carries the TLS session to the server)."""
        loop = asyncio.get_running_loop()
        authority = f"{self.host}:{self.port}" if ":" not in self.host else f"[{self.host}]:{self.port}"
        await loop.sock_sendall(sock, f"CONNECT {authority} HTTP/1.1\r\nHost: {authority}\r\n{self._proxy_auth}\r\n"
                                .encode("latin-1"))
        buf = b""
        while b"\r\n\r\n" not in buf:
            chunk = await loop.sock_recv(sock, 4096)
            if not chunk:
                raise ConnectionFailed("proxy closed the connection", True, False)
            buf += chunk
            if len(buf) > 65536:
                raise ConnectionFailed("bad proxy response", True, False)
        # a proxy answers CONNECT with a head only: nothing of the tunnel follows before our hello
        line = buf.split(b"\r\n", 1)[0].split(b" ", 2)
        try:
            status = int(line[1])
        except (IndexError, ValueError):
            raise ConnectionFailed("bad proxy response", True, False) from None
        if status != 200:
            raise ConnectionFailed(f"proxy CONNECT {authority}: HTTP {status}", True, False)

    async def _dial_addr(self, host: str, port: int) -> _socket.socket:
        loop = asyncio.get_running_loop()
        infos = await loop.getaddrinfo(host, port, type=_socket.SOCK_STREAM)
        err: Optional[BaseException] = None
        for family, type_, proto, _, addr in infos:
            sock = _socket.socket(family, type_, proto)
            try:
                sock.setblocking(False)
                await loop.sock_connect(sock, addr)
            except OSError as e:
                sock.close()
                err = e
                continue
            except BaseException:
                sock.close()
                raise
            try:
                sock.setsockopt(_socket.IPPROTO_TCP, _socket.TCP_NODELAY, 1)
            except OSError:
                pass
            keepalive_socket(sock)
            return sock
        raise err if err is not None else OSError(f"no address for {host}:{port}")

    async def _open_native(self):
        """A native connection (``_netconn.Conn``), TLS handshake done."""
        loop = asyncio.get_running_loop()
        sock = await self._dial()
        ctx = self.ssl
        try:
            if ctx is None:
                conn = self._netconn.Conn(loop, sock.fileno())
            else:
                # the extension's own SSL_CTX when it has the PEM material; the hostname policy
                # is the ssl.SSLContext's either way
                conn = self._netconn.Conn(loop, sock.fileno(), self._native_tls or ctx,
                                          self.server_hostname or self.host, ctx.check_hostname,
                                          ctx.hostname_checks_common_name)
        except BaseException:
            sock.close()
            raise
        sock.detach()  # the connection owns the descriptor now
        if ctx is not None:
            try:
                await conn.handshake()
            except BaseException:
                conn.close()
                raise
        return conn

    def _take_idle(self) -> Optional[_Conn]:
        while self._pidle:
            c = self._pidle.pop()
            if c.alive and not c.closing():
                return c
        return None

    def _give_back(self, c: _Conn) -> None:
        if c.alive and not self._closed and len(self._pidle) < self.max_idle and c.fut is None \
                and c.ssl_gen == self._ssl_gen:
            self._pidle.append(c)
        else:
            c.close()

    async def request(self, method: str, path: str, body: Optional[bytes] = None,
                      content_type: str = "application/json") -> Tuple[int, bytes]:
        status, raw, _ = await self.request_full(method, path, body, content_type)
        return status, raw

    def start(self, method: str, path: str, body: Optional[bytes] = None, content_type: str = "application/json",
              accept: str = "application/json") -> Optional["asyncio.Future[Tuple[int, bytes, Optional[int]]]"]:
        """The native pool's request on an idle connection, sent now: the response future, or
        None (no native pool, or nothing idle -- use :meth:`request_full`).  A caller awaiting
        it retries a ``ConnectionFailed(no_response, reused)`` once with ``request_full(...,
        fresh=True)`` and, when cancelled, hands the future to :meth:`discard`."""
        np = self._np
        if np is None:
            return None
        fut = np.request(method, path, body, content_type, accept)
        if fut is not None and self._sweeper is None:
            self._sweeper = asyncio.get_running_loop().call_later(self._sweep_every, self._sweep)
        return fut

    def discard(self, fut: "asyncio.Future[Any]") -> None:
        """The request of ``fut`` (from :meth:`start`) was abandoned: close its connection."""
        if self._np is not None:
            self._np.discard(fut)

    async def request_full(self, method: str, path: str, body: Optional[bytes] = None,
                           content_type: str = "application/json",
                           accept: str = "application/json", fresh: bool = False) -> Tuple[int, bytes, Optional[int]]:
        """``(status, body, Retry-After seconds or None)``.  ``fresh``: on a new connection."""
        np = self._np
        if np is not None:
            # native pool: head built, idle connection taken, sent, and given back when the
            # response completes -- all in C++; Python only connects when no connection is idle
            fut = None if fresh else np.request(method, path, body, content_type, accept)
            if fut is None:
                fut = np.request_on(await self._connect(), method, path, body, content_type, accept)
            if self._sweeper is None:
                self._sweeper = asyncio.get_running_loop().call_later(self._sweep_every, self._sweep)
            try:
                return await fut
            except ConnectionFailed as e:
                if not (e.no_response and e.reused):
                    raise
            except asyncio.CancelledError:
                np.discard(fut)  # abandoned mid-exchange: the connection cannot be reused
                raise
            # a stale keep-alive connection: once more on a fresh one
            fut = np.request_on(await self._connect(), method, path, body, content_type, accept)
            try:
                return await fut
            except asyncio.CancelledError:
                np.discard(fut)
                raise
        head = f"{method} {self._target}{path} HTTP/1.1\r\n{self._fixed}Accept: {accept}\r\n"
        if body is not None:
            head += f"Content-Type: {content_type}\r\nContent-Length: {len(body)}\r\n\r\n"
            data = head.encode("latin-1") + body
        else:
            data = (head + ("Content-Length: 0\r\n\r\n" if method in ("POST", "PUT", "PATCH") else "\r\n")
                    ).encode("latin-1")
        loop = asyncio.get_running_loop()
        for attempt in ((1,) if fresh else (0, 1)):
            conn = self._take_idle() if attempt == 0 else None
            if conn is None:
                conn = await self._connect()
            fut = conn.send(data)
            conn.deadline = loop.time() + self.timeout
            self._busy.add(conn)
            if self._sweeper is None:
                self._sweeper = loop.call_later(self._sweep_every, self._sweep)
            try:
                status, raw, retry_after = await fut
            except ConnectionFailed as e:
                conn.alive = False
                conn.close()
                if attempt == 0 and e.no_response and e.reused:
                    continue  # stale keep-alive connection: retry once on a fresh one
                raise
            except BaseException:  # deadline (TimeoutError), cancellation, anything else
                conn.alive = False
                conn.close()
                raise
            finally:
                self._busy.discard(conn)
            self._give_back(conn)
            return status, raw, retry_after
        raise ConnectionFailed("unreachable", True, False)  # pragma: no cover

    def _sweep(self) -> None:
        """Fail every in-flight request past its deadline; re-arm while any is in flight."""
        self._sweeper = None
        np = self._np
        if not self._busy and (np is None or not np.busy):
            return
        loop = asyncio.get_running_loop()
        now = loop.time()
        for c in [c for c in self._busy if c.deadline <= now]:
            if c.fut is not None:
                _expire(c.fut)
        if self._busy or (np is not None and np.sweep(now)):
            self._sweeper = loop.call_later(self._sweep_every, self._sweep)

    async def open_stream(self, path: str, decode, accept: str = "application/json") -> Stream:
        """GET ``path`` on a dedicated connection and stream its body line by line
        (``decode`` turns each non-empty line into an item).  Raises
        :class:`HttpStatusError` for an error status."""
        if self._netconn is not None:
            nc = await asyncio.wait_for(self._open_native(), self.timeout)
            try:
                head = nc.open_stream(f"GET {self._target}{path} HTTP/1.1\r\n{self._fixed}Accept: {accept}\r\n\r\n"
                                      .encode("latin-1"), decode)
                await asyncio.wait_for(head, self.timeout)
            except BaseException:
                nc.close()
                raise
            return NativeStream(nc)
        conn = await self._open(lambda: _StreamConn(decode))
        conn.head = asyncio.get_running_loop().create_future()
        assert conn.transport is not None
        conn.transport.write(f"GET {self._target}{path} HTTP/1.1\r\n{self._fixed}Accept: {accept}\r\n\r\n"
                             .encode("latin-1"))
        try:
            await asyncio.wait_for(conn.head, self.timeout)
        except BaseException:
            conn.close()
            raise
        return Stream(conn)

    async def close(self) -> None:
        self._closed = True
        if self._sweeper is not None:
            self._sweeper.cancel()
            self._sweeper = None
        if self._np is not None:
            self._np.close()
        while self._pidle:
            self._pidle.pop().close()


def encode_query(params: Dict[str, str]) -> str:
    if not params:
        return ""
    from urllib.parse import urlencode

    return "?" + urlencode(params)


__all__: List[str] = ["HttpPool", "ConnectionFailed", "HttpStatusError", "Stream", "NativeStream", "encode_query"]
