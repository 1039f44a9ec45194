"""HTTP transport: the Kubernetes REST protocol.

Works against a real kube-apiserver (kubeconfig / in-cluster config) and the
framework's fake apiserver served by :mod:`cron_operator_amd.apiserver.http`.
Requests, watch streams and discovery go through the lean keep-alive pool of
:mod:`.fasthttp` (``fast=True``, the default) or aiohttp (``fast=False``, imported only
then: it costs a process ~13 MiB); aiohttp watch streams are read line by line
(newline-delimited JSON) with a large line limit so big objects fit.
"""
from __future__ import annotations

import asyncio
import json
import re
from typing import TYPE_CHECKING, Any, Dict, List, Optional, Tuple
from urllib.parse import quote

from ..api import errors
from ..api.meta import GroupVersion, GroupVersionResource
from ..utils import jsonutil
from . import metrics
from .client import ACCEPT, DECODE, DISCARD, PATCH_CONTENT_TYPES, Transport, WatchStream
from .fasthttp import ConnectionFailed, HttpPool, HttpStatusError, Stream, encode_query
from .kubeconfig import RestConfig

if TYPE_CHECKING:
    import aiohttp


_PREFIXES: Dict[Tuple[GroupVersionResource, str], str] = {}
# characters quote(..., safe="") leaves alone: a Kubernetes name (DNS-1123) never needs quoting
_UNRESERVED = re.compile(r"[A-Za-z0-9._~-]+").fullmatch


def resource_path(gvr: GroupVersionResource, namespace: str = "", name: str = "", sub: str = "") -> str:
    """The REST path of a resource (collection when ``name`` is empty).  The collection
    prefix is memoised per (resource, namespace); names are only quoted when they need it
    (a per-name memo would grow with every job ever deleted)."""
    key = (gvr, namespace)
    base = _PREFIXES.get(key)
    if base is None:
        if len(_PREFIXES) >= 4096:
            _PREFIXES.clear()
        base = _PREFIXES[key] = _collection_path(gvr, namespace)
    if name:
        base += "/" + (name if _UNRESERVED(name) else quote(name, safe=""))
    if sub:
        base += "/" + sub
    return base


def _collection_path(gvr: GroupVersionResource, namespace: str) -> str:
    base = f"/api/{gvr.version}" if not gvr.group else f"/apis/{gvr.group}/{gvr.version}"
    if namespace:
        base += f"/namespaces/{quote(namespace, safe='')}"
    return base + f"/{gvr.resource}"


def _clean(params: Optional[Dict[str, Any]]) -> Dict[str, str]:
    out: Dict[str, str] = {}
    if not params:
        return out
    for k, v in params.items():
        if k == "patchType" or k.startswith("_") or v is None or v == "":
            continue
        out[k] = str(v)
    return out


class _HttpWatch(WatchStream):
    def __init__(self, resp: aiohttp.ClientResponse, decoder: Any = None):
        self._resp = resp
        self._done = False
        self._decode = decoder or _decode_event

    async def __anext__(self) -> Tuple[str, Dict[str, Any]]:
        import aiohttp

        if self._done:
            raise StopAsyncIteration
        while True:
            try:
                line = await self._resp.content.readline()
            except (aiohttp.ClientError, asyncio.TimeoutError, ValueError):
                self.stop()
                raise StopAsyncIteration
            if not line:
                self.stop()
                raise StopAsyncIteration
            line = line.strip()
            if not line:
                continue
            return self._decode(line)

    def stop(self) -> None:
        if not self._done:
            self._done = True
            self._resp.close()


_NO_PARAMS: Dict[str, Any] = {}  # read-only
_COLLECTION_VERBS = frozenset(("list", "create", "deletecollection"))
_METHODS = {"get": "GET", "list": "GET", "create": "POST", "update": "PUT", "patch": "PATCH",
            "delete": "DELETE", "deletecollection": "DELETE"}


def _decode_event(line: bytes) -> Tuple[str, Dict[str, Any]]:
    ev = jsonutil.loads(line)
    return ev.get("type", ""), ev.get("object") or {}


class _FastWatch(WatchStream):
    def __init__(self, stream: Stream):
        self._s = stream

    def __anext__(self):  # the stream's own awaitable: no extra coroutine frame per event
        return self._s.__anext__()

    def take_ready(self) -> List[Tuple[str, Dict[str, Any]]]:
        return self._s.take_ready()

    def wait_ready(self):
        return self._s.wait_ready()

    def stop(self) -> None:
        self._s.close()


def _status_error(status: int, raw: bytes) -> errors.ApiError:
    try:
        body: Any = jsonutil.loads(raw)
    except ValueError:
        body = raw.decode(errors="replace")
    return errors.ApiError.from_status(status, body)


class HttpTransport(Transport):
    def __init__(self, config: RestConfig, pool_size: int = 64, timeout: float = 60.0, fast: bool = True,
                 max_retries: int = 10):
        self.config = config
        # client-go rest.Request: a 429/5xx carrying Retry-After is retried after that many seconds,
        # up to maxRetries (10) times -- how an apiserver under API Priority and Fairness sheds load
        self.max_retries = max_retries
        self.retries = 0
        # set by a Client that retries itself (Client._do): each retry then goes through the QPS
        # bucket and the in-flight gate again, and no gate slot is held while Retry-After elapses
        self.retry_in_client = False
        self.host = config.host.split("://", 1)[-1]
        self._pool_size = pool_size
        self._timeout = timeout
        self._session: Optional[aiohttp.ClientSession] = None
        self.fast = fast
        self._pool: Optional[HttpPool] = None
        self._token = ""  # the bearer token the pool/session headers carry
        self._cert_generation = 0  # the exec-plugin client certificate the pool's TLS context holds
        # resolved once, at construction: a bad proxy fails (or is reported) at startup,
        # not on every request
        self._proxy: Optional[str] = config.proxy()
        self._exec_lock: Optional[asyncio.Lock] = None

    def _fast_pool(self) -> HttpPool:
        if self._pool is None:
            self._token = self.config.token()
            self._pool = HttpPool(self.config.host, ssl_context=self.config.ssl_context() or None,
                                  headers=self.config.auth_headers(self._token), max_idle=self._pool_size,
                                  timeout=self._timeout, server_hostname=self.config.tls_server_name or None,
                                  proxy=self._proxy or "", tls_material=self.config.tls_material())
            self._cert_generation = self.config.cert_generation
        elif self.config.rotating:
            self._rotate_token()
        return self._pool

    def _rotate_token(self) -> None:
        """Re-stamp ``Authorization`` when the token file's content or the exec plugin's token
        changed, and switch new connections to a rotated exec client certificate (client-go
        closes the old connections then; here idle ones are dropped, busy ones finish)."""
        tok = self.config.token()
        if self.config.cert_generation != self._cert_generation and self._pool is not None:
            self._cert_generation = self.config.cert_generation
            ctx = self.config.ssl_context()
            if ctx is not None:
                self._pool.set_ssl(ctx, self.config.tls_material())
        if tok == self._token:
            return
        self._token = tok
        hdrs = self.config.auth_headers(tok)
        if self._pool is not None:
            self._pool.set_headers(hdrs)
        if self._session is not None and not self._session.closed:
            self._session.headers.update(hdrs)

    async def _fresh_exec(self) -> None:
        """Run a stale exec credential plugin off the event loop, once for all waiting requests."""
        if self._exec_lock is None:
            self._exec_lock = asyncio.Lock()
        async with self._exec_lock:
            if self.config.exec_stale():
                await asyncio.get_running_loop().run_in_executor(None, self.config.refresh_exec)

    def _unauthorized(self) -> None:
        """A 401: drop the cached file token / exec credential so the next request refreshes it."""
        if self.config.rotating:
            self.config.reset_token()

    def _tls_kw(self) -> Dict[str, Any]:
        """Per-request aiohttp options: kubeconfig ``tls-server-name`` (verify the certificate
        against this name) and the proxy (kubeconfig ``proxy-url`` or the environment)."""
        kw: Dict[str, Any] = {}
        name = self.config.tls_server_name
        if name and self.config.host.startswith("https://"):
            kw["server_hostname"] = name
        if self._proxy:
            kw["proxy"] = self._proxy if "://" in self._proxy else "http://" + self._proxy
        return kw

    def _sess(self) -> aiohttp.ClientSession:
        import aiohttp

        if self.config.rotating and self._session is not None:
            self._rotate_token()
        if self._session is None or self._session.closed:
            self._token = self.config.token()
            conn = aiohttp.TCPConnector(limit=self._pool_size, ssl=self.config.ssl_context() or False,
                                        keepalive_timeout=120)
            self._session = aiohttp.ClientSession(connector=conn, headers=self.config.auth_headers(self._token),
                                                  read_bufsize=1 << 20, json_serialize=jsonutil.dumps)
        return self._session

    async def _raise(self, resp: aiohttp.ClientResponse) -> None:
        if resp.status == 401:
            self._unauthorized()
        raw = await resp.read()
        try:
            body: Any = json.loads(raw)
        except ValueError:
            body = raw.decode(errors="replace")
        raise errors.ApiError.from_status(resp.status, body)

    async def request(self, verb: str, gvr: GroupVersionResource, namespace: str = "", name: str = "",
                      subresource: str = "", body: Any = None, params: Optional[Dict[str, Any]] = None) -> Any:
        cfg = self.config
        if cfg.exec_provider is not None and cfg.exec_stale():
            await self._fresh_exec()
        params = params or _NO_PARAMS
        method = _METHODS[verb]
        path = resource_path(gvr, namespace, name if verb not in _COLLECTION_VERBS else "", subresource)
        if self.fast:
            data = body if body is None or body.__class__ is bytes else jsonutil.dumpb(body)
            if params:
                ctype = PATCH_CONTENT_TYPES[params.get("patchType", "merge")] if verb == "patch" else \
                    "application/json"
                q = _clean(params)
                target = path + encode_query(q) if q else path
                accept = params.get(ACCEPT) or "application/json"
            else:
                ctype = PATCH_CONTENT_TYPES["merge"] if verb == "patch" else "application/json"
                target, accept = path, "application/json"
            pool = self._pool if self._pool is not None and not cfg.rotating else self._fast_pool()
            attempt = 0
            while True:
                if attempt:
                    if cfg.exec_provider is not None and cfg.exec_stale():
                        await self._fresh_exec()  # expired while waiting out Retry-After: refresh off the loop
                    pool = self._fast_pool()  # a token rotated meanwhile is stamped on the retry
                # an idle native connection takes the request at once (no extra coroutine frame)
                fut = pool.start(method, target, data, ctype, accept)
                try:
                    if fut is not None:
                        try:
                            status, raw, retry_after = await fut
                        except ConnectionFailed as e:
                            if not (e.no_response and e.reused):
                                raise
                            # a stale keep-alive connection: once more on a fresh one
                            status, raw, retry_after = await pool.request_full(method, target, data, ctype, accept,
                                                                               fresh=True)
                        except asyncio.CancelledError:
                            pool.discard(fut)  # abandoned mid-exchange: the connection cannot be reused
                            raise
                    else:
                        status, raw, retry_after = await pool.request_full(method, target, data, ctype, accept)
                except (ConnectionFailed, OSError, asyncio.TimeoutError) as e:
                    raise errors.ApiError(503, "ServiceUnavailable", f"connection error: {e}") from None
                if retry_after is None or not (status == 429 or status >= 500) or attempt >= self.max_retries \
                        or self.retry_in_client:
                    break
                attempt += 1
                self.retries += 1
                metrics.REST_RETRIES.labels(str(status), method, self.host).inc()
                await asyncio.sleep(max(0, retry_after))
            if status >= 400:
                if status == 401:
                    self._unauthorized()
                try:
                    err_body: Any = jsonutil.loads(raw)
                except ValueError:
                    err_body = raw.decode(errors="replace")
                err = errors.ApiError.from_status(status, err_body)
                if err.retry_after is None and retry_after is not None:
                    err.retry_after = retry_after  # the Retry-After header (a Status body may omit it)
                raise err
            if params.get(DISCARD):
                return None
            if not raw:
                return None
            dec = params.get(DECODE)
            return dec.loads(raw) if dec is not None else jsonutil.loads(raw)
        import aiohttp

        url = self.config.host + path
        headers = {"Accept": params.get(ACCEPT) or "application/json"}
        data = None
        if body is not None:
            data = body if body.__class__ is bytes else jsonutil.dumpb(body)
            headers["Content-Type"] = PATCH_CONTENT_TYPES[params.get("patchType", "merge")] if verb == "patch" \
                else "application/json"
        timeout = aiohttp.ClientTimeout(total=self._timeout)
        try:
            async with self._sess().request(method, url, params=_clean(params), data=data, headers=headers,
                                            timeout=timeout, **self._tls_kw()) as resp:
                if resp.status >= 400:
                    await self._raise(resp)
                raw = await resp.read()
        except aiohttp.ClientConnectionError as e:
            raise errors.ApiError(503, "ServiceUnavailable", f"connection error: {e}") from None
        if not raw:
            return None
        dec = params.get(DECODE) if params else None
        return dec.loads(raw) if dec is not None else jsonutil.loads(raw)

    async def watch(self, gvr: GroupVersionResource, namespace: str = "",
                    params: Optional[Dict[str, Any]] = None, decoder: Any = None) -> WatchStream:
        if self.config.exec_provider is not None and self.config.exec_stale():
            await self._fresh_exec()
        p = _clean(params)
        p["watch"] = "true"
        if self.fast:
            try:
                stream = await self._fast_pool().open_stream(resource_path(gvr, namespace) + encode_query(p),
                                                             decoder or _decode_event)
            except HttpStatusError as e:
                if e.status == 401:
                    self._unauthorized()
                raise _status_error(e.status, e.body) from None
            except (ConnectionFailed, OSError, asyncio.TimeoutError) as e:
                raise errors.ApiError(503, "ServiceUnavailable", f"connection error: {e}") from None
            return _FastWatch(stream)
        import aiohttp

        url = self.config.host + resource_path(gvr, namespace)
        timeout = aiohttp.ClientTimeout(total=None, sock_connect=self._timeout)
        try:
            resp = await self._sess().get(url, params=p, timeout=timeout, **self._tls_kw())
        except aiohttp.ClientConnectionError as e:
            raise errors.ApiError(503, "ServiceUnavailable", f"connection error: {e}") from None
        if resp.status >= 400:
            try:
                await self._raise(resp)
            finally:
                resp.release()
        return _HttpWatch(resp, decoder)

    async def discover(self, group_version: GroupVersion) -> List[Dict[str, Any]]:
        if self.config.exec_provider is not None and self.config.exec_stale():
            await self._fresh_exec()
        path = f"/api/{group_version.version}" if not group_version.group else \
            f"/apis/{group_version.group}/{group_version.version}"
        if self.fast:
            try:
                status, raw, _ = await self._fast_pool().request_full("GET", path, None, "application/json",
                                                                      "application/json")
            except (ConnectionFailed, OSError, asyncio.TimeoutError) as e:
                raise errors.ApiError(503, "ServiceUnavailable", f"connection error: {e}") from None
            if status >= 400:
                if status == 401:
                    self._unauthorized()
                raise _status_error(status, raw)
            return (jsonutil.loads(raw) if raw else {}).get("resources") or []
        import aiohttp

        try:
            async with self._sess().get(self.config.host + path, **self._tls_kw()) as resp:
                if resp.status >= 400:
                    await self._raise(resp)
                doc = json.loads(await resp.read())
        except aiohttp.ClientConnectionError as e:
            raise errors.ApiError(503, "ServiceUnavailable", f"connection error: {e}") from None
        return doc.get("resources") or []

    async def close(self) -> None:
        if self._pool is not None:
            await self._pool.close()
            self._pool = None
        if self._session is not None:
            await self._session.close()
            self._session = None
