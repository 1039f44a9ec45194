"""Kubernetes API client: transports, REST mapping, throttling, request metrics.

Counterpart of the client-go/controller-runtime client the reference talks to
the apiserver with (the only process boundary).  Layers:

* :class:`Transport` -- raw verbs against one apiserver.  :class:`InMemoryTransport`
  calls the fake :class:`~cron_operator_amd.apiserver.server.APIServer` directly
  (tests, single-process bench); :class:`~cron_operator_amd.runtime.http.HttpTransport`
  speaks the Kubernetes REST protocol to any apiserver (real clusters, the fake
  apiserver served over HTTP).
* :class:`RESTMapper` -- GVK -> resource via discovery, cached.
* :class:`Client` -- typed-ish convenience on top: ``get/list/create/update/patch/
  delete/watch`` by GVR or GVK, a ``status`` sub-client (``client.Status()``),
  merge-patch from an old object (``client.MergeFrom``), the client-side token
  bucket (``--qps``/``--burst``) and ``rest_client_*`` metrics.
"""
from __future__ import annotations

import asyncio
import time
from typing import Any, Dict, List, Optional, Tuple, Union

from ..api import errors
from ..api.meta import GroupVersion, GroupVersionKind, GroupVersionResource
from ..utils import jsonutil
from ..utils.gotime import format_duration
from . import metrics, tracing
from .ratelimit import PRIORITY_HIGH, PRIORITY_LOW, PRIORITY_NORMAL, InflightGate, TokenBucket, make_client_limiter

GVRorGVK = Union[GroupVersionResource, GroupVersionKind]

MERGE = "merge"
JSON_PATCH = "json"
STRATEGIC = "strategic"

PATCH_CONTENT_TYPES = {
    MERGE: "application/merge-patch+json",
    JSON_PATCH: "application/json-patch+json",
    STRATEGIC: "application/strategic-merge-patch+json",
}


# request-parameter keys (never sent as query parameters):
# client-go rest.Request throttling thresholds [ext] (rest/request.go longThrottleLatency,
# extraLongThrottleLatency)
LONG_THROTTLE_LATENCY = 0.050
EXTRA_LONG_THROTTLE_LATENCY = 1.0


class ThrottledLogger:
    """client-go's ``globalThrottledLogger`` [ext]: the first *enabled* setting decides --
    with V(2) on, at most one line per second at V(2); otherwise at most one Info line per
    10 s -- so a starved client reports it without flooding the log."""

    SETTINGS = ((2, 1.0), (0, 10.0))  # (verbosity, min interval s)

    def __init__(self, settings: Tuple[Tuple[int, float], ...] = SETTINGS, clock=time.monotonic):
        self.settings = settings
        self.clock = clock
        self._last: Dict[int, float] = {}
        self.lines = 0

    def info(self, log: Any, msg: str) -> bool:
        for level, interval in self.settings:
            lg = log.v(level)
            if not lg.enabled():
                continue
            now = self.clock()
            last = self._last.get(level)
            if last is not None and now - last < interval:
                return False
            self._last[level] = now
            self.lines += 1
            lg.info(msg)
            return True
        return False


THROTTLED_LOGGER = ThrottledLogger()


def _throttle_log():
    from ..utils.logging import get_logger

    return get_logger("rest")


DISCARD = "_discardResponse"   # the caller ignores the response body
DECODE = "_decode"             # a jsonutil.Codec for the response body (e.g. one that skips spec)
ACCEPT = "_accept"             # Accept header override (server-side printing)
TABLE_ACCEPT = "application/json;as=Table;v=v1;g=meta.k8s.io,application/json"


class Transport:
    host = "in-memory"

    async def request(self, verb: str, gvr: GroupVersionResource, namespace: str = "", name: str = "",
                      subresource: str = "", body: Any = None, params: Optional[Dict[str, Any]] = None) -> Any:
        raise NotImplementedError

    async def watch(self, gvr: GroupVersionResource, namespace: str = "",
                    params: Optional[Dict[str, Any]] = None, decoder: Any = None) -> "WatchStream":
        """``decoder``: turns one event line into ``(type, object)`` (a ``jsonutil.Codec``);
        transports that do not decode bytes ignore it."""
        raise NotImplementedError

    async def discover(self, group_version: GroupVersion) -> List[Dict[str, Any]]:
        raise NotImplementedError

    async def close(self) -> None:
        pass


class WatchStream:
    """Async iterator of ``(type, object)``; ``stop()`` ends it."""

    def __aiter__(self):
        return self

    async def __anext__(self) -> Tuple[str, Dict[str, Any]]:
        raise NotImplementedError

    def stop(self) -> None:
        raise NotImplementedError


class _MemWatch(WatchStream):
    def __init__(self, w):
        self._w = w

    async def __anext__(self) -> Tuple[str, Dict[str, Any]]:
        return await self._w.__anext__()

    def stop(self) -> None:
        self._w.stop()


class InMemoryTransport(Transport):
    """Direct calls into an in-process fake APIServer (same event loop)."""

    host = "in-memory"

    def __init__(self, server, yield_every: int = 1):
        self.server = server
        self._yield_every = max(1, yield_every)
        self._n = 0

    async def _gate(self, verb: str, resource: str, sub: str, name: str) -> None:
        faults = self.server.faults
        delay = faults.delay_for(verb) if faults.latency else 0.0
        if delay > 0:
            await asyncio.sleep(delay)
        else:
            self._n += 1
            if self._n % self._yield_every == 0:
                await asyncio.sleep(0)  # a real round trip yields to other tasks
        if faults.faults:
            faults.check(verb, resource, sub or None, name or None)

    async def request(self, verb: str, gvr: GroupVersionResource, namespace: str = "", name: str = "",
                      subresource: str = "", body: Any = None, params: Optional[Dict[str, Any]] = None) -> Any:
        params = params or {}
        await self._gate(verb, gvr.resource, subresource, name)
        if params.get(ACCEPT) and verb in ("get", "list"):
            from ..apiserver.table import printer_columns_of, to_table, wants_table

            if wants_table(params[ACCEPT]):
                s = self.server
                if name:
                    objs = [s.get(gvr, namespace, name)]
                else:
                    objs = s.list(gvr, namespace or None, params.get("labelSelector"))["items"]
                return to_table(printer_columns_of(s.resource(gvr)), objs, s.clock.now_ns())
        if body.__class__ is bytes:  # pre-encoded by the caller (Codec.dumpb)
            body = jsonutil.loads(body)
        out = self._apply(verb, gvr, namespace, name, subresource, body, params)
        faults = self.server.faults
        if faults.faults:
            faults.check(verb, gvr.resource, subresource or None, name or None, after=True)
        return out

    def _apply(self, verb: str, gvr: GroupVersionResource, namespace: str, name: str, subresource: str, body: Any,
               params: Dict[str, Any]) -> Any:
        s = self.server
        if verb == "get":
            return s.get(gvr, namespace, name)
        if verb == "list":
            return s.list(gvr, namespace or None, params.get("labelSelector"), params.get("fieldSelector"),
                          int(params.get("limit") or 0), params.get("continue"))
        if verb == "create":
            return s.create(gvr, namespace, body, dry_run=bool(params.get("dryRun")))
        if verb == "update":
            return s.update(gvr, namespace, name, body, subresource or None)
        if verb == "patch":
            return s.patch(gvr, namespace, name, body, params.get("patchType", MERGE), subresource or None)
        if verb == "delete":
            opts = body or {}
            return s.delete(gvr, namespace, name, opts.get("propagationPolicy"), opts.get("preconditions"))
        if verb == "deletecollection":
            return s.delete_collection(gvr, namespace or None, params.get("labelSelector"))
        raise ValueError(f"unknown verb {verb}")

    async def watch(self, gvr: GroupVersionResource, namespace: str = "",
                    params: Optional[Dict[str, Any]] = None, decoder: Any = None) -> WatchStream:
        params = params or {}
        await self._gate("watch", gvr.resource, "", "")
        w = self.server.watch(gvr, namespace or None, str(params.get("resourceVersion") or ""),
                              params.get("labelSelector"), params.get("fieldSelector"),
                              bool(params.get("allowWatchBookmarks")))
        return _MemWatch(w)

    async def discover(self, group_version: GroupVersion) -> List[Dict[str, Any]]:
        return [ri.discovery_entry() for ri in self.server.resources()
                if ri.group == group_version.group and ri.version == group_version.version]


class NoKindMatchError(errors.ApiError):
    def __init__(self, gvk: GroupVersionKind):
        super().__init__(404, "NotFound", f'no matches for kind "{gvk.kind}" in version "{gvk.api_version}"')
        self.gvk = gvk


class RESTMapper:
    """GVK <-> GVR via discovery (``meta.RESTMapper``), with a negative cache that
    is refreshed on miss (CRDs may be installed after start)."""

    def __init__(self, transport: Transport):
        self.transport = transport
        self._gvk: Dict[GroupVersionKind, Tuple[GroupVersionResource, bool]] = {}
        self._gvr: Dict[GroupVersionResource, Tuple[GroupVersionKind, bool]] = {}
        self._loaded: Dict[GroupVersion, float] = {}

    async def _load(self, gv: GroupVersion, force: bool = False) -> None:
        if not force and gv in self._loaded:
            return
        try:
            entries = await self.transport.discover(gv)
        except errors.ApiError as e:
            if e.code == 404:
                entries = []
            else:
                raise
        for e in entries:
            name = e.get("name", "")
            if "/" in name:
                continue
            gvr = GroupVersionResource(gv.group, gv.version, name)
            gvk = GroupVersionKind(gv.group, gv.version, e.get("kind", ""))
            self._gvk[gvk] = (gvr, bool(e.get("namespaced", True)))
            self._gvr[gvr] = (gvk, bool(e.get("namespaced", True)))
        self._loaded[gv] = time.monotonic()

    async def resource_for(self, gvk: GroupVersionKind) -> Tuple[GroupVersionResource, bool]:
        hit = self._gvk.get(gvk)
        if hit is not None:
            return hit
        await self._load(gvk.group_version())
        hit = self._gvk.get(gvk)
        if hit is None:
            await self._load(gvk.group_version(), force=True)
            hit = self._gvk.get(gvk)
        if hit is None:
            raise NoKindMatchError(gvk)
        return hit

    async def kind_for(self, gvr: GroupVersionResource) -> Tuple[GroupVersionKind, bool]:
        hit = self._gvr.get(gvr)
        if hit is None:
            await self._load(GroupVersion(gvr.group, gvr.version), force=True)
            hit = self._gvr.get(gvr)
        if hit is None:
            raise errors.ApiError(404, "NotFound", f"no matches for {gvr}")
        return hit

    def register(self, gvk: GroupVersionKind, gvr: GroupVersionResource, namespaced: bool = True) -> None:
        self._gvk[gvk] = (gvr, namespaced)
        self._gvr[gvr] = (gvk, namespaced)


class Client:
    """The controller's API client (controller-runtime ``client.Client`` analog)."""

    def __init__(self, transport: Transport, qps: float = 30.0, burst: int = 50,
                 limiter: Optional[TokenBucket] = None, mapper: Optional[RESTMapper] = None,
                 max_inflight: int = 0, gauges: bool = True, low_reserve: int = 0):
        """``max_inflight`` > 0 caps concurrent requests (watches excluded); excess requests
        wait in priority order (:class:`~.ratelimit.InflightGate`).  ``gauges``: publish this
        client's gates as ``rest_client_requests_{in_flight,waiting}`` (the main client does; a
        derived side client does not overwrite its series).  ``low_reserve``: burst tokens a
        low-priority request may not spend (:class:`~.ratelimit.TokenBucket`; -1: the whole burst)."""
        self.transport = transport
        self.limiter = limiter if limiter is not None else make_client_limiter(qps, burst, low_reserve=low_reserve)
        self.inflight: Optional[InflightGate] = InflightGate(max_inflight) if max_inflight > 0 else None
        self.mapper = mapper or RESTMapper(transport)
        self.host = getattr(transport, "host", "in-memory")
        cfg = getattr(transport, "config", None)
        self.url_base = getattr(cfg, "host", "") if cfg is not None else ""
        self.requests = 0
        self.requests_by_verb: Dict[str, int] = {}
        self._m_verb: Dict[str, Tuple[Dict[str, Any], Any]] = {}  # verb -> ({code: counter}, latency histogram)
        self._m_rl: Dict[str, Any] = {}
        if gauges:
            self._observe_gates()
        # Retry-After retries (429 / 5xx from an apiserver shedding load, client-go rest.Request):
        # an HTTP transport leaves them to the client, so each attempt is throttled and gated anew
        self._retries_here = hasattr(transport, "retry_in_client")
        if self._retries_here:
            transport.retry_in_client = True  # type: ignore[attr-defined]

    def _observe_gates(self) -> None:
        """Scrape-time series of the request gates (``rest_client_requests_in_flight`` /
        ``_waiting``): read from the gates when /metrics is served, no per-request cost."""
        if self.inflight is not None:
            metrics.REST_INFLIGHT.observe((self.host,), self.inflight, lambda g: g.inflight)
        for gate_name, gate in (("rate_limiter", self.limiter), ("in_flight", self.inflight)):
            if gate is None:
                continue
            for prio, label in ((PRIORITY_HIGH, "high"), (PRIORITY_NORMAL, "normal"), (PRIORITY_LOW, "low")):
                metrics.REST_WAITING.observe((self.host, gate_name, label), gate,
                                             lambda g, p=prio: g.waiting_at(p))

    def derive(self) -> "Client":
        """A side client over the same transport (connections, credentials, REST mapping) with
        its **own** QPS bucket of the same ``qps``/``burst`` and **no** in-flight cap.

        controller-runtime builds the leader-election resource lock from a copy of the rest
        config (``leaderelection.NewResourceLock`` -> ``NewForConfig``) [ext], so the Lease
        requests get a token bucket of their own: the reference's ``--qps``/``--burst``
        (``/root/reference/cmd/operator/start.go:152-154``) bound the reconciler's traffic
        and, separately, the lock's -- a throttled tick can never hold a renewal back."""
        lim = self.limiter
        side = Client(self.transport, limiter=TokenBucket(lim.qps, lim.burst, lim.max_defer) if lim else None,
                      qps=-1 if lim is None else lim.qps, mapper=self.mapper, gauges=False)
        return side

    def gate_saturated(self) -> bool:
        """Is the in-flight cap the bottleneck right now (every slot taken, QPS bucket idle)?
        A reconcile then runs its writes on its worker instead of as a deferred tail: more
        queued requests would only wait in the gate (and cost CPU), not reorder anything --
        reordering happens while the QPS bucket is backed up, and there tails are cheap."""
        g = self.inflight
        if g is None or g.inflight + g.waiting < g.limit:
            return False
        lim = self.limiter
        return lim is None or not lim.waiting

    # -- plumbing
    def _gvr_now(self, target: GVRorGVK) -> Optional[GroupVersionResource]:
        """The resource of ``target`` without a discovery round trip (None: not known yet)."""
        if target.__class__ is GroupVersionResource:
            return target  # type: ignore[return-value]
        hit = self.mapper._gvk.get(target)  # type: ignore[arg-type]
        return hit[0] if hit is not None else None

    async def _gvr(self, target: GVRorGVK) -> GroupVersionResource:
        if isinstance(target, GroupVersionResource):
            return target
        return (await self.mapper.resource_for(target))[0]

    async def _throttle(self, verb: str, gvr: GroupVersionResource, namespace: str, name: str,
                        subresource: str, priority: int = PRIORITY_NORMAL) -> None:
        if self.limiter is not None:
            d = await self.limiter.wait(priority)
            m = self._m_rl.get(verb)
            if m is None:
                m = self._m_rl[verb] = metrics.REST_RATE_LIMIT.labels(verb, self.host)
            m.observe(d)
            if d > LONG_THROTTLE_LATENCY:
                self._log_throttle(d, verb, gvr, namespace, name, subresource)

    def _log_throttle(self, d: float, verb: str, gvr: GroupVersionResource, namespace: str, name: str,
                      subresource: str) -> None:
        """client-go ``tryThrottleWithInfo`` [ext]: a wait on the QPS bucket above 50 ms is
        logged at V(3); above 1 s through the process-wide throttled logger, so a starved
        operator says so -- the reference sets ``--qps``/``--burst`` on this rest config
        (``/root/reference/cmd/operator/start.go:152-154,218-219``)."""
        log = _throttle_log()
        v3 = log.v(3).enabled()
        if not v3 and d <= EXTRA_LONG_THROTTLE_LATENCY:
            return
        from .http import resource_path

        msg = (f"Waited for {format_duration(int(d * 1e9))} due to client-side throttling, not priority and "
               f"fairness, request: {self._METHOD.get(verb, verb.upper())}:{self.url_base}"
               f"{resource_path(gvr, namespace, name, subresource)}")
        if v3:
            log.v(3).info(msg)
        if d > EXTRA_LONG_THROTTLE_LATENCY:
            THROTTLED_LOGGER.info(log, msg)

    _METHOD = {"get": "GET", "list": "GET", "watch": "GET", "create": "POST", "update": "PUT", "patch": "PATCH",
               "delete": "DELETE", "deletecollection": "DELETE"}

    async def _do(self, verb: str, gvr: GroupVersionResource, namespace: str = "", name: str = "",
                  subresource: str = "", body: Any = None, params: Optional[Dict[str, Any]] = None,
                  priority: int = PRIORITY_NORMAL) -> Any:
        attempt = 0
        while True:
            if self.limiter is not None:
                await self._throttle(verb, gvr, namespace, name, subresource, priority)
            gate = self.inflight
            try:
                if gate is None:
                    return await self._send(verb, gvr, namespace, name, subresource, body, params)
                await gate.acquire(priority)
                try:
                    return await self._send(verb, gvr, namespace, name, subresource, body, params)
                finally:
                    gate.release()
            except errors.ApiError as e:
                if not self._retries_here or e.retry_after is None or not (e.code == 429 or e.code >= 500) \
                        or attempt >= self.transport.max_retries:  # type: ignore[attr-defined]
                    raise
                wait, code = max(0, e.retry_after), e.code
            # client-go: wait out Retry-After, then the retry passes the rate limiter again -- and
            # here the in-flight gate: no slot is held while the apiserver asks us to back off
            attempt += 1
            self.transport.retries += 1  # type: ignore[attr-defined]
            metrics.REST_RETRIES.labels(str(code), self._METHOD.get(verb, verb.upper()), self.host).inc()
            await asyncio.sleep(wait)

    async def _send(self, verb: str, gvr: GroupVersionResource, namespace: str, name: str, subresource: str,
                    body: Any, params: Optional[Dict[str, Any]]) -> Any:
        self.requests += 1
        rbv = self.requests_by_verb
        rbv[verb] = rbv.get(verb, 0) + 1
        if tracing.get_tracer().enabled:
            return await self._do_traced(verb, gvr, namespace, name, subresource, body, params)
        t0 = time.perf_counter()
        code = "200"
        try:
            return await self.transport.request(verb, gvr, namespace, name, subresource, body, params)
        except errors.ApiError as e:
            code = str(e.code)
            raise
        except Exception:
            code = "<error>"
            raise
        finally:
            self._observe(code, verb, t0)

    async def _do_traced(self, verb: str, gvr: GroupVersionResource, namespace: str, name: str, subresource: str,
                         body: Any, params: Optional[Dict[str, Any]]) -> Any:
        t0 = time.perf_counter()
        code = "200"
        with tracing.span("http." + verb, resource=gvr.resource + ("/" + subresource if subresource else ""),
                          namespace=namespace, name=name) as sp:
            try:
                return await self.transport.request(verb, gvr, namespace, name, subresource, body, params)
            except errors.ApiError as e:
                code = str(e.code)
                sp.set(code=e.code)
                raise
            except Exception:
                code = "<error>"
                raise
            finally:
                self._observe(code, verb, t0)

    def _observe(self, code: str, verb: str, t0: float) -> None:
        """``rest_client_requests_total`` and ``rest_client_request_duration_seconds``."""
        ms = self._m_verb.get(verb)
        if ms is None:
            ms = self._m_verb[verb] = ({}, metrics.REST_LATENCY.labels(verb.upper(), self.host))
        m = ms[0].get(code)
        if m is None:
            m = ms[0][code] = metrics.REST_REQUESTS.labels(code, self.host, self._METHOD.get(verb, verb.upper()))
        m.inc()
        ms[1].observe(time.perf_counter() - t0)

    # -- verbs
    async def get(self, target: GVRorGVK, namespace: str, name: str,
                  priority: int = PRIORITY_NORMAL) -> Dict[str, Any]:
        gvr = self._gvr_now(target) or await self._gvr(target)
        return await self._do("get", gvr, namespace, name, priority=priority)

    async def list(self, target: GVRorGVK, namespace: str = "", label_selector: Optional[str] = None,
                   field_selector: Optional[str] = None, limit: int = 0,
                   continue_: Optional[str] = None, decoder: Any = None) -> Dict[str, Any]:
        """``decoder``: a ``jsonutil.Codec`` for the response body (HTTP transports; paths
        under ``items/*``), e.g. one sharing recurring subtrees with an informer's watch codec."""
        params: Dict[str, Any] = {}
        if decoder is not None:
            params[DECODE] = decoder
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        if limit:
            params["limit"] = limit
        if continue_:
            params["continue"] = continue_
        gvr = self._gvr_now(target) or await self._gvr(target)
        return await self._do("list", gvr, namespace, params=params)

    async def table(self, target: GVRorGVK, namespace: str = "", name: str = "",
                    label_selector: Optional[str] = None) -> Dict[str, Any]:
        """``kubectl get`` data: a ``meta.k8s.io/v1`` Table from server-side printing (HTTP transports)."""
        params: Dict[str, Any] = {ACCEPT: TABLE_ACCEPT}
        if label_selector:
            params["labelSelector"] = label_selector
        gvr = self._gvr_now(target) or await self._gvr(target)
        return await self._do("get" if name else "list", gvr, namespace, name, params=params)

    async def list_all(self, target: GVRorGVK, namespace: str = "", label_selector: Optional[str] = None,
                       page_size: int = 500) -> Dict[str, Any]:
        """Paged LIST (client-go pager) returning one merged list."""
        out: Optional[Dict[str, Any]] = None
        cont = None
        while True:
            page = await self.list(target, namespace, label_selector, limit=page_size, continue_=cont)
            if out is None:
                out = page
            else:
                out["items"].extend(page["items"])
                out["metadata"]["resourceVersion"] = page["metadata"].get("resourceVersion")
            cont = (page.get("metadata") or {}).get("continue")
            if not cont:
                break
        assert out is not None
        out["metadata"].pop("continue", None)
        return out

    async def create(self, target: GVRorGVK, obj: Dict[str, Any], namespace: Optional[str] = None,
                     dry_run: bool = False, decoder: Any = None, priority: int = PRIORITY_NORMAL) -> Dict[str, Any]:
        """``decoder``: a ``jsonutil.Codec`` for the returned object, e.g. one that skips the
        ``spec`` the caller never reads (HTTP transports; others return the whole object).
        ``priority``: the request's class on a backed-up QPS bucket (``ratelimit.PRIORITY_*``)."""
        ns = namespace if namespace is not None else (obj.get("metadata") or {}).get("namespace", "")
        gvr = self._gvr_now(target) or await self._gvr(target)
        params: Optional[Dict[str, Any]] = None
        if dry_run or decoder is not None:
            params = {"dryRun": "All"} if dry_run else {}
            if decoder is not None:
                params[DECODE] = decoder
        return await self._do("create", gvr, ns, body=obj, params=params, priority=priority)

    async def update(self, target: GVRorGVK, obj: Dict[str, Any], subresource: str = "",
                     priority: int = PRIORITY_NORMAL) -> Dict[str, Any]:
        m = obj.get("metadata") or {}
        gvr = self._gvr_now(target) or await self._gvr(target)
        return await self._do("update", gvr, m.get("namespace", ""), m.get("name", ""),
                              subresource, body=obj, priority=priority)

    async def patch(self, target: GVRorGVK, namespace: str, name: str, patch: Any, patch_type: str = MERGE,
                    subresource: str = "", discard_response: bool = False,
                    priority: int = PRIORITY_NORMAL) -> Dict[str, Any]:
        """``discard_response``: the caller does not read the result, so an HTTP transport
        need not decode the returned object (it is still received, and errors still raise).
        ``patch`` may be bytes already encoded by the caller (``Codec.dumpb``)."""
        params: Dict[str, Any] = {"patchType": patch_type}
        if discard_response:
            params[DISCARD] = True
        gvr = self._gvr_now(target) or await self._gvr(target)
        return await self._do("patch", gvr, namespace, name, subresource, body=patch,
                              params=params, priority=priority)

    async def delete(self, target: GVRorGVK, namespace: str, name: str, propagation_policy: Optional[str] = None,
                     preconditions: Optional[Dict[str, str]] = None, discard_response: bool = False,
                     priority: int = PRIORITY_NORMAL) -> Any:
        opts: Dict[str, Any] = {}
        if propagation_policy:
            opts["propagationPolicy"] = propagation_policy
        if preconditions:
            opts["preconditions"] = preconditions
        gvr = self._gvr_now(target) or await self._gvr(target)
        return await self._do("delete", gvr, namespace, name, body=opts or None,
                              params={DISCARD: True} if discard_response else None, priority=priority)

    async def delete_all_of(self, target: GVRorGVK, namespace: str = "", label_selector: Optional[str] = None) -> Any:
        params = {"labelSelector": label_selector} if label_selector else {}
        gvr = self._gvr_now(target) or await self._gvr(target)
        return await self._do("deletecollection", gvr, namespace, params=params)

    async def watch(self, target: GVRorGVK, namespace: str = "", resource_version: str = "",
                    label_selector: Optional[str] = None, field_selector: Optional[str] = None,
                    allow_bookmarks: bool = True, timeout_seconds: Optional[int] = None,
                    decoder: Any = None) -> WatchStream:
        gvr = self._gvr_now(target) or await self._gvr(target)
        await self._throttle("watch", gvr, namespace, "", "")
        self.requests += 1
        self.requests_by_verb["watch"] = self.requests_by_verb.get("watch", 0) + 1
        params: Dict[str, Any] = {"watch": "true", "resourceVersion": resource_version,
                                  "allowWatchBookmarks": "true" if allow_bookmarks else "false"}
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        if timeout_seconds:
            params["timeoutSeconds"] = timeout_seconds
        try:
            w = await self.transport.watch(gvr, namespace, params, decoder) if decoder is not None \
                else await self.transport.watch(gvr, namespace, params)
        except errors.ApiError as e:
            metrics.REST_REQUESTS.labels(str(e.code), self.host, "GET").inc()
            raise
        metrics.REST_REQUESTS.labels("200", self.host, "GET").inc()
        return w

    # -- controller-runtime idioms
    async def patch_status_from(self, target: GVRorGVK, old: Dict[str, Any], new: Dict[str, Any]) -> Dict[str, Any]:
        """``client.Status().Patch(ctx, new, client.MergeFrom(old))``."""
        patch = jsonutil.create_merge_patch(old, new)
        m = new.get("metadata") or {}
        return await self.patch(target, m.get("namespace", ""), m.get("name", ""), patch, MERGE, "status")

    async def update_status(self, target: GVRorGVK, obj: Dict[str, Any]) -> Dict[str, Any]:
        """``client.Status().Update(ctx, obj)``."""
        return await self.update(target, obj, "status")

    async def close(self) -> None:
        await self.transport.close()
