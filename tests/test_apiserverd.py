"""The native fake apiserver (``_apiserverd``, ``ops/csrc/apiserverd.cpp``) against the Python one.

The Python :class:`~cron_operator_amd.apiserver.server.APIServer` behind
:class:`~cron_operator_amd.apiserver.http.APIServerApp` is the envtest analog the suite trusts
(``tests/test_apiserver.py``).  The benchmark serves the same contract natively, so every
request here goes to both and the answers must agree: status code, reason and the decoded
body, resourceVersions included (only the random ``uid`` is masked).  A scripted stream covers
each verb's edges (defaulting, validation, AlreadyExists, preconditions, no-op writes,
finalizers, selectors, paging); a generated one interleaves them at random.  Watches are compared
over HTTP: the same writes, the same event stream per selector, resumed from a resourceVersion.
"""
from __future__ import annotations

import asyncio
import json
from typing import Any, Dict, List, Optional, Tuple
from urllib.parse import parse_qsl

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from cron_operator_amd.api.v1alpha1 import new_cron
from cron_operator_amd.api.v1alpha1.crd import crd
from cron_operator_amd.apiserver.http import APIServerApp, Request
from cron_operator_amd.apiserver.native import NativeAPIServer, load
from cron_operator_amd.apiserver.server import APIServer
from cron_operator_amd.bench.harness import pytorchjob_template
from cron_operator_amd.trainingop.crds import kubeflow_crds
from cron_operator_amd.utils.clock import FakeClock

pytestmark = pytest.mark.skipif(load() is None, reason="_apiserverd did not build")

T0 = 1767268800 * 10**9
NS = "bench"
CRONS = "/apis/apps.kubedl.io/v1alpha1/namespaces/bench/crons"
JOBS = "/apis/kubeflow.org/v1/namespaces/bench/pytorchjobs"
MERGE = "application/merge-patch+json"


class Pair:
    """One request stream, two servers."""

    def __init__(self) -> None:
        self.py = APIServer(FakeClock(T0))
        self.py.install_crd(crd())
        for c in kubeflow_crds():
            self.py.install_crd(c)
        self.app = APIServerApp(self.py)
        self.nat = NativeAPIServer(T0)
        self.nat.install_crd(crd())
        for c in kubeflow_crds():
            self.nat.install_crd(c)

    def py_call(self, method: str, path: str, query: str, body: bytes, ctype: str) -> Tuple[int, Any]:
        q: Dict[str, str] = {}
        for k, v in parse_qsl(query, keep_blank_values=True):
            q.setdefault(k, v)
        hdrs = {"content-type": ctype} if ctype else {}
        r = self.app.dispatch(Request(method, path, q, hdrs, body))
        assert not asyncio.isfuture(r)
        return r.status, json.loads(r.body) if r.body[:1] in (b"{", b"[") else r.body

    def nat_call(self, method: str, path: str, query: str, body: bytes, ctype: str) -> Tuple[int, Any]:
        status, raw = self.nat.srv.request(method, path, query, body, ctype)
        return status, json.loads(raw) if raw[:1] in (b"{", b"[") else raw

    def both(self, method: str, path: str, body: Any = None, query: str = "",
             ctype: str = "application/json", message: bool = True) -> Tuple[int, Any]:
        """``message=False``: the Status messages may differ (a JSON decoder's own wording)."""
        raw = body if isinstance(body, bytes) else (json.dumps(body).encode() if body is not None else b"")
        a = _norm(self.py_call(method, path, query, raw, ctype if raw else ""))
        b = _norm(self.nat_call(method, path, query, raw, ctype if raw else ""))
        if "limit=" not in query:  # an unpaged LIST: Python answers in insertion order, native in key
            for x in (a, b):       # order (as etcd does); paged LISTs are key-ordered by both
                if isinstance(x[1], dict) and isinstance(x[1].get("items"), list):
                    x[1]["items"].sort(key=lambda o: (o["metadata"].get("namespace", ""), o["metadata"]["name"]))
        if not message:
            for x in (a, b):
                if isinstance(x[1], dict):
                    x[1]["message"] = x[1].get("message", "").split(":", 1)[0]
        assert a == b, f"{method} {path}?{query}\n python: {a}\n native: {b}"
        return b


def _norm(x: Any) -> Any:
    """Mask what differs by design: random uids (and the generated-name suffix)."""
    if isinstance(x, dict):
        out = {}
        for k, v in x.items():
            if k == "uid" and isinstance(v, str):
                out[k] = "<uid>"
            else:
                out[k] = _norm(v)
        return out
    if isinstance(x, list):
        return [_norm(v) for v in x]
    if isinstance(x, tuple):
        return tuple(_norm(v) for v in x)
    return x


def _job(name: str, labels: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
    j = pytorchjob_template()
    j["metadata"] = {"name": name, "labels": dict(labels or {"app": "bench"})}
    return j


def test_scripted_stream_agrees():
    p = Pair()
    p.both("POST", "/api/v1/namespaces", {"metadata": {"name": NS}})
    p.both("POST", "/api/v1/namespaces", {"metadata": {"name": NS}})  # AlreadyExists
    # Crons: defaulting (concurrencyPolicy Allow), validation (enum), required fields
    c = new_cron("c1", NS, "* * * * *", pytorchjob_template(), history_limit=3).to_dict()
    c["spec"].pop("concurrencyPolicy", None)
    created = p.both("POST", CRONS, c)[1]
    assert created["spec"]["concurrencyPolicy"] == "Allow"
    bad = new_cron("c2", NS, "* * * * *", pytorchjob_template()).to_dict()
    bad["spec"]["concurrencyPolicy"] = "Sometimes"
    assert p.both("POST", CRONS, bad)[0] == 422
    nosched = new_cron("c3", NS, "* * * * *", pytorchjob_template()).to_dict()
    del nosched["spec"]["schedule"]
    assert p.both("POST", CRONS, nosched)[0] == 422
    assert p.both("POST", CRONS, {**c, "metadata": {"name": "Bad_Name"}})[0] == 422
    assert p.both("POST", "/apis/apps.kubedl.io/v1alpha1/namespaces/nowhere/crons",
                  {**c, "metadata": {"name": "x"}})[0] == 404
    assert p.both("POST", CRONS, b"{not json", message=False)[0] == 400
    # status writes: ignore everything but status; the main resource ignores status
    st = {"status": {"lastScheduleTime": "2026-01-01T12:01:00Z",
                     "active": [{"kind": "PyTorchJob", "name": "c1-1", "namespace": NS}]}}
    p.both("PATCH", CRONS + "/c1/status", st, ctype=MERGE)
    p.both("PATCH", CRONS + "/c1/status", st, ctype=MERGE)  # no-op: same resourceVersion
    assert p.both("PATCH", CRONS + "/c1/status", {"status": {"lastScheduleTime": "yesterday"}},
                  ctype=MERGE)[0] == 422
    # pruning inside a subtree whose request bytes the native parser keeps as its encoding
    pruned = p.both("PATCH", CRONS + "/c1/status", {"status": {"history": [
        {"uid": "u1", "object": {"kind": "PyTorchJob", "name": "c1-0", "extra": True}, "status": "Succeeded",
         "bogus": 1}]}}, ctype=MERGE)[1]
    assert "bogus" not in pruned["status"]["history"][0]
    # a repeated key: the last value wins, and the bytes sent are not the stored object's
    p.both("PATCH", CRONS + "/c1/status", b'{"status":{"history":[{"uid":"u2","uid":"u3","object":{"kind":"PyTorchJob",'
                                          b'"name":"c1-9"},"status":"Failed"}]}}', ctype=MERGE)
    assert p.nat_call("GET", CRONS + "/c1", "", b"", "")[1]["status"]["history"][0]["uid"] == "u3"
    p.both("PATCH", CRONS + "/c1", {"status": {"active": None}, "metadata": {"labels": {"a": "1"}}}, ctype=MERGE)
    spec = p.both("PATCH", CRONS + "/c1", {"spec": {"suspend": True}}, ctype=MERGE)[1]
    assert spec["metadata"]["generation"] == 2
    # optimistic concurrency
    assert p.both("PATCH", CRONS + "/c1", {"metadata": {"resourceVersion": "1"}, "spec": {"suspend": False}},
                  ctype=MERGE)[0] == 409
    cur = p.both("GET", CRONS + "/c1")[1]
    cur["spec"]["historyLimit"] = 5
    p.both("PUT", CRONS + "/c1", cur)
    assert p.both("PUT", CRONS + "/c1", cur)[0] == 409  # stale resourceVersion now
    assert p.both("PATCH", CRONS + "/c1", {"spec": {}}, ctype="application/strategic-merge-patch+json")[0] == 415
    assert p.both("PATCH", CRONS + "/c1", {"spec": {}}, ctype="text/plain")[0] == 415
    # jobs: labels, selectors, paging
    for i in range(7):
        p.both("POST", JOBS, _job(f"j{i}", {"app": "bench", "kubedl.io/cron-name": f"c{i % 3}",
                                            **({"tier": "gold"} if i % 2 else {})}))
    for sel in ("", "kubedl.io/cron-name=c1", "kubedl.io/cron-name==c2", "kubedl.io/cron-name!=c1",
                "kubedl.io/cron-name in (c0,c2)", "kubedl.io/cron-name notin (c0, c2)", "tier", "!tier",
                "tier,kubedl.io/cron-name=c0", "app=bench,tier!=gold", "nope=x"):
        p.both("GET", JOBS, query=f"labelSelector={sel}")
    p.both("GET", JOBS, query="fieldSelector=metadata.name=j3")
    p.both("GET", JOBS, query="fieldSelector=metadata.name!=j3,metadata.namespace=bench")
    assert p.both("GET", JOBS, query="labelSelector=a in b")[0] == 400
    page = p.both("GET", JOBS, query="limit=3")[1]
    while page["metadata"].get("continue"):
        page = p.both("GET", JOBS, query=f"limit=3&continue={page['metadata']['continue']}")[1]
    assert p.both("GET", JOBS, query="limit=2&continue=garbage")[0] == 400
    p.both("GET", "/apis/kubeflow.org/v1/pytorchjobs")  # all namespaces
    # deletes: preconditions, finalizers, collections
    assert p.both("DELETE", JOBS + "/j0", {"preconditions": {"uid": "nope"}}, message=False)[0] == 409  # names the uid
    p.both("DELETE", JOBS + "/j0", {"propagationPolicy": "Background"})
    assert p.both("DELETE", JOBS + "/j0")[0] == 404
    p.both("PATCH", JOBS + "/j1", {"metadata": {"finalizers": ["example.com/hold"]}}, ctype=MERGE)
    p.both("DELETE", JOBS + "/j1")  # marks deletionTimestamp
    p.both("DELETE", JOBS + "/j1")  # already terminating: unchanged
    p.both("PATCH", JOBS + "/j1", {"metadata": {"finalizers": None}}, ctype=MERGE)  # drained: gone
    assert p.both("GET", JOBS + "/j1")[0] == 404
    p.both("DELETE", JOBS, query="labelSelector=tier%3Dgold")
    p.both("GET", JOBS)
    # routing and discovery
    for path in ("/apis/kubeflow.org/v1", "/apis/apps.kubedl.io/v1alpha1", "/apis/nope/v1", "/version",
                 "/apis/kubeflow.org/v1/namespaces/bench/nothings", "/apis/apiextensions.k8s.io/v1/namespaces/x/"
                 "customresourcedefinitions", "/api/v1/namespaces/bench"):
        p.both("GET", path)
    assert p.both("POST", "/apis/kubeflow.org/v1/namespaces/bench/pytorchjobs", [1, 2])[0] == 400


OPS = st.lists(st.tuples(st.sampled_from(["create", "status", "label", "delete", "get", "list", "put"]),
                         st.integers(0, 4), st.integers(0, 3)), min_size=5, max_size=40)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(OPS)
def test_generated_streams_agree(ops: List[Tuple[str, int, int]]):
    p = Pair()
    p.both("POST", "/api/v1/namespaces", {"metadata": {"name": NS}})
    phases = ["Created", "Running", "Succeeded", "Failed"]
    for op, i, k in ops:
        name = f"j{i}"
        if op == "create":
            p.both("POST", JOBS, _job(name, {"app": "bench", "kubedl.io/cron-name": f"c{k}"}))
        elif op == "status":
            p.both("PATCH", f"{JOBS}/{name}/status", {"status": {"conditions": [
                {"type": phases[k], "status": "True", "lastTransitionTime": "2026-01-01T12:00:00Z"}],
                "completionTime": "2026-01-01T12:00:30Z" if k >= 2 else None}}, ctype=MERGE)
        elif op == "label":
            p.both("PATCH", f"{JOBS}/{name}", {"metadata": {"labels": {"kubedl.io/shard": f"{k}-of-4"}}},
                   ctype=MERGE)
        elif op == "delete":
            p.both("DELETE", f"{JOBS}/{name}")
        elif op == "get":
            p.both("GET", f"{JOBS}/{name}")
        elif op == "put":
            status, cur = p.nat_call("GET", f"{JOBS}/{name}", "", b"", "")
            if status == 200:
                cur["spec"]["runPolicy"] = {"backoffLimit": k}
                p.both("PUT", f"{JOBS}/{name}", cur)
        else:
            p.both("GET", JOBS, query=f"labelSelector=kubedl.io/cron-name=c{k}")
            p.both("GET", JOBS, query=f"labelSelector=kubedl.io/shard notin ({k}-of-4)")


# --------------------------------------------------------------------------- watches


async def _read_events(reader: asyncio.StreamReader, n: int, timeout: float = 5.0) -> List[Dict[str, Any]]:
    """``n`` events off a chunked watch response (the head already consumed)."""
    out: List[Dict[str, Any]] = []
    buf = b""
    while len(out) < n:
        size_line = await asyncio.wait_for(reader.readline(), timeout)
        size = int(size_line.strip() or b"0", 16)
        if size == 0:
            break
        buf += await asyncio.wait_for(reader.readexactly(size + 2), timeout)
        buf = buf[:-2] if buf.endswith(b"\r\n") else buf
        *lines, buf = buf.split(b"\n")
        out += [json.loads(ln) for ln in lines if ln.strip()]
    return out


async def _open_watch(port: int, path: str, query: str) -> Tuple[asyncio.StreamReader, asyncio.StreamWriter]:
    r, w = await asyncio.open_connection("127.0.0.1", port)
    w.write(f"GET {path}?watch=true&{query} HTTP/1.1\r\nHost: x\r\n\r\n".encode())
    await w.drain()
    head = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
    assert head.startswith(b"HTTP/1.1 200") and b"chunked" in head.lower(), head
    return r, w


def _summ(evs: List[Dict[str, Any]]) -> List[Tuple[str, str, str]]:
    return [(e["type"], e["object"]["metadata"]["name"], e["object"]["metadata"]["resourceVersion"]) for e in evs]


async def test_watch_streams_agree_over_http():
    """The same writes, watched through each server's HTTP front end with a label selector:
    the same ADDED / MODIFIED / DELETED sequence (a relabel moves an object out of scope as
    DELETED and into another as ADDED), the same resourceVersions, and the same replay when a
    watch resumes from a resourceVersion."""
    p = Pair()
    app_port = await p.app.start("127.0.0.1", 0)
    nat_port = p.nat.start("127.0.0.1", 0)
    try:
        p.both("POST", "/api/v1/namespaces", {"metadata": {"name": NS}})
        p.both("POST", JOBS, _job("w0", {"app": "bench", "kubedl.io/shard": "0-of-2"}))
        rv0 = p.both("GET", JOBS)[1]["metadata"]["resourceVersion"]
        sels = ["labelSelector=kubedl.io/shard%3D0-of-2", "labelSelector=kubedl.io/shard%3D1-of-2",
                "labelSelector=kubedl.io/shard"]
        streams = {}
        for port, tag in ((app_port, "py"), (nat_port, "nat")):
            for s in sels:
                streams[(tag, s)] = await _open_watch(port, JOBS, s + "&resourceVersion=0")
        p.both("POST", JOBS, _job("w1", {"app": "bench", "kubedl.io/shard": "1-of-2"}))
        p.both("PATCH", f"{JOBS}/w0/status", {"status": {"startTime": "2026-01-01T12:00:00Z"}}, ctype=MERGE)
        p.both("PATCH", f"{JOBS}/w0", {"metadata": {"labels": {"kubedl.io/shard": "1-of-2"}}}, ctype=MERGE)
        p.both("DELETE", f"{JOBS}/w1")
        want = {sels[0]: 3, sels[1]: 3, sels[2]: 5}
        for s in sels:
            a = await _read_events(streams[("py", s)][0], want[s])
            b = await _read_events(streams[("nat", s)][0], want[s])
            assert _summ(a) == _summ(b), (s, _summ(a), _summ(b))
            assert _norm(a) == _norm(b)
        # resume from a resourceVersion: the log replayed with the same scope transitions
        for port, tag in ((app_port, "py"), (nat_port, "nat")):
            streams[(tag, "resume")] = await _open_watch(port, JOBS, f"{sels[1]}&resourceVersion={rv0}")
        a = await _read_events(streams[("py", "resume")][0], 3)
        b = await _read_events(streams[("nat", "resume")][0], 3)
        assert _summ(a) == _summ(b) and [e["type"] for e in b] == ["ADDED", "ADDED", "DELETED"], _summ(b)
        for _, w in streams.values():
            w.close()
    finally:
        await p.app.stop()
        p.nat.stop()


async def test_watch_timeout_ends_the_stream_and_the_connection_serves_on():
    """``timeoutSeconds`` ends the chunked body with its terminator; the kept-alive connection
    then answers the next request (what an informer's re-watch relies on)."""
    nat = NativeAPIServer(T0, bookmark_interval=0.2)
    port = nat.start("127.0.0.1", 0)
    try:
        r, w = await _open_watch(port, "/api/v1/namespaces", "timeoutSeconds=0.5&allowWatchBookmarks=true")
        evs = await _read_events(r, 5, timeout=5)  # 4 synthetic ADDED + a BOOKMARK (0.2 s)
        assert [e["type"] for e in evs[:4]] == ["ADDED"] * 4 and evs[4]["type"] == "BOOKMARK"
        while True:  # drain bookmarks up to the terminating chunk
            line = await asyncio.wait_for(r.readline(), 5)
            if line.strip() == b"0":
                await r.readline()
                break
            await r.readexactly(int(line.strip(), 16) + 2)
        w.write(b"GET /version HTTP/1.1\r\nHost: x\r\n\r\n")
        await w.drain()
        head = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
        assert head.startswith(b"HTTP/1.1 200")
        w.close()
    finally:
        nat.stop()


async def test_too_old_resource_version_is_gone_and_the_log_stays_bounded():
    """The event log keeps ``watch_window`` events per resource (the soak's memory bound): a
    watch from before that answers 410 Expired, as kube-apiserver's watch cache does."""
    nat = NativeAPIServer(T0, watch_window=50)
    srv = nat.srv
    srv.request("POST", "/api/v1/namespaces", "", b'{"metadata":{"name":"bench"}}', "application/json")
    for i in range(200):
        srv.request("POST", "/api/v1/namespaces/bench/configmaps", "",
                    json.dumps({"metadata": {"name": f"m{i}"}}).encode(), "application/json")
    assert srv.log_sizes()["/configmaps"] == 50
    port = nat.start("127.0.0.1", 0)
    try:
        r, w = await asyncio.open_connection("127.0.0.1", port)
        w.write(b"GET /api/v1/namespaces/bench/configmaps?watch=true&resourceVersion=10 HTTP/1.1\r\nHost: x\r\n\r\n")
        await w.drain()
        head = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
        assert head.startswith(b"HTTP/1.1 410"), head
        w.close()
    finally:
        nat.stop()


async def test_the_log_replays_bytes_and_scope_only():
    """The watch log keeps each event's bytes and its object's name, namespace and labels, not
    the object: a resume replays the events as they were sent (a relabel still moves an object
    between label scopes, a metadata.name field selector still filters), and a resume with a
    field selector on any other field answers 410 so the client relists."""
    nat = NativeAPIServer(T0)
    srv = nat.srv
    srv.request("POST", "/api/v1/namespaces", "", b'{"metadata":{"name":"bench"}}', "application/json")
    st, raw = srv.request("GET", "/api/v1/namespaces/bench/configmaps")
    rv0 = json.loads(raw)["metadata"]["resourceVersion"]
    cm = "/api/v1/namespaces/bench/configmaps"
    for i in range(3):
        srv.request("POST", cm, "", json.dumps({"metadata": {"name": f"m{i}", "labels": {"a": "x"}},
                                                "data": {"k": str(i)}}).encode(), "application/json")
    srv.request("PATCH", f"{cm}/m1", "", b'{"metadata":{"labels":{"a":"y"}},"data":{"k":"changed"}}', MERGE)
    srv.request("DELETE", f"{cm}/m2", "", b"{}", "application/json")
    port = nat.start("127.0.0.1", 0)
    try:
        r, w = await _open_watch(port, cm, f"labelSelector=a%3Dx&resourceVersion={rv0}")
        evs = await _read_events(r, 5)
        assert [(e["type"], e["object"]["metadata"]["name"]) for e in evs] == [
            ("ADDED", "m0"), ("ADDED", "m1"), ("ADDED", "m2"), ("DELETED", "m1"), ("DELETED", "m2")], evs
        assert evs[3]["object"]["data"] == {"k": "changed"}  # the bytes of the event, as first sent
        w.close()
        r, w = await _open_watch(port, cm, f"fieldSelector=metadata.name%3Dm1&resourceVersion={rv0}")
        evs = await _read_events(r, 2)
        assert [(e["type"], e["object"]["metadata"]["name"]) for e in evs] == [("ADDED", "m1"), ("MODIFIED", "m1")]
        w.close()
        r, w = await asyncio.open_connection("127.0.0.1", port)
        w.write(f"GET {cm}?watch=true&fieldSelector=data.k%3D1&resourceVersion={rv0} HTTP/1.1\r\nHost: x\r\n\r\n"
                .encode())
        await w.drain()
        head = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
        assert head.startswith(b"HTTP/1.1 410"), head
        w.close()
    finally:
        nat.stop()


async def test_tls_requests_and_a_watch(tmp_path):
    """The deployment-shaped arm's transport: HTTPS on the server's own OpenSSL context, a
    request and a watch over it, verified against the self-signed CA (CN=localhost)."""
    import ssl

    from cron_operator_amd.runtime.servers import self_signed_cert

    cert, key = self_signed_cert(str(tmp_path), host="localhost")
    nat = NativeAPIServer(T0)
    port = nat.start("127.0.0.1", 0, cert, key)
    ctx = ssl.create_default_context(cafile=cert)
    try:
        r, w = await asyncio.open_connection("127.0.0.1", port, ssl=ctx, server_hostname="localhost")
        body = b'{"metadata":{"name":"bench"}}'
        w.write(b"POST /api/v1/namespaces HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                b"Content-Length: %d\r\n\r\n" % len(body) + body)
        await w.drain()
        head = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
        assert head.startswith(b"HTTP/1.1 201"), head
        n = int([ln for ln in head.split(b"\r\n") if ln.lower().startswith(b"content-length")][0].split(b":")[1])
        assert json.loads(await r.readexactly(n))["metadata"]["name"] == "bench"
        w.write(b"GET /api/v1/namespaces/bench/configmaps?watch=true&resourceVersion=0 HTTP/1.1\r\nHost: x\r\n\r\n")
        await w.drain()
        head = await asyncio.wait_for(r.readuntil(b"\r\n\r\n"), 5)
        assert head.startswith(b"HTTP/1.1 200") and b"chunked" in head.lower(), head
        nat.srv.request("POST", "/api/v1/namespaces/bench/configmaps", "", b'{"metadata":{"name":"m"}}',
                        "application/json")
        evs = await _read_events(r, 1)
        assert evs[0]["type"] == "ADDED" and evs[0]["object"]["metadata"]["name"] == "m"
        w.close()
    finally:
        nat.stop()


def test_bench_controls_complete_and_lifecycle():
    """The /debug/fake controls the harness drives: a lifecycle stage reaches every unfinished
    job (their new resourceVersions returned), ``complete`` finishes them, stats count verbs."""
    nat = NativeAPIServer(T0)
    for c in kubeflow_crds():
        nat.install_crd(c)
    srv = nat.srv
    srv.request("POST", "/api/v1/namespaces", "", b'{"metadata":{"name":"bench"}}', "application/json")
    for i in range(5):
        srv.request("POST", JOBS, "", json.dumps(_job(f"j{i}")).encode(), "application/json")

    def ctl(what: str, body: Dict[str, Any]) -> Dict[str, Any]:
        st_, raw = nat.fallback("POST", f"/debug/fake/{what}", "", {}, json.dumps(body).encode())
        assert st_ == 200, raw
        return json.loads(raw)

    rvs = ctl("lifecycle", {"namespace": NS, "stage": 0, "start": "2026-01-01T12:00:00Z",
                            "end": "2026-01-01T12:00:30Z"})["resourceVersions"]
    assert sorted(rvs) == [f"{NS}/j{i}" for i in range(5)]
    # perTurn on a server that is not running: applied at once, as without it
    assert ctl("complete", {"namespace": NS, "time": "2026-01-01T12:00:30Z", "perTurn": 2}) == \
        {"completed": 5, "queued": False}
    assert ctl("complete", {"namespace": NS, "time": "2026-01-01T12:00:30Z"}) == {"completed": 0, "queued": False}
    job = json.loads(srv.request("GET", JOBS + "/j0")[1])
    assert job["status"]["completionTime"] == "2026-01-01T12:00:30Z"
    assert job["status"]["conditions"][-1]["type"] == "Succeeded"
    stats = json.loads(nat.fallback("GET", "/debug/fake/stats", "", {}, b"")[1])
    assert stats["by_verb"]["patch"] == 10 and stats["native"] is True
    assert nat.fallback("POST", "/debug/fake/faults", "", {}, b'{"faults":[{"verb":"create"}]}')[0] == 501


async def test_interleaved_completion_writes_are_applied_a_few_per_turn():
    """``complete`` with ``perTurn`` on a running server answers at once with the number queued;
    the server thread then applies that many per loop turn, serving other requests between them:
    a GET sent right after the control is answered while writes are still queued, and a watch
    sees every job's MODIFIED event."""
    nat = NativeAPIServer(T0)
    for c in kubeflow_crds():
        nat.install_crd(c)
    srv = nat.srv
    srv.request("POST", "/api/v1/namespaces", "", b'{"metadata":{"name":"bench"}}', "application/json")
    n = 400
    for i in range(n):
        srv.request("POST", JOBS, "", json.dumps(_job(f"j{i}")).encode(), "application/json")
    port = nat.start("127.0.0.1", 0)
    try:
        r, w = await _open_watch(port, JOBS, "resourceVersion=" + json.loads(srv.request("GET", JOBS)[1])
                                 ["metadata"]["resourceVersion"])
        cr, cw = await asyncio.open_connection("127.0.0.1", port)

        async def call(method: str, path: str, body: bytes = b"") -> Tuple[bytes, bytes]:
            cw.write(f"{method} {path} HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                     f"Content-Length: {len(body)}\r\n\r\n".encode() + body)
            await cw.drain()
            head = await asyncio.wait_for(cr.readuntil(b"\r\n\r\n"), 5)
            ln = int([x for x in head.split(b"\r\n") if x.lower().startswith(b"content-length")][0].split(b":")[1])
            return head, await cr.readexactly(ln)

        head, body = await call("POST", "/debug/fake/complete",
                                json.dumps({"namespace": NS, "time": "2026-01-01T12:00:30Z", "perTurn": 1}).encode())
        assert head.startswith(b"HTTP/1.1 200") and json.loads(body) == {"completed": n, "queued": True}
        head, body = await call("GET", JOBS + "?limit=1")  # served between the queued writes
        assert head.startswith(b"HTTP/1.1 200")
        evs = await _read_events(r, n, timeout=20)
        assert {e["type"] for e in evs} == {"MODIFIED"} and len({e["object"]["metadata"]["name"] for e in evs}) == n
        assert all(e["object"]["status"]["completionTime"] == "2026-01-01T12:00:30Z" for e in evs)
        head, body = await call("POST", "/debug/fake/complete",
                                json.dumps({"namespace": NS, "time": "2026-01-01T12:00:30Z", "perTurn": 1}).encode())
        assert json.loads(body) == {"completed": 0, "queued": True}
        w.close()
        cw.close()
    finally:
        nat.stop()
