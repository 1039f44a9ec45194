"""The lean HTTP/1.1 client (runtime/fasthttp.py) against hand-written server replies."""
from __future__ import annotations

import asyncio

import pytest

from cron_operator_amd.runtime import fasthttp
from cron_operator_amd.runtime.fasthttp import ConnectionFailed, HttpPool, encode_query


@pytest.fixture(autouse=True, params=["native", "python"])
def pool_mode(request, monkeypatch):
    """Every test runs on the native connections (``_netconn``) and on the asyncio protocols."""
    if request.param == "native":
        from cron_operator_amd.ops import netconn_native

        if netconn_native.load() is None:
            pytest.skip("_netconn extension not built")
        monkeypatch.setattr(fasthttp, "DEFAULT_NATIVE", True)
    else:
        monkeypatch.setattr(fasthttp, "DEFAULT_NATIVE", False)
    return request.param


async def serve(replies, record=None):
    """A TCP server that answers successive requests on a connection with ``replies`` (bytes or callables)."""
    it = iter(replies)

    async def handle(reader, writer):
        try:
            while True:
                head = await reader.readuntil(b"\r\n\r\n")
                clen = 0
                for line in head.split(b"\r\n"):
                    if line.lower().startswith(b"content-length:"):
                        clen = int(line.split(b":")[1])
                body = await reader.readexactly(clen) if clen else b""
                if record is not None:
                    record.append((head, body))
                r = next(it)
                if r is None:  # close without answering
                    writer.close()
                    return
                writer.write(r)
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionResetError, StopIteration):
            writer.close()

    srv = await asyncio.start_server(handle, "127.0.0.1", 0)
    return srv, srv.sockets[0].getsockname()[1]


async def test_content_length_keepalive_and_headers():
    rec = []
    srv, port = await serve([b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\n{}",
                             b"HTTP/1.1 201 Created\r\nContent-Length: 7\r\n\r\n{\"a\":1}"], rec)
    pool = HttpPool(f"http://127.0.0.1:{port}", headers={"Authorization": "Bearer t"})
    try:
        assert await pool.request("GET", "/x") == (200, b"{}")
        assert await pool.request("POST", "/y", b'{"k":1}') == (201, b'{"a":1}')
        assert pool.connects == 1  # kept alive
        head0, _ = rec[0]
        assert head0.startswith(b"GET /x HTTP/1.1\r\n") and b"Authorization: Bearer t" in head0
        head1, body1 = rec[1]
        assert b"Content-Type: application/json" in head1 and body1 == b'{"k":1}'
    finally:
        await pool.close()
        srv.close()


async def test_chunked_and_split_packets():
    body = b"4\r\nWiki\r\n6;ext=1\r\npedia \r\nE\r\nin \r\n\r\nchunks.\r\n0\r\nX-Trailer: 1\r\n\r\n"
    srv, port = await serve([b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n" + body,
                             b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n0\r\n\r\n"])
    pool = HttpPool(f"http://127.0.0.1:{port}")
    try:
        st, raw = await pool.request("GET", "/c")
        assert st == 200 and raw == b"Wikipedia in \r\n\r\nchunks."
        assert await pool.request("GET", "/empty") == (200, b"")
        assert pool.connects == 1
    finally:
        await pool.close()
        srv.close()


async def test_parser_handles_byte_by_byte_delivery():
    from cron_operator_amd.runtime.fasthttp import _Conn

    loop = asyncio.get_running_loop()

    class T:
        def write(self, d):
            pass

        def is_closing(self):
            return False

        def close(self):
            pass

    c = _Conn()
    c.connection_made(T())
    fut = c.send(b"GET / HTTP/1.1\r\n\r\n")
    for b in b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n0\r\n\r\n":
        c.data_received(bytes([b]))
    assert fut.done() and fut.result() == (200, b"abc", None)
    assert loop is asyncio.get_running_loop()


async def test_connection_close_and_read_to_eof():
    srv, port = await serve([b"HTTP/1.1 200 OK\r\nConnection: close\r\nContent-Length: 1\r\n\r\na"])
    pool = HttpPool(f"http://127.0.0.1:{port}")
    try:
        assert await pool.request("GET", "/") == (200, b"a")
        assert not pool._idle  # closed, not pooled
    finally:
        await pool.close()
        srv.close()

    async def eof_server(reader, writer):
        await reader.readuntil(b"\r\n\r\n")
        writer.write(b"HTTP/1.0 200 OK\r\n\r\nuntil-close")
        await writer.drain()
        writer.close()

    srv2 = await asyncio.start_server(eof_server, "127.0.0.1", 0)
    pool2 = HttpPool(f"http://127.0.0.1:{srv2.sockets[0].getsockname()[1]}")
    try:
        assert await pool2.request("GET", "/") == (200, b"until-close")
    finally:
        await pool2.close()
        srv2.close()


async def test_stale_keepalive_is_retried_once():
    # first connection: one good reply then the server drops the idle connection
    srv, port = await serve([b"HTTP/1.1 200 OK\r\nContent-Length: 1\r\n\r\n1", None,
                             b"HTTP/1.1 200 OK\r\nContent-Length: 1\r\n\r\n2"])
    pool = HttpPool(f"http://127.0.0.1:{port}")
    try:
        assert await pool.request("GET", "/") == (200, b"1")
        assert await pool.request("GET", "/") == (200, b"2")  # retried on a fresh connection
        assert pool.connects == 2
    finally:
        await pool.close()
        srv.close()


async def test_fresh_connection_failure_raises_and_timeout():
    srv, port = await serve([None])
    pool = HttpPool(f"http://127.0.0.1:{port}")
    try:
        with pytest.raises(ConnectionFailed):
            await pool.request("GET", "/")
    finally:
        await pool.close()
        srv.close()

    async def silent(reader, writer):
        await asyncio.sleep(5)

    srv2 = await asyncio.start_server(silent, "127.0.0.1", 0)
    pool2 = HttpPool(f"http://127.0.0.1:{srv2.sockets[0].getsockname()[1]}", timeout=0.2)
    try:
        with pytest.raises(asyncio.TimeoutError):
            await pool2.request("GET", "/")
    finally:
        await pool2.close()
        srv2.close()


def test_encode_query():
    assert encode_query({}) == ""
    assert encode_query({"labelSelector": "kubedl.io/cron-name=a b"}) == "?labelSelector=kubedl.io%2Fcron-name%3Da+b"


async def test_retry_after_429_is_honoured_by_http_transport():
    """client-go semantics: 429 + Retry-After is retried (here with Retry-After: 0), 429 without it is not."""
    from cron_operator_amd.api import errors
    from cron_operator_amd.api.v1alpha1 import CRON_GVR
    from cron_operator_amd.apiserver.http import APIServerApp
    from cron_operator_amd.runtime.client import Client
    from cron_operator_amd.runtime.http import HttpTransport
    from cron_operator_amd.runtime.kubeconfig import RestConfig
    from cron_operator_amd.testing.env import TestEnv

    env = TestEnv()
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0)
    tr = HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}"))
    client = Client(tr, qps=-1)
    try:
        env.server.faults.add(verb="list", resource="crons", code=429, reason="TooManyRequests", times=3,
                              retry_after=0)
        assert (await client.list(CRON_GVR, "default"))["items"] == []
        assert tr.retries == 3
        env.server.faults.add(verb="list", resource="crons", code=429, reason="TooManyRequests", times=1)
        with pytest.raises(errors.ApiError) as ei:
            await client.list(CRON_GVR, "default")
        assert ei.value.code == 429 and tr.retries == 3
        env.server.faults.add(verb="get", resource="crons", code=503, reason="ServiceUnavailable", retry_after=0)
        tr.max_retries = 2
        with pytest.raises(errors.ApiError) as ei:
            await client.get(CRON_GVR, "default", "x")
        assert ei.value.code == 503 and ei.value.retry_after == 0 and tr.retries == 5
    finally:
        await client.close()
        await app.stop()


async def test_https_apiserver_with_ca_and_bearer_token(tmp_path):
    """TLS end to end: the fake apiserver serves HTTPS, the client verifies it against the CA from the
    kubeconfig-style RestConfig, sends a bearer token, and watches over the same TLS endpoint."""
    import ssl

    from cron_operator_amd.api.v1alpha1 import CRON_GVR, new_cron
    from cron_operator_amd.apiserver.http import APIServerApp
    from cron_operator_amd.runtime.client import Client
    from cron_operator_amd.runtime.http import HttpTransport
    from cron_operator_amd.runtime.kubeconfig import RestConfig
    from cron_operator_amd.runtime.servers import self_signed_cert
    from cron_operator_amd.testing.env import TestEnv

    cert, key = self_signed_cert(str(tmp_path), host="localhost")
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(cert, key)
    env = TestEnv()
    env.server.tokens = {"tok": {"username": "admin", "groups": ["system:masters"]}}
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0, ssl_context=ctx)
    with open(cert, "rb") as fh:
        ca = fh.read()
    cfg = RestConfig(host=f"https://127.0.0.1:{port}", bearer_token="tok", ca_data=ca, tls_server_name="localhost")
    client = Client(HttpTransport(cfg), qps=-1)
    try:
        obj = new_cron("tls", "default", "@daily", {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob"}).to_dict()
        created = await client.create(CRON_GVR, obj, "default")
        w = await client.watch(CRON_GVR, "default", resource_version=created["metadata"]["resourceVersion"])
        await client.patch(CRON_GVR, "default", "tls", {"metadata": {"labels": {"a": "b"}}})
        et, ev = await asyncio.wait_for(w.__anext__(), 5)
        assert et == "MODIFIED" and ev["metadata"]["labels"] == {"a": "b"}
        w.stop()
        # wrong token over TLS -> 401
        bad = Client(HttpTransport(RestConfig(host=cfg.host, bearer_token="nope", ca_data=ca,
                                              tls_server_name="localhost")), qps=-1)
        from cron_operator_amd.api import errors

        with pytest.raises(errors.ApiError) as ei:
            await bad.get(CRON_GVR, "default", "tls")
        assert ei.value.code == 401
        await bad.close()
    finally:
        await client.close()
        await app.stop()


async def test_stream_chunked_lines_split_across_chunks():
    body_lines = [b'{"type":"ADDED","object":{"a":1}}', b'{"type":"MODIFIED","object":{"a":2}}']
    payload = b"\n".join(body_lines) + b"\n"
    # split the payload mid-line across chunks, deliver in small TCP writes
    chunks = [payload[:10], payload[10:40], payload[40:]]
    wire = b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n" + b"".join(
        b"%x\r\n" % len(c) + c + b"\r\n" for c in chunks) + b"0\r\n\r\n"

    async def handle(reader, writer):
        await reader.readuntil(b"\r\n\r\n")
        for i in range(0, len(wire), 7):
            writer.write(wire[i:i + 7])
            await writer.drain()
            await asyncio.sleep(0)
        writer.close()

    srv = await asyncio.start_server(handle, "127.0.0.1", 0)
    pool = HttpPool(f"http://127.0.0.1:{srv.sockets[0].getsockname()[1]}")
    import json

    try:
        st = await pool.open_stream("/w?watch=true", json.loads)
        got = [x async for x in st]
        assert got == [{"type": "ADDED", "object": {"a": 1}}, {"type": "MODIFIED", "object": {"a": 2}}]
    finally:
        await pool.close()
        srv.close()


async def test_stream_error_status_raises():
    from cron_operator_amd.runtime.fasthttp import HttpStatusError

    body = b'{"kind":"Status","code":410,"reason":"Expired","message":"too old"}'
    srv, port = await serve([b"HTTP/1.1 410 Gone\r\nContent-Length: %d\r\n\r\n" % len(body) + body])
    pool = HttpPool(f"http://127.0.0.1:{port}")
    try:
        with pytest.raises(HttpStatusError) as ei:
            await pool.open_stream("/w", lambda b: b)
        assert ei.value.status == 410 and b"Expired" in ei.value.body
    finally:
        await pool.close()
        srv.close()
