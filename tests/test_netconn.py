"""The native HTTP/1.1 connection (``ops/csrc/netconn.cpp``) where it differs from the asyncio
protocols it replaces: TLS through OpenSSL on the caller's ``ssl.SSLContext`` (verification,
hostname checks, SNI), bodies larger than a socket buffer in both directions, and the stream
mode's end-of-stream, decode-error and cancellation paths.  ``tests/test_fasthttp.py`` runs the
shared behaviour (keep-alive, chunking, retries, deadlines, streams) on both implementations."""
from __future__ import annotations

import asyncio
import json
import ssl

import pytest

from cron_operator_amd.ops import netconn_native
from cron_operator_amd.runtime.fasthttp import ConnectionFailed, HttpPool, HttpStatusError, NativeStream

nc = netconn_native.load()
pytestmark = pytest.mark.skipif(nc is None, reason="_netconn extension not built")


async def _server(handler, ssl_context=None):
    srv = await asyncio.start_server(handler, "127.0.0.1", 0, ssl=ssl_context)
    return srv, srv.sockets[0].getsockname()[1]


async def _read_request(reader):
    head = await reader.readuntil(b"\r\n\r\n")
    clen = 0
    for line in head.split(b"\r\n"):
        if line.lower().startswith(b"content-length:"):
            clen = int(line.split(b":")[1])
    body = await reader.readexactly(clen) if clen else b""
    return head, body


@pytest.fixture(scope="module")
def certs(tmp_path_factory):
    from cron_operator_amd.runtime.servers import self_signed_cert

    d = tmp_path_factory.mktemp("certs")
    cert, key = self_signed_cert(str(d), host="localhost")
    (d / "other").mkdir()
    other_cert, _ = self_signed_cert(str(d / "other"), host="localhost")
    return cert, key, other_cert


def _server_ctx(cert, key):
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(cert, key)
    return ctx


async def _echo_tls_server(cert, key):
    async def handle(reader, writer):
        try:
            while True:
                head, body = await _read_request(reader)
                payload = json.dumps({"path": head.split(b" ")[1].decode(), "n": len(body)}).encode()
                writer.write(b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(payload) + payload)
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionResetError, ssl.SSLError):
            writer.close()

    return await _server(handle, _server_ctx(cert, key))


def test_ssl_context_layout_is_recognised():
    ctx = ssl.create_default_context()
    assert nc.ssl_context_supported(ctx)
    ctx.check_hostname = False
    ctx.verify_mode = ssl.CERT_NONE
    assert nc.ssl_context_supported(ctx)
    assert not nc.ssl_context_supported(object())


async def test_tls_verified_against_ca_with_hostname(certs):
    cert, key, _ = certs
    srv, port = await _echo_tls_server(cert, key)
    ctx = ssl.create_default_context(cafile=cert)
    pool = HttpPool(f"https://127.0.0.1:{port}", ssl_context=ctx, server_hostname="localhost", native=True)
    try:
        st, raw = await pool.request("POST", "/tls", b"x" * 1000)
        assert st == 200 and json.loads(raw) == {"path": "/tls", "n": 1000}
        st, raw = await pool.request("GET", "/again")
        assert json.loads(raw)["path"] == "/again" and pool.connects == 1  # kept alive over TLS
        conn = pool._idle[0]
        assert conn.tls and conn.tls_version.startswith("TLS")
    finally:
        await pool.close()
        srv.close()


async def test_tls_rejects_wrong_hostname_and_untrusted_ca(certs):
    cert, key, other = certs
    srv, port = await _echo_tls_server(cert, key)
    try:
        # the certificate is for "localhost"
        bad_host = HttpPool(f"https://127.0.0.1:{port}", ssl_context=ssl.create_default_context(cafile=cert),
                            server_hostname="not-localhost", native=True)
        with pytest.raises(ssl.SSLError, match="verify"):
            await bad_host.request("GET", "/")
        await bad_host.close()
        # a CA that did not sign it
        untrusted = HttpPool(f"https://127.0.0.1:{port}", ssl_context=ssl.create_default_context(cafile=other),
                             server_hostname="localhost", native=True)
        with pytest.raises(ssl.SSLError, match="verify"):
            await untrusted.request("GET", "/")
        await untrusted.close()
        # insecure-skip-tls-verify: no verification at all
        ctx = ssl.create_default_context()
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
        insecure = HttpPool(f"https://127.0.0.1:{port}", ssl_context=ctx, native=True)
        assert (await insecure.request("GET", "/ok"))[0] == 200
        await insecure.close()
    finally:
        srv.close()


async def test_large_bodies_both_ways():
    """A request body far larger than the socket send buffer (the native writer waits for
    writability) and a response body delivered in many reads, Content-Length and chunked."""
    big = bytes(range(256)) * (16 * 1024)  # 4 MiB

    async def handle(reader, writer):
        try:
            while True:
                head, body = await _read_request(reader)
                await asyncio.sleep(0.05)  # let the client's send buffer fill up
                if b"/chunked" in head:
                    writer.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n")
                    for i in range(0, len(big), 100_000):
                        c = big[i:i + 100_000]
                        writer.write(b"%x\r\n" % len(c) + c + b"\r\n")
                        await writer.drain()
                    writer.write(b"0\r\n\r\n")
                else:
                    writer.write(b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(body) + body)
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionResetError):
            writer.close()

    srv, port = await _server(handle)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        st, raw = await pool.request("POST", "/echo", big)
        assert st == 200 and raw == big
        st, raw = await pool.request("GET", "/chunked")
        assert st == 200 and raw == big
        assert pool.connects == 1
    finally:
        await pool.close()
        srv.close()


async def test_interim_response_and_retry_after():
    async def handle(reader, writer):
        await _read_request(reader)
        writer.write(b"HTTP/1.1 100 Continue\r\n\r\nHTTP/1.1 429 Too Many Requests\r\nRetry-After: 3\r\n"
                     b"Content-Length: 2\r\n\r\n{}")
        await writer.drain()
        writer.close()

    srv, port = await _server(handle)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        assert await pool.request_full("GET", "/") == (429, b"{}", 3)
    finally:
        await pool.close()
        srv.close()


async def test_malformed_response_fails_the_request():
    async def handle(reader, writer):
        await _read_request(reader)
        writer.write(b"HTTP/1.1 200 OK\r\nContent-Length: nope\r\n\r\n")
        await writer.drain()

    srv, port = await _server(handle)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        with pytest.raises(ConnectionFailed, match="bad HTTP response"):
            await pool.request("GET", "/")
        assert not pool._idle
    finally:
        await pool.close()
        srv.close()


def _chunk(b: bytes) -> bytes:
    return b"%x\r\n" % len(b) + b + b"\r\n"


async def test_stream_terminal_chunk_ends_iteration_and_wait():
    async def handle(reader, writer):
        await reader.readuntil(b"\r\n\r\n")
        writer.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n")
        writer.write(_chunk(b'{"a":1}\n{"a":2}\n'))
        await writer.drain()
        await asyncio.sleep(0.05)
        writer.write(_chunk(b'{"a":3}\n') + b"0\r\n\r\n")
        await writer.drain()
        await asyncio.sleep(1)  # the connection stays open: the terminal chunk alone ends the stream

    srv, port = await _server(handle)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        st = await pool.open_stream("/w", json.loads)
        assert isinstance(st, NativeStream)
        got = []
        while await asyncio.wait_for(st.wait_ready(), 2):
            got.extend(st.take_ready())
        assert got == [{"a": 1}, {"a": 2}, {"a": 3}]
        st.close()
    finally:
        await pool.close()
        srv.close()


async def test_stream_decode_error_ends_the_stream():
    async def handle(reader, writer):
        await reader.readuntil(b"\r\n\r\n")
        writer.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n" +
                     _chunk(b'{"ok":1}\nnot json\n{"x":2}\n'))
        await writer.drain()
        await asyncio.sleep(1)

    srv, port = await _server(handle)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        st = await pool.open_stream("/w", json.loads)
        got = [x async for x in st]
        assert got == [{"ok": 1}]
        assert isinstance(st._n.error, ValueError) and st._n.done
    finally:
        await pool.close()
        srv.close()


async def test_stream_error_status_chunked_body():
    body = b'{"kind":"Status","code":403,"reason":"Forbidden"}'

    async def handle(reader, writer):
        await reader.readuntil(b"\r\n\r\n")
        writer.write(b"HTTP/1.1 403 Forbidden\r\nTransfer-Encoding: chunked\r\n\r\n" + _chunk(body[:10]) +
                     _chunk(body[10:]) + b"0\r\n\r\n")
        await writer.drain()

    srv, port = await _server(handle)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        with pytest.raises(HttpStatusError) as ei:
            await pool.open_stream("/w", json.loads)
        assert ei.value.status == 403 and ei.value.body == body
    finally:
        await pool.close()
        srv.close()


async def test_cancelled_wait_does_not_poison_the_next_one():
    gate = asyncio.Event()

    async def handle(reader, writer):
        await reader.readuntil(b"\r\n\r\n")
        writer.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n")
        await writer.drain()
        await gate.wait()
        writer.write(_chunk(b'{"late":true}\n'))
        await writer.drain()
        await asyncio.sleep(1)

    srv, port = await _server(handle)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        st = await pool.open_stream("/w", json.loads)
        t = asyncio.ensure_future(st.wait_ready())
        await asyncio.sleep(0.05)
        t.cancel()
        with pytest.raises(asyncio.CancelledError):
            await t
        gate.set()
        assert await asyncio.wait_for(st.wait_ready(), 2)
        assert st.take_ready() == [{"late": True}]
        st.close()
        assert st._n.done and not await st.wait_ready()
    finally:
        await pool.close()
        srv.close()


async def test_closed_connection_fails_fast_and_close_fails_inflight():
    async def silent(reader, writer):
        await asyncio.sleep(2)

    srv, port = await _server(silent)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        conn = await pool._connect()
        fut = conn.send(b"GET / HTTP/1.1\r\nHost: x\r\n\r\n")
        conn.close()
        with pytest.raises(ConnectionFailed) as ei:
            await fut
        assert ei.value.no_response
        with pytest.raises(ConnectionFailed):
            await conn.send(b"GET / HTTP/1.1\r\n\r\n")
        assert conn.closing() and conn.fd == -1
    finally:
        await pool.close()
        srv.close()


async def test_watch_and_requests_over_tls_against_fake_apiserver(certs):
    """The operator's client over native TLS end to end: CREATE, PATCH and a WATCH stream."""
    from cron_operator_amd.api.v1alpha1 import CRON_GVR, new_cron
    from cron_operator_amd.apiserver.http import APIServerApp
    from cron_operator_amd.runtime.client import Client
    from cron_operator_amd.runtime.http import HttpTransport
    from cron_operator_amd.runtime.kubeconfig import RestConfig
    from cron_operator_amd.testing.env import TestEnv

    cert, key, _ = certs
    env = TestEnv()
    app = APIServerApp(env.server)
    port = await app.start("127.0.0.1", 0, ssl_context=_server_ctx(cert, key))
    with open(cert, "rb") as fh:
        ca = fh.read()
    tr = HttpTransport(RestConfig(host=f"https://127.0.0.1:{port}", ca_data=ca, tls_server_name="localhost"))
    client = Client(tr, qps=-1)
    try:
        obj = new_cron("tls", "default", "@daily", {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob"}).to_dict()
        created = await client.create(CRON_GVR, obj, "default")
        assert tr._fast_pool().native
        w = await client.watch(CRON_GVR, "default", resource_version=created["metadata"]["resourceVersion"])
        for i in range(20):
            await client.patch(CRON_GVR, "default", "tls", {"metadata": {"labels": {"i": str(i)}}})
        seen = []
        while len(seen) < 20:
            et, ev = await asyncio.wait_for(w.__anext__(), 5)
            seen.append(ev["metadata"]["labels"]["i"])
        assert seen == [str(i) for i in range(20)]
        w.stop()
    finally:
        await client.close()
        await app.stop()


async def test_early_response_to_unsent_body_retires_the_connection():
    """A server may answer before reading the whole request (413 on a huge body).  The unsent
    tail must never precede the next request on that connection: it is not reused."""
    big = b"x" * (8 << 20)

    async def handle(reader, writer):
        await reader.readuntil(b"\r\n\r\n")
        writer.write(b"HTTP/1.1 413 Request Entity Too Large\r\nContent-Length: 0\r\n\r\n")
        await writer.drain()
        await asyncio.sleep(1)  # never reads the body

    srv, port = await _server(handle)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        st, raw = await asyncio.wait_for(pool.request("POST", "/big", big), 5)
        assert st == 413 and raw == b""
        assert not pool._idle
    finally:
        await pool.close()
        srv.close()


async def test_tls_client_certificate_is_presented(tmp_path):
    """mTLS (a kubeconfig's client-certificate-data): the native handshake presents the
    certificate the SSLContext holds; without it the server refuses the connection."""
    from cron_operator_amd.runtime.servers import self_signed_cert

    (tmp_path / "srv").mkdir()
    (tmp_path / "cli").mkdir()
    scert, skey = self_signed_cert(str(tmp_path / "srv"), host="localhost")
    ccert, ckey = self_signed_cert(str(tmp_path / "cli"), host="operator")
    sctx = _server_ctx(scert, skey)
    sctx.verify_mode = ssl.CERT_REQUIRED
    sctx.load_verify_locations(cafile=ccert)
    peers = []

    async def handle(reader, writer):
        try:
            peers.append(writer.get_extra_info("peercert"))
            await _read_request(reader)
            writer.write(b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nok")
            await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionResetError, ssl.SSLError):
            pass
        writer.close()

    srv, port = await _server(handle, sctx)
    try:
        ctx = ssl.create_default_context(cafile=scert)
        ctx.load_cert_chain(ccert, ckey)
        pool = HttpPool(f"https://127.0.0.1:{port}", ssl_context=ctx, server_hostname="localhost", native=True)
        assert await pool.request("GET", "/") == (200, b"ok")
        await pool.close()
        assert peers and dict(x[0] for x in peers[0]["subject"])["commonName"] == "operator"
        anon = HttpPool(f"https://127.0.0.1:{port}", ssl_context=ssl.create_default_context(cafile=scert),
                        server_hostname="localhost", native=True)
        with pytest.raises((ssl.SSLError, ConnectionFailed)):
            await anon.request("GET", "/")
        await anon.close()
    finally:
        srv.close()


# ----------------------------------------------------------------------------- the native pool


async def _capture_server(responses=None, delay=0.0):
    """A keep-alive server recording every request's exact bytes (head + body)."""
    seen = []
    conns = []

    async def handle(reader, writer):
        conns.append(writer)
        try:
            while True:
                head, body = await _read_request(reader)
                seen.append(head + body)
                if delay:
                    await asyncio.sleep(delay)
                payload = b'{"ok":true}'
                writer.write(b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(payload) + payload)
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionResetError):
            writer.close()

    srv, port = await _server(handle)
    return srv, port, seen, conns


async def test_pool_request_bytes_equal_the_python_path():
    """The request the native pool builds is byte for byte the asyncio path's: target prefix,
    fixed headers (rotated ones too), Accept, and the body framing of every verb."""
    srv, port, seen, _ = await _capture_server()
    calls = [("GET", "/api/v1/namespaces/a/pods?watch=false", None, "application/json", "application/json"),
             ("POST", "/apis/x/v1/things", b'{"a":1}', "application/json", "application/json"),
             ("PATCH", "/apis/x/v1/things/a/status", b'{"s":2}', "application/merge-patch+json", "application/json"),
             ("PUT", "/empty", None, "application/json", "application/json;as=Table;v=v1;g=meta.k8s.io"),
             ("DELETE", "/apis/x/v1/things/b", None, "application/json", "application/json")]
    try:
        for native in (True, False):
            pool = HttpPool(f"http://127.0.0.1:{port}/base", headers={"Authorization": "Bearer t0"}, native=native)
            assert (pool._np is not None) == native
            try:
                for args in calls:
                    assert (await pool.request_full(*args))[0] == 200
                pool.set_headers({"Authorization": "Bearer t1"})
                await pool.request_full(*calls[0])
            finally:
                await pool.close()
        n = len(calls) + 1
        assert len(seen) == 2 * n
        assert seen[:n] == seen[n:]
        assert b"Bearer t1" in seen[n - 1] and seen[0].startswith(b"GET /base/api/v1/namespaces/a/pods?watch=false ")
        assert b"Content-Length: 0\r\n\r\n" in seen[3] and b"Content-Length" not in seen[0]
    finally:
        srv.close()


async def test_pool_reuses_keeps_at_most_max_idle_and_reports_busy():
    srv, port, seen, conns = await _capture_server(delay=0.05)
    pool = HttpPool(f"http://127.0.0.1:{port}", max_idle=2, native=True)
    try:
        out = await asyncio.gather(*(pool.request("GET", f"/{i}") for i in range(4)))
        assert all(st == 200 for st, _ in out)
        assert pool.connects == 4 and len(pool._idle) == 2 and pool._np.busy == 0
        await pool.request("GET", "/again")
        assert pool.connects == 4  # reused
        # the connections over max_idle were closed: the server saw EOF on them
        await asyncio.sleep(0.05)
        assert sum(w.is_closing() for w in conns) == 2
    finally:
        await pool.close()
        srv.close()


async def test_pool_deadline_sweep_fails_the_request_and_closes_it():
    hold = asyncio.Event()

    async def handle(reader, writer):
        await _read_request(reader)
        await hold.wait()  # never answers
        writer.close()

    srv, port = await _server(handle)
    pool = HttpPool(f"http://127.0.0.1:{port}", timeout=0.2, native=True)
    try:
        t0 = asyncio.get_running_loop().time()
        with pytest.raises(asyncio.TimeoutError):
            await pool.request("GET", "/slow")
        assert asyncio.get_running_loop().time() - t0 < 2.0
        assert pool._np.busy == 0 and not pool._idle
    finally:
        hold.set()
        await pool.close()
        srv.close()


async def test_pool_cancelled_request_does_not_return_its_connection():
    got = asyncio.Event()
    closed = asyncio.Event()

    async def handle(reader, writer):
        await _read_request(reader)
        got.set()
        try:
            await reader.read()  # EOF when the client drops the connection
        finally:
            closed.set()
            writer.close()

    srv, port = await _server(handle)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        task = asyncio.ensure_future(pool.request("GET", "/hang"))
        await asyncio.wait_for(got.wait(), 5)
        task.cancel()
        with pytest.raises(asyncio.CancelledError):
            await task
        await asyncio.wait_for(closed.wait(), 5)
        assert pool._np.busy == 0 and not pool._idle
    finally:
        await pool.close()
        srv.close()


async def test_pool_closed_while_busy_closes_the_connection_after_its_response():
    srv, port, seen, conns = await _capture_server(delay=0.1)
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        task = asyncio.ensure_future(pool.request("GET", "/x"))
        await asyncio.sleep(0.03)
        await pool.close()
        assert (await task)[0] == 200  # the exchange in flight completes
        assert not pool._idle and pool._np.busy == 0
        await asyncio.sleep(0.05)
        assert conns[0].is_closing()
    finally:
        srv.close()


async def test_pool_ssl_generation_retires_idle_connections():
    srv, port, seen, conns = await _capture_server()
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    try:
        await pool.request("GET", "/a")
        assert len(pool._idle) == 1
        pool._np.ssl_gen += 1  # what set_ssl does for a rotated client certificate
        pool._np.close_idle()
        assert not pool._idle
        await pool.request("GET", "/b")
        # the new connection was made for the pool's old generation (pool._ssl_gen is still 0):
        # it is closed when its response completes instead of going back to the idle list
        assert pool.connects == 2 and not pool._idle
    finally:
        await pool.close()
        srv.close()


async def test_pool_objects_are_released():
    """No references leak through the busy/idle lists: after many requests and a close, the
    pool and its connections are freed by reference counting and the cycle collector."""
    import gc
    import weakref

    srv, port, seen, _ = await _capture_server()
    pool = HttpPool(f"http://127.0.0.1:{port}", native=True)
    for _ in range(200):
        await pool.request("POST", "/x", b"{}")
    refs = [weakref.ref(c) for c in pool._idle] + [weakref.ref(pool._np)]
    await pool.close()
    del pool
    gc.collect()
    assert all(r() is None for r in refs)
    srv.close()


async def test_pool_unencodable_path_fails_like_the_python_path_without_leaking():
    srv, port, seen, conns = await _capture_server()
    try:
        for native in (True, False):
            pool = HttpPool(f"http://127.0.0.1:{port}", native=native)
            try:
                with pytest.raises(UnicodeEncodeError):
                    await pool.request("GET", "/café☃")
                if native:
                    assert pool._np.busy == 0 and not pool._idle
                assert (await pool.request("GET", "/ok"))[0] == 200
            finally:
                await pool.close()
        await asyncio.sleep(0.05)
        assert all(c.is_closing() for c in conns[:1])  # the native pool's first connection was closed
    finally:
        srv.close()
