"""The probe / metrics HTTP server (``runtime/miniweb.py``): routing, keep-alive, pipelining,
error statuses and the connection deadlines a framework's server would have applied."""
from __future__ import annotations

import asyncio

import pytest

from cron_operator_amd.runtime import miniweb as web


async def _server():
    app = web.Router()

    async def hello(req: web.Request) -> web.Response:
        return web.Response(text=f"hi {req.query.get('who', '')} {req.headers.get('X-Test', '')}")

    async def check(req: web.Request) -> web.Response:
        return web.json_response({"check": req.match_info["check"]})

    async def boom(req: web.Request) -> web.Response:
        raise RuntimeError("broken")

    app.add_get("/hello", hello)
    app.add_get("/healthz/{check}", check)
    app.add_get("/boom", boom)
    srv = web.Server(app)
    await srv.start("127.0.0.1", 0)
    return srv


async def _exchange(port: int, raw: bytes, read_until_close: bool = True) -> bytes:
    r, w = await asyncio.open_connection("127.0.0.1", port)
    w.write(raw)
    await w.drain()
    data = await asyncio.wait_for(r.read() if read_until_close else r.read(65536), 5)
    w.close()
    return data


async def test_routes_query_headers_and_errors():
    srv = await _server()
    try:
        out = await _exchange(srv.port, b"GET /hello?who=me HTTP/1.1\r\nX-Test: t\r\nConnection: close\r\n\r\n")
        assert out.startswith(b"HTTP/1.1 200 OK\r\n") and out.endswith(b"hi me t")
        out = await _exchange(srv.port, b"GET /healthz/ping HTTP/1.0\r\n\r\n")
        assert b'{"check": "ping"}' in out and b"Connection: close" in out
        assert (await _exchange(srv.port, b"GET /nope HTTP/1.0\r\n\r\n")).startswith(b"HTTP/1.1 404 ")
        assert (await _exchange(srv.port, b"POST /hello HTTP/1.0\r\nContent-Length: 2\r\n\r\nab")).startswith(
            b"HTTP/1.1 405 ")
        assert (await _exchange(srv.port, b"GET /boom HTTP/1.0\r\n\r\n")).startswith(b"HTTP/1.1 500 ")
        assert (await _exchange(srv.port, b"garbage\r\n\r\n")).startswith(b"HTTP/1.1 400 ")
        head = await _exchange(srv.port, b"HEAD /hello HTTP/1.0\r\n\r\n")
        assert head.startswith(b"HTTP/1.1 200 ") and head.endswith(b"\r\n\r\n")  # no body
        big = b"GET /hello HTTP/1.1\r\nX-Big: " + b"a" * (web.MAX_HEAD + 10)
        assert (await _exchange(srv.port, big)).startswith(b"HTTP/1.1 431 ")
    finally:
        await srv.stop()


async def test_keep_alive_and_pipelined_requests_answer_in_order():
    srv = await _server()
    try:
        r, w = await asyncio.open_connection("127.0.0.1", srv.port)
        w.write(b"GET /hello?who=a HTTP/1.1\r\n\r\nGET /hello?who=b HTTP/1.1\r\n\r\n")
        await w.drain()
        got = b""
        while got.count(b"HTTP/1.1 200") < 2:
            got += await asyncio.wait_for(r.read(4096), 5)
        assert got.index(b"hi a") < got.index(b"hi b")
        w.write(b"GET /healthz/x HTTP/1.1\r\n\r\n")  # the same connection, later
        await w.drain()
        assert b'"check": "x"' in await asyncio.wait_for(r.read(4096), 5)
        w.close()
    finally:
        await srv.stop()


@pytest.mark.parametrize("partial", [b"", b"GET /hel"])
async def test_idle_and_trickling_connections_are_closed(monkeypatch, partial):
    monkeypatch.setattr(web, "IDLE_TIMEOUT", 0.2)
    monkeypatch.setattr(web, "REQUEST_TIMEOUT", 0.2)
    srv = await _server()
    try:
        r, w = await asyncio.open_connection("127.0.0.1", srv.port)
        if partial:
            w.write(partial)
            await w.drain()
        assert await asyncio.wait_for(r.read(), 3) == b""  # closed by the server, nothing answered
        assert not srv._conns
        w.close()
    finally:
        await srv.stop()
