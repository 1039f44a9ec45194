"""Native HTTP/1.1 framing (ops/csrc/httpcodec.cpp) against the pure-Python parsers it
replaces: the fake apiserver's request parser (``_ServerConn._next_request_py``) and the
client's response parser (``_Conn._parse_py``).  Same messages, same split points, same
results -- a hand-written corpus plus hypothesis-generated messages."""
from __future__ import annotations

import asyncio

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from cron_operator_amd.apiserver import http as srvhttp
from cron_operator_amd.ops import httpcodec_native
from cron_operator_amd.runtime import fasthttp

codec = httpcodec_native.load()
pytestmark = pytest.mark.skipif(codec is None, reason="_httpcodec not built")


class _Transport:
    def __init__(self):
        self.out = bytearray()
        self.closed = False

    def write(self, b):
        self.out += b

    def close(self):
        self.closed = True

    def is_closing(self):
        return self.closed


def _server_parse(chunks, native):
    """Feed ``chunks`` to a server connection; collect every request the parser yields."""
    conn = srvhttp._ServerConn.__new__(srvhttp._ServerConn)
    srvhttp._ServerConn.__init__(conn, None)
    conn.transport = _Transport()
    got = []
    nxt = conn._next_request if native else conn._next_request_py
    for c in chunks:
        conn.buf += c
        while not conn.closed:
            r = nxt()
            if r is None:
                break
            req, keep = r
            got.append((req.method, req.path, req.query, req.headers, req.body, keep))
    return got, bytes(conn.buf), bytes(conn.transport.out), conn.closed


REQUESTS = [
    b"GET /api/v1/namespaces HTTP/1.1\r\nHost: x\r\n\r\n",
    b"PATCH /apis/apps.kubedl.io/v1alpha1/namespaces/d/crons/c/status HTTP/1.1\r\nHost: x\r\n"
    b"Content-Type: application/merge-patch+json\r\nContent-Length: 13\r\n\r\n{\"status\":{}}",
    b"POST /x HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n4;ext=1\r\nWiki\r\n5\r\npedia\r\n0\r\nT: 1\r\n\r\n",
    b"GET /w?watch=true&labelSelector=kubedl.io%2Fshard%3D1&x&&y=2&watch=false HTTP/1.1\r\n\r\n",
    b"GET /a%20b/%E2%9C%93 HTTP/1.1\r\nX-Dup: 1\r\nx-dup: 2\r\nNoColonHeader\r\n  Spaced-Key  :  v v  \r\n\r\n",
    b"GET / HTTP/1.0\r\nConnection: keep-alive\r\n\r\n",
    b"GET / HTTP/1.0\r\n\r\n",
    b"DELETE /x HTTP/1.1\r\nConnection: close\r\nContent-Length: 0\r\n\r\n",
    b"GET / HTTP/1.1\r\nConnection: Keep-Alive\r\nContent-Length:\r\n\r\n",
    b"put /lower HTTP/1.1\r\nContent-Length: 3\r\n\r\nabc",
]


@pytest.mark.parametrize("msg", REQUESTS)
def test_request_corpus_matches_python(msg):
    for split in (None, 1, 7):
        chunks = [msg] if split is None else [msg[i:i + split] for i in range(0, len(msg), split)]
        assert _server_parse(chunks, True) == _server_parse(chunks, False)


def test_pipelined_requests_and_leftover():
    msg = REQUESTS[1] + REQUESTS[0] + REQUESTS[2] + b"GET /partial HTTP/1.1\r\nHo"
    n, p = _server_parse([msg], True), _server_parse([msg], False)
    assert n == p and len(n[0]) == 3 and n[1] == b"GET /partial HTTP/1.1\r\nHo"


def test_expect_continue_and_errors():
    head = b"PUT /x HTTP/1.1\r\nExpect: 100-continue\r\nContent-Length: 4\r\n\r\n"
    for native in (True, False):
        got, rest, out, closed = _server_parse([head], native)
        assert got == [] and out == b"HTTP/1.1 100 Continue\r\n\r\n" and not closed
        got, rest, out, closed = _server_parse([head, b"ab", b"cd"], native)
        assert got[0][4] == b"abcd" and out.count(b"100 Continue") == 1
    # framing errors answer and close (the Python parser raised on a bad chunk size)
    for bad, status in ((b"GARBAGE\r\n\r\n", b"400"), (b"GET / HTTP/1.1\r\nContent-Length: x\r\n\r\n", b"400"),
                        (b"POST / HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n", b"400"),
                        (b"POST / HTTP/1.1\r\nContent-Length: %d\r\n\r\n" % (srvhttp.MAX_BODY + 1), b"413")):
        got, _, out, closed = _server_parse([bad], True)
        assert got == [] and closed and out.startswith(b"HTTP/1.1 " + status)
    got, _, out, closed = _server_parse([b"x" * ((1 << 20) + 1)], True)
    assert closed and out.startswith(b"HTTP/1.1 431")


_token = st.text(alphabet="abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-_", min_size=1, max_size=12)
_value = st.text(alphabet="abcdefghijklmnopqrstuvwxyz0123456789 ;=/,.-_\t", max_size=20)


@st.composite
def _request(draw):
    method = draw(st.sampled_from(["GET", "PUT", "POST", "PATCH", "DELETE", "get"]))
    path = "/" + "/".join(draw(st.lists(_token, max_size=4)))
    if draw(st.booleans()):
        path += "?" + "&".join(f"{k}={v}" for k, v in draw(st.lists(st.tuples(_token, _token), max_size=3)))
    version = draw(st.sampled_from(["HTTP/1.1", "HTTP/1.0"]))
    headers = draw(st.lists(st.tuples(_token, _value), max_size=5))
    if draw(st.booleans()):
        headers.append(("Connection", draw(st.sampled_from(["close", "keep-alive", "Upgrade"]))))
    body = draw(st.binary(max_size=64))
    chunked = draw(st.booleans())
    head = f"{method} {path} {version}\r\n" + "".join(f"{k}: {v}\r\n" for k, v in headers)
    if chunked:
        sizes = draw(st.lists(st.integers(1, 16), max_size=5))
        parts, pos = [], 0
        for n in sizes:
            if pos >= len(body):
                break
            part = body[pos:pos + n]
            parts.append(b"%x\r\n" % len(part) + part + b"\r\n")
            pos += len(part)
        msg = (head + "Transfer-Encoding: chunked\r\n\r\n").encode("latin-1") + b"".join(parts) + b"0\r\n\r\n"
    else:
        msg = (head + f"Content-Length: {len(body)}\r\n\r\n").encode("latin-1") + body
    return msg


@settings(max_examples=200, deadline=None)
@given(st.lists(_request(), min_size=1, max_size=3), st.integers(1, 40))
def test_request_property_matches_python(msgs, split):
    data = b"".join(msgs)
    chunks = [data[i:i + split] for i in range(0, len(data), split)]
    assert _server_parse(chunks, True) == _server_parse(chunks, False)


# ------------------------------------------------------------------ responses (client side)


def _client_parse(chunks, native, monkeypatch):
    monkeypatch.setattr(fasthttp, "_codec", codec if native else None)
    loop = asyncio.new_event_loop()
    try:
        conn = fasthttp._Conn()
        conn.transport = _Transport()
        results = []
        conn.fut = loop.create_future()
        for c in chunks:
            conn.data_received(c)
            while conn.fut is None or conn.fut.done():
                if conn.fut is not None:
                    results.append(conn.fut.result() if conn.fut.exception() is None else repr(conn.fut.exception()))
                conn.fut = loop.create_future()
                if not conn.buf:
                    break
                conn._parse()
        return results, bytes(conn.buf), conn.alive
    finally:
        loop.close()


RESPONSES = [
    b"HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\n{}",
    b"HTTP/1.1 429 Too Many Requests\r\nRetry-After: 2\r\nContent-Length: 0\r\n\r\n",
    b"HTTP/1.1 200 OK\r\nRetry-After: 2\r\nContent-Length: 0\r\n\r\n",
    b"HTTP/1.1 503 Unavailable\r\nRetry-After: soon\r\nContent-Length: 1\r\n\r\nx",
    b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n4\r\nWiki\r\n6;e=1\r\npedia \r\n0\r\nX-T: 1\r\n\r\n",
    b"HTTP/1.1 204 No Content\r\n\r\n",
    b"HTTP/1.0 200 OK\r\nContent-Length: 1\r\n\r\na",
    b"HTTP/1.0 200 OK\r\nConnection: keep-alive\r\nContent-Length: 1\r\n\r\na",
    b"HTTP/1.1 200 OK\r\nConnection: close\r\nContent-Length: 1\r\n\r\na",
    b"HTTP/1.1 100 Continue\r\n\r\nHTTP/1.1 201 Created\r\nContent-Length: 2\r\n\r\nok",
]


@pytest.mark.parametrize("msg", RESPONSES)
def test_response_corpus_matches_python(msg, monkeypatch):
    for split in (None, 1, 5):
        chunks = [msg] if split is None else [msg[i:i + split] for i in range(0, len(msg), split)]
        assert _client_parse(chunks, True, monkeypatch) == _client_parse(chunks, False, monkeypatch)


def test_response_read_until_close_falls_back():
    assert codec.parse_response(b"HTTP/1.1 200 OK\r\n\r\nabc") == -1
    assert codec.parse_response(b"HTTP/1.1 100 Continue\r\n\r\n") == -1
    assert codec.parse_response(b"HTTP/1.1 200 OK\r\nContent-Length: 5\r\n\r\nab") is None
    msg = b"HTTP/1.1 429 X\r\nRetry-After: 7\r\nContent-Length: 0\r\n\r\n"
    assert codec.parse_response(msg + b"HTTP/1.1") == (429, b"", len(msg), False, 7)


@settings(max_examples=150, deadline=None)
@given(st.integers(200, 599).filter(lambda s: s not in (204, 304)),  # no body allowed: framing differs
       st.binary(max_size=80), st.booleans(), st.booleans(),
       st.sampled_from(["", "close", "keep-alive"]), st.integers(1, 30))
def test_response_property_matches_python(status, body, chunked, http10, conn, split):
    import pytest as _pytest

    head = f"HTTP/{'1.0' if http10 else '1.1'} {status} X\r\n"
    if conn:
        head += f"Connection: {conn}\r\n"
    if status >= 400:
        head += "Retry-After: 1\r\n"
    if chunked:
        msg = (head + "Transfer-Encoding: chunked\r\n\r\n").encode() + (
            (b"%x\r\n" % len(body) + body + b"\r\n") if body else b"") + b"0\r\n\r\n"
    else:
        msg = (head + f"Content-Length: {len(body)}\r\n\r\n").encode() + body
    chunks = [msg[i:i + split] for i in range(0, len(msg), split)]
    mp = _pytest.MonkeyPatch()
    try:
        assert _client_parse(chunks, True, mp) == _client_parse(chunks, False, mp)
    finally:
        mp.undo()
