"""HTTP proxies (client-go: kubeconfig ``proxy-url``, else ``HTTPS_PROXY``/``HTTP_PROXY`` minus
``NO_PROXY``): absolute-form requests to plain servers, ``CONNECT`` tunnels to TLS ones, for
both request/response verbs and watch streams, through a small relay proxy that records what
it was asked."""
from __future__ import annotations

import asyncio
import base64
import os
import ssl
import tempfile

import pytest
import yaml

from cron_operator_amd.api import errors
from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.apiserver.http import APIServerApp, _origin_form
from cron_operator_amd.runtime.client import Client
from cron_operator_amd.runtime.http import HttpTransport
from cron_operator_amd.runtime.kubeconfig import ConfigError, RestConfig, _no_proxy_match, load_kubeconfig, \
    proxy_from_environment
from cron_operator_amd.runtime.servers import self_signed_cert
from cron_operator_amd.testing.env import TestEnv

CM = GroupVersionResource("", "v1", "configmaps")


class RelayProxy:
    """A forward proxy: ``CONNECT host:port`` opens a tunnel; an absolute-form request is
    relayed, with every later byte of the connection, to the host it names."""

    def __init__(self, require_auth: str = ""):
        self.heads: list = []
        self.require_auth = require_auth
        self.server = None
        self.port = 0

    async def start(self) -> int:
        self.server = await asyncio.start_server(self._handle, "127.0.0.1", 0)
        self.port = self.server.sockets[0].getsockname()[1]
        return self.port

    async def stop(self) -> None:
        self.server.close()
        await self.server.wait_closed()

    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        try:
            head = await reader.readuntil(b"\r\n\r\n")
        except (asyncio.IncompleteReadError, ConnectionError):
            writer.close()
            return
        text = head.decode("latin-1")
        self.heads.append(text)
        method, target, _ = text.split("\r\n", 1)[0].split(" ", 2)
        if self.require_auth and f"Proxy-Authorization: Basic {self.require_auth}" not in text:
            writer.write(b"HTTP/1.1 407 Proxy Authentication Required\r\nContent-Length: 0\r\n\r\n")
            await writer.drain()
            writer.close()
            return
        if method == "CONNECT":
            host, port = target.rsplit(":", 1)
            ur, uw = await asyncio.open_connection(host, int(port))
            writer.write(b"HTTP/1.1 200 Connection established\r\n\r\n")
        else:
            authority = target.split("://", 1)[1].split("/", 1)[0]
            host, port = authority.rsplit(":", 1)
            ur, uw = await asyncio.open_connection(host, int(port))
            uw.write(head)

        async def pipe(r: asyncio.StreamReader, w: asyncio.StreamWriter) -> None:
            try:
                while True:
                    data = await r.read(65536)
                    if not data:
                        break
                    w.write(data)
                    await w.drain()
            except (ConnectionError, asyncio.CancelledError):
                pass
            finally:
                w.close()

        await asyncio.gather(pipe(reader, uw), pipe(ur, writer))


def _auth(user: str, pw: str) -> str:
    return base64.b64encode(f"{user}:{pw}".encode()).decode()


@pytest.mark.parametrize("tls", [False, True])
@pytest.mark.parametrize("fast", [True, False])
async def test_requests_and_watch_through_proxy(tls, fast):
    env = TestEnv()
    app = APIServerApp(env.server)
    with tempfile.TemporaryDirectory() as d:
        ctx = None
        if tls:
            crt, key = self_signed_cert(d)
            ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
            ctx.load_cert_chain(crt, key)
        port = await app.start("127.0.0.1", 0, ssl_context=ctx)
        proxy = RelayProxy(require_auth=_auth("op", "p@ss"))
        pport = await proxy.start()
        scheme = "https" if tls else "http"
        cfg = RestConfig(host=f"{scheme}://127.0.0.1:{port}", insecure=tls,
                         proxy_url=f"http://op:p%40ss@127.0.0.1:{pport}")
        c = Client(HttpTransport(cfg, fast=fast), qps=-1)
        try:
            if fast:
                from cron_operator_amd.ops import netconn_native

                # the native connections go through the proxy too (absolute form / CONNECT tunnel)
                assert c.transport._fast_pool().native == (netconn_native.load() is not None)
            await c.create(CM, {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "a"}}, "default")
            assert (await c.get(CM, "default", "a"))["metadata"]["name"] == "a"
            with pytest.raises(errors.ApiError) as e:
                await c.get(CM, "default", "missing")
            assert e.value.code == 404
            w = await c.watch(CM, "default", resource_version="0")
            ev = await asyncio.wait_for(w.__anext__(), 10)
            assert ev[0] == "ADDED" and ev[1]["metadata"]["name"] == "a"
            w.stop()
        finally:
            await c.close()
            await app.stop()
            await proxy.stop()
    assert proxy.heads, "nothing went through the proxy"
    for h in proxy.heads:
        first = h.split("\r\n", 1)[0]
        if tls:
            assert first == f"CONNECT 127.0.0.1:{port} HTTP/1.1"
        else:
            assert first.split(" ")[1].startswith(f"http://127.0.0.1:{port}/api/v1/")
        assert f"Proxy-Authorization: Basic {_auth('op', 'p@ss')}" in h


async def test_proxy_refusal_surfaces_as_connection_error():
    env = TestEnv()
    app = APIServerApp(env.server)
    with tempfile.TemporaryDirectory() as d:
        crt, key = self_signed_cert(d)
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(crt, key)
        port = await app.start("127.0.0.1", 0, ssl_context=ctx)
        proxy = RelayProxy(require_auth="nope")
        pport = await proxy.start()
        c = Client(HttpTransport(RestConfig(host=f"https://127.0.0.1:{port}", insecure=True,
                                            proxy_url=f"http://127.0.0.1:{pport}")), qps=-1)
        try:
            with pytest.raises(errors.ApiError) as e:
                await c.get(CM, "default", "a")
            assert e.value.code == 503 and "407" in e.value.message
        finally:
            await c.close()
            await app.stop()
            await proxy.stop()


@pytest.mark.parametrize("host,port,entries,hit", [
    ("api.example.com", 443, "*", True),
    ("api.example.com", 443, "example.com", True),
    ("example.com", 443, "example.com", True),
    ("example.com", 443, ".example.com", False),      # leading dot: subdomains only
    ("api.example.com", 443, ".example.com", True),
    ("api.example.com", 443, "*.example.com", True),
    ("badexample.com", 443, "example.com", False),
    ("api.example.com", 443, "example.com:6443", False),
    ("api.example.com", 6443, "example.com:6443", True),
    ("10.1.2.3", 443, "10.0.0.0/8", True),
    ("11.1.2.3", 443, "10.0.0.0/8", False),
    ("10.1.2.3", 443, "10.1.2.3", True),
    ("10.1.2.3", 443, "10.1.2.3:80", False),
    ("fd00::1", 443, "fd00::/8", True),
    ("fd00::1", 443, "[fd00::1]:443", True),
    ("API.Example.COM", 443, " other.org , EXAMPLE.com ", True),
])
def test_no_proxy_rules(host, port, entries, hit):
    assert _no_proxy_match(host, port, entries) is hit


def test_proxy_from_environment(monkeypatch):
    for n in ("HTTPS_PROXY", "https_proxy", "HTTP_PROXY", "http_proxy", "NO_PROXY", "no_proxy"):
        monkeypatch.delenv(n, raising=False)
    assert proxy_from_environment("https://api.example.com") == ""
    monkeypatch.setenv("https_proxy", "http://lower:3128")
    assert proxy_from_environment("https://api.example.com") == "http://lower:3128"
    monkeypatch.setenv("HTTPS_PROXY", "http://upper:3128")
    assert proxy_from_environment("https://api.example.com") == "http://upper:3128"
    assert proxy_from_environment("http://api.example.com") == ""  # HTTP_PROXY for http servers
    monkeypatch.setenv("HTTP_PROXY", "plain:8080")
    assert proxy_from_environment("http://api.example.com") == "plain:8080"
    # loopback is never proxied
    assert proxy_from_environment("https://127.0.0.1:6443") == ""
    assert proxy_from_environment("https://localhost:6443") == ""
    assert proxy_from_environment("https://[::1]:6443") == ""
    monkeypatch.setenv("NO_PROXY", "example.com,10.96.0.0/12")
    assert proxy_from_environment("https://api.example.com") == ""
    assert proxy_from_environment("https://10.96.0.1:443") == ""
    assert proxy_from_environment("https://api.other.org") == "http://upper:3128"
    monkeypatch.setenv("HTTPS_PROXY", "socks5://s:1080")
    with pytest.raises(ConfigError, match="only http://"):
        proxy_from_environment("https://api.other.org")
    # a client built in such an environment connects directly (warned once, at construction)
    # instead of failing every request
    from cron_operator_amd.runtime.http import HttpTransport

    cfg = RestConfig(host="https://api.other.org")
    assert cfg.proxy() == ""
    t = HttpTransport(cfg)
    assert t._proxy == "" and t._fast_pool()._proxy is None


def test_kubeconfig_proxy_url():
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "kc")

        def write(proxy: str) -> None:
            doc = {"current-context": "c",
                   "clusters": [{"name": "c", "cluster": {"server": "https://127.0.0.1:6443", "proxy-url": proxy}}],
                   "users": [{"name": "u", "user": {"token": "t"}}],
                   "contexts": [{"name": "c", "context": {"cluster": "c", "user": "u"}}]}
            with open(p, "w") as fh:
                yaml.safe_dump(doc, fh)

        write("http://proxy.corp:3128")
        cfg = load_kubeconfig(p)
        assert cfg.proxy() == "http://proxy.corp:3128"  # proxy-url applies even to loopback
        write("https://proxy.corp:3128")
        with pytest.raises(ConfigError, match="only http://"):
            load_kubeconfig(p)


@pytest.mark.parametrize("target,origin", [
    ("/api/v1/pods?watch=true", "/api/v1/pods?watch=true"),
    ("http://h:1/api/v1/pods?watch=true", "/api/v1/pods?watch=true"),
    ("HTTPS://h/apis", "/apis"),
    ("http://h:1", "/"),
    ("http://h:1?x=1", "/?x=1"),
])
def test_absolute_form_targets(target, origin):
    assert _origin_form(target) == origin
