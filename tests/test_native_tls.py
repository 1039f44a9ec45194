"""Native TLS without CPython internals: ``_netconn.TlsContext`` and the shared-OpenSSL guard.

The native connections (``ops/csrc/netconn.cpp``) build their own ``SSL_CTX`` from the
kubeconfig's PEM material with the libssl the extension links.  A plain ``ssl.SSLContext``
is driven natively only when CPython's ``_ssl`` provably runs on that same libssl
(``configure`` checks the build number and, with ``dlopen``/``dlsym``, that ``_ssl``'s
``SSL_CTX_new`` is the extension's own).  A forced mismatch must fall back to asyncio's TLS
transports -- or keep the native path through a ``TlsContext`` -- with identical results.
Reference: the operator's rest config is client-go's (``/root/reference/cmd/operator/start.go:152-154``),
which verifies the apiserver against the kubeconfig CA and presents its client certificate.
"""
from __future__ import annotations

import asyncio
import ssl

import pytest

from cron_operator_amd.ops import netconn_native
from cron_operator_amd.runtime.fasthttp import ConnectionFailed, HttpPool
from cron_operator_amd.runtime.kubeconfig import RestConfig

nc = netconn_native.load()
pytestmark = pytest.mark.skipif(nc is None, reason="_netconn extension not built")


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    from cron_operator_amd.runtime.servers import self_signed_cert

    d = tmp_path_factory.mktemp("pki")
    (d / "srv").mkdir()
    (d / "cli").mkdir()
    (d / "other").mkdir()
    scert, skey = self_signed_cert(str(d / "srv"), host="localhost")
    ccert, ckey = self_signed_cert(str(d / "cli"), host="operator")
    other, _ = self_signed_cert(str(d / "other"), host="localhost")
    rd = lambda p: open(p, "rb").read()  # noqa: E731
    return {"scert": scert, "skey": skey, "ccert": ccert, "ckey": ckey, "other": other,
            "scert_pem": rd(scert), "ccert_pem": rd(ccert), "ckey_pem": rd(ckey), "other_pem": rd(other)}


async def _server(pki, mtls=False):
    sctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    sctx.load_cert_chain(pki["scert"], pki["skey"])
    if mtls:
        sctx.verify_mode = ssl.CERT_REQUIRED
        sctx.load_verify_locations(cafile=pki["ccert"])
    peers = []

    async def handle(reader, writer):
        try:
            peers.append(writer.get_extra_info("peercert"))
            while True:
                head = await reader.readuntil(b"\r\n\r\n")
                path = head.split(b" ")[1]
                writer.write(b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n" % len(path) + path)
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionResetError, ssl.SSLError):
            pass
        writer.close()

    srv = await asyncio.start_server(handle, "127.0.0.1", 0, ssl=sctx)
    return srv, srv.sockets[0].getsockname()[1], peers


@pytest.fixture
def forced_mismatch(monkeypatch):
    """Reload the extension's configuration as if CPython's ssl module reported another
    OpenSSL build; restore the real configuration afterwards."""
    monkeypatch.setattr(netconn_native, "_ssl_version_number", lambda: 0x1010107F)  # 1.1.1g
    netconn_native._reset_for_tests()
    m = netconn_native.load()
    yield m
    monkeypatch.undo()
    netconn_native._reset_for_tests()
    netconn_native.load()


def test_openssl_is_reported_and_shared_on_this_interpreter():
    num, text, shared = nc.openssl()
    assert num > 0 and "OpenSSL" in text
    assert shared is True  # the system python links the system libssl the extension links
    assert nc.ssl_context_supported(ssl.create_default_context())
    assert "native" in netconn_native.status()


def test_forced_version_mismatch_refuses_ssl_contexts(forced_mismatch):
    m = forced_mismatch
    assert m.openssl()[2] is False
    # the SSLContext is refused before its SSL_CTX is read at all; a TlsContext is unaffected
    assert not m.ssl_context_supported(ssl.create_default_context())
    assert m.ssl_context_supported(m.TlsContext(verify=False))


def test_wrong_ssl_module_path_is_not_trusted():
    """configure() with an _ssl path that is not loaded (or not _ssl): not shared."""
    import asyncio as aio

    from cron_operator_amd.runtime.fasthttp import HttpStatusError

    try:
        nc.configure(ConnectionFailed, HttpStatusError, ssl.SSLError, aio.TimeoutError, "/nonexistent/_ssl.so",
                     ssl.OPENSSL_VERSION_NUMBER)
        assert nc.openssl()[2] is False
        assert not nc.ssl_context_supported(ssl.create_default_context())
    finally:
        netconn_native._reset_for_tests()
        netconn_native.load()


async def test_mismatch_falls_back_to_asyncio_tls_with_identical_results(pki, forced_mismatch):
    srv, port, _ = await _server(pki)
    try:
        ctx = ssl.create_default_context(cafile=pki["scert"])
        url = f"https://127.0.0.1:{port}"
        fallback = HttpPool(url, ssl_context=ctx, server_hostname="localhost")
        assert fallback.native is False  # asyncio's TLS transports
        own = HttpPool(url, ssl_context=ctx, server_hostname="localhost",
                       tls_material={"cadata": pki["scert_pem"], "verify": True})
        assert own.native is True  # the extension's own SSL_CTX
        for pool in (fallback, own):
            assert await pool.request("GET", "/a/b") == (200, b"/a/b")
            assert await pool.request("GET", "/c") == (200, b"/c")
            await pool.close()
    finally:
        srv.close()


async def test_tls_context_verifies_ca_and_hostname(pki):
    srv, port, _ = await _server(pki)
    url = f"https://127.0.0.1:{port}"
    try:
        good = HttpPool(url, ssl_context=ssl.create_default_context(cafile=pki["scert"]),
                        server_hostname="localhost", tls_material={"cadata": pki["scert_pem"]}, native=True)
        assert good._native_tls is not None
        assert await good.request("GET", "/ok") == (200, b"/ok")
        await good.close()
        # a CA that did not sign the server's certificate
        bad_ca = HttpPool(url, ssl_context=ssl.create_default_context(cafile=pki["other"]),
                          server_hostname="localhost", tls_material={"cadata": pki["other_pem"]}, native=True)
        with pytest.raises((ssl.SSLError, ConnectionFailed)):
            await bad_ca.request("GET", "/")
        await bad_ca.close()
        # the right CA, the wrong name
        bad_name = HttpPool(url, ssl_context=ssl.create_default_context(cafile=pki["scert"]),
                            server_hostname="apiserver.example", tls_material={"cadata": pki["scert_pem"]},
                            native=True)
        with pytest.raises((ssl.SSLError, ConnectionFailed)):
            await bad_name.request("GET", "/")
        await bad_name.close()
    finally:
        srv.close()


async def test_tls_context_presents_the_client_certificate(pki):
    srv, port, peers = await _server(pki, mtls=True)
    url = f"https://127.0.0.1:{port}"
    try:
        ctx = ssl.create_default_context(cafile=pki["scert"])
        ctx.load_cert_chain(pki["ccert"], pki["ckey"])
        pool = HttpPool(url, ssl_context=ctx, server_hostname="localhost", native=True,
                        tls_material={"cadata": pki["scert_pem"], "certdata": pki["ccert_pem"],
                                      "keydata": pki["ckey_pem"]})
        assert await pool.request("GET", "/m") == (200, b"/m")
        await pool.close()
        assert dict(x[0] for x in peers[-1]["subject"])["commonName"] == "operator"
    finally:
        srv.close()


def test_tls_context_rejects_bad_material(pki):
    with pytest.raises(ssl.SSLError):
        nc.TlsContext(cadata=b"not a certificate")
    with pytest.raises(ssl.SSLError):
        nc.TlsContext(cadata=pki["scert_pem"], certdata=pki["ccert_pem"], keydata=b"garbage")
    with pytest.raises(ssl.SSLError):  # a key that is not the certificate's
        nc.TlsContext(certdata=pki["ccert_pem"], keydata=open(pki["skey"], "rb").read(), verify=False)
    assert nc.TlsContext(verify=False).verify is False
    assert nc.TlsContext(cadata=pki["scert_pem"]).verify is True


def test_rest_config_tls_material(pki, tmp_path):
    rc = RestConfig(host="https://10.0.0.1:6443", ca_data=pki["scert_pem"], cert_data=pki["ccert_pem"],
                    key_data=pki["ckey_pem"])
    m = rc.tls_material()
    assert m["cadata"] == pki["scert_pem"] and m["certdata"] == pki["ccert_pem"] and m["verify"] is True
    rc2 = RestConfig(host="https://10.0.0.1:6443", insecure=True)
    assert rc2.tls_material()["verify"] is False and rc2.tls_material()["cadata"] is None
    rc3 = RestConfig(host="https://10.0.0.1:6443", ca_file=pki["scert"], cert_file=pki["ccert"], key_file=pki["ckey"])
    m3 = rc3.tls_material()
    assert m3["cafile"] == pki["scert"] and m3["certdata"] == pki["ccert_pem"] and m3["keydata"] == pki["ckey_pem"]
    assert RestConfig(host="http://127.0.0.1:8080").tls_material() is None
