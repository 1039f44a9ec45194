"""Loader for the ``_netconn`` extension (``csrc/netconn.cpp``).

``load()`` returns the module, or ``None`` when ``CRON_OPERATOR_NATIVE_HTTP=python`` or the
extension cannot be built/imported -- then ``runtime/fasthttp.py`` keeps its asyncio
protocols (with ``=native`` a failure raises instead).  The exception classes the native
connection raises are installed here (``configure``), so callers see the same
``ConnectionFailed``/``HttpStatusError``/``ssl.SSLError`` on both paths.

TLS: the native connections use a ``_netconn.TlsContext`` -- an ``SSL_CTX`` the extension
builds from the kubeconfig's PEM material with the libssl it links (:func:`tls_context`).
An ``ssl.SSLContext`` is accepted natively only when CPython's ``_ssl`` module is proven to
run on that same libssl: ``configure`` receives ``_ssl``'s file and
``ssl.OPENSSL_VERSION_NUMBER`` and checks, with ``dlopen``/``dlsym``, that ``_ssl`` resolves
``SSL_CTX_new`` to the extension's own function and that the build numbers agree.  An
interpreter with its own OpenSSL (pyenv, conda, python.org builds) therefore never has its
``SSL_CTX`` driven by a different libssl; such a pool keeps asyncio's TLS transports unless
it has the PEM material for a ``TlsContext``.
"""
from __future__ import annotations

import importlib
import os
import threading

from . import build as _build

_mod = None
_tried = False
_lock = threading.Lock()


def mode() -> str:
    return os.environ.get("CRON_OPERATOR_NATIVE_HTTP", "auto").lower()


def load():
    global _mod, _tried
    if _tried:
        return _mod
    with _lock:
        if not _tried:
            want = mode()
            if want != "python":
                try:
                    if _build.needs_build("_netconn"):
                        _build.build_extension("_netconn")
                    m = importlib.import_module("cron_operator_amd.ops._netconn")
                    import asyncio
                    import ssl

                    from ..runtime.fasthttp import ConnectionFailed, HttpStatusError

                    import _ssl

                    m.configure(ConnectionFailed, HttpStatusError, ssl.SSLError, asyncio.TimeoutError,
                                getattr(_ssl, "__file__", None), _ssl_version_number())
                    _mod = m
                except Exception:  # noqa: BLE001 - the asyncio protocols remain
                    if want == "native":
                        raise
                    _mod = None
            _tried = True
    return _mod


def _ssl_version_number() -> int:
    """CPython's ``ssl.OPENSSL_VERSION_NUMBER`` (the hook tests override to force a mismatch)."""
    import ssl

    return int(ssl.OPENSSL_VERSION_NUMBER)


def status() -> str:
    """``native`` (TLS through the extension's own OpenSSL, and whether CPython's ``ssl`` shares
    it), or ``asyncio``."""
    m = load()
    if m is None:
        return "asyncio"
    num, text, shared = m.openssl()
    return f"native ({text}{', shared with ssl' if shared else ''})"


def tls_context(material):
    """A ``TlsContext`` from :meth:`RestConfig.tls_material` output, or None (extension missing)."""
    m = load()
    if m is None or material is None:
        return None
    return m.TlsContext(cadata=material.get("cadata"), cafile=material.get("cafile"),
                        certdata=material.get("certdata"), keydata=material.get("keydata"),
                        verify=material.get("verify", True))


def _reset_for_tests() -> None:
    global _mod, _tried
    _mod, _tried = None, False
