"""Loader for the ``_netconn`` extension (``csrc/netconn.cpp``).

``load()`` returns the module, or ``None`` when ``CRON_OPERATOR_NATIVE_HTTP=python`` or the
extension cannot be built/imported -- then ``runtime/fasthttp.py`` keeps its asyncio
protocols (with ``=native`` a failure raises instead).  The exception classes the native
connection raises are installed here (``configure``), so callers see the same
``ConnectionFailed``/``HttpStatusError``/``ssl.SSLError`` on both paths.
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

                    m.configure(ConnectionFailed, HttpStatusError, ssl.SSLError, asyncio.TimeoutError)
                    _mod = m
                except Exception:  # noqa: BLE001 - the asyncio protocols remain
                    if want == "native":
                        raise
                    _mod = None
            _tried = True
    return _mod
