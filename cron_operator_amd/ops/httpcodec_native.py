"""Loader for the ``_httpcodec`` extension (``csrc/httpcodec.cpp``).

``load()`` returns the module, or ``None`` when ``CRON_OPERATOR_HTTPCODEC=python``
or the extension cannot be built/imported (then the pure-Python parsers in
``runtime/fasthttp.py`` and ``apiserver/http.py`` run; with ``=native`` a failure
raises instead).
"""
from __future__ import annotations

import importlib
import os
import threading

from . import build as _build

_mod = None
_tried = False
_lock = threading.Lock()


def load():
    global _mod, _tried
    if _tried:
        return _mod
    with _lock:
        if not _tried:
            want = os.environ.get("CRON_OPERATOR_HTTPCODEC", "auto").lower()
            if want != "python":
                try:
                    if _build.needs_build("_httpcodec"):
                        _build.build_extension("_httpcodec")
                    _mod = importlib.import_module("cron_operator_amd.ops._httpcodec")
                except Exception:  # noqa: BLE001 - pure-Python fallback
                    if want == "native":
                        raise
                    _mod = None
            _tried = True
    return _mod
