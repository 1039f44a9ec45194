"""Loader for the ``_fastjson`` extension (``csrc/fastjson.cpp``)."""
from __future__ import annotations

import importlib
import threading

from . import build as _build

_mod = None
_lock = threading.Lock()


def load(build_if_missing: bool = True):
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None:
            if build_if_missing and _build.needs_build("_fastjson"):
                _build.build_extension("_fastjson")
            _mod = importlib.import_module("cron_operator_amd.ops._fastjson")
    return _mod
