"""Loader for the ``_aioloop`` extension (``csrc/aioloop.cpp``).

``load()`` returns the configured module, or ``None`` when ``CRON_OPERATOR_NATIVE_LOOP=python``
or the extension cannot be built/imported -- then the operator runs on asyncio's own loop
(with ``=native`` a failure raises instead).  ``configure`` hands the extension the pieces of
asyncio it defers to: the selector class it can poll natively, ``heapq``'s heap operations on
the timer heap, asyncio's callback formatting, and ``BaseEventLoop``'s Python ``call_soon`` /
``_run_once`` for debug mode.
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
    return os.environ.get("CRON_OPERATOR_NATIVE_LOOP", "auto").lower()


def load():
    global _mod, _tried
    if _tried:
        return _mod
    with _lock:
        if not _tried:
            want = mode()
            if want != "python":
                try:
                    if _build.needs_build("_aioloop"):
                        _build.build_extension("_aioloop")
                    m = importlib.import_module("cron_operator_amd.ops._aioloop")
                    import heapq
                    import selectors
                    from asyncio import base_events, format_helpers

                    m.configure(selectors.EpollSelector if hasattr(selectors, "EpollSelector") else type(None),
                                heapq.heappop, heapq.heapify, format_helpers._format_callback_source,
                                base_events.BaseEventLoop.call_soon, base_events.BaseEventLoop._run_once)
                    _mod = m
                except Exception:  # noqa: BLE001 - asyncio's own loop remains
                    if want == "native":
                        raise
                    _mod = None
            _tried = True
    return _mod
