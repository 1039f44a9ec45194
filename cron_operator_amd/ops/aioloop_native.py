"""Loader for the ``_aioloop`` extension (``csrc/aioloop.cpp``).

``load()`` returns the configured module, or ``None`` when ``CRON_OPERATOR_NATIVE_LOOP=python``
or the extension cannot be built/imported -- then the operator runs on asyncio's own loop
(with ``=native`` a failure raises instead).  ``configure`` hands the extension the pieces of
asyncio it defers to: the selector class it can poll natively, ``heapq``'s heap operations on
the timer heap, asyncio's callback formatting, and ``BaseEventLoop``'s Python ``call_soon`` /
``_run_once`` for debug mode.

**Interpreter gate.**  The core re-implements CPython's private ``BaseEventLoop._run_once``,
``Handle`` and selector bookkeeping (``_ready``, ``_scheduled``, ``_timer_cancelled_count``,
``_fd_to_key``) as they are in the minor versions listed in :data:`SUPPORTED`.  Those are
private and change between releases, so on any other interpreter the loader does not load
the extension at all and asyncio's own loop runs (``=native`` raises instead); the reason is
logged once.  :func:`status` says which loop runs and why.
"""
from __future__ import annotations

import importlib
import os
import platform
import sys
import threading

from . import build as _build

# CPython minor versions whose asyncio internals aioloop.cpp was written against
SUPPORTED = ((3, 10),)

_mod = None
_tried = False
_reason = ""
_lock = threading.Lock()


def interpreter_supported(version=None, implementation=None) -> bool:
    v = tuple((version or sys.version_info)[:2])
    return (implementation or platform.python_implementation()) == "CPython" and v in SUPPORTED


def status() -> str:
    """``native``, or ``asyncio: <reason>`` (after :func:`load`)."""
    load()
    return "native" if _mod is not None else f"asyncio: {_reason}"


def mode() -> str:
    return os.environ.get("CRON_OPERATOR_NATIVE_LOOP", "auto").lower()


def load():
    global _mod, _tried, _reason
    if _tried:
        return _mod
    with _lock:
        if not _tried:
            want = mode()
            if want == "python":
                _reason = "CRON_OPERATOR_NATIVE_LOOP=python"
            elif not interpreter_supported():
                _reason = (f"{platform.python_implementation()} {sys.version_info[0]}.{sys.version_info[1]} is not "
                           f"one of the versions the native core targets "
                           f"({', '.join('%d.%d' % v for v in SUPPORTED)})")
                if want == "native":
                    _tried = True
                    raise RuntimeError(f"native event loop unavailable: {_reason}")
                _log_fallback(_reason)
            else:
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
                except Exception as e:  # noqa: BLE001 - asyncio's own loop remains
                    if want == "native":
                        raise
                    _mod = None
                    _reason = f"extension unavailable: {e}"
                    _log_fallback(_reason)
            _tried = True
    return _mod


def _log_fallback(reason: str) -> None:
    from ..utils.logging import get_logger

    get_logger("aioloop").info("running on asyncio's event loop", reason=reason)


def _reset_for_tests() -> None:
    global _mod, _tried, _reason
    _mod, _tried, _reason = None, False, ""
