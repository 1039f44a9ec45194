"""The operator's event loop: asyncio's selector loop with a native core.

controller-runtime runs the manager, informers and reconcile workers as goroutines on Go's
scheduler (``/root/reference/cmd/operator/start.go:156-209``); this operator runs them as
asyncio tasks on one loop per process.  ``NativeEventLoop`` is ``asyncio.SelectorEventLoop``
with ``call_soon`` and ``_run_once`` -- the per-wake-up machinery every response, watch batch
and work-queue hand-off goes through -- implemented in C++ (``ops/csrc/aioloop.cpp``); all
other behaviour is asyncio's own code on the same ready queue, timer heap and selector.

``install()`` makes ``asyncio.run`` / ``asyncio.new_event_loop`` build it (an event-loop
policy, as uvloop installs itself).  The operator's entry points call it (``cmd/main.py``
``start``/``supervisor``, the bench's operator processes); the fake apiserver fixture keeps
asyncio's stock loop.  ``CRON_OPERATOR_NATIVE_LOOP=python`` (or no native build) leaves
asyncio's loop in place everywhere.
"""
from __future__ import annotations

import asyncio
from typing import Optional, Type

from ..ops import aioloop_native

_loop_cls: Optional[Type[asyncio.AbstractEventLoop]] = None


def loop_class() -> Optional[Type[asyncio.AbstractEventLoop]]:
    """``NativeEventLoop``, or None without the native extension."""
    global _loop_cls
    if _loop_cls is None:
        m = aioloop_native.load()
        if m is None:
            return None

        class NativeEventLoop(m.LoopCore, asyncio.SelectorEventLoop):  # type: ignore[misc,name-defined]
            """asyncio.SelectorEventLoop with native call_soon/_run_once (``_aioloop.LoopCore``)."""

        _loop_cls = NativeEventLoop
    return _loop_cls


def new_event_loop() -> asyncio.AbstractEventLoop:
    cls = loop_class()
    return cls() if cls is not None else asyncio.SelectorEventLoop()


class NativeLoopPolicy(asyncio.DefaultEventLoopPolicy):  # type: ignore[misc,valid-type]
    """The default policy (child watchers and all) building ``NativeEventLoop``s."""

    def new_event_loop(self) -> asyncio.AbstractEventLoop:
        return new_event_loop()


def install() -> bool:
    """Make new event loops native (True), or leave asyncio's policy alone (False: disabled or
    not built)."""
    if loop_class() is None:
        return False
    if not isinstance(asyncio.get_event_loop_policy(), NativeLoopPolicy):
        asyncio.set_event_loop_policy(NativeLoopPolicy())
    return True


def active() -> bool:
    """True when the running loop is the native one."""
    cls = loop_class()
    try:
        return cls is not None and isinstance(asyncio.get_running_loop(), cls)
    except RuntimeError:
        return False
