"""asyncio helpers that never swallow the caller's own cancellation.

The tempting shutdown idiom::

    task.cancel()
    try:
        await task
    except (asyncio.CancelledError, Exception):
        pass

drops a cancellation aimed at the *caller*: when the caller is cancelled while it
awaits ``task``, the ``CancelledError`` it receives is caught like the task's own
and the caller carries on (Python 3.10 has no ``Task.cancelling()`` to tell the two
apart).  ``asyncio.wait`` never raises a child's exception and raises
``CancelledError`` only for the caller, without touching the children -- so waiting
through it keeps both apart.  controller-runtime's equivalent is a context whose
cancellation reaches every goroutine below it (``cmd/operator/start.go:205-209``).
"""
from __future__ import annotations

import asyncio
import functools
from typing import Iterable, Optional


def consume(tasks: Iterable[Optional["asyncio.Future"]]) -> None:
    """Mark the outcome of every finished task as retrieved (no "exception was never
    retrieved" warnings); errors are dropped -- callers log them where they happen."""
    for t in tasks:
        if t is not None and t.done() and not t.cancelled():
            t.exception()


def _wake(waiter: "asyncio.Future", _t: "asyncio.Future") -> None:
    if not waiter.done():
        waiter.set_result(None)


async def wait_one(t: "asyncio.Future") -> None:
    """Wait until ``t`` has finished, whatever its outcome (``asyncio.wait`` for one task,
    minus its sets and counters: this runs once per reconcile that GCs a child).  The caller
    awaits a private future, so cancelling the caller cancels only that future."""
    if t.done():
        return
    waiter = t.get_loop().create_future()
    cb = functools.partial(_wake, waiter)
    t.add_done_callback(cb)
    try:
        await waiter
    finally:
        t.remove_done_callback(cb)


async def wait_all(tasks: Iterable[Optional["asyncio.Future"]]) -> None:
    """Wait until every task has finished, whatever its outcome.  If the caller is
    cancelled meanwhile, ``CancelledError`` propagates and the tasks keep running."""
    live = [t for t in tasks if t is not None]
    for t in live:
        if not t.done():
            await wait_one(t)
    consume(live)


async def cancel_and_wait(*tasks: Optional["asyncio.Future"]) -> None:
    """Cancel the tasks and wait until they have finished.  A cancellation of the
    caller while it waits propagates (the tasks are already cancelled)."""
    live = [t for t in tasks if t is not None]
    for t in live:
        t.cancel()
    await wait_all(live)


def cancel_all(tasks: Iterable[Optional["asyncio.Future"]]) -> None:
    for t in tasks:
        if t is not None:
            t.cancel()
