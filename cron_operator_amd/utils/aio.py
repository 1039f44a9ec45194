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
from typing import Iterable, Optional


def consume(tasks: Iterable[Optional["asyncio.Future"]]) -> None:
    """Mark the outcome of every finished task as retrieved (no "exception was never
    retrieved" warnings); errors are dropped -- callers log them where they happen."""
    for t in tasks:
        if t is not None and t.done() and not t.cancelled():
            t.exception()


async def wait_all(tasks: Iterable[Optional["asyncio.Future"]]) -> None:
    """Wait until every task has finished, whatever its outcome.  If the caller is
    cancelled meanwhile, ``CancelledError`` propagates and the tasks keep running."""
    live = [t for t in tasks if t is not None]
    if live:
        await asyncio.wait(live)
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
