"""The work queue's native core (``ops/csrc/workqueue.cpp``) against its Python twin
(``parallel/workqueue.py``): the same keys come out in the same order after any sequence of
adds (with priorities), gets, dones and shutdown, with the same dedupe/parking counts and the
same metered depth, adds, queue-latency and work-duration samples.  Every other queue test
(``tests/test_runtime.py``) runs on whichever core is active."""
from __future__ import annotations

import asyncio
import itertools

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from cron_operator_amd.parallel import workqueue as wq
from cron_operator_amd.parallel.workqueue import ShutDown, WorkQueue

_ids = itertools.count()


def _pair():
    n = next(_ids)
    nat = WorkQueue(f"native-{n}")
    py = WorkQueue(f"python-{n}", native=False)
    if nat._core is None:
        pytest.skip("_workqueue not built or disabled")
    assert py._core is None
    return nat, py


def _state(q: WorkQueue):
    return (len(q), q.processing(), q.idle(), q.adds, q.gets, q._m_depth.value, q._m_adds.value,
            q._m_latency.count, q._m_work.count)


_OPS = st.lists(st.one_of(
    st.tuples(st.just("add"), st.integers(0, 5), st.integers(0, 3)),
    st.tuples(st.just("get"), st.just(0), st.just(0)),
    st.tuples(st.just("done"), st.integers(0, 5), st.just(0)),
    st.tuples(st.just("shutdown"), st.just(0), st.just(0)),
), max_size=80)


@settings(max_examples=300, deadline=None)
@given(_OPS)
def test_native_core_matches_python_core(ops):
    nat, py = _pair()
    for op, k, p in ops:
        if op == "add":
            nat.add(("ns", f"k{k}"), p)
            py.add(("ns", f"k{k}"), p)
        elif op == "get":
            a, b = nat._core.pop(), py._pop()
            assert a == b or (a is wq._EMPTY and b is wq._EMPTY)
        elif op == "done":
            nat.done(("ns", f"k{k}"))
            py.done(("ns", f"k{k}"))
        else:
            nat.shutdown()
            py.shutdown()
        assert _state(nat) == _state(py)
    # drain: the rest comes out in the same order
    while True:
        a, b = nat._core.pop(), py._pop()
        assert a == b or (a is wq._EMPTY and b is wq._EMPTY)
        if a is wq._EMPTY:
            break


async def test_native_get_waits_is_woken_and_serialises_keys():
    nat, _ = _pair()
    got = []

    async def worker():
        while True:
            try:
                k = await nat.get()
            except ShutDown:
                return
            got.append(k)
            await asyncio.sleep(0)
            nat.add(k)  # parked while processing: comes back after done
            nat.done(k)

    t = asyncio.get_running_loop().create_task(worker())
    await asyncio.sleep(0)
    nat.add("a")
    for _ in range(20):
        await asyncio.sleep(0)
    nat.shutdown()
    await asyncio.wait_for(t, 5)
    assert got[:3] == ["a", "a", "a"] and nat.adds >= 2


async def test_native_get_cancelled_waiter_is_removed():
    nat, _ = _pair()
    t = asyncio.get_running_loop().create_task(nat.get())
    await asyncio.sleep(0)
    t.cancel()
    with pytest.raises(asyncio.CancelledError):
        await t
    nat.add("x")  # no cancelled future is woken instead of a live getter
    t2 = asyncio.get_running_loop().create_task(nat.get())
    assert await asyncio.wait_for(t2, 5) == "x"


async def test_native_shutdown_wakes_getters():
    nat, _ = _pair()
    ts = [asyncio.get_running_loop().create_task(nat.get()) for _ in range(3)]
    await asyncio.sleep(0)
    nat.shutdown()
    for t in ts:
        with pytest.raises(ShutDown):
            await asyncio.wait_for(t, 5)
    nat.add("late")
    assert len(nat) == 0


def test_unfinished_metrics_read_the_native_start_times():
    nat, _ = _pair()
    nat.add("a")
    assert nat._core.pop() == "a"
    nat.update_unfinished_metrics()
    assert nat._m_unfinished.value >= 0 and nat._m_longest.value >= 0
    assert len(nat._core.started()) == 1
    nat.done("a")
    assert nat._core.started() == [] and nat.idle()
