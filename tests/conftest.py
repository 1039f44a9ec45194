"""Shared pytest configuration.

* ``gpu`` marker: tests that need a real MI355X (``-m gpu`` on the GPU box).
* ``async def`` tests run in a fresh asyncio loop (no pytest-asyncio in the image).
"""
from __future__ import annotations

import asyncio
import inspect
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# the fake apiserver and reconciler log at info; keep test output quiet
from cron_operator_amd.utils.logging import new_from_options, set_logger  # noqa: E402

set_logger(new_from_options(encoder="console", level="error", stream=open(os.devnull, "w")))

# every asyncio test runs on the operator's loop (native call_soon/_run_once, runtime/aioloop.py)
# unless CRON_OPERATOR_NATIVE_LOOP=python selects asyncio's stock loop (CI runs both tiers)
from cron_operator_amd.runtime import aioloop as _aioloop  # noqa: E402

_aioloop.install()


# Property tests draw the same examples on every run (a CI run must not turn red on a
# fresh random draw); HYPOTHESIS_RANDOM=1 explores new examples when hunting for bugs.
try:
    from hypothesis import settings as _hyp_settings

    _hyp_settings.register_profile("repo", derandomize=os.environ.get("HYPOTHESIS_RANDOM") != "1")
    _hyp_settings.load_profile("repo")
except ImportError:  # pragma: no cover - hypothesis is a test dependency
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) visible to PyTorch")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.hookimpl(tryfirst=True)
def pytest_pyfunc_call(pyfuncitem):
    fn = pyfuncitem.obj
    if inspect.iscoroutinefunction(fn):
        sig = inspect.signature(fn)
        kwargs = {k: v for k, v in pyfuncitem.funcargs.items() if k in sig.parameters}
        timeout = 120
        m = pyfuncitem.get_closest_marker("timeout")
        if m and m.args:
            timeout = m.args[0]

        async def runner():
            return await asyncio.wait_for(fn(**kwargs), timeout)

        asyncio.run(runner())
        return True
    return None
