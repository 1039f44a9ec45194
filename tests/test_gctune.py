"""Collector tuning (``utils/gctune.py``): thresholds, the environment override, and the
per-generation time the bench reports."""
from __future__ import annotations

import gc

from cron_operator_amd.utils import gctune


def test_thresholds_from_the_environment(monkeypatch):
    before = gc.get_threshold()
    try:
        monkeypatch.setattr(gctune, "_ENABLED", True)
        monkeypatch.setenv("CRON_OPERATOR_GC_THRESHOLDS", "123456,7,8")
        gctune.tune()
        assert gc.get_threshold() == (123456, 7, 8)
        for bad in ("1,2", "a,b,c", "-1,2,3", ""):
            monkeypatch.setenv("CRON_OPERATOR_GC_THRESHOLDS", bad)
            gctune.tune()
            assert gc.get_threshold() == gctune.DEFAULT_THRESHOLDS, bad
        monkeypatch.setattr(gctune, "_ENABLED", False)
        gc.set_threshold(*before)
        gctune.tune()
        assert gc.get_threshold() == before  # tuning off: left alone
    finally:
        gc.set_threshold(*before)


def test_gc_stats_split_time_by_generation():
    st = gctune.GcStats().start()
    try:
        gc.collect(0)
        gc.collect(2)
    finally:
        st.stop()
    d = st.to_dict()
    assert d["collections"][0] >= 1 and d["collections"][2] >= 1
    assert len(d["ms_by_generation"]) == 3 and abs(sum(d["ms_by_generation"]) - d["ms"]) < 0.1
