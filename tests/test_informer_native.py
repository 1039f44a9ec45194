"""The informer's native event bookkeeping (``_fastjson.store_apply``) against the Python
path it replaces: the same store, derived memos, namespace and label indexes, and the same
handler calls, for random event sequences including malformed objects (which the native
call hands back to Python untouched).  CPU only."""
from __future__ import annotations

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from cron_operator_amd.runtime.informer import EventHandler, Informer, label_index
from cron_operator_amd.utils import jsonutil

pytestmark = pytest.mark.skipif(jsonutil.store_apply is None, reason="_fastjson not built")

LABEL = "kubedl.io/cron-name"

names = st.sampled_from(["a", "b", "c", "", "d/e"])
namespaces = st.one_of(st.sampled_from(["ns1", "ns2", ""]), st.none(), st.just(5))
label_vals = st.one_of(st.sampled_from(["x", "y", ""]), st.none(), st.just(3))


@st.composite
def objects(draw):
    kind = draw(st.integers(0, 9))
    if kind == 0:
        return {"metadata": draw(st.sampled_from([None, [], "m", 0, 1, {}]))}
    m = {}
    if draw(st.booleans()):
        m["name"] = draw(names)
    if draw(st.integers(0, 3)):
        m["namespace"] = draw(namespaces)
    r = draw(st.integers(0, 4))
    if r == 1:
        m["labels"] = {LABEL: draw(label_vals)}
    elif r == 2:
        m["labels"] = draw(st.sampled_from([None, [], "l", {}]))
    elif r == 3:
        m["labels"] = {"other": "z", LABEL: draw(label_vals)}
    m["resourceVersion"] = str(draw(st.integers(0, 99)))
    return {"metadata": m, "v": draw(st.integers(0, 3))}


def _informer(native: bool, log, keep=None):
    inf = Informer(None, "things", indexers={"cron": label_index(LABEL)}, keep=keep)
    if not native:
        inf._napply = None
    else:
        assert inf._napply is not None
    inf.set_derive(lambda o: ("d", (o.get("metadata") or {}).get("resourceVersion") if isinstance(
        o.get("metadata"), dict) else None))
    inf.add_handler(EventHandler(on_add=lambda o: log.append(("add", id(o))),
                                 on_update=lambda old, o: log.append(("upd", id(old), id(o))),
                                 on_delete=lambda o: log.append(("del", id(o)))))
    return inf


def _apply(inf, etype, obj):
    try:
        inf._apply(etype, obj)
        return None
    except Exception as e:  # noqa: BLE001 - both paths must fail the same way
        return type(e)


def _state(inf):
    return (dict(inf.store), dict(inf.derived),
            {n: {v: set(s) for v, s in idx.items()} for n, idx in inf.indices.items()}, inf.events)


def _keep_odd(o):
    """An informer ``keep`` filter (a shard's share): objects whose ``v`` is odd."""
    return o.get("v", 0) % 2 == 1


@pytest.mark.parametrize("keep", [None, _keep_odd], ids=["all", "keep-filter"])
@settings(max_examples=300, deadline=None)
@given(events=st.lists(st.tuples(st.sampled_from(["ADDED", "MODIFIED", "DELETED"]), objects()), max_size=40))
def test_native_bookkeeping_matches_python(keep, events):
    la, lb = [], []
    a, b = _informer(True, la, keep), _informer(False, lb, keep)
    for etype, obj in events:
        # each informer gets its own copy (transforms and stores may keep the object)
        ea = _apply(a, etype, jsonutil.deepcopy(obj))
        eb = _apply(b, etype, jsonutil.deepcopy(obj))
        assert ea == eb
    sa, sb = _state(a), _state(b)
    assert sa[0].keys() == sb[0].keys()
    assert all(jsonutil.json_equal(sa[0][k], sb[0][k]) for k in sa[0])
    assert sa[1] == sb[1] and sa[2] == sb[2] and sa[3] == sb[3]
    assert [e[0] for e in la] == [e[0] for e in lb]
    if keep is not None:
        assert all(keep(o) for o in sa[0].values())  # a rejected version never stays stored


def test_native_path_is_taken_for_regular_objects_and_keeps_identity():
    log = []
    inf = _informer(True, log)
    o1 = {"metadata": {"name": "j1", "namespace": "ns", "labels": {LABEL: "c1"}, "resourceVersion": "1"}}
    inf._apply("ADDED", o1)
    assert inf.store["ns/j1"] is o1 and inf.indices["cron"] == {"ns/c1": {"ns/j1"}}
    assert inf.indices["namespace"] == {"ns": {"ns/j1"}}
    o2 = {"metadata": {"name": "j1", "namespace": "ns", "labels": {LABEL: "c2"}, "resourceVersion": "2"}}
    inf._apply("MODIFIED", o2)
    assert inf.indices["cron"] == {"ns/c2": {"ns/j1"}} and inf.derived["ns/j1"] == ("d", "2")
    inf._apply("DELETED", o2)
    assert not inf.store and not inf.derived and inf.indices == {"namespace": {}, "cron": {}}
    assert [e[0] for e in log] == ["add", "upd", "del"]
    assert log[1][1] == id(o1) and log[1][2] == id(o2)


def test_unknown_index_function_keeps_the_python_path():
    inf = Informer(None, "things", indexers={"custom": lambda o: ["k"]})
    assert inf._napply is None
    inf2 = Informer(None, "things")
    assert inf2._napply is not None
    inf2.add_indexer("custom", lambda o: ["k"])
    assert inf2._napply is None


@settings(max_examples=200, deadline=None)
@given(st.dictionaries(st.text(max_size=3), st.integers()), st.sets(st.text(max_size=3), max_size=8))
def test_pick_matches_the_comprehension(d, keys):
    try:
        want = [d[k] for k in keys]
    except KeyError:
        with pytest.raises(KeyError):
            jsonutil.pick(d, keys)
        return
    assert jsonutil.pick(d, keys) == want == jsonutil.py_pick(d, keys)
