"""Fake apiserver fidelity (the envtest analog, SURVEY section 4 "Implication").

CRUD, label/field selectors, paging, resourceVersion + watch semantics
(resume, 410, filtered transitions), the status subresource, merge/JSON
patch, no-op writes, optimistic concurrency, CRD defaulting/enum/required,
finalizers, ownerReference GC and fault injection -- in-process and over HTTP.
"""
from __future__ import annotations

import asyncio

import pytest

from cron_operator_amd.api import errors
from cron_operator_amd.api.meta import GroupVersionResource
from cron_operator_amd.api.selectors import (
    SelectorError,
    matches_fields,
    matches_labels,
    parse_field_selector,
    parse_label_selector,
)
from cron_operator_amd.api.v1alpha1 import CRON_GVR, new_cron
from cron_operator_amd.api.v1alpha1.crd import crd
from cron_operator_amd.apiserver import schema as sch
from cron_operator_amd.apiserver.server import APIServer
from cron_operator_amd.trainingop.crds import kubeflow_crds
from cron_operator_amd.utils.clock import FakeClock

PT = GroupVersionResource("kubeflow.org", "v1", "pytorchjobs")
CM = GroupVersionResource("", "v1", "configmaps")
NSR = GroupVersionResource("", "v1", "namespaces")


def mk(gc=False):
    s = APIServer(FakeClock(1767268805 * 10**9), gc=gc)
    s.install_crd(crd())
    for c in kubeflow_crds():
        s.install_crd(c)
    return s


def cm(name, labels=None, **data):
    m = {"name": name}
    if labels:
        m["labels"] = labels
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": m, "data": data}


# ---------------------------------------------------------------- selectors


@pytest.mark.parametrize("sel,labels,ok", [
    ("a=b", {"a": "b"}, True), ("a==b", {"a": "b"}, True), ("a!=b", {"a": "c"}, True), ("a!=b", {}, True),
    ("a", {"a": ""}, True), ("!a", {"a": "x"}, False), ("a in (x, y)", {"a": "y"}, True),
    ("a notin (x)", {"a": "x"}, False), ("a=b,c=d", {"a": "b", "c": "e"}, False),
    ("kubedl.io/cron-name=c1", {"kubedl.io/cron-name": "c1"}, True), ("", {}, True),
])
def test_label_selectors(sel, labels, ok):
    assert matches_labels(parse_label_selector(sel), labels) == ok


def test_label_selector_errors():
    with pytest.raises(SelectorError):
        parse_label_selector("a in x")
    with pytest.raises(SelectorError):
        parse_label_selector("a=b c=d")


def test_field_selectors():
    obj = {"metadata": {"name": "n", "namespace": "ns"}}
    assert matches_fields(parse_field_selector("metadata.name=n,metadata.namespace!=x"), obj)
    assert not matches_fields(parse_field_selector("metadata.name==m"), obj)


# ---------------------------------------------------------------- CRUD and RV


def test_create_get_list_update_delete():
    s = mk()
    a = s.create(CM, "default", cm("a", {"app": "x"}, k="1"))
    assert a["metadata"]["uid"] and a["metadata"]["resourceVersion"] and a["metadata"]["generation"] == 1
    assert a["metadata"]["creationTimestamp"] == "2026-01-01T12:00:05Z"  # second precision
    with pytest.raises(errors.ApiError) as e:
        s.create(CM, "default", cm("a"))
    assert errors.is_already_exists(e.value) and e.value.code == 409
    s.create(CM, "default", cm("b", {"app": "y"}))
    assert [o["metadata"]["name"] for o in s.list(CM, "default", "app=x")["items"]] == ["a"]
    a["data"]["k"] = "2"
    u = s.update(CM, "default", "a", a)
    assert int(u["metadata"]["resourceVersion"]) > int(a["metadata"]["resourceVersion"])
    with pytest.raises(errors.ApiError) as e:
        s.update(CM, "default", "a", a)  # stale RV
    assert errors.is_conflict(e.value)
    s.delete(CM, "default", "a")
    with pytest.raises(errors.ApiError) as e:
        s.get(CM, "default", "a")
    assert errors.is_not_found(e.value)
    assert e.value.message == 'configmaps "a" not found'


def test_namespace_must_exist_and_generate_name():
    s = mk()
    with pytest.raises(errors.ApiError) as e:
        s.create(CM, "nope", cm("a"))
    assert errors.is_not_found(e.value)
    s.create_namespace("nope")
    o = s.create(CM, "nope", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"generateName": "x-"}})
    assert o["metadata"]["name"].startswith("x-") and len(o["metadata"]["name"]) == 7


def test_invalid_name_rejected():
    s = mk()
    with pytest.raises(errors.ApiError) as e:
        s.create(CM, "default", cm("Bad_Name"))
    assert errors.is_invalid(e.value)


def test_paging():
    s = mk()
    for i in range(7):
        s.create(CM, "default", cm(f"c{i}"))
    page = s.list(CM, "default", limit=3)
    names = [o["metadata"]["name"] for o in page["items"]]
    while page["metadata"].get("continue"):
        page = s.list(CM, "default", limit=3, continue_=page["metadata"]["continue"])
        names += [o["metadata"]["name"] for o in page["items"]]
    assert names == [f"c{i}" for i in range(7)]


def test_noop_update_and_patch_keep_rv():
    s = mk()
    a = s.create(CM, "default", cm("a", k="1"))
    rv = a["metadata"]["resourceVersion"]
    assert s.update(CM, "default", "a", a)["metadata"]["resourceVersion"] == rv
    assert s.patch(CM, "default", "a", {"data": {"k": "1"}})["metadata"]["resourceVersion"] == rv
    assert s.patch(CM, "default", "a", {})["metadata"]["resourceVersion"] == rv


def test_merge_and_json_patch():
    s = mk()
    s.create(CM, "default", cm("a", k="1", j="2"))
    o = s.patch(CM, "default", "a", {"data": {"k": None, "z": "3"}})
    assert o["data"] == {"j": "2", "z": "3"}
    o = s.patch(CM, "default", "a", [{"op": "replace", "path": "/data/j", "value": "9"},
                                     {"op": "add", "path": "/metadata/labels", "value": {"l": "v"}}], "json")
    assert o["data"]["j"] == "9" and o["metadata"]["labels"] == {"l": "v"}
    with pytest.raises(errors.ApiError):
        s.patch(CM, "default", "a", [{"op": "test", "path": "/data/j", "value": "0"}], "json")


# ---------------------------------------------------------------- CRD admission + status subresource


def test_cron_crd_defaulting_and_validation():
    s = mk()
    c = new_cron("c", "default", "* * * * *", {"apiVersion": "kubeflow.org/v1", "kind": "PyTorchJob",
                                               "anything": {"kept": True}})
    d = c.to_dict()
    d["spec"]["unknownField"] = 1
    out = s.create(CRON_GVR, "default", d)
    assert out["spec"]["concurrencyPolicy"] == "Allow"  # default
    assert "unknownField" not in out["spec"]  # pruned
    assert out["spec"]["template"]["workload"]["anything"] == {"kept": True}  # preserve-unknown-fields
    bad = new_cron("b", "default", "* * * * *", {"apiVersion": "v1", "kind": "X"}, concurrency_policy="Sometimes")
    with pytest.raises(errors.ApiError) as e:
        s.create(CRON_GVR, "default", bad.to_dict())
    assert errors.is_invalid(e.value) and "Unsupported value" in e.value.message
    missing = {"apiVersion": "apps.kubedl.io/v1alpha1", "kind": "Cron", "metadata": {"name": "m"},
               "spec": {"schedule": "* * * * *"}}
    with pytest.raises(errors.ApiError) as e:
        s.create(CRON_GVR, "default", missing)
    assert "spec.template: Required value" in e.value.message
    wrong_type = new_cron("w", "default", "* * * * *", {"apiVersion": "v1", "kind": "X"}).to_dict()
    wrong_type["spec"]["suspend"] = "yes"
    with pytest.raises(errors.ApiError) as e:
        s.create(CRON_GVR, "default", wrong_type)
    assert "must be of type boolean" in e.value.message


def test_compiled_schema_matches_slow_path():
    schema = crd()["spec"]["versions"][0]["schema"]["openAPIV3Schema"]
    fast = sch.CompiledSchema(schema)
    good = new_cron("c", "ns", "* * * * *", {"apiVersion": "a/b", "kind": "K"}).to_dict()
    good["status"] = {"history": [{"object": {"kind": "K", "name": "n"}, "status": "Succeeded",
                                   "created": "2026-01-01T00:00:00Z"}]}
    assert fast(good) and sch.validate(good, schema) == []
    bad = dict(good)
    bad["status"] = {"history": [{"object": {"kind": "K", "name": "n"}}]}  # status missing
    assert not fast(bad) and sch.validate(bad, schema)


def test_status_subresource_semantics():
    s = mk()
    c = s.create(CRON_GVR, "default", new_cron("c", "default", "* * * * *",
                                               {"apiVersion": "a/v1", "kind": "K"}).to_dict())
    # status is ignored on create and on main-resource update
    c["status"] = {"lastScheduleTime": "2026-01-01T00:00:00Z"}
    c["spec"]["schedule"] = "*/2 * * * *"
    u = s.update(CRON_GVR, "default", "c", c)
    assert "status" not in u and u["metadata"]["generation"] == 2
    # status update ignores spec changes and does not bump generation
    u["status"] = {"lastScheduleTime": "2026-01-01T00:00:00Z"}
    u["spec"]["schedule"] = "@daily"
    v = s.update(CRON_GVR, "default", "c", u, "status")
    assert v["status"]["lastScheduleTime"] == "2026-01-01T00:00:00Z"
    assert v["spec"]["schedule"] == "*/2 * * * *" and v["metadata"]["generation"] == 2
    w = s.patch(CRON_GVR, "default", "c", {"status": {"active": [{"name": "x"}]}}, "merge", "status")
    assert w["status"]["active"] == [{"name": "x"}]


def test_finalizers_and_deletion_timestamp():
    s = mk()
    o = s.create(CM, "default", dict(cm("a"), metadata={"name": "a", "finalizers": ["x/y"]}))
    d = s.delete(CM, "default", "a")
    assert d["metadata"]["deletionTimestamp"]
    assert s.get(CM, "default", "a")["metadata"]["deletionTimestamp"]
    got = s.get(CM, "default", "a")
    got["metadata"]["finalizers"] = []
    s.update(CM, "default", "a", got)
    with pytest.raises(errors.ApiError):
        s.get(CM, "default", "a")
    assert o


def test_delete_preconditions():
    s = mk()
    s.create(CM, "default", cm("a"))
    with pytest.raises(errors.ApiError) as e:
        s.delete(CM, "default", "a", preconditions={"uid": "wrong"})
    assert errors.is_conflict(e.value)


# ---------------------------------------------------------------- garbage collection


def test_owner_gc_background_and_orphan():
    s = mk(gc=True)
    owner = s.create(CM, "default", cm("owner"))
    ref = {"apiVersion": "v1", "kind": "ConfigMap", "name": "owner", "uid": owner["metadata"]["uid"],
           "controller": True, "blockOwnerDeletion": True}
    for n in ("d1", "d2"):
        s.create(CM, "default", dict(cm(n), metadata={"name": n, "ownerReferences": [ref]}))
    s.delete(CM, "default", "owner")
    s.run_gc()
    assert [o["metadata"]["name"] for o in s.list(CM, "default")["items"]] == []
    owner = s.create(CM, "default", cm("owner2"))
    ref["uid"], ref["name"] = owner["metadata"]["uid"], "owner2"
    s.create(CM, "default", dict(cm("d3"), metadata={"name": "d3", "ownerReferences": [ref]}))
    s.delete(CM, "default", "owner2", propagation_policy="Orphan")
    s.run_gc()
    d3 = s.get(CM, "default", "d3")
    assert "ownerReferences" not in d3["metadata"]


def test_no_gc_by_default_like_envtest():
    s = mk(gc=False)
    owner = s.create(CM, "default", cm("owner"))
    ref = {"apiVersion": "v1", "kind": "ConfigMap", "name": "owner", "uid": owner["metadata"]["uid"],
           "controller": True}
    s.create(CM, "default", dict(cm("d"), metadata={"name": "d", "ownerReferences": [ref]}))
    s.delete(CM, "default", "owner")
    s.run_gc()
    assert s.get(CM, "default", "d")


# ---------------------------------------------------------------- watch


async def _drain(w, n, timeout=1.0):
    out = []
    for _ in range(n):
        out.append(await asyncio.wait_for(w.__anext__(), timeout))
    return out


async def test_watch_initial_and_resume():
    s = mk()
    s.create(CM, "default", cm("a"))
    w = s.watch(CM, "default")
    evs = await _drain(w, 1)
    assert evs[0][0] == "ADDED" and evs[0][1]["metadata"]["name"] == "a"
    rv = s.current_rv()
    s.create(CM, "default", cm("b"))
    s.patch(CM, "default", "b", {"data": {"x": "1"}})
    s.delete(CM, "default", "b")
    assert [e[0] for e in await _drain(w, 3)] == ["ADDED", "MODIFIED", "DELETED"]
    w2 = s.watch(CM, "default", str(rv))
    assert [e[0] for e in await _drain(w2, 3)] == ["ADDED", "MODIFIED", "DELETED"]
    w.stop()
    w2.stop()


async def test_watch_gone_when_too_old():
    s = APIServer(FakeClock(0), watch_window=3)
    for i in range(10):
        s.create(CM, "default", cm(f"c{i}"))
    with pytest.raises(errors.ApiError) as e:
        s.watch(CM, "default", "1")
    assert errors.is_gone(e.value) and e.value.code == 410


async def test_filtered_watch_transitions():
    s = mk()
    w = s.watch(CM, "default", str(s.current_rv()), label_selector="app=x")
    s.create(CM, "default", cm("a", {"app": "y"}))
    s.patch(CM, "default", "a", {"metadata": {"labels": {"app": "x"}}})  # starts matching
    s.patch(CM, "default", "a", {"metadata": {"labels": {"app": "z"}}})  # stops matching
    evs = await _drain(w, 2)
    assert [e[0] for e in evs] == ["ADDED", "DELETED"]
    w.stop()


# ---------------------------------------------------------------- faults


def test_fault_injection():
    s = mk()
    s.faults.add(verb="create", resource="configmaps", code=503, reason="ServiceUnavailable", times=1)
    with pytest.raises(errors.ApiError) as e:
        s.faults.check("create", "configmaps")
    assert e.value.code == 503
    s.faults.check("create", "configmaps")  # times exhausted


# ---------------------------------------------------------------- compiled schema == slow path (property test)
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

_vals = st.recursive(st.none() | st.booleans() | st.integers(-5, 5) | st.text(max_size=4)
                     | st.sampled_from(["Allow", "Forbid", "Replace", "2026-01-01T00:00:00Z", "* * * * *"]),
                     lambda c: st.lists(c, max_size=3) | st.dictionaries(
                         st.sampled_from(["schedule", "suspend", "concurrencyPolicy", "historyLimit", "deadline",
                                          "template", "workload", "active", "history", "status", "object", "kind",
                                          "name", "uid", "created", "finished", "lastScheduleTime", "x"]), c,
                         max_size=4), max_leaves=12)


_PATHS = [("spec", "schedule"), ("spec", "suspend"), ("spec", "concurrencyPolicy"), ("spec", "historyLimit"),
          ("spec", "deadline"), ("spec", "template"), ("spec", "x"), ("status", "lastScheduleTime"),
          ("status", "active"), ("status", "history"), ("status", "x"), ("spec", "template", "workload"),
          ("status", "history", 0, "status"), ("status", "history", 0, "object"), ("status", "history", 0, "created"),
          ("status", "history", 0, "object", "name"), ("status", "active", 0, "uid"), ("status", "active", 0, "x")]


@settings(max_examples=400, deadline=None)
@given(mutations=st.lists(st.tuples(st.sampled_from(_PATHS), _vals | st.just("<delete>")), max_size=3))
def test_compiled_schema_property_matches_prune_default_validate(mutations):
    """Start from a valid Cron, apply up to three random field mutations, and require the compiled
    one-pass checker to agree with prune + default + validate on validity and on the pruned object."""
    import copy as _copy

    schema = crd()["spec"]["versions"][0]["schema"]["openAPIV3Schema"]
    obj = new_cron("c", "ns", "* * * * *", {"apiVersion": "a/b", "kind": "K"}, history_limit=3).to_dict()
    obj["status"] = {"lastScheduleTime": "2026-01-01T00:00:00Z",
                     "active": [{"kind": "K", "name": "a", "uid": "u1", "apiVersion": "a/b"}],
                     "history": [{"object": {"kind": "K", "name": "n", "apiGroup": "a/b"}, "status": "Succeeded",
                                  "uid": "u2", "created": "2026-01-01T00:00:00Z"}]}
    for path, val in mutations:
        cur = obj
        for p in path[:-1]:
            if isinstance(cur, dict) and p in cur:
                cur = cur[p]
            elif isinstance(cur, list) and isinstance(p, int) and p < len(cur):
                cur = cur[p]
            else:
                cur = None
                break
        if isinstance(cur, dict):
            if val == "<delete>":
                cur.pop(path[-1], None)
            else:
                cur[path[-1]] = _copy.deepcopy(val)
    a = _copy.deepcopy(obj)
    b = _copy.deepcopy(obj)
    ok_fast = sch.CompiledSchema(schema)(a)
    sch.prune(b, schema)
    sch.apply_defaults(b, schema)
    ok_slow = sch.validate(b, schema) == []
    assert ok_fast == ok_slow, (obj, sch.validate(b, schema))
    if ok_fast:
        assert a == b


async def test_http_writes_never_mutate_stored_objects():
    """The HTTP front end hands request bodies over without copies and status merges share
    untouched subtrees; previously stored objects (already sent in watch events) stay intact."""
    import copy as _copy

    from cron_operator_amd.apiserver.http import APIServerApp
    from cron_operator_amd.runtime.client import Client
    from cron_operator_amd.runtime.http import HttpTransport
    from cron_operator_amd.runtime.kubeconfig import RestConfig

    s = mk()
    app = APIServerApp(s)
    port = await app.start("127.0.0.1", 0)
    client = Client(HttpTransport(RestConfig(host=f"http://127.0.0.1:{port}")), qps=-1)
    try:
        await client.create(CRON_GVR, new_cron("m", "default", "* * * * *", {"apiVersion": "a/b", "kind": "K"})
                            .to_dict(), "default")
        ri = s.resource(CRON_GVR)
        v1 = s._get_raw(ri, "default", "m")
        snap1 = _copy.deepcopy(v1)
        await client.patch(CRON_GVR, "default", "m", {"status": {"lastScheduleTime": "2026-01-01T00:00:00Z",
                                                                 "history": [{"object": {"kind": "K", "name": "a"},
                                                                              "status": "Succeeded"}]}},
                           "merge", "status")
        v2 = s._get_raw(ri, "default", "m")
        snap2 = _copy.deepcopy(v2)
        await client.patch(CRON_GVR, "default", "m", {"status": {"lastScheduleTime": "2026-01-01T00:01:00Z"}},
                           "merge", "status")
        await client.patch(CRON_GVR, "default", "m", {"spec": {"suspend": True}, "metadata": {"labels": {"x": "y"}}})
        v4 = s._get_raw(ri, "default", "m")
        assert v1 == snap1 and v2 == snap2  # earlier versions untouched
        assert v4["spec"]["suspend"] is True and v4["metadata"]["labels"] == {"x": "y"}
        assert v4["status"]["history"] == snap2["status"]["history"]
        assert int(v4["metadata"]["resourceVersion"]) > int(v2["metadata"]["resourceVersion"])
        assert v4["metadata"]["generation"] == 2 and v2["metadata"].get("generation", 1) == 1
    finally:
        await client.close()
        await app.stop()


@settings(max_examples=300, deadline=None)
@given(key=st.sampled_from(["lastScheduleTime", "active", "history", "x"]), val=_vals | st.just("<delete>"))
def test_incremental_status_admission_matches_full(key, val):
    """check_changed (skip fields shared by identity with the admitted old status) == full check."""
    import copy as _copy

    schema = crd()["spec"]["versions"][0]["schema"]["openAPIV3Schema"]["properties"]["status"]
    cs = sch.CompiledSchema(schema, root=False)
    old = {"lastScheduleTime": "2026-01-01T00:00:00Z",
           "active": [{"kind": "K", "name": "a", "uid": "u1", "apiVersion": "a/b"}],
           "history": [{"object": {"kind": "K", "name": "n"}, "status": "Succeeded", "uid": "u2"}]}
    assert cs(_copy.deepcopy(old))
    new = dict(old)  # shares every untouched field with old, like a structural-sharing merge
    if val == "<delete>":
        new.pop(key, None)
    else:
        new[key] = _copy.deepcopy(val)
    full = _copy.deepcopy(new)
    assert cs.check_changed(new, old) == cs(full)
    if cs(_copy.deepcopy(new)):
        assert new == full


_HIST = [{"object": {"kind": "K", "name": f"n{i}", "apiGroup": "a/b"}, "status": "Succeeded", "uid": f"u{i}",
          "created": "2026-01-01T00:00:00Z", "finished": "2026-01-01T00:01:00Z"} for i in range(6)]


@settings(max_examples=300, deadline=None)
@given(picks=st.lists(st.integers(0, 5) | _vals, max_size=8))
def test_elementwise_status_admission_matches_full(picks):
    """Array elements equal (not identical) to the old ones are skipped; the verdict and the
    pruned result still match a full check, whatever mix of old and new elements arrives."""
    import copy as _copy

    schema = crd()["spec"]["versions"][0]["schema"]["openAPIV3Schema"]["properties"]["status"]
    cs = sch.CompiledSchema(schema, root=False)
    old = {"lastScheduleTime": "2026-01-01T00:00:00Z", "history": _copy.deepcopy(_HIST)}
    assert cs(_copy.deepcopy(old))
    hist = [_copy.deepcopy(_HIST[p]) if type(p) is int else _copy.deepcopy(p) for p in picks]
    new = {"lastScheduleTime": "2026-01-01T00:00:00Z", "history": hist}  # equal, not identical, values
    full = _copy.deepcopy(new)
    assert cs.check_changed(new, old) == cs(full)
    if cs(_copy.deepcopy(new)):
        assert new == full


_SELS = ["", "s=0", "s=1", "s=0,k", "s notin (0,1)", "k", "!s", "s in (1,2)", "s=2,k=a", "k=a"]
_OPS = st.lists(st.tuples(st.sampled_from(["create", "label", "unlabel", "delete"]), st.integers(0, 3),
                          st.sampled_from(["s", "k"]), st.sampled_from(["0", "1", "2", "a"])), max_size=25)


@settings(max_examples=150, deadline=None)
@given(ops=_OPS, sels=st.lists(st.sampled_from(_SELS), min_size=1, max_size=6))
def test_indexed_watch_fanout_matches_per_watcher_selectors(ops, sels):
    """The label-pinned watcher index and the shared per-selector evaluation deliver exactly the
    events a per-watcher selector check would (ADDED/DELETED on label transitions included)."""
    from cron_operator_amd.api.selectors import matches_labels, parse_label_selector

    s = mk()
    ws = [s.watch(CM, "default", label_selector=sel or None) for sel in sels]
    want = [[] for _ in sels]
    cur = {}
    for op, i, key, val in ops:
        name = f"o{i}"
        old = cur.get(name)
        if op == "create" and old is None:
            new = {key: val}
            s.create(CM, "default", cm(name, dict(new)))
        elif op in ("label", "unlabel") and old is not None:
            new = dict(old)
            if op == "label":
                new[key] = val
            else:
                new.pop(key, None)
            if new == old:
                continue  # a no-op patch writes nothing and emits no event
            s.patch(CM, "default", name, {"metadata": {"labels": {key: val if op == "label" else None}}})
        elif op == "delete" and old is not None:
            new = None
            s.delete(CM, "default", name)
        else:
            continue
        for j, sel in enumerate(sels):
            reqs = parse_label_selector(sel)
            was = old is not None and matches_labels(reqs, old)
            now = new is not None and matches_labels(reqs, new)
            if new is None:
                ev = "DELETED" if was else None
            elif old is None:
                ev = "ADDED" if now else None
            else:
                ev = {(True, True): "MODIFIED", (True, False): "DELETED", (False, True): "ADDED"}.get((was, now))
            if ev:
                want[j].append((ev, name))
        if new is None:
            cur.pop(name, None)
        else:
            cur[name] = new
    for j, w in enumerate(ws):
        got = []
        while not w.queue.empty():
            etype, obj = w.queue.get_nowait()
            got.append((etype, obj["metadata"]["name"]))
        assert got == want[j], sels[j]


def test_label_index_answers_pinned_selectors_like_a_scan():
    """A LIST that pins ``key=value`` reads the label index (built on first use, kept current by
    every write); its answer equals a full scan's, in key order, across label edits, deletes,
    namespaces and paging."""
    import random

    from cron_operator_amd.api.selectors import compile_selectors

    s = mk()
    s.create_namespace("other")
    rng = random.Random(3)
    live = {}
    for step in range(400):
        ns = rng.choice(["default", "other"])
        name = f"c{rng.randrange(40)}"
        op = rng.random()
        cur = live.get((ns, name))
        if cur is None:
            labels = {"k": rng.choice(["a", "b"]), "z": "1"} if rng.random() < 0.8 else {"z": "1"}
            live[(ns, name)] = s.create(CM, ns, cm(name, labels))
        elif op < 0.4:
            s.delete(CM, ns, name)
            del live[(ns, name)]
        else:
            v = rng.choice(["a", "b", None])
            live[(ns, name)] = s.patch(CM, ns, name, {"metadata": {"labels": {"k": v}}}, "merge")
        if step % 20 == 0:
            for sel in ("k=a", "k=b", "k=a,z=1", "k=a,z!=1"):
                for lns in ("default", "other", None):
                    got = [(o["metadata"]["namespace"], o["metadata"]["name"]) for o in s.list(CM, lns, sel)["items"]]
                    pred = compile_selectors(sel, None)
                    want = sorted((k for k, o in live.items() if (lns is None or k[0] == lns) and pred(o)),
                                  key=lambda k: (k[0], k[1]) if lns is None else k[1])
                    if lns is None:
                        assert sorted(got) == sorted(want), (sel, lns)
                    else:
                        assert got == sorted(want, key=lambda k: k[1]), (sel, lns)
    assert ("", "configmaps") in s._label_idx and "k" in s._label_idx[("", "configmaps")]
    page = s.list(CM, "default", "k=a", limit=2)
    names = [o["metadata"]["name"] for o in page["items"]]
    while page["metadata"].get("continue"):
        page = s.list(CM, "default", "k=a", limit=2, continue_=page["metadata"]["continue"])
        names += [o["metadata"]["name"] for o in page["items"]]
    assert names == sorted(n for (ns, n), o in live.items() if ns == "default"
                           and (o["metadata"].get("labels") or {}).get("k") == "a")
