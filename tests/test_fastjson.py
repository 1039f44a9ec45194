"""Native JSON decoder (``_fastjson.loads``) against ``json.loads`` as the oracle."""
from __future__ import annotations

import json
import math

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from cron_operator_amd.ops import fastjson_native

m = fastjson_native.load()

json_values = st.recursive(
    st.none() | st.booleans() | st.integers(min_value=-(10 ** 30), max_value=10 ** 30)
    | st.floats(allow_nan=False, allow_infinity=False) | st.text(max_size=20),
    lambda children: st.lists(children, max_size=5) | st.dictionaries(st.text(max_size=12), children, max_size=5),
    max_leaves=40)


@settings(max_examples=400, deadline=None)
@given(json_values, st.booleans(), st.booleans())
def test_roundtrip_matches_json(v, ascii_only, pretty):
    s = json.dumps(v, ensure_ascii=ascii_only, indent=2 if pretty else None)
    want = json.loads(s)
    assert m.loads(s) == want
    assert m.loads(s.encode()) == want
    assert m.loads(bytearray(s.encode())) == want
    assert repr(m.loads(s)) == repr(want)  # int vs float, -0.0, key order


@pytest.mark.parametrize("doc", [
    '{}', '[]', '0', '-0', '-0.0', '1.5e10', '1E-5', '2.5E+3', '123456789012345678901234567890',
    '-12345678901234567', '"a\\u00e9\\ud83d\\ude00\\ud800x"', '"\\"\\\\\\/\\b\\f\\n\\r\\t"', '"héllo ✓"',
    '{"a":1,"a":2}', '[1,[2,[3,{"x":null,"y":true,"z":false}]]]', ' \n {"k" : [ 1 , 2 ] } \t', '1e400',
    '"\\ud800"', '"\\udc00\\ud800"', '"\U0001F600"', '-1e-400',
])
def test_edge_cases(doc):
    assert repr(m.loads(doc)) == repr(json.loads(doc))


def test_non_finite():
    assert math.isnan(m.loads("NaN"))
    assert m.loads("Infinity") == math.inf and m.loads("-Infinity") == -math.inf
    assert m.loads(b"\xef\xbb\xbf[1]") == [1]  # UTF-8 BOM on bytes is skipped, like json.loads
    with pytest.raises(ValueError):
        m.loads("﻿[1]")


@pytest.mark.parametrize("bad", ['', '{', '[1,]', '{"a"}', '{"a" 1}', '01', '1.', '"abc', '"\x01"', 'tru', '{"a":1}x',
                                 '"\\x"', '-', '[1 2]', b'"\xff"', '"\\u12"', "{'a':1}", '[1,,2]', '{"a":1,}'])
def test_rejects_what_json_rejects(bad):
    with pytest.raises(ValueError):
        json.loads(bad)
    with pytest.raises(ValueError):
        m.loads(bad)


def test_deep_nesting_and_types():
    with pytest.raises((ValueError, RecursionError)):
        m.loads("[" * 5000 + "]" * 5000)
    with pytest.raises(TypeError):
        m.loads(1)


def test_keys_are_shared_and_cache_clear():
    a = m.loads('{"metadata":{"name":"x"}}')
    b = m.loads(b'{"metadata":{"name":"y"}}')
    assert next(iter(a)) is next(iter(b))  # interned through the key cache
    m.clear_key_cache()
    assert m.loads('{"metadata":1}') == {"metadata": 1}


def test_recurring_short_values_are_shared():
    """Short ASCII values recur across cached objects (apiVersion, kind, condition types,
    namespaces, timestamps): decoded trees share one str per value.  Longer, escaped and
    non-ASCII values still decode to equal (fresh) strings."""
    doc = ('{"apiVersion":"kubeflow.org/v1","kind":"PyTorchJob","status":"Succeeded",'
           '"long":"%s","esc":"a\\"b","uni":"caf\u00e9","n":""}' % ("x" * 80))
    a, b = m.loads(doc), m.loads(doc.encode())
    assert a == b == json.loads(doc)
    for k in ("apiVersion", "kind", "status", "n"):
        assert a[k] is b[k], k
    # many one-off values (slot collisions, replacement) never change what decodes
    for i in range(50_000):
        assert m.loads('{"v":"uid-%d"}' % i)["v"] == "uid-%d" % i
    assert m.loads('{"v":"kubeflow.org/v1"}')["v"] == "kubeflow.org/v1"
    m.clear_key_cache()
    assert m.loads(doc) == json.loads(doc)


def _ref_dumps(v):
    return json.dumps(v, separators=(",", ":"), ensure_ascii=False)


@settings(max_examples=400, deadline=None)
@given(json_values)
def test_encoder_matches_json(v):
    assert m.dumps(v) == _ref_dumps(v)
    assert m.dumpb(v) == _ref_dumps(v).encode()


@settings(max_examples=120, deadline=None)
@given(st.dictionaries(st.text(max_size=8), json_values, max_size=5),
       st.dictionaries(st.text(max_size=8), json_values, max_size=5))
def test_dumpb_shared_matches_dumpb(a, b):
    """Subtrees shared by identity between successive (immutable) objects reuse their bytes;
    the output is always dumpb's."""
    cache = {}
    objs = [a, b, dict(a, **{k: v for k, v in b.items() if k not in a}), {"x": a, "y": [b, a]}, dict(a)]
    for _ in range(2):
        for o in objs:
            assert m.dumpb_shared(o, cache) == m.dumpb(o)
    for k, (obj, raw) in cache.items():
        assert id(obj) == k and raw == m.dumpb(obj) and len(raw) >= 64
    vol = {}
    for o in objs:
        assert m.dumpb_shared(o, vol, ("x",)) == m.dumpb(o)
    assert all(obj is not objs[3]["x"] for obj, _ in vol.values())


def test_dumpb_shared_reuses_spec_bytes():
    spec = {"template": {"workload": {"kind": "PyTorchJob", "spec": {"replicas": list(range(40))}}}}
    cache = {}
    old = {"apiVersion": "v1", "spec": spec, "status": {"n": 1}}
    m.dumpb_shared(old, cache)
    assert id(spec) in cache
    new = dict(old, status={"n": 2})  # a status write shares spec by identity
    assert m.dumpb_shared(new, cache) == m.dumpb(new)
    with pytest.raises(TypeError):
        m.dumpb_shared(new, [])


@pytest.mark.parametrize("v", [float("inf"), float("-inf"), -0.0, 1e-7, 2 ** 80, -(2 ** 70), "\x00\x1f\u2028\"\\",
                               (1, [2, (3,)]), {1: "a", 2.5: "b", None: "c", False: "d"}, 123456789.123])
def test_encoder_edge_cases(v):
    assert m.dumps(v) == _ref_dumps(v)


def test_encoder_nan_and_errors():
    assert m.dumps(float("nan")) == "NaN"
    with pytest.raises(TypeError):
        m.dumpb(object())
    with pytest.raises(TypeError):
        m.dumpb({(1, 2): 3})
    with pytest.raises(UnicodeEncodeError):
        m.dumpb("\ud800")
    deep = []
    cur = deep
    for _ in range(3000):
        nxt = []
        cur.append(nxt)
        cur = nxt
    with pytest.raises(ValueError):
        m.dumpb(deep)


def test_decoded_and_copied_trees_are_exempt_from_cyclic_gc():
    """JSON trees are acyclic: the native decoder and deepcopy untrack their containers so
    young-generation GC passes do not walk the informer caches; refcounting still frees
    them, and CPython re-tracks a dict that later receives a container."""
    import gc
    import weakref

    from cron_operator_amd.ops import _fastjson as fj

    doc = fj.loads(b'{"metadata":{"labels":{"a":"b"},"ownerReferences":[{"uid":"1"}]},"items":[[],{}]}')
    nodes = [doc, doc["metadata"], doc["metadata"]["ownerReferences"], doc["metadata"]["ownerReferences"][0],
             doc["items"], doc["items"][0], doc["items"][1]]
    assert not any(gc.is_tracked(n) for n in nodes)
    cp = fj.deepcopy(doc)
    assert cp == doc and not gc.is_tracked(cp) and not gc.is_tracked(cp["metadata"]["ownerReferences"])

    class Probe:  # a tracked object referenced from an untracked tree stays alive while the tree is
        pass

    p = Probe()
    ref = weakref.ref(p)
    doc["items"].append(p)
    del p
    gc.collect()
    assert ref() is not None
    del doc, nodes
    gc.collect()
    assert ref() is None  # freed by refcounting once the tree goes
    cp["metadata"]["new"] = {"x": []}
    assert gc.is_tracked(cp["metadata"])
    prev = fj.set_gc_untrack(False)
    try:
        assert prev is True and gc.is_tracked(fj.loads(b'{"a":[1]}')["a"])
    finally:
        fj.set_gc_untrack(prev)


# ------------------------------------------------------------------ plan codecs (skip / memo paths)

from cron_operator_amd.utils import jsonutil  # noqa: E402

doc_trees = st.dictionaries(st.sampled_from(["spec", "status", "metadata", "x", "items"]),
                            json_values, max_size=5)


@settings(max_examples=300, deadline=None)
@given(doc_trees, st.lists(st.lists(st.sampled_from(["spec", "status", "metadata", "x", "items", "*"]),
                                    min_size=1, max_size=3), max_size=3))
def test_codec_skip_matches_python_twin(doc, skips):
    """Decoding with skipped paths == json.loads followed by deleting those paths (the twin)."""
    raw = json.dumps(doc)
    native = m.Codec(skip=skips)
    twin = jsonutil.PyCodec(skip=skips)
    assert repr(native.loads(raw)) == repr(twin.loads(raw))
    event = json.dumps({"type": "MODIFIED", "object": doc})
    prefixed = [["object"] + p for p in skips]
    assert repr(m.Codec(skip=prefixed)(event)) == repr(jsonutil.PyCodec(skip=prefixed)(event))


@settings(max_examples=200, deadline=None)
@given(doc_trees, doc_trees)
def test_codec_memo_is_exact(a, b):
    """Memoised paths give the same value as a plain decode -- only identity differs."""
    memo = m.Memo(64)
    c = m.Codec(memo_paths=[("spec",), ("status", "*"), ("items", "*")], memo=memo)
    for doc in (a, b, a, b):
        raw = json.dumps(doc)
        assert repr(c.loads(raw)) == repr(json.loads(raw))


def test_codec_memo_reuses_objects_across_documents_and_from_the_encoder():
    memo = m.Memo()
    enc = m.Codec(memo_paths=[("status", "history", "*")], memo=memo)
    dec = m.Codec(memo_paths=[("object", "spec"), ("object", "status", "history", "*")], memo=memo)
    entries = [{"uid": f"u{i}", "object": {"apiGroup": "kubeflow.org/v1", "kind": "PyTorchJob", "name": f"j{i}"},
                "status": "Succeeded", "created": "2026-01-01T12:00:00Z"} for i in range(3)]
    patch = {"status": {"history": entries}}
    body = enc.dumpb(patch)
    assert body == json.dumps(patch, separators=(",", ":"), ensure_ascii=False).encode()
    obj = {"metadata": {"name": "c", "resourceVersion": "7"}, "spec": {"schedule": "* * * * *"},
           "status": {"history": entries, "lastScheduleTime": "2026-01-01T12:01:00Z"}}
    t, o = dec(json.dumps({"type": "MODIFIED", "object": obj}, separators=(",", ":")).encode())
    assert t == "MODIFIED" and o == obj
    assert all(x is y for x, y in zip(o["status"]["history"], entries))  # the encoder's own dicts
    _, o2 = dec(json.dumps({"type": "MODIFIED", "object": obj}, separators=(",", ":")).encode())
    assert o2["spec"] is o["spec"] and o2["metadata"] is not o["metadata"]
    st_ = memo.stats()
    assert st_["hits"] >= 7 and st_["stores"] >= 4
    memo.clear()
    assert memo.stats()["used"] == 0



def test_memo_forget_drops_exactly_that_entry():
    memo = m.Memo()
    enc = m.Codec(memo_paths=[("status", "history", "*")], memo=memo)
    dec = m.Codec(memo_paths=[("object", "status", "history", "*")], memo=memo)
    entries = [{"uid": f"u{i}", "status": "Succeeded"} for i in range(3)]
    enc.dumpb({"status": {"history": entries}})
    used = memo.stats()["used"]
    assert memo.forget(entries[0]) is True and memo.stats()["used"] == used - 1
    assert memo.forget(entries[0]) is False and memo.forget({"uid": "u1", "status": "Succeeded"}) is False
    ev = json.dumps({"type": "MODIFIED", "object": {"status": {"history": entries}}}, separators=(",", ":"))
    _, o = dec(ev.encode())
    # the forgotten entry decodes afresh (equal, not identical); the others are still shared
    assert o["status"]["history"] == entries
    assert o["status"]["history"][0] is not entries[0]
    assert o["status"]["history"][1] is entries[1] and o["status"]["history"][2] is entries[2]
    # and the encoder re-encodes it (byte-exact) instead of copying remembered bytes
    assert enc.dumpb({"status": {"history": entries}}) == \
        json.dumps({"status": {"history": entries}}, separators=(",", ":")).encode()


def test_reconciler_forgets_history_entries_it_rotates_out():
    """A Cron's history keeps historyLimit entries; the entries it drops are forgotten by the
    shared wire memo, so the memo holds the live set instead of every entry ever written."""
    from cron_operator_amd.bench.harness import BenchConfig, run_sync
    from cron_operator_amd.controller import reconciler as rc

    made = []
    orig = rc.WireCodecs.__init__

    def spy(self, *a, **k):
        orig(self, *a, **k)
        made.append(self)

    rc.WireCodecs.__init__ = spy
    try:
        run_sync(BenchConfig(n_crons=30, steps=30, warmup=1, shards=1, transport="http"))
    finally:
        rc.WireCodecs.__init__ = orig
    used = [c.memo.stats()["used"] for c in made]
    # live: 10 history entries + a few per-Cron values (labels, owner references, spec) each;
    # without forgetting, 30 more entries per tick stay (~1250 after 30 ticks)
    assert used and max(used) < 30 * 16, used

@settings(max_examples=200, deadline=None)
@given(st.lists(json_values, max_size=4), json_values)
def test_codec_encoder_reuses_remembered_bytes_by_identity(entries, other):
    """Values at memo paths met again by identity are copied from the bytes the encoder
    remembered -- the output stays byte-identical to a plain encode -- while values the decoder
    remembered (a peer's encoding, maybe formatted differently) are encoded anew."""
    memo = m.Memo(64)
    enc = m.Codec(memo_paths=[("h", "*")], memo=memo)
    doc = {"h": entries, "o": other}
    plain = m.dumpb(doc)
    assert enc.dumpb(doc) == plain
    assert enc.dumpb(doc) == plain
    if entries:
        assert memo.stats()["reuses"] >= 1
    # the decoder remembers a peer's spacing; encoding that object must not copy those bytes
    dec = m.Codec(memo_paths=[("h", "*")], memo=memo)
    peer = json.dumps({"h": [{"k": [1, 2]}]}, separators=(", ", ": "))
    got = dec.loads(peer)
    assert enc.dumpb(got) == m.dumpb(got)


def test_codec_event_shape_and_errors():
    c = m.Codec(skip=[("object", "spec")])
    assert c(b'{"type":"ADDED","object":{"spec":{"big":[1,2,3]},"metadata":{"name":"a"}}}') == \
        ("ADDED", {"metadata": {"name": "a"}})
    assert c(b'{"type":"BOOKMARK"}') == ("BOOKMARK", {})
    assert c(b'{"object":{"x":1}}') == ("", {"x": 1})
    for bad in (b'{"type":"A","object":{"spec":{"a":[1,2}}', b'{"type":"A","object":{"spec":"open}}', b'{',
                b'{"type":"A","object":{"spec":{"a":1}}}x', b'{"type":"A","object":{"spec":]}}'):
        with pytest.raises(ValueError):
            c(bad)
    with pytest.raises(TypeError):
        m.Codec(skip=[("a", 1)])
    with pytest.raises(ValueError):
        m.Codec(skip=[()])
    with pytest.raises(TypeError):
        m.Codec(memo_paths=[("a",)], memo=object())


@settings(max_examples=200, deadline=None)
@given(st.dictionaries(st.text(max_size=6), json_values, max_size=5),
       st.dictionaries(st.text(max_size=6), json_values, max_size=5))
def test_merge_patch_share_equals_copy(old, new):
    shared = m.create_merge_patch(old, new, True)
    assert shared == m.create_merge_patch(old, new) == jsonutil.py_create_merge_patch(old, new)
    assert jsonutil.py_create_merge_patch(old, new, True) == shared


def test_memo_grows_with_its_working_set_and_forgets_exactly():
    """The memo starts small, doubles once half full instead of evicting values still in use
    (up to max_slots), and forget() drops exactly the entry of each value -- used returns to 0."""
    memo = m.Memo(64, 4096)
    enc = m.Codec(memo_paths=[("h", "*")], memo=memo)
    dec = m.Codec(memo_paths=[("h", "*")], memo=memo)
    entries = [{"uid": f"u{i}", "status": "Succeeded", "n": i} for i in range(1000)]
    for i in range(0, 1000, 50):
        enc.dumpb({"h": entries[i:i + 50]})
    st = memo.stats()
    assert st["grows"] >= 4 and st["slots"] >= 2048 and st["used"] >= 990, st
    # the watch echo of every entry decodes to the encoder's own dicts
    got = dec.loads(json.dumps({"h": entries}, separators=(",", ":")))["h"]
    shared = sum(a is b for a, b in zip(got, entries))
    assert shared >= 990
    for e in entries:
        memo.forget(e)
    # left: only the decoder's own copies of the few entries that had been evicted
    assert memo.stats()["used"] == len(entries) - shared


def test_memo_is_bounded_by_max_slots():
    memo = m.Memo(64, 256)
    enc = m.Codec(memo_paths=[("h", "*")], memo=memo)
    for i in range(0, 5000, 100):
        enc.dumpb({"h": [{"uid": f"v{j}"} for j in range(i, i + 100)]})
    st = memo.stats()
    assert st["slots"] == 256 and st["used"] <= 256 and st["evictions"] > 0, st


def test_codec_raw_paths_keep_the_exact_json_text_also_below_a_memo_path():
    """raw paths: the value's own JSON text comes back as bytes (spacing and key order as sent),
    also inside a memoised value; the encoder writes such bytes back verbatim."""
    memo = m.Memo()
    dec = m.Codec(memo_paths=[("object", "spec")], raw_paths=[("object", "spec", "template", "workload")],
                  memo=memo)
    wl = '{"kind": "PyTorchJob",  "spec": {"b": [1, 2], "a": {}}}'
    line = ('{"type":"ADDED","object":{"metadata":{"name":"c"},"spec":{"schedule":"* * * * *",'
            '"template":{"workload":' + wl + '}}}}').encode()
    t, o = dec(line)
    assert t == "ADDED" and o["spec"]["template"]["workload"] == wl.encode()
    _, o2 = dec(line)
    assert o2["spec"] is o["spec"]  # the memoised spec holds the raw text
    enc = m.Codec(raw_paths=[("spec", "template", "workload")])
    assert json.loads(enc.dumpb(o)) == {"metadata": {"name": "c"},
                                        "spec": {"schedule": "* * * * *", "template": {"workload": json.loads(wl)}}}
    # the Python twin: the same tree, its text re-encoded compactly
    py = jsonutil.PyCodec(raw_paths=[("object", "spec", "template", "workload")])
    _, p = py(line)
    assert json.loads(p["spec"]["template"]["workload"]) == json.loads(wl)


# ------------------------------------------------------------------ route paths (hash-routed shards)

LBL = "kubedl.io/cron-name"
route_meta = st.fixed_dictionaries({}, optional={
    "name": st.one_of(st.text(max_size=6), st.integers(0, 3)),
    "namespace": st.one_of(st.sampled_from(["", "ns", "tëam"]), st.none(), st.just("\ud800")),
    "labels": st.one_of(st.dictionaries(st.sampled_from([LBL, "app"]), st.one_of(st.text(max_size=6), st.none()),
                                        max_size=2), st.text(max_size=2)),
})
route_objs = st.lists(st.fixed_dictionaries({"metadata": route_meta}, optional={
    "apiVersion": st.just("v1"), "spec": json_values, "status": json_values}), max_size=6)


@settings(max_examples=300, deadline=None)
@given(route_objs, st.integers(1, 4), st.data(), st.sampled_from([None, LBL]))
def test_codec_route_paths_match_python_twin_and_shard_of(items, count, data, label):
    """Another shard's objects keep their members up to ``metadata`` (natively: the rest is
    never built); this shard's, and anything the test cannot hash, decode whole.  The cut
    agrees with ``shard_of`` -- what the informer's keep filter then applies."""
    from cron_operator_amd.runtime.controller import shard_of

    index = data.draw(st.integers(0, count - 1))
    raw = json.dumps({"kind": "List", "items": items})
    kw = {"route_paths": [("items", "*")], "route": (index, count, label)}
    native = m.Codec(**kw).loads(raw)
    twin = jsonutil.PyCodec(**kw).loads(raw)
    assert repr(native) == repr(twin)
    for full, got in zip(json.loads(raw)["items"], native["items"]):
        md = full["metadata"]
        labels = md.get("labels")
        if label:  # routed by the cron-name label: an object without it is this shard's
            key = labels.get(LBL) if isinstance(labels, dict) and LBL in labels else None
        else:
            key = md.get("name", "")
        ns = md.get("namespace", "")
        hashable = isinstance(ns, str) and isinstance(key, str) and "\ud800" not in ns + key
        mine = not hashable or count == 1 or shard_of(ns, key, count) == index
        keys = list(full)
        cut = {k: full[k] for k in keys[:keys.index("metadata") + 1]}  # members up to metadata
        assert repr(got) == repr(full if mine else cut)
    ev = json.dumps({"type": "ADDED", "object": items[0]}) if items else None
    if ev:
        kw1 = {"route_paths": [("object",)], "route": (index, count, label)}
        assert repr(m.Codec(**kw1)(ev)) == repr(jsonutil.PyCodec(**kw1)(ev))


def test_codec_route_paths_check_their_arguments_and_syntax():
    for bad in [(2, 2, None), (0, 0, None), (0, 2, 5), "x", None]:
        with pytest.raises((ValueError, TypeError)):
            m.Codec(route_paths=[("object",)], route=bad)
        with pytest.raises((ValueError, TypeError)):
            jsonutil.PyCodec(route_paths=[("object",)], route=bad)
    c = m.Codec(route_paths=[("object",)], route=(0, 2, None))  # "a" hashes to shard 1 of 2
    from cron_operator_amd.runtime.controller import shard_of

    assert shard_of("", "a", 2) == 1
    ok = b'{"type": "ADDED", "object": {"metadata": {"name": "a"}, "spec": {"x": [1, {"y": 2}]}, "z": 1}}'
    assert c(ok) == ("ADDED", {"metadata": {"name": "a"}})
    head = b'{"object": {"metadata": {"name": "a"}'
    for tail in (b', "spec" 1}}', b',}}', b' "x": 1}}', b', "x": [}}', b', "x": 1'):
        broken = head + tail
        with pytest.raises(ValueError):
            c.loads(broken)
        with pytest.raises(ValueError):
            json.loads(broken)
