// Native JSON-tree helpers (CPython extension `_fastjson`).
//
// Kubernetes objects are handled as Python dict/list trees by the fake
// apiserver, the informer cache and the reconciler.  Copy-on-read, the status
// "semantic DeepEqual" check and the merge-patch computation of the deferred
// status write (reference: internal/controller/cron_controller.go:107-120) run
// on every request/reconcile, so they are done here instead of in Python
// recursion.  Semantics are identical to utils/jsonutil.py (py_* functions),
// which the tests use as the oracle.
//
//   deepcopy(tree) -> tree           dicts/lists copied, scalars shared (immutable)
//   json_equal(a, b) -> bool         structural equality; bool is never equal to int
//   create_merge_patch(old, new)     RFC 7386 patch turning old into new
//   loads(bytes | str) -> tree       JSON decoder (json.loads semantics for UTF-8 input)
//   dumpb(tree) -> bytes             compact UTF-8 JSON, byte-identical to
//                                    json.dumps(tree, separators=(",", ":"), ensure_ascii=False).encode()
//   dumps(tree) -> str               the same as str
//   dumpb_shared(tree, cache, volatile_keys=()) -> bytes
//                                    dumpb for trees that are never mutated (the fake
//                                    apiserver's stored objects): the top-level container
//                                    values, except under volatile_keys, are cached by
//                                    identity in `cache` and reused
//
// loads: every API response and watch event the operator receives is decoded,
// and in the 1000-Cron bench that was the largest single item of operator CPU
// (~50 us per Cron/PyTorchJob object with CPython's json).  The decoder here is
// a single-pass recursive-descent parser that builds the Python objects
// directly and interns object keys through a process-wide cache: Kubernetes
// objects repeat the same few hundred keys ("metadata", "name", ...), so a key
// costs one hash probe instead of a str allocation + hash.  Semantics follow
// json.loads: duplicate keys keep the last value, NaN/Infinity/-Infinity are
// accepted, control characters inside strings and lone trailing data are
// errors (ValueError), \uXXXX escapes combine surrogate pairs and keep lone
// surrogates, numbers with a fraction/exponent become float (correctly
// rounded, via PyOS_string_to_double), the rest int (arbitrary precision).
//
// GC: a JSON tree cannot contain a reference cycle, so the dicts and lists that
// loads() and deepcopy() build are removed from the cyclic collector's lists
// (PyObject_GC_UnTrack) -- reference counting alone frees them.  The operator
// caches ~12k such trees in the 1000-Cron bench; every young-generation pass
// used to walk all of the recently replaced ones (~47 ms per pass, measured).
// set_gc_untrack(False) restores normal tracking.  An untracked dict that later
// receives a container value is re-tracked by CPython itself.

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#if defined(__SSE2__)
#include <emmintrin.h>
#endif

namespace {

bool g_untrack = true;

// A finished JSON container: exempt it from cyclic GC (see the header comment).
inline PyObject* acyclic(PyObject* c) {
  if (c != nullptr && g_untrack && PyObject_GC_IsTracked(c)) PyObject_GC_UnTrack(c);
  return c;
}

PyObject* deepcopy_impl(PyObject* x, int depth);

inline bool is_container(PyObject* x) { return PyDict_CheckExact(x) || PyList_CheckExact(x); }

PyObject* deepcopy_impl(PyObject* x, int depth) {
  if (depth > 512) {
    PyErr_SetString(PyExc_RecursionError, "JSON tree too deep");
    return nullptr;
  }
  if (PyDict_CheckExact(x)) {
    PyObject* out = _PyDict_NewPresized(PyDict_GET_SIZE(x));
    if (!out) return nullptr;
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(x, &pos, &k, &v)) {
      PyObject* cv;
      if (is_container(v)) {
        cv = deepcopy_impl(v, depth + 1);
        if (!cv) {
          Py_DECREF(out);
          return nullptr;
        }
      } else {
        Py_INCREF(v);
        cv = v;
      }
      const int rc = PyDict_SetItem(out, k, cv);
      Py_DECREF(cv);
      if (rc < 0) {
        Py_DECREF(out);
        return nullptr;
      }
    }
    return acyclic(out);
  }
  if (PyList_CheckExact(x)) {
    const Py_ssize_t n = PyList_GET_SIZE(x);
    PyObject* out = PyList_New(n);
    if (!out) return nullptr;
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* v = PyList_GET_ITEM(x, i);
      PyObject* cv;
      if (is_container(v)) {
        cv = deepcopy_impl(v, depth + 1);
        if (!cv) {
          Py_DECREF(out);
          return nullptr;
        }
      } else {
        Py_INCREF(v);
        cv = v;
      }
      PyList_SET_ITEM(out, i, cv);
    }
    return acyclic(out);
  }
  Py_INCREF(x);
  return x;
}

// -1 error, 0 not equal, 1 equal
int equal_impl(PyObject* a, PyObject* b, int depth) {
  if (a == b) return 1;
  if (depth > 512) {
    PyErr_SetString(PyExc_RecursionError, "JSON tree too deep");
    return -1;
  }
  const bool da = PyDict_CheckExact(a), db = PyDict_CheckExact(b);
  if (da || db) {
    if (!(da && db)) return 0;
    if (PyDict_GET_SIZE(a) != PyDict_GET_SIZE(b)) return 0;
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(a, &pos, &k, &v)) {
      PyObject* w = PyDict_GetItemWithError(b, k);
      if (!w) return PyErr_Occurred() ? -1 : 0;
      const int r = equal_impl(v, w, depth + 1);
      if (r != 1) return r;
    }
    return 1;
  }
  const bool la = PyList_CheckExact(a), lb = PyList_CheckExact(b);
  if (la || lb) {
    if (!(la && lb)) return 0;
    const Py_ssize_t n = PyList_GET_SIZE(a);
    if (n != PyList_GET_SIZE(b)) return 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
      const int r = equal_impl(PyList_GET_ITEM(a, i), PyList_GET_ITEM(b, i), depth + 1);
      if (r != 1) return r;
    }
    return 1;
  }
  const bool ba = PyBool_Check(a), bb = PyBool_Check(b);
  if (ba || bb) return (ba && bb && a == b) ? 1 : 0;
  return PyObject_RichCompareBool(a, b, Py_EQ);
}

// share: the patch references `nw`'s subtrees instead of copying them (a patch that is
// only serialised and dropped; `nw` must not change while the patch lives)
inline PyObject* patch_value(PyObject* v, int depth, bool share) {
  if (share) {
    Py_INCREF(v);
    return v;
  }
  return deepcopy_impl(v, depth);
}

PyObject* merge_patch_impl(PyObject* old, PyObject* nw, int depth, bool share = false) {
  if (!PyDict_CheckExact(old) || !PyDict_CheckExact(nw)) return patch_value(nw, depth, share);
  PyObject* patch = PyDict_New();
  if (!patch) return nullptr;
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  while (PyDict_Next(nw, &pos, &k, &v)) {
    PyObject* ov = PyDict_GetItemWithError(old, k);
    PyObject* entry = nullptr;
    if (!ov) {
      if (PyErr_Occurred()) goto fail;
      entry = patch_value(v, depth + 1, share);
      if (!entry) goto fail;
    } else if (PyDict_CheckExact(ov) && PyDict_CheckExact(v)) {
      PyObject* sub = merge_patch_impl(ov, v, depth + 1, share);
      if (!sub) goto fail;
      if (PyDict_GET_SIZE(sub) == 0) {
        Py_DECREF(sub);
        continue;
      }
      entry = sub;
    } else {
      const int eq = equal_impl(ov, v, depth + 1);
      if (eq < 0) goto fail;
      if (eq == 1) continue;
      entry = patch_value(v, depth + 1, share);
      if (!entry) goto fail;
    }
    if (PyDict_SetItem(patch, k, entry) < 0) {
      Py_DECREF(entry);
      goto fail;
    }
    Py_DECREF(entry);
  }
  pos = 0;
  while (PyDict_Next(old, &pos, &k, &v)) {
    const int has = PyDict_Contains(nw, k);
    if (has < 0) goto fail;
    if (!has && PyDict_SetItem(patch, k, Py_None) < 0) goto fail;
  }
  return patch;
fail:
  Py_DECREF(patch);
  return nullptr;
}


// ---------------------------------------------------------------------------------------- decoder

constexpr int kMaxDepth = 1000;
constexpr size_t kKeySlots = 8192;   // power of two
constexpr size_t kMaxKeyLen = 64;

struct KeySlot {
  uint64_t hash;
  PyObject* str;  // strong ref; nullptr = empty
  uint32_t len;
};
KeySlot g_keys[kKeySlots];
size_t g_keys_used = 0;

inline uint64_t fnv1a(const char* p, size_t n) {
  uint64_t h = 1469598103934665603ULL;
  for (size_t i = 0; i < n; ++i) {
    h ^= static_cast<unsigned char>(p[i]);
    h *= 1099511628211ULL;
  }
  return h;
}

// Short ASCII *values* recur across objects and watch events: apiVersion/kind, condition
// types, statuses and reasons, namespaces, label values, the tick's timestamps, and an
// object's own name/uid in each of its versions.  A direct-mapped cache hands back the
// existing str, so decoded trees share those strings with the trees already cached: an
// informer holding 11k jobs keeps one "kubeflow.org/v1" instead of 11k.  Strings are
// immutable, so the sharing is invisible.  Second-chance replacement: a slot hit since it
// was last probed survives one miss, so one-off strings (resourceVersions, fresh uids) do
// not evict the recurring ones.
constexpr size_t kValSlots = 16384;  // power of two
constexpr size_t kMaxValLen = 48;

struct ValSlot {
  uint64_t hash;
  PyObject* str;  // strong ref; nullptr = empty
  uint32_t len;
  bool hot;
};
ValSlot g_vals[kValSlots];

void clear_keys() {
  for (auto& s : g_keys) {
    Py_CLEAR(s.str);
    s.hash = 0;
    s.len = 0;
  }
  g_keys_used = 0;
  for (auto& s : g_vals) {
    Py_CLEAR(s.str);
    s.hash = 0;
    s.len = 0;
    s.hot = false;
  }
}

// ASCII key without escapes -> cached str (new reference)
PyObject* cached_key(const char* p, size_t n) {
  const uint64_t h = fnv1a(p, n);
  size_t i = h & (kKeySlots - 1);
  for (size_t probe = 0; probe < 16; ++probe, i = (i + 1) & (kKeySlots - 1)) {
    KeySlot& s = g_keys[i];
    if (s.str == nullptr) {
      if (g_keys_used > kKeySlots / 2) break;  // keep probes short; fall through to a fresh str
      PyObject* str = PyUnicode_New(static_cast<Py_ssize_t>(n), 127);
      if (!str) return nullptr;
      std::memcpy(PyUnicode_DATA(str), p, n);
      PyUnicode_InternInPlace(&str);
      s.hash = h;
      s.len = static_cast<uint32_t>(n);
      s.str = str;
      ++g_keys_used;
      Py_INCREF(str);
      return str;
    }
    if (s.hash == h && s.len == n && std::memcmp(PyUnicode_DATA(s.str), p, n) == 0) {
      Py_INCREF(s.str);
      return s.str;
    }
  }
  PyObject* str = PyUnicode_New(static_cast<Py_ssize_t>(n), 127);
  if (!str) return nullptr;
  std::memcpy(PyUnicode_DATA(str), p, n);
  return str;
}

// ASCII value without escapes -> shared str (new reference)
PyObject* cached_value(const char* p, size_t n) {
  const uint64_t h = fnv1a(p, n);
  ValSlot& s = g_vals[h & (kValSlots - 1)];
  if (s.str != nullptr && s.hash == h && s.len == n && std::memcmp(PyUnicode_DATA(s.str), p, n) == 0) {
    s.hot = true;
    Py_INCREF(s.str);
    return s.str;
  }
  PyObject* str = PyUnicode_New(static_cast<Py_ssize_t>(n), 127);
  if (!str) return nullptr;
  std::memcpy(PyUnicode_DATA(str), p, n);
  if (s.str != nullptr && s.hot) {
    s.hot = false;  // second chance: keep the recurring string, do not cache this one
    return str;
  }
  Py_INCREF(str);
  Py_XSETREF(s.str, str);
  s.hash = h;
  s.len = static_cast<uint32_t>(n);
  s.hot = false;
  return str;
}

// ------------------------------------------------------------------------ decode/encode plans
//
// A Plan names JSON paths -- object keys, "*" for any list element -- where the codec
// acts instead of building or writing the value plainly:
//
//   skip   the decoder scans past the value and leaves its key out.  A child informer
//          never reads a PyTorchJob's `spec` (the bulk of the object); skipping it at
//          decode time saves building it only for the informer to drop it.
//   memo   the decoder scans the value's bytes and, when the Memo holds an object that
//          was decoded from -- or encoded to -- exactly those bytes, returns that object
//          instead of building a new one; otherwise it builds and remembers it.  The
//          encoder remembers the bytes of each value it writes at a memo path.
//   raw    the decoder returns the value's JSON text (bytes) and the encoder writes it back.
//   route  (hash-routed shards) once the object's `metadata` is decoded, an object that
//          hashes to another shard gets the rest of its members skipped: a shard that
//          watches the whole fleet builds only its own share, and only the metadata of
//          the rest, which its informer's keep filter then drops.
//
// Memo values are shared between trees, so they must never be mutated -- the informer
// cache and the reconciler's status entries are read-only by contract already.  Byte
// equality of the scanned span implies JSON equality, so a hit is exact; a span that
// does not match just costs the scan.  A Cron's status write therefore comes back on
// the watch with the reconciler's own history-entry dicts (same objects), which makes
// the own-write check and the next merge patch compare them by identity.  The other way
// round, the encoder copies the bytes it remembered for a memo value it meets again by
// identity: the reconciler's status write re-sends the same history-entry dicts on every
// tick, so only the changed entries are encoded (a 10-entry status patch: 12 -> 1.3 us).

enum Action : uint8_t { kActNone = 0, kActSkip = 1, kActMemo = 2, kActRaw = 3, kActRoute = 4 };

struct PlanNode {
  std::vector<std::pair<std::string, int>> kids;
  int any = -1;  // child for list elements ("*")
  Action act = kActNone;
};

struct Plan {
  std::vector<PlanNode> nodes;  // nodes[0]: the root
  // route paths (hash-routed shards): an object there whose key hashes to another shard keeps
  // only what precedes and includes its `metadata`; the rest is skipped, never built.  The key
  // is `namespace/name`, or `namespace/<labels[route_label]>` when a label is given (an object
  // without that label is this shard's), hashed as runtime/controller.py shard_of does
  uint32_t route_index = 0, route_count = 0;
  std::string route_label;
  bool route_by_label = false;

  static bool utf8_of(PyObject* s, const char** d, Py_ssize_t* n) {
    if (!PyUnicode_CheckExact(s)) return false;
    *d = PyUnicode_AsUTF8AndSize(s, n);
    if (*d == nullptr) {
      PyErr_Clear();
      return false;
    }
    return true;
  }
  // true only when the object surely belongs to another shard (anything unexpected: kept)
  bool foreign(PyObject* meta) const {
    if (route_count <= 1 || !PyDict_CheckExact(meta)) return false;
    const char* ns = "";
    Py_ssize_t nn = 0;
    PyObject* nsv = PyDict_GetItemString(meta, "namespace");
    if (nsv != nullptr && !utf8_of(nsv, &ns, &nn)) return false;
    PyObject* keyv;
    if (route_by_label) {
      PyObject* labels = PyDict_GetItemString(meta, "labels");
      if (labels == nullptr || !PyDict_CheckExact(labels)) return false;
      keyv = PyDict_GetItemString(labels, route_label.c_str());
      if (keyv == nullptr) return false;
    } else {
      keyv = PyDict_GetItemString(meta, "name");
    }
    const char* key = "";
    Py_ssize_t kn = 0;
    if (keyv != nullptr && !utf8_of(keyv, &key, &kn)) return false;
    uint32_t h = 0x811C9DC5u;
    auto mix = [&h](const char* b, Py_ssize_t n) {
      for (Py_ssize_t i = 0; i < n; ++i) h = (h ^ static_cast<uint8_t>(b[i])) * 0x01000193u;
    };
    mix(ns, nn);
    mix("/", 1);
    mix(key, kn);
    return h % route_count != route_index;
  }

  int child(int node, const char* k, size_t n) const {
    if (node < 0) return -1;
    for (const auto& kv : nodes[static_cast<size_t>(node)].kids)
      if (kv.first.size() == n && std::memcmp(kv.first.data(), k, n) == 0) return kv.second;
    return -1;
  }
  int element(int node) const { return node < 0 ? -1 : nodes[static_cast<size_t>(node)].any; }
  Action act(int node) const { return node < 0 ? kActNone : nodes[static_cast<size_t>(node)].act; }

  // path: a sequence of str; returns false (with a Python error) on bad input
  bool add(PyObject* path, Action a) {
    PyObject* seq = PySequence_Fast(path, "a plan path must be a sequence of str");
    if (!seq) return false;
    int node = 0;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    if (n == 0) {
      Py_DECREF(seq);
      PyErr_SetString(PyExc_ValueError, "empty plan path");
      return false;
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* e = PySequence_Fast_GET_ITEM(seq, i);
      Py_ssize_t len;
      const char* k = PyUnicode_Check(e) ? PyUnicode_AsUTF8AndSize(e, &len) : nullptr;
      if (!k) {
        Py_DECREF(seq);
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_TypeError, "plan path elements must be str");
        return false;
      }
      int next;
      if (len == 1 && k[0] == '*') {
        next = nodes[static_cast<size_t>(node)].any;
        if (next < 0) {
          next = static_cast<int>(nodes.size());
          nodes.emplace_back();
          nodes[static_cast<size_t>(node)].any = next;
        }
      } else {
        next = child(node, k, static_cast<size_t>(len));
        if (next < 0) {
          next = static_cast<int>(nodes.size());
          nodes.emplace_back();
          nodes[static_cast<size_t>(node)].kids.emplace_back(std::string(k, static_cast<size_t>(len)), next);
        }
      }
      node = next;
    }
    Py_DECREF(seq);
    nodes[static_cast<size_t>(node)].act = a;
    return true;
  }
};

inline uint64_t span_hash(const char* p, size_t n) {
  // 8 bytes per step (multiply / xor-shift mixing); the tail byte by byte
  uint64_t h = 0x9E3779B97F4A7C15ULL ^ (n * 0xff51afd7ed558ccdULL);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, p + i, 8);
    h ^= w * 0xc4ceb9fe1a85ec53ULL;
    h = (h << 27) | (h >> 37);
    h *= 0x9E3779B97F4A7C15ULL;
  }
  for (; i < n; ++i) {
    h ^= static_cast<unsigned char>(p[i]);
    h *= 1099511628211ULL;
  }
  h ^= h >> 33;
  return h;
}

struct MemoSlot {
  uint64_t hash = 0;
  char* bytes = nullptr;    // malloc'd copy of the value's JSON (nullptr: empty slot)
  PyObject* obj = nullptr;  // strong ref
  uint32_t len = 0;
  uint32_t stamp = 0;       // table clock at the last hit / store (least recently used goes first)
  bool canonical = false;   // `bytes` is this encoder's own output for `obj` (not a peer's encoding)
};

// bytes -> object, plus object -> slot: the encoder copies the remembered bytes of a memo value
// it meets again (by identity) instead of encoding it anew.  A slot holds a strong reference to
// its object, so a pointer match is that very object; memo values are never mutated (the
// contract above), so their canonical bytes stay exact.
//
// 4-way set associative with two candidate sets per value, least recently used way replaced.  Once half full, the table doubles (up to
// `max_slots`) instead of replacing a way that was used within the last table-size operations: the working set
// -- a 10,000-Cron shard remembers ~10 history entries plus a labels map and an owner reference
// per Cron, ~120,000 values -- then fits instead of thrashing (a missed label map is a fresh copy
// in every cached child).  The object -> slot index is an exact open-addressed map, so
// forget() always drops the entry of a value that rotated out and the live count stays the
// working set (40-byte slots; the bytes live in their own allocation).
struct MemoTable {
  static constexpr size_t kWays = 4;
  static constexpr uint32_t kTomb = 0xFFFFFFFFu;
  std::vector<MemoSlot> slots;
  std::vector<uint32_t> by_obj;  // open addressing: slot index + 1; 0 empty, kTomb deleted
  size_t mask = 0, omask = 0, max_slots = 0, used = 0, tombs = 0;
  uint32_t clock = 0;
  uint64_t hits = 0, misses = 0, stores = 0, reuses = 0, evictions = 0, grows = 0;

  static size_t pow2(size_t n) {
    size_t cap = 64;
    while (cap < n) cap <<= 1;
    return cap;
  }
  MemoTable(size_t n, size_t max_n) {
    const size_t cap = pow2(n);
    max_slots = std::max(cap, pow2(max_n));
    slots.resize(cap);
    by_obj.assign(cap * 2, 0);
    mask = cap - 1;
    omask = cap * 2 - 1;
  }
  ~MemoTable() { clear(); }
  static void release(MemoSlot& sl) {
    Py_CLEAR(sl.obj);
    std::free(sl.bytes);
    sl.bytes = nullptr;
    sl.len = 0;
    sl.hash = 0;
    sl.canonical = false;
  }
  void clear() {
    for (auto& sl : slots) release(sl);
    std::fill(by_obj.begin(), by_obj.end(), 0);
    used = 0;
    tombs = 0;
  }
  static inline size_t ptr_hash(const PyObject* o) {
    uint64_t x = reinterpret_cast<uintptr_t>(o) >> 4;
    x *= 0x9E3779B97F4A7C15ULL;
    return static_cast<size_t>(x >> 17);
  }
  // two candidate sets per value (two-choice hashing: a set overflows far less often than with one)
  inline size_t bucket(uint64_t h) const { return static_cast<size_t>(h) & mask & ~(kWays - 1); }
  inline size_t bucket2(uint64_t h) const {
    return static_cast<size_t>((h >> 32) ^ (h * 0x9E3779B97F4A7C15ULL >> 29)) & mask & ~(kWays - 1);
  }
  // position in by_obj of the entry for `o`, or SIZE_MAX
  size_t find_obj(const PyObject* o) const {
    for (size_t i = ptr_hash(o) & omask;; i = (i + 1) & omask) {
      const uint32_t e = by_obj[i];
      if (e == 0) return SIZE_MAX;
      if (e != kTomb && slots[e - 1].obj == o) return i;
    }
  }
  void map_obj(size_t slot) {
    const PyObject* o = slots[slot].obj;
    const size_t at = find_obj(o);
    if (at != SIZE_MAX) {  // the same object under other bytes: the newest slot answers for it
      by_obj[at] = static_cast<uint32_t>(slot + 1);
      return;
    }
    for (size_t i = ptr_hash(o) & omask;; i = (i + 1) & omask) {
      const uint32_t e = by_obj[i];
      if (e == 0 || e == kTomb) {
        if (e == kTomb) --tombs;
        by_obj[i] = static_cast<uint32_t>(slot + 1);
        return;
      }
    }
  }
  void unmap_obj(size_t slot) {
    const size_t at = find_obj(slots[slot].obj);
    if (at != SIZE_MAX && by_obj[at] == slot + 1) {
      by_obj[at] = kTomb;
      ++tombs;
    }
  }
  // (once the slots are consistent again: after a store or a forget)
  inline void maybe_reindex() {
    if (tombs > by_obj.size() / 4) reindex();
  }
  void reindex() {
    std::fill(by_obj.begin(), by_obj.end(), 0);
    tombs = 0;
    for (size_t i = 0; i < slots.size(); ++i)
      if (slots[i].obj != nullptr) map_obj(i);
  }
  static inline bool same(const MemoSlot& sl, const char* p, size_t n, uint64_t h) {
    return sl.obj != nullptr && sl.hash == h && sl.len == n && std::memcmp(sl.bytes, p, n) == 0;
  }
  PyObject* find(const char* p, size_t n, uint64_t h) {  // borrowed
    const size_t bs[2] = {bucket(h), bucket2(h)};
    for (const size_t b : bs) {
      for (size_t w = 0; w < kWays; ++w) {
        MemoSlot& sl = slots[b + w];
        if (same(sl, p, n, h)) {
          ++hits;
          sl.stamp = ++clock;
          return sl.obj;
        }
      }
    }
    ++misses;
    return nullptr;
  }
  // double the table (every remembered value re-placed; one that finds its new set full is dropped)
  void grow() {
    std::vector<MemoSlot> old;
    old.swap(slots);
    const size_t cap = old.size() * 2;
    slots.resize(cap);
    by_obj.assign(cap * 2, 0);
    mask = cap - 1;
    omask = cap * 2 - 1;
    used = 0;
    tombs = 0;
    ++grows;
    for (auto& o : old) {
      if (o.obj == nullptr) continue;
      size_t at = SIZE_MAX;
      for (const size_t b : {bucket(o.hash), bucket2(o.hash)}) {
        for (size_t w = 0; w < kWays && at == SIZE_MAX; ++w)
          if (slots[b + w].obj == nullptr) at = b + w;
      }
      if (at == SIZE_MAX) {
        release(o);
        continue;
      }
      slots[at] = o;
      o.obj = nullptr;
      o.bytes = nullptr;
      map_obj(at);
      ++used;
    }
  }
  void store(const char* p, size_t n, uint64_t h, PyObject* o, bool canonical) {
    if (n > 0xFFFFFFFFu) return;
    const size_t bs[2] = {bucket(h), bucket2(h)};
    size_t i = SIZE_MAX;
    for (const size_t b : bs) {  // the same bytes again: replace that entry
      for (size_t w = 0; w < kWays && i == SIZE_MAX; ++w)
        if (same(slots[b + w], p, n, h)) i = b + w;
    }
    for (const size_t b : bs) {  // else a free way of either set
      for (size_t w = 0; w < kWays && i == SIZE_MAX; ++w)
        if (slots[b + w].obj == nullptr) i = b + w;
    }
    if (i == SIZE_MAX) {  // else the least recently used of the 8
      size_t lru = bs[0];
      for (const size_t b : bs)
        for (size_t w = 0; w < kWays; ++w)
          if (static_cast<uint32_t>(clock - slots[b + w].stamp) > static_cast<uint32_t>(clock - slots[lru].stamp))
            lru = b + w;
      if (used * 2 > slots.size() && slots.size() < max_slots &&
          static_cast<uint32_t>(clock - slots[lru].stamp) < slots.size()) {
        grow();
        store(p, n, h, o, canonical);
        return;
      }
      i = lru;
      ++evictions;
    }
    char* copy = static_cast<char*>(std::malloc(n ? n : 1));
    if (copy == nullptr) return;  // out of memory: simply not remembered
    std::memcpy(copy, p, n);
    MemoSlot& sl = slots[i];
    if (sl.obj != nullptr) {
      unmap_obj(i);
      release(sl);
    } else {
      ++used;
    }
    Py_INCREF(o);
    sl.obj = o;
    sl.bytes = copy;
    sl.len = static_cast<uint32_t>(n);
    sl.hash = h;
    sl.canonical = canonical;
    sl.stamp = ++clock;
    map_obj(i);
    ++stores;
    maybe_reindex();
  }
  // drop the slot holding exactly `o` (false: nothing remembers it)
  bool forget(const PyObject* o) {
    const size_t at = find_obj(o);
    if (at == SIZE_MAX) return false;
    const size_t i = by_obj[at] - 1;
    by_obj[at] = kTomb;
    release(slots[i]);
    --used;
    ++tombs;
    maybe_reindex();
    return true;
  }
  // this encoder's bytes for exactly `o` (nullptr when not remembered or a peer's bytes)
  const MemoSlot* canonical_bytes(const PyObject* o) {
    const size_t at = find_obj(o);
    if (at == SIZE_MAX) return nullptr;
    MemoSlot& sl = slots[by_obj[at] - 1];
    if (!sl.canonical) return nullptr;
    ++reuses;
    sl.stamp = ++clock;
    return &sl;
  }
};

struct Decoder {
  const char* begin;
  const char* p;
  const char* end;
  std::vector<Py_UCS4> ubuf;
  const Plan* plan = nullptr;
  MemoTable* memo = nullptr;

  PyObject* fail(const char* msg) {
    if (!PyErr_Occurred()) {
      PyErr_Format(PyExc_ValueError, "%s: char %zd", msg, static_cast<Py_ssize_t>(p - begin));
    }
    return nullptr;
  }

  inline void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }

  static inline int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }

  bool hex4(Py_UCS4* out) {
    if (end - p < 4) return false;
    Py_UCS4 v = 0;
    for (int i = 0; i < 4; ++i) {
      const int h = hexval(p[i]);
      if (h < 0) return false;
      v = (v << 4) | static_cast<Py_UCS4>(h);
    }
    p += 4;
    *out = v;
    return true;
  }

  // decode one UTF-8 sequence at p (p < end, *p >= 0x80)
  bool utf8(Py_UCS4* out) {
    const unsigned char c = static_cast<unsigned char>(*p);
    int n;
    Py_UCS4 v;
    if ((c & 0xE0) == 0xC0) { n = 1; v = c & 0x1F; }
    else if ((c & 0xF0) == 0xE0) { n = 2; v = c & 0x0F; }
    else if ((c & 0xF8) == 0xF0) { n = 3; v = c & 0x07; }
    else return false;
    if (end - p <= n) return false;
    for (int i = 1; i <= n; ++i) {
      const unsigned char cc = static_cast<unsigned char>(p[i]);
      if ((cc & 0xC0) != 0x80) return false;
      v = (v << 6) | (cc & 0x3F);
    }
    if ((n == 1 && v < 0x80) || (n == 2 && v < 0x800) || (n == 3 && (v < 0x10000 || v > 0x10FFFF))) return false;
    if (v >= 0xD800 && v <= 0xDFFF) return false;
    p += n + 1;
    *out = v;
    return true;
  }

  // p is just past the opening quote
  PyObject* string(bool key) {
    const char* s = p;
    bool ascii = true;
#if defined(__SSE2__)
    // 16 bytes at a time while none is '"', a backslash, a control character or non-ASCII
    // (a signed compare below 0x20 catches both < 0x20 and >= 0x80)
    {
      const __m128i lim = _mm_set1_epi8(0x20), quote = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\');
      while (end - p >= 16) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
        const __m128i hit = _mm_or_si128(_mm_cmplt_epi8(v, lim),
                                         _mm_or_si128(_mm_cmpeq_epi8(v, quote), _mm_cmpeq_epi8(v, bs)));
        if (_mm_movemask_epi8(hit) != 0) break;
        p += 16;
      }
    }
#endif
    while (p < end) {
      const unsigned char c = static_cast<unsigned char>(*p);
      if (c == '"') break;
      if (c == '\\') goto slow;
      if (c < 0x20) return fail("Invalid control character");
      if (c >= 0x80) ascii = false;
      ++p;
    }
    if (p >= end) return fail("Unterminated string");
    {
      const size_t n = static_cast<size_t>(p - s);
      ++p;  // closing quote
      if (ascii) {
        if (key && n <= kMaxKeyLen) return cached_key(s, n);
        if (!key && n <= kMaxValLen) return cached_value(s, n);
        PyObject* str = PyUnicode_New(static_cast<Py_ssize_t>(n), 127);
        if (!str) return nullptr;
        std::memcpy(PyUnicode_DATA(str), s, n);
        return str;
      }
      PyObject* str = PyUnicode_DecodeUTF8(s, static_cast<Py_ssize_t>(n), "strict");
      if (!str) {
        PyErr_Clear();
        return fail("Invalid UTF-8 in string");
      }
      return str;
    }
  slow:
    ubuf.clear();
    for (const char* q = s; q < p; ) {  // the run before the first backslash
      const unsigned char c = static_cast<unsigned char>(*q);
      if (c < 0x80) { ubuf.push_back(c); ++q; continue; }
      const char* save = p;
      p = q;
      Py_UCS4 v;
      if (!utf8(&v)) return fail("Invalid UTF-8 in string");
      q = p;
      p = save;
      ubuf.push_back(v);
    }
    while (true) {
      if (p >= end) return fail("Unterminated string");
      const unsigned char c = static_cast<unsigned char>(*p);
      if (c == '"') { ++p; break; }
      if (c < 0x20) return fail("Invalid control character");
      if (c == '\\') {
        ++p;
        if (p >= end) return fail("Unterminated string");
        const char e = *p++;
        Py_UCS4 v;
        switch (e) {
          case '"': v = '"'; break;
          case '\\': v = '\\'; break;
          case '/': v = '/'; break;
          case 'b': v = '\b'; break;
          case 'f': v = '\f'; break;
          case 'n': v = '\n'; break;
          case 'r': v = '\r'; break;
          case 't': v = '\t'; break;
          case 'u': {
            if (!hex4(&v)) return fail("Invalid \\uXXXX escape");
            if (v >= 0xD800 && v <= 0xDBFF && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              const char* save = p;
              p += 2;
              Py_UCS4 lo;
              if (hex4(&lo) && lo >= 0xDC00 && lo <= 0xDFFF) {
                v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
              } else {
                p = save;  // lone high surrogate: kept as is (json.loads does the same)
              }
            }
            break;
          }
          default:
            --p;
            return fail("Invalid \\escape");
        }
        ubuf.push_back(v);
        continue;
      }
      if (c >= 0x80) {
        Py_UCS4 v;
        if (!utf8(&v)) return fail("Invalid UTF-8 in string");
        ubuf.push_back(v);
        continue;
      }
      ubuf.push_back(c);
      ++p;
    }
    PyObject* str = PyUnicode_FromKindAndData(PyUnicode_4BYTE_KIND, ubuf.data(), static_cast<Py_ssize_t>(ubuf.size()));
    if (str && key) PyUnicode_InternInPlace(&str);
    return str;
  }

  PyObject* number() {
    const char* s = p;
    bool is_float = false;
    if (*p == '-') {
      ++p;
      if (p < end && *p == 'I') {
        if (end - p >= 8 && std::memcmp(p, "Infinity", 8) == 0) {
          p += 8;
          return PyFloat_FromDouble(-Py_HUGE_VAL);
        }
        return fail("Expecting value");
      }
    }
    if (p >= end) return fail("Expecting value");
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < end && *p >= '0' && *p <= '9') ++p;
    } else {
      p = s;
      return fail("Expecting value");
    }
    if (p < end && *p == '.' && p + 1 < end && p[1] >= '0' && p[1] <= '9') {
      is_float = true;
      ++p;
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      const char* save = p;
      ++p;
      if (p < end && (*p == '+' || *p == '-')) ++p;
      if (p < end && *p >= '0' && *p <= '9') {
        is_float = true;
        while (p < end && *p >= '0' && *p <= '9') ++p;
      } else {
        p = save;  // "1e" -> the number ends before 'e' (then: extra data)
      }
    }
    const size_t n = static_cast<size_t>(p - s);
    char small[64];
    std::string big;
    const char* z;
    if (n < sizeof(small)) {
      std::memcpy(small, s, n);
      small[n] = 0;
      z = small;
    } else {
      big.assign(s, n);
      z = big.c_str();
    }
    if (is_float) {
      const double d = PyOS_string_to_double(z, nullptr, nullptr);
      if (d == -1.0 && PyErr_Occurred()) return nullptr;
      return PyFloat_FromDouble(d);
    }
    if (n <= 18) return PyLong_FromLongLong(std::strtoll(z, nullptr, 10));
    return PyLong_FromString(z, nullptr, 10);
  }

  // scan past one string (p just past its opening quote); no validation
  bool skip_string() {
#if defined(__SSE2__)
    {
      const __m128i quote = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\');
      while (end - p >= 16) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
        if (_mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(v, quote), _mm_cmpeq_epi8(v, bs))) != 0) break;
        p += 16;
      }
    }
#endif
    while (p < end) {
      const char c = *p;
      if (c == '\\') {
        if (end - p < 2) break;
        p += 2;
        continue;
      }
      ++p;
      if (c == '"') return true;
    }
    fail("Unterminated string");
    return false;
  }

  // scan past one value (p at its first byte, whitespace skipped); structure only
  // the members left in an object (after a value): `, "key": value ...}` skipped up to and
  // including the closing brace, with the same syntax checks as a decode
  bool skip_members() {
    while (true) {
      ws();
      if (p < end && *p == '}') {
        ++p;
        return true;
      }
      if (p >= end || *p != ',') {
        fail("Expecting ',' delimiter");
        return false;
      }
      ++p;
      ws();
      if (p >= end || *p != '"') {
        fail("Expecting property name enclosed in double quotes");
        return false;
      }
      if (!skip_value()) return false;
      ws();
      if (p >= end || *p != ':') {
        fail("Expecting ':' delimiter");
        return false;
      }
      ++p;
      ws();
      if (!skip_value()) return false;
    }
  }

  bool skip_value() {
    if (p >= end) {
      fail("Expecting value");
      return false;
    }
    const char c0 = *p;
    if (c0 == '"') {
      ++p;
      return skip_string();
    }
    if (c0 == '{' || c0 == '[') {
      int d = 0;
      while (p < end) {
        const char c = *p;
        if (c == '"') {
          ++p;
          if (!skip_string()) return false;
          continue;
        }
        ++p;
        if (c == '{' || c == '[') {
          if (++d > kMaxDepth) {
            PyErr_SetString(PyExc_RecursionError, "JSON nested too deeply");
            return false;
          }
        } else if (c == '}' || c == ']') {
          if (--d == 0) return true;
        }
      }
      fail("Unterminated container");
      return false;
    }
    const char* s = p;
    while (p < end && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n' && *p != '\r' &&
           *p != '\t')
      ++p;
    if (p == s) {
      fail("Expecting value");
      return false;
    }
    return true;
  }

  // a value at a memo path: reuse the object remembered for exactly these bytes
  // a value at a raw path: its JSON text, undecoded
  PyObject* raw_value() {
    ws();
    const char* s = p;
    if (!skip_value()) return nullptr;
    return PyBytes_FromStringAndSize(s, static_cast<Py_ssize_t>(p - s));
  }

  PyObject* memo_value(int depth, int node) {
    ws();
    const char* s = p;
    if (!skip_value()) return nullptr;
    const size_t n = static_cast<size_t>(p - s);
    const uint64_t h = span_hash(s, n);
    PyObject* hit = memo->find(s, n, h);
    if (hit != nullptr) {
      Py_INCREF(hit);
      return hit;
    }
    const char* after = p;
    p = s;
    PyObject* v = value(depth, node, true);  // plan paths below the memo path still apply
    if (!v) return nullptr;
    if (p != after) {  // cannot happen for well-formed input: keep the parse, do not remember it
      return v;
    }
    memo->store(s, n, h, v, false);
    return v;
  }

  static inline bool key_bytes(PyObject* k, const char** d, size_t* n) {
    if (!PyUnicode_IS_COMPACT_ASCII(k)) return false;
    *d = static_cast<const char*>(PyUnicode_DATA(k));
    *n = static_cast<size_t>(PyUnicode_GET_LENGTH(k));
    return true;
  }

  PyObject* value(int depth, int node = -1, bool no_memo = false) {
    if (depth > kMaxDepth) {
      PyErr_SetString(PyExc_RecursionError, "JSON nested too deeply");
      return nullptr;
    }
    if (node >= 0) {
      const Action a = plan->act(node);
      if (a == kActMemo && memo != nullptr && !no_memo) return memo_value(depth, node);
      if (a == kActRaw) return raw_value();
    }
    ws();
    if (p >= end) return fail("Expecting value");
    switch (*p) {
      case '{': {
        ++p;
        PyObject* d = PyDict_New();
        if (!d) return nullptr;
        ws();
        if (p < end && *p == '}') { ++p; return acyclic(d); }
        while (true) {
          ws();
          if (p >= end || *p != '"') { Py_DECREF(d); return fail("Expecting property name enclosed in double quotes"); }
          ++p;
          PyObject* k = string(true);
          if (!k) { Py_DECREF(d); return nullptr; }
          ws();
          if (p >= end || *p != ':') { Py_DECREF(k); Py_DECREF(d); return fail("Expecting ':' delimiter"); }
          ++p;
          int kid = -1;
          bool route_meta = false;
          if (node >= 0) {
            const char* kd;
            size_t kn;
            if (key_bytes(k, &kd, &kn)) {
              kid = plan->child(node, kd, kn);
              route_meta = plan->act(node) == kActRoute && kn == 8 && std::memcmp(kd, "metadata", 8) == 0;
            }
            if (kid >= 0 && plan->act(kid) == kActSkip) {
              Py_DECREF(k);
              ws();
              if (!skip_value()) { Py_DECREF(d); return nullptr; }
              ws();
              if (p < end && *p == ',') { ++p; continue; }
              if (p < end && *p == '}') { ++p; return acyclic(d); }
              Py_DECREF(d);
              return fail("Expecting ',' delimiter");
            }
          }
          PyObject* v = value(depth + 1, kid);
          if (!v) { Py_DECREF(k); Py_DECREF(d); return nullptr; }
          const int rc = PyDict_SetItem(d, k, v);
          const bool away = rc >= 0 && route_meta && plan->foreign(v);
          Py_DECREF(k);
          Py_DECREF(v);
          if (rc < 0) { Py_DECREF(d); return nullptr; }
          if (away) {  // another shard's object: its remaining members are skipped
            if (!skip_members()) { Py_DECREF(d); return nullptr; }
            return acyclic(d);
          }
          ws();
          if (p < end && *p == ',') { ++p; continue; }
          if (p < end && *p == '}') { ++p; return acyclic(d); }
          Py_DECREF(d);
          return fail("Expecting ',' delimiter");
        }
      }
      case '[': {
        ++p;
        std::vector<PyObject*> items;
        ws();
        if (p < end && *p == ']') { ++p; return acyclic(PyList_New(0)); }
        const int elem = node >= 0 ? plan->element(node) : -1;
        while (true) {
          PyObject* v = value(depth + 1, elem);
          if (!v) {
            for (PyObject* o : items) Py_DECREF(o);
            return nullptr;
          }
          items.push_back(v);
          ws();
          if (p < end && *p == ',') { ++p; continue; }
          if (p < end && *p == ']') { ++p; break; }
          for (PyObject* o : items) Py_DECREF(o);
          return fail("Expecting ',' delimiter");
        }
        PyObject* l = PyList_New(static_cast<Py_ssize_t>(items.size()));
        if (!l) {
          for (PyObject* o : items) Py_DECREF(o);
          return nullptr;
        }
        for (size_t i = 0; i < items.size(); ++i) PyList_SET_ITEM(l, static_cast<Py_ssize_t>(i), items[i]);
        return acyclic(l);
      }
      case '"':
        ++p;
        return string(false);
      case 't':
        if (end - p >= 4 && std::memcmp(p, "true", 4) == 0) { p += 4; Py_RETURN_TRUE; }
        return fail("Expecting value");
      case 'f':
        if (end - p >= 5 && std::memcmp(p, "false", 5) == 0) { p += 5; Py_RETURN_FALSE; }
        return fail("Expecting value");
      case 'n':
        if (end - p >= 4 && std::memcmp(p, "null", 4) == 0) { p += 4; Py_RETURN_NONE; }
        return fail("Expecting value");
      case 'N':
        if (end - p >= 3 && std::memcmp(p, "NaN", 3) == 0) { p += 3; return PyFloat_FromDouble(Py_NAN); }
        return fail("Expecting value");
      case 'I':
        if (end - p >= 8 && std::memcmp(p, "Infinity", 8) == 0) { p += 8; return PyFloat_FromDouble(Py_HUGE_VAL); }
        return fail("Expecting value");
      default:
        return number();
    }
  }
};

PyObject* py_loads(PyObject*, PyObject* arg) {
  const char* data;
  Py_ssize_t n;
  bool from_bytes = false;
  if (PyBytes_Check(arg)) {
    data = PyBytes_AS_STRING(arg);
    n = PyBytes_GET_SIZE(arg);
    from_bytes = true;
  } else if (PyByteArray_Check(arg)) {
    data = PyByteArray_AS_STRING(arg);
    n = PyByteArray_GET_SIZE(arg);
    from_bytes = true;
  } else if (PyUnicode_Check(arg)) {
    data = PyUnicode_AsUTF8AndSize(arg, &n);
    if (!data) return nullptr;
    if (n >= 3 && std::memcmp(data, "\xEF\xBB\xBF", 3) == 0) {
      PyErr_SetString(PyExc_ValueError, "Unexpected UTF-8 BOM (decode using utf-8-sig)");
      return nullptr;
    }
  } else {
    PyErr_Format(PyExc_TypeError, "the JSON object must be str, bytes or bytearray, not %s", Py_TYPE(arg)->tp_name);
    return nullptr;
  }
  if (from_bytes && n >= 3 && std::memcmp(data, "\xEF\xBB\xBF", 3) == 0) {
    data += 3;
    n -= 3;
  }
  Decoder d{data, data, data + n, {}};
  PyObject* v = d.value(0);
  if (!v) return nullptr;
  d.ws();
  if (d.p != d.end) {
    Py_DECREF(v);
    return d.fail("Extra data");
  }
  return v;
}


// ---------------------------------------------------------------------------------------- encoder
//
// The fake apiserver encodes every response and watch event and the operator every
// request body; CPython's encoder re-enters Python for each container.  This writes
// straight into one growing buffer.  Output matches json.dumps(separators=(",", ":"),
// ensure_ascii=False): floats via repr (PyOS_double_to_string 'r'), NaN/Infinity
// literals, non-str keys coerced like json (True -> "true", 1 -> "1", None -> "null"),
// tuples as arrays, control characters escaped as \uXXXX except the short forms.

struct Encoder {
  std::string out;
  // dumpb_shared: id(subtree) -> (subtree, bytes) for the top-level values of immutable trees,
  // except those under a key in `volatile_keys` (they change on every write: never reused)
  PyObject* shared = nullptr;
  PyObject* volatile_keys = nullptr;
  // Codec.dumpb: values written at memo paths are remembered (bytes -> object) afterwards,
  // and a value met again by identity is copied from its remembered bytes
  const Plan* plan = nullptr;
  MemoTable* memo = nullptr;
  struct Rec {
    size_t start, end;
    PyObject* obj;  // borrowed: alive for the whole encode (the caller holds the tree)
  };
  std::vector<Rec> recs;

  bool str(PyObject* u) {
    Py_ssize_t n;
    const char* p;
    if (PyUnicode_IS_COMPACT_ASCII(u)) {  // the common case: the bytes are the str's own data
      p = static_cast<const char*>(PyUnicode_DATA(u));
      n = PyUnicode_GET_LENGTH(u);
    } else {
      p = PyUnicode_AsUTF8AndSize(u, &n);
      if (!p) return false;  // lone surrogates: UnicodeEncodeError, like json.dumps(...).encode()
    }
    out.push_back('"');
    const char* run = p;
    const char* e = p + n;
    const char* q = p;
#if defined(__SSE2__)
    // 16 bytes at a time until one needs escaping: < 0x20 (unsigned), '"' or backslash
    {
      const __m128i lim = _mm_set1_epi8(0x1F), quote = _mm_set1_epi8('"'), bs = _mm_set1_epi8('\\');
      while (e - q >= 16) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(q));
        const __m128i ctl = _mm_cmpeq_epi8(_mm_min_epu8(v, lim), v);
        const __m128i hit = _mm_or_si128(ctl, _mm_or_si128(_mm_cmpeq_epi8(v, quote), _mm_cmpeq_epi8(v, bs)));
        if (_mm_movemask_epi8(hit) != 0) break;
        q += 16;
      }
    }
#endif
    for (; q < e; ++q) {
      const unsigned char c = static_cast<unsigned char>(*q);
      if (c >= 0x20 && c != '"' && c != '\\') continue;
      out.append(run, static_cast<size_t>(q - run));
      run = q + 1;
      switch (c) {
        case '"': out.append("\\\""); break;
        case '\\': out.append("\\\\"); break;
        case '\n': out.append("\\n"); break;
        case '\r': out.append("\\r"); break;
        case '\t': out.append("\\t"); break;
        case '\b': out.append("\\b"); break;
        case '\f': out.append("\\f"); break;
        default: {
          static const char hex[] = "0123456789abcdef";
          char buf[7] = {'\\', 'u', '0', '0', hex[c >> 4], hex[c & 15], 0};
          out.append(buf, 6);
        }
      }
    }
    out.append(run, static_cast<size_t>(e - run));
    out.push_back('"');
    return true;
  }

  bool flt(double d) {
    if (d != d) { out.append("NaN"); return true; }
    if (d == Py_HUGE_VAL) { out.append("Infinity"); return true; }
    if (d == -Py_HUGE_VAL) { out.append("-Infinity"); return true; }
    char* r = PyOS_double_to_string(d, 'r', 0, Py_DTSF_ADD_DOT_0, nullptr);
    if (!r) return false;
    out.append(r);
    PyMem_Free(r);
    return true;
  }

  bool integer(PyObject* o) {
    int overflow = 0;
    const long long v = PyLong_AsLongLongAndOverflow(o, &overflow);
    if (v == -1 && PyErr_Occurred()) return false;
    if (!overflow) {
      char buf[24];
      char* w = buf + sizeof(buf);
      unsigned long long u = v < 0 ? 0ULL - static_cast<unsigned long long>(v) : static_cast<unsigned long long>(v);
      do {
        *--w = static_cast<char>('0' + u % 10);
        u /= 10;
      } while (u);
      if (v < 0) *--w = '-';
      out.append(w, static_cast<size_t>(buf + sizeof(buf) - w));
      return true;
    }
    PyObject* s = PyLong_Type.tp_repr(o);
    if (!s) return false;
    Py_ssize_t n;
    const char* p = PyUnicode_AsUTF8AndSize(s, &n);
    if (p) out.append(p, static_cast<size_t>(n));
    Py_DECREF(s);
    return p != nullptr;
  }

  bool key(PyObject* k) {
    if (PyUnicode_Check(k)) return str(k);
    if (k == Py_True) { out.append("\"true\""); return true; }
    if (k == Py_False) { out.append("\"false\""); return true; }
    if (k == Py_None) { out.append("\"null\""); return true; }
    if (PyLong_Check(k)) {
      out.push_back('"');
      if (!integer(k)) return false;
      out.push_back('"');
      return true;
    }
    if (PyFloat_Check(k)) {
      out.push_back('"');
      if (!flt(PyFloat_AS_DOUBLE(k))) return false;
      out.push_back('"');
      return true;
    }
    PyErr_Format(PyExc_TypeError, "keys must be str, int, float, bool or None, not %s", Py_TYPE(k)->tp_name);
    return false;
  }

  bool value(PyObject* o, int depth, int node = -1, bool no_memo = false) {
    if (depth > kMaxDepth) {
      PyErr_SetString(PyExc_ValueError, "Circular reference detected");
      return false;
    }
    if (node >= 0 && plan->act(node) == kActRaw && PyBytes_Check(o)) {  // raw JSON text, as decoded
      out.append(PyBytes_AS_STRING(o), static_cast<size_t>(PyBytes_GET_SIZE(o)));
      return true;
    }
    if (node >= 0 && !no_memo && plan->act(node) == kActMemo) {
      if (memo != nullptr) {
        const MemoSlot* b = memo->canonical_bytes(o);
        if (b != nullptr) {
          out.append(b->bytes, b->len);
          return true;
        }
      }
      const size_t start = out.size();
      if (!value(o, depth, node, true)) return false;  // plan paths below the memo path still apply
      recs.push_back(Rec{start, out.size(), o});
      return true;
    }
    if (o == Py_None) { out.append("null"); return true; }
    if (o == Py_True) { out.append("true"); return true; }
    if (o == Py_False) { out.append("false"); return true; }
    if (PyUnicode_Check(o)) return str(o);
    if (PyLong_Check(o)) return integer(o);
    if (PyFloat_Check(o)) return flt(PyFloat_AS_DOUBLE(o));
    return container(o, depth, node);
  }

  // A subtree shared by identity with one encoded before (a status write keeps the stored
  // object's spec, a tombstone everything but its metadata) is copied from its bytes.
  bool cached(PyObject* o, int depth) {
    PyObject* id = PyLong_FromVoidPtr(o);
    if (!id) return false;
    PyObject* hit = PyDict_GetItemWithError(shared, id);  // borrowed
    if (hit != nullptr && PyTuple_GET_ITEM(hit, 0) == o) {
      PyObject* b = PyTuple_GET_ITEM(hit, 1);
      out.append(PyBytes_AS_STRING(b), static_cast<size_t>(PyBytes_GET_SIZE(b)));
      Py_DECREF(id);
      return true;
    }
    if (PyErr_Occurred()) {
      Py_DECREF(id);
      return false;
    }
    const size_t start = out.size();
    if (!container(o, depth)) {
      Py_DECREF(id);
      return false;
    }
    const size_t n = out.size() - start;
    int rc = 0;
    if (n >= kSharedMin) {
      PyObject* b = PyBytes_FromStringAndSize(out.data() + start, static_cast<Py_ssize_t>(n));
      PyObject* t = b ? PyTuple_Pack(2, o, b) : nullptr;  // holds o: its id stays unique while cached
      rc = t ? PyDict_SetItem(shared, id, t) : -1;
      Py_XDECREF(b);
      Py_XDECREF(t);
    }
    Py_DECREF(id);
    return rc == 0;
  }

  static constexpr size_t kSharedMin = 64;

  bool container(PyObject* o, int depth, int node = -1) {
    if (PyDict_Check(o)) {
      out.push_back('{');
      Py_ssize_t pos = 0;
      PyObject *k, *v;
      bool first = true;
      while (PyDict_Next(o, &pos, &k, &v)) {
        if (!first) out.push_back(',');
        first = false;
        if (!key(k)) return false;
        out.push_back(':');
        if (depth == 0 && shared != nullptr && (PyDict_CheckExact(v) || PyList_CheckExact(v))) {
          const int vol = volatile_keys != nullptr ? PySequence_Contains(volatile_keys, k) : 0;
          if (vol < 0) return false;
          if (!(vol ? value(v, depth + 1) : cached(v, depth + 1))) return false;
          continue;
        }
        int kid = -1;
        if (node >= 0 && PyUnicode_IS_COMPACT_ASCII(k))
          kid = plan->child(node, static_cast<const char*>(PyUnicode_DATA(k)),
                            static_cast<size_t>(PyUnicode_GET_LENGTH(k)));
        if (!value(v, depth + 1, kid)) return false;
      }
      out.push_back('}');
      return true;
    }
    if (PyList_Check(o) || PyTuple_Check(o)) {
      PyObject* seq = o;
      const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
      PyObject** items = PySequence_Fast_ITEMS(seq);
      const int elem = node >= 0 ? plan->element(node) : -1;
      out.push_back('[');
      for (Py_ssize_t i = 0; i < n; ++i) {
        if (i) out.push_back(',');
        if (!value(items[i], depth + 1, elem)) return false;
      }
      out.push_back(']');
      return true;
    }
    PyErr_Format(PyExc_TypeError, "Object of type %s is not JSON serializable", Py_TYPE(o)->tp_name);
    return false;
  }
};

PyObject* py_dumpb(PyObject*, PyObject* o) {
  Encoder e;
  e.out.reserve(1024);
  if (!e.value(o, 0)) return nullptr;
  return PyBytes_FromStringAndSize(e.out.data(), static_cast<Py_ssize_t>(e.out.size()));
}

PyObject* py_dumpb_shared(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if ((nargs != 2 && nargs != 3) || !PyDict_CheckExact(args[1])) {
    PyErr_SetString(PyExc_TypeError, "dumpb_shared(tree, cache: dict, volatile_keys=())");
    return nullptr;
  }
  Encoder e;
  e.shared = args[1];
  e.volatile_keys = nargs == 3 ? args[2] : nullptr;
  e.out.reserve(1024);
  if (!e.value(args[0], 0)) return nullptr;
  return PyBytes_FromStringAndSize(e.out.data(), static_cast<Py_ssize_t>(e.out.size()));
}

PyObject* py_dumps(PyObject*, PyObject* o) {
  Encoder e;
  e.out.reserve(1024);
  if (!e.value(o, 0)) return nullptr;
  return PyUnicode_DecodeUTF8(e.out.data(), static_cast<Py_ssize_t>(e.out.size()), "strict");
}

PyObject* py_clear_key_cache(PyObject*, PyObject*) {
  clear_keys();
  Py_RETURN_NONE;
}

PyObject* py_deepcopy(PyObject*, PyObject* x) { return deepcopy_impl(x, 0); }

PyObject* py_json_equal(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "json_equal(a, b)");
    return nullptr;
  }
  const int r = equal_impl(args[0], args[1], 0);
  if (r < 0) return nullptr;
  return PyBool_FromLong(r);
}

PyObject* py_merge_patch(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2 && nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "create_merge_patch(old, new, share=False)");
    return nullptr;
  }
  int share = 0;
  if (nargs == 3 && (share = PyObject_IsTrue(args[2])) < 0) return nullptr;
  return merge_patch_impl(args[0], args[1], 0, share != 0);
}

// ---------------------------------------------------------------------- kubeflow job status
//
// kubeflow_summary(status) -> None | (finished, last_type, n_conditions, completion_time, terminal_ltt)
//
// What the reconciler's classification reads from a training-operator JobStatus
// (models/kubeflow.py, models/workload.py classify; reference cron_util.go:73-114): whether a
// Succeeded/Failed condition is True, the last condition's type, and the raw completionTime /
// the terminal condition's lastTransitionTime strings.  Only exactly-typed input is taken
// (str/None string fields, int/None counts, RFC 3339 times as time.Parse(time.RFC3339)
// accepts them, in ASCII); anything else returns None and the Python converter -- the oracle
// of tests/test_kubeflow_status.py -- decides, raising its precise ConversionError.

// ASCII RFC 3339 with the Python parser's field ranges (a subset of what it accepts)
bool rfc3339_ok(PyObject* v) {
  if (!PyUnicode_IS_COMPACT_ASCII(v)) return false;
  const char* s = static_cast<const char*>(PyUnicode_DATA(v));
  const Py_ssize_t n = PyUnicode_GET_LENGTH(v);
  if (n < 20) return false;
  auto dig = [s](Py_ssize_t i) { return s[i] >= '0' && s[i] <= '9'; };
  static const int kDigits[] = {0, 1, 2, 3, 5, 6, 8, 9, 11, 12, 14, 15, 17, 18};
  for (int i : kDigits)
    if (!dig(i)) return false;
  if (s[4] != '-' || s[7] != '-' || (s[10] != 'T' && s[10] != 't') || s[13] != ':' || s[16] != ':') return false;
  auto two = [s](int i) { return (s[i] - '0') * 10 + (s[i + 1] - '0'); };
  const int mo = two(5), d = two(8), hh = two(11), mi = two(14), ss = two(17);
  if (mo < 1 || mo > 12 || d < 1 || d > 31 || hh > 23 || mi > 59 || ss > 59) return false;
  Py_ssize_t i = 19;
  if (s[i] == '.') {
    const Py_ssize_t b = ++i;
    while (i < n && dig(i)) ++i;
    if (i - b < 1 || i - b > 9) return false;
  }
  if (i < n && (s[i] == 'Z' || s[i] == 'z')) return i + 1 == n;
  return n - i == 6 && (s[i] == '+' || s[i] == '-') && dig(i + 1) && dig(i + 2) && s[i + 3] == ':' &&
         dig(i + 4) && dig(i + 5);
}

// a time field: absent/None/"" (no time) or a valid string; false -> the strict path decides
inline bool time_ok(PyObject* v) {
  if (v == nullptr || v == Py_None) return true;
  if (!PyUnicode_CheckExact(v)) return false;
  return PyUnicode_GET_LENGTH(v) == 0 || rfc3339_ok(v);
}

inline bool str_or_none(PyObject* v) { return v == nullptr || v == Py_None || PyUnicode_CheckExact(v); }
inline bool int_or_none(PyObject* v) { return v == nullptr || v == Py_None || PyLong_CheckExact(v); }

inline bool eq_ascii(PyObject* v, const char* lit) {
  return v != nullptr && PyUnicode_CheckExact(v) && PyUnicode_IS_COMPACT_ASCII(v) &&
         std::strcmp(static_cast<const char*>(PyUnicode_DATA(v)), lit) == 0 &&
         static_cast<size_t>(PyUnicode_GET_LENGTH(v)) == std::strlen(lit);
}

PyObject* py_kubeflow_summary(PyObject*, PyObject* st) {
  if (!PyDict_CheckExact(st)) Py_RETURN_NONE;
  PyObject* conds = PyDict_GetItemString(st, "conditions");  // borrowed
  bool finished = false;
  PyObject* last = nullptr;
  PyObject* tltt = nullptr;  // lastTransitionTime of the last True Succeeded/Failed condition
  Py_ssize_t nconds = 0;
  if (conds != nullptr && conds != Py_None) {
    if (!PyList_CheckExact(conds)) Py_RETURN_NONE;
    nconds = PyList_GET_SIZE(conds);
    for (Py_ssize_t i = 0; i < nconds; ++i) {
      PyObject* c = PyList_GET_ITEM(conds, i);
      if (!PyDict_CheckExact(c)) Py_RETURN_NONE;
      PyObject* type = PyDict_GetItemString(c, "type");
      PyObject* status = PyDict_GetItemString(c, "status");
      PyObject* ltt = PyDict_GetItemString(c, "lastTransitionTime");
      if (!str_or_none(type) || !str_or_none(status) || !str_or_none(PyDict_GetItemString(c, "reason")) ||
          !str_or_none(PyDict_GetItemString(c, "message")) || !time_ok(PyDict_GetItemString(c, "lastUpdateTime")) ||
          !time_ok(ltt))
        Py_RETURN_NONE;
      if ((eq_ascii(type, "Succeeded") || eq_ascii(type, "Failed")) && eq_ascii(status, "True")) {
        finished = true;
        tltt = ltt;
      }
      last = type;
    }
  }
  PyObject* rs = PyDict_GetItemString(st, "replicaStatuses");
  if (rs != nullptr && rs != Py_None) {
    if (!PyDict_CheckExact(rs)) Py_RETURN_NONE;
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    while (PyDict_Next(rs, &pos, &k, &v)) {
      if (v == Py_None) continue;
      if (!PyDict_CheckExact(v)) Py_RETURN_NONE;
      PyObject* sel = PyDict_GetItemString(v, "labelSelector");
      if (!int_or_none(PyDict_GetItemString(v, "active")) || !int_or_none(PyDict_GetItemString(v, "succeeded")) ||
          !int_or_none(PyDict_GetItemString(v, "failed")) || !str_or_none(PyDict_GetItemString(v, "selector")) ||
          !(sel == nullptr || sel == Py_None || PyDict_CheckExact(sel)))
        Py_RETURN_NONE;
    }
  }
  PyObject* comp = PyDict_GetItemString(st, "completionTime");
  if (!time_ok(PyDict_GetItemString(st, "startTime")) || !time_ok(comp) ||
      !time_ok(PyDict_GetItemString(st, "lastReconcileTime")))
    Py_RETURN_NONE;
  auto text = [](PyObject* v) -> PyObject* {  // a non-empty time string, else None
    if (v == nullptr || v == Py_None || PyUnicode_GET_LENGTH(v) == 0) Py_RETURN_NONE;
    Py_INCREF(v);
    return v;
  };
  PyObject* last_s = (last == nullptr || last == Py_None) ? PyUnicode_FromStringAndSize("", 0) : (Py_INCREF(last), last);
  PyObject* comp_s = text(comp);
  PyObject* tltt_s = text(tltt);
  return Py_BuildValue("(ONnNN)", finished ? Py_True : Py_False, last_s, nconds, comp_s, tltt_s);
}

PyObject* py_set_gc_untrack(PyObject*, PyObject* arg) {
  const int on = PyObject_IsTrue(arg);
  if (on < 0) return nullptr;
  PyObject* prev = g_untrack ? Py_True : Py_False;
  g_untrack = on != 0;
  Py_INCREF(prev);
  return prev;
}

// ---------------------------------------------------------------------------- Memo / Codec types

struct MemoObject {
  PyObject_HEAD
  MemoTable* table;
};

// ---------------------------------------------------------------------------------------------
// store_apply: the bookkeeping of one informer event (runtime/informer.py Informer._apply) on the
// informer's own dicts -- the store key (`ns/name`, or `name` without a namespace), the store
// write or delete, the derived-memo drop, and the namespace and label indexes -- so that only
// the event handlers stay in Python.  Anything irregular (metadata, namespace, name or label of
// an unexpected type) returns None before a single dict is touched, and the Python path decides.

PyObject *s_metadata_key, *s_namespace_key, *s_name_key, *s_labels_key, *s_empty;  // interned at import

// obj["metadata"] as a dict (nullptr: absent or falsy -> empty; `bad`: present but not a dict)
PyObject* meta_of(PyObject* obj, bool* bad) {
  PyObject* m = PyDict_GetItemWithError(obj, s_metadata_key);
  if (!m) return nullptr;  // absent (or a lookup error, surfaced by the caller's PyErr_Occurred)
  if (PyDict_CheckExact(m)) return PyDict_GET_SIZE(m) ? m : nullptr;
  const int t = PyObject_IsTrue(m);
  if (t != 0) *bad = true;  // truthy non-dict: Python's `.get` would raise
  return nullptr;
}

// m.get(k, "") as an exact str (nullptr + bad when present but not a str)
PyObject* str_field(PyObject* m, PyObject* k, bool* bad) {
  if (!m) return nullptr;
  PyObject* v = PyDict_GetItemWithError(m, k);
  if (!v) return nullptr;
  if (!PyUnicode_CheckExact(v)) {
    *bad = true;
    return nullptr;
  }
  return v;
}

// The store key; nullptr + bad on irregular input.  New reference.
PyObject* store_key(PyObject* m, bool* bad) {
  PyObject* ns = str_field(m, s_namespace_key, bad);
  PyObject* name = str_field(m, s_name_key, bad);
  if (*bad) return nullptr;
  if (!name) name = s_empty;
  if (!ns || PyUnicode_GET_LENGTH(ns) == 0) {
    Py_INCREF(name);
    return name;
  }
  return PyUnicode_FromFormat("%U/%U", ns, name);
}

// The index values of `m` for one indexer: label == nullptr -> [namespace]; else
// [ns/<label value>] or [] (returned as a new str, or nullptr for "no value").  bad on irregular.
PyObject* index_value(PyObject* m, PyObject* label, bool* bad, bool* none) {
  PyObject* ns = str_field(m, s_namespace_key, bad);
  if (*bad) return nullptr;
  if (!label) {
    *none = false;
    PyObject* v = ns ? ns : s_empty;
    Py_INCREF(v);
    return v;
  }
  PyObject* labels = m ? PyDict_GetItemWithError(m, s_labels_key) : nullptr;
  if (labels && !PyDict_CheckExact(labels)) {
    if (PyObject_IsTrue(labels) != 0) {
      *bad = true;
      return nullptr;
    }
    labels = nullptr;
  }
  PyObject* v = labels ? PyDict_GetItemWithError(labels, label) : nullptr;
  if (!v || v == Py_None) {
    *none = true;
    return nullptr;
  }
  if (!PyUnicode_CheckExact(v)) {
    *bad = true;
    return nullptr;
  }
  *none = false;
  return PyUnicode_FromFormat("%U/%U", ns ? ns : s_empty, v);
}

bool index_remove(PyObject* idx, PyObject* value, PyObject* key) {
  PyObject* s = PyDict_GetItemWithError(idx, value);
  if (!s) return !PyErr_Occurred();
  if (PySet_Discard(s, key) < 0) return false;
  if (PySet_GET_SIZE(s) == 0 && PyDict_DelItem(idx, value) < 0) return false;
  return true;
}

bool index_add(PyObject* idx, PyObject* value, PyObject* key) {
  PyObject* s = PyDict_GetItemWithError(idx, value);
  if (!s) {
    if (PyErr_Occurred()) return false;
    s = PySet_New(nullptr);
    if (!s) return false;
    const int r = PyDict_SetItem(idx, value, s);
    Py_DECREF(s);
    if (r < 0) return false;
  }
  return PySet_Add(s, key) == 0;
}

// store_apply(store, derived, indices, spec, deleting, obj) -> (key, old) | None
//   spec: tuple of (index name, label or None); None: the namespace index
PyObject* py_store_apply(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 6 || !PyDict_CheckExact(args[0]) || !PyDict_CheckExact(args[1]) || !PyDict_CheckExact(args[2]) ||
      !PyTuple_CheckExact(args[3])) {
    PyErr_SetString(PyExc_TypeError, "store_apply(store, derived, indices, spec, deleting, obj)");
    return nullptr;
  }
  PyObject *store = args[0], *derived = args[1], *indices = args[2], *spec = args[3], *obj = args[5];
  const int deleting = PyObject_IsTrue(args[4]);
  if (deleting < 0) return nullptr;
  if (!PyDict_CheckExact(obj)) Py_RETURN_NONE;
  bool bad = false;
  PyObject* m = meta_of(obj, &bad);
  if (PyErr_Occurred()) return nullptr;
  PyObject* key = bad ? nullptr : store_key(m, &bad);
  if (!key) {
    if (PyErr_Occurred()) return nullptr;
    Py_RETURN_NONE;
  }
  PyObject* old = PyDict_GetItemWithError(store, key);  // borrowed
  if (!old && PyErr_Occurred()) {
    Py_DECREF(key);
    return nullptr;
  }
  PyObject* om = nullptr;
  if (old) {
    if (!PyDict_CheckExact(old)) {
      Py_DECREF(key);
      Py_RETURN_NONE;
    }
    om = meta_of(old, &bad);
  }
  const Py_ssize_t ni = PyTuple_GET_SIZE(spec);
  // index values, all computed (and validated) before anything changes
  std::vector<PyObject*> names(ni), ov(ni, nullptr), nv(ni, nullptr), idxs(ni);
  std::vector<char> is_ns(ni), have_ov(ni, 0), have_nv(ni, 0);
  bool ok = !bad && !PyErr_Occurred();
  for (Py_ssize_t i = 0; ok && i < ni; ++i) {
    PyObject* e = PyTuple_GET_ITEM(spec, i);
    if (!PyTuple_CheckExact(e) || PyTuple_GET_SIZE(e) != 2) {
      ok = false;
      break;
    }
    names[i] = PyTuple_GET_ITEM(e, 0);
    PyObject* label = PyTuple_GET_ITEM(e, 1);
    is_ns[i] = label == Py_None;
    idxs[i] = PyDict_GetItemWithError(indices, names[i]);
    if (!idxs[i] || !PyDict_CheckExact(idxs[i])) {
      ok = false;
      break;
    }
    bool none = false;
    const bool update = old && !deleting;
    if (old && !(update && is_ns[i])) {
      ov[i] = index_value(om, is_ns[i] ? nullptr : label, &bad, &none);
      have_ov[i] = !none && ov[i];
    }
    if (!deleting && !(update && is_ns[i])) {
      none = false;
      nv[i] = index_value(m, is_ns[i] ? nullptr : label, &bad, &none);
      have_nv[i] = !none && nv[i];
    }
    if (bad || PyErr_Occurred()) ok = false;
  }
  PyObject* result = nullptr;
  if (ok) {
    bool done = true;
    Py_XINCREF(old);  // the store drops or replaces its reference below; we return it
    if (deleting) {
      if (old) {
        done = PyDict_DelItem(store, key) == 0;
        if (done) {
          PyObject* d = PyDict_GetItemWithError(derived, key);
          if (d) done = PyDict_DelItem(derived, key) == 0;
          else done = !PyErr_Occurred();
        }
        for (Py_ssize_t i = 0; done && i < ni; ++i)
          if (have_ov[i]) done = index_remove(idxs[i], ov[i], key);
      }
    } else {
      done = PyDict_SetItem(store, key, obj) == 0;
      for (Py_ssize_t i = 0; done && i < ni; ++i) {
        if (old && is_ns[i]) continue;  // the key carries the namespace: an update cannot move it
        if (old) {
          const bool same = have_ov[i] == have_nv[i] &&
                            (!have_ov[i] || PyUnicode_Compare(ov[i], nv[i]) == 0);
          if (same) continue;
          if (have_ov[i]) done = index_remove(idxs[i], ov[i], key);
        }
        if (done && have_nv[i]) done = index_add(idxs[i], nv[i], key);
      }
    }
    if (done) result = PyTuple_Pack(2, key, old ? old : Py_None);
    Py_XDECREF(old);
    if (!done && !PyErr_Occurred()) PyErr_SetString(PyExc_RuntimeError, "store_apply failed");
  } else if (!PyErr_Occurred()) {
    result = Py_None;
    Py_INCREF(result);
  }
  Py_XDECREF(key);
  for (Py_ssize_t i = 0; i < ni; ++i) {
    Py_XDECREF(ov[i]);
    Py_XDECREF(nv[i]);
  }
  return result;
}

// pick(mapping, keys) -> [mapping[k] for k in keys] (KeyError for a missing key)
PyObject* py_pick(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 2 || !PyDict_Check(args[0])) {
    PyErr_SetString(PyExc_TypeError, "pick(dict, keys)");
    return nullptr;
  }
  PyObject* it = PyObject_GetIter(args[1]);
  if (!it) return nullptr;
  PyObject* out = PyList_New(0);
  PyObject* k;
  while (out && (k = PyIter_Next(it))) {
    PyObject* v = PyDict_GetItemWithError(args[0], k);
    if (!v) {
      if (!PyErr_Occurred()) PyErr_SetObject(PyExc_KeyError, k);
      Py_CLEAR(out);
    } else if (PyList_Append(out, v) < 0) {
      Py_CLEAR(out);
    }
    Py_DECREF(k);
  }
  Py_DECREF(it);
  if (out && PyErr_Occurred()) Py_CLEAR(out);
  return out;
}

void memo_dealloc(PyObject* self) {
  delete reinterpret_cast<MemoObject*>(self)->table;
  Py_TYPE(self)->tp_free(self);
}

PyObject* memo_new(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  static const char* kw[] = {"slots", "max_slots", nullptr};
  Py_ssize_t n = 1 << 14, max_n = -1;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|nn", const_cast<char**>(kw), &n, &max_n)) return nullptr;
  if (max_n < 0) max_n = std::max<Py_ssize_t>(n, 1 << 19);
  if (n < 1 || n > (1 << 24) || max_n < n || max_n > (1 << 24)) {
    PyErr_SetString(PyExc_ValueError, "slots must be in [1, 2**24] and max_slots in [slots, 2**24]");
    return nullptr;
  }
  PyObject* self = type->tp_alloc(type, 0);
  if (!self) return nullptr;
  reinterpret_cast<MemoObject*>(self)->table = new MemoTable(static_cast<size_t>(n), static_cast<size_t>(max_n));
  return self;
}

PyObject* memo_stats(PyObject* self, PyObject*) {
  MemoTable* t = reinterpret_cast<MemoObject*>(self)->table;
  size_t used = 0;
  for (const auto& sl : t->slots) used += sl.obj != nullptr;  // (== t->used)
  return Py_BuildValue("{s:K,s:K,s:K,s:K,s:K,s:K,s:n,s:n,s:n}", "hits", static_cast<unsigned long long>(t->hits),
                       "misses", static_cast<unsigned long long>(t->misses), "stores",
                       static_cast<unsigned long long>(t->stores), "reuses",
                       static_cast<unsigned long long>(t->reuses), "evictions",
                       static_cast<unsigned long long>(t->evictions), "grows",
                       static_cast<unsigned long long>(t->grows), "used", static_cast<Py_ssize_t>(used),
                       "slots", static_cast<Py_ssize_t>(t->slots.size()),
                       "max_slots", static_cast<Py_ssize_t>(t->max_slots));
}

PyObject* memo_clear(PyObject* self, PyObject*) {
  reinterpret_cast<MemoObject*>(self)->table->clear();
  Py_RETURN_NONE;
}

PyObject* memo_forget(PyObject* self, PyObject* o) {
  return PyBool_FromLong(reinterpret_cast<MemoObject*>(self)->table->forget(o));
}

PyMethodDef memo_methods[] = {
    {"stats", memo_stats, METH_NOARGS, "hits, misses, stores, used and total slots"},
    {"clear", memo_clear, METH_NOARGS, "drop every remembered object"},
    {"forget", memo_forget, METH_O,
     "forget(obj) -> bool: drop the entry remembering exactly obj (a value that will not be met again)"},
    {nullptr, nullptr, 0, nullptr}};

PyTypeObject MemoType = {PyVarObject_HEAD_INIT(nullptr, 0)};

struct CodecObject {
  PyObject_HEAD
  Plan* plan;
  PyObject* memo;  // MemoObject or nullptr
  vectorcallfunc vectorcall;
};

void codec_dealloc(PyObject* self) {
  CodecObject* c = reinterpret_cast<CodecObject*>(self);
  delete c->plan;
  Py_XDECREF(c->memo);
  Py_TYPE(self)->tp_free(self);
}

inline MemoTable* codec_memo(CodecObject* c) {
  return c->memo != nullptr ? reinterpret_cast<MemoObject*>(c->memo)->table : nullptr;
}

bool buffer_of(PyObject* arg, const char** data, Py_ssize_t* n) {
  if (PyBytes_Check(arg)) {
    *data = PyBytes_AS_STRING(arg);
    *n = PyBytes_GET_SIZE(arg);
    return true;
  }
  if (PyByteArray_Check(arg)) {
    *data = PyByteArray_AS_STRING(arg);
    *n = PyByteArray_GET_SIZE(arg);
    return true;
  }
  if (PyUnicode_Check(arg)) {
    *data = PyUnicode_AsUTF8AndSize(arg, n);
    return *data != nullptr;
  }
  PyErr_Format(PyExc_TypeError, "the JSON object must be str, bytes or bytearray, not %s", Py_TYPE(arg)->tp_name);
  return false;
}

PyObject* codec_decode(CodecObject* c, PyObject* arg) {
  const char* data;
  Py_ssize_t n;
  if (!buffer_of(arg, &data, &n)) return nullptr;
  Decoder d{data, data, data + n, {}};
  d.plan = c->plan;
  d.memo = codec_memo(c);
  PyObject* v = d.value(0, 0);
  if (!v) return nullptr;
  d.ws();
  if (d.p != d.end) {
    Py_DECREF(v);
    return d.fail("Extra data");
  }
  return v;
}

PyObject* codec_new(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  static const char* kw[] = {"skip", "memo_paths", "memo", "raw_paths", "route_paths", "route", nullptr};
  PyObject* skip = nullptr;
  PyObject* memo_paths = nullptr;
  PyObject* memo = nullptr;
  PyObject* raw_paths = nullptr;
  PyObject* route_paths = nullptr;
  PyObject* route = nullptr;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "|OOOOOO", const_cast<char**>(kw), &skip, &memo_paths, &memo,
                                   &raw_paths, &route_paths, &route))
    return nullptr;
  unsigned int r_index = 0, r_count = 0;
  PyObject* r_label = Py_None;
  const bool routed = route_paths != nullptr && route_paths != Py_None;
  if (routed) {
    // route = (index, count, label or None)
    if (route == nullptr || !PyTuple_Check(route) ||
        !PyArg_ParseTuple(route, "IIO", &r_index, &r_count, &r_label) || r_count < 1 || r_index >= r_count ||
        (r_label != Py_None && !PyUnicode_Check(r_label))) {
      if (!PyErr_Occurred())
        PyErr_SetString(PyExc_ValueError, "route must be (index, count, label or None) with 0 <= index < count");
      return nullptr;
    }
  }
  if (memo == Py_None) memo = nullptr;
  if (memo != nullptr && !PyObject_TypeCheck(memo, &MemoType)) {
    PyErr_SetString(PyExc_TypeError, "memo must be a Memo");
    return nullptr;
  }
  auto plan = new Plan();
  plan->nodes.emplace_back();
  auto add_all = [&](PyObject* paths, Action a) -> bool {
    if (paths == nullptr || paths == Py_None) return true;
    PyObject* seq = PySequence_Fast(paths, "paths must be a sequence of paths");
    if (!seq) return false;
    for (Py_ssize_t i = 0; i < PySequence_Fast_GET_SIZE(seq); ++i) {
      if (!plan->add(PySequence_Fast_GET_ITEM(seq, i), a)) {
        Py_DECREF(seq);
        return false;
      }
    }
    Py_DECREF(seq);
    return true;
  };
  if (!add_all(skip, kActSkip) || !add_all(memo_paths, kActMemo) || !add_all(raw_paths, kActRaw) ||
      (routed && !add_all(route_paths, kActRoute))) {
    delete plan;
    return nullptr;
  }
  if (routed) {
    plan->route_index = r_index;
    plan->route_count = r_count;
    if (r_label != Py_None) {
      Py_ssize_t ln = 0;
      const char* l = PyUnicode_AsUTF8AndSize(r_label, &ln);
      if (l == nullptr) {
        delete plan;
        return nullptr;
      }
      plan->route_label.assign(l, static_cast<size_t>(ln));
      plan->route_by_label = true;
    }
  }
  PyObject* self = type->tp_alloc(type, 0);
  if (!self) {
    delete plan;
    return nullptr;
  }
  CodecObject* c = reinterpret_cast<CodecObject*>(self);
  c->plan = plan;
  Py_XINCREF(memo);
  c->memo = memo;
  c->vectorcall = nullptr;  // set by the type's init below
  return self;
}

// codec(line) -> (type, object): one watch event ({"type": ..., "object": {...}})
PyObject* codec_vectorcall(PyObject* self, PyObject* const* args, size_t nargsf, PyObject* kwnames) {
  if (PyVectorcall_NARGS(nargsf) != 1 || (kwnames && PyTuple_GET_SIZE(kwnames))) {
    PyErr_SetString(PyExc_TypeError, "codec(line) takes exactly one argument");
    return nullptr;
  }
  PyObject* ev = codec_decode(reinterpret_cast<CodecObject*>(self), args[0]);
  if (!ev) return nullptr;
  PyObject* type = nullptr;
  PyObject* obj = nullptr;
  if (PyDict_CheckExact(ev)) {
    type = PyDict_GetItemString(ev, "type");   // borrowed
    obj = PyDict_GetItemString(ev, "object");  // borrowed
  }
  PyObject* t = (type != nullptr && PyObject_IsTrue(type) == 1) ? type : nullptr;
  PyObject* o = (obj != nullptr && PyObject_IsTrue(obj) == 1) ? obj : nullptr;
  PyObject* out = PyTuple_New(2);
  if (!out) {
    Py_DECREF(ev);
    return nullptr;
  }
  if (t) {
    Py_INCREF(t);
  } else {
    t = PyUnicode_FromStringAndSize("", 0);
  }
  if (o) {
    Py_INCREF(o);
  } else {
    o = PyDict_New();
  }
  PyTuple_SET_ITEM(out, 0, t);
  PyTuple_SET_ITEM(out, 1, o);
  Py_DECREF(ev);
  if (!t || !o) {
    Py_DECREF(out);
    return nullptr;
  }
  return out;
}

PyObject* codec_call(PyObject* self, PyObject* args, PyObject* kwds) {
  if (kwds && PyDict_GET_SIZE(kwds)) {
    PyErr_SetString(PyExc_TypeError, "codec(line) takes no keyword arguments");
    return nullptr;
  }
  return codec_vectorcall(self, &PyTuple_GET_ITEM(args, 0), static_cast<size_t>(PyTuple_GET_SIZE(args)), nullptr);
}

PyObject* codec_loads(PyObject* self, PyObject* arg) { return codec_decode(reinterpret_cast<CodecObject*>(self), arg); }

PyObject* codec_dumpb(PyObject* self, PyObject* o) {
  CodecObject* c = reinterpret_cast<CodecObject*>(self);
  Encoder e;
  e.plan = c->plan;
  MemoTable* m = codec_memo(c);
  e.memo = m;
  e.out.reserve(4096);
  if (!e.value(o, 0, 0)) return nullptr;
  if (m != nullptr) {
    for (const auto& r : e.recs) {
      const char* p = e.out.data() + r.start;
      const size_t n = r.end - r.start;
      m->store(p, n, span_hash(p, n), r.obj, true);
    }
  }
  return PyBytes_FromStringAndSize(e.out.data(), static_cast<Py_ssize_t>(e.out.size()));
}

PyMethodDef codec_methods[] = {
    {"loads", codec_loads, METH_O, "decode a JSON document with this codec's plan"},
    {"dumpb", codec_dumpb, METH_O, "encode compactly; remember the values written at memo paths"},
    {nullptr, nullptr, 0, nullptr}};

PyMemberDef codec_members[] = {
    {"memo", T_OBJECT, offsetof(CodecObject, memo), READONLY, "the shared Memo (or None)"},
    {nullptr, 0, 0, 0, nullptr}};

PyTypeObject CodecType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyObject* codec_new_vc(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  PyObject* self = codec_new(type, args, kwds);
  if (self) reinterpret_cast<CodecObject*>(self)->vectorcall = codec_vectorcall;
  return self;
}

PyMethodDef methods[] = {
    {"deepcopy", py_deepcopy, METH_O, "copy a JSON tree"},
    {"json_equal", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(py_json_equal)), METH_FASTCALL,
     "structural JSON equality"},
    {"create_merge_patch", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(py_merge_patch)),
     METH_FASTCALL, "RFC 7386 merge patch from old to new"},
    {"loads", py_loads, METH_O, "decode JSON (bytes, bytearray or str)"},
    {"dumpb", py_dumpb, METH_O, "compact JSON as UTF-8 bytes"},
    {"dumps", py_dumps, METH_O, "compact JSON as str"},
    {"dumpb_shared", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(py_dumpb_shared)),
     METH_FASTCALL, "dumpb of an immutable tree, reusing the bytes of subtrees cached by identity"},
    {"clear_key_cache", py_clear_key_cache, METH_NOARGS, "drop the interned-key cache"},
    {"pick", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(py_pick)), METH_FASTCALL,
     "pick(dict, keys) -> [dict[k] for k in keys]"},
    {"store_apply", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(py_store_apply)), METH_FASTCALL,
     "store_apply(store, derived, indices, spec, deleting, obj) -> (key, old) | None: an informer event's "
     "store/index bookkeeping"},
    {"kubeflow_summary", py_kubeflow_summary, METH_O,
     "kubeflow_summary(status) -> None | (finished, last_type, n_conditions, completion_time, terminal_ltt)"},
    {"set_gc_untrack", py_set_gc_untrack, METH_O,
     "set_gc_untrack(bool) -> previous: exempt decoded/copied containers from cyclic GC"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_fastjson", "Native JSON-tree helpers", -1, methods,
                      nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__fastjson(void) {
  MemoType.tp_name = "_fastjson.Memo";
  MemoType.tp_basicsize = sizeof(MemoObject);
  MemoType.tp_flags = Py_TPFLAGS_DEFAULT;
  MemoType.tp_doc = "Memo(slots=16384, max_slots=524288): bytes -> decoded object table shared by Codecs (grows to max_slots)";
  MemoType.tp_new = memo_new;
  MemoType.tp_dealloc = memo_dealloc;
  MemoType.tp_methods = memo_methods;
  CodecType.tp_name = "_fastjson.Codec";
  CodecType.tp_basicsize = sizeof(CodecObject);
  CodecType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_VECTORCALL;
  CodecType.tp_doc =
      "Codec(skip=(), memo_paths=(), memo=None, raw_paths=(), route_paths=None, route=None): JSON decode/encode "
      "with skipped, memoised, raw and routed paths; "
      "calling it decodes one watch event line into (type, object)";
  CodecType.tp_new = codec_new_vc;
  CodecType.tp_dealloc = codec_dealloc;
  CodecType.tp_methods = codec_methods;
  CodecType.tp_members = codec_members;
  CodecType.tp_call = codec_call;
  CodecType.tp_vectorcall_offset = offsetof(CodecObject, vectorcall);
  if (PyType_Ready(&MemoType) < 0 || PyType_Ready(&CodecType) < 0) return nullptr;
  if (!(s_metadata_key = PyUnicode_InternFromString("metadata")) ||
      !(s_namespace_key = PyUnicode_InternFromString("namespace")) ||
      !(s_name_key = PyUnicode_InternFromString("name")) || !(s_labels_key = PyUnicode_InternFromString("labels")) ||
      !(s_empty = PyUnicode_InternFromString("")))
    return nullptr;
  PyObject* m = PyModule_Create(&moddef);
  if (!m) return nullptr;
  Py_INCREF(&MemoType);
  Py_INCREF(&CodecType);
  if (PyModule_AddObject(m, "Memo", reinterpret_cast<PyObject*>(&MemoType)) < 0 ||
      PyModule_AddObject(m, "Codec", reinterpret_cast<PyObject*>(&CodecType)) < 0) {
    Py_DECREF(m);
    return nullptr;
  }
  return m;
}
