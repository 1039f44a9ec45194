// Native core of the controller's work queue (CPython extension `_workqueue`).
//
// controller-runtime's workers pull keys from client-go's rate-limited work queue
// (reference: MaxConcurrentReconciles workers, /root/reference/cmd/operator/start.go:215 and
// SURVEY 2.3 "controller parallelism"): a key is queued at most once, a key added while a
// worker holds it is parked ("dirty") and re-queued when the worker is done, and queue depth,
// adds, queue latency and work duration are metered.  Every Cron fire passes through the
// queue twice (its tick and its job's completion), so the bookkeeping runs here:
//
//   Core(depth_gauge, adds_counter, latency_histogram, work_histogram, empty)
//     add(item, priority=0)   dedupe (a more urgent add raises the priority; the stale heap
//                             entry is skipped later), park while processing, else push and
//                             wake one waiting future
//     pop()                   the most urgent queued item (FIFO within a priority), now in
//                             processing; `empty` when nothing is queued
//     done(item)              end of processing: observe work time, re-queue a parked item
//     add_waiter(fut) / remove_waiter(fut) / shutdown()
//     len(), processing(), idle(), started() (start times of items in flight), .adds, .gets,
//     .shut
//
// parallel/workqueue.py keeps the delaying (add_after/add_at, one clock timer for the queue)
// and rate-limiting layers in Python and its own pure-Python core as the fallback and the
// oracle of tests/test_workqueue_native.py.  Times come from the same clock as
// time.perf_counter() (CLOCK_MONOTONIC).  Single-threaded: the operator's loop thread.

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <time.h>

#include <algorithm>
#include <deque>
#include <vector>

namespace {

struct Entry {
  long long negp;
  unsigned long long seq;
  PyObject* item;  // strong reference held by the heap
};

// min-heap on (negp, seq): std heap functions build a max-heap, so "less" is reversed
struct EntryAfter {
  bool operator()(const Entry& a, const Entry& b) const {
    return a.negp != b.negp ? a.negp > b.negp : a.seq > b.seq;
  }
};

struct CoreObject {
  PyObject_HEAD
  std::vector<Entry>* heap;
  std::deque<PyObject*>* waiters;  // futures (strong references)
  PyObject* queued;                // dict item -> (negp, seq) of its live heap entry
  PyObject* processing;            // set
  PyObject* dirty;                 // dict item -> best priority requested while processing
  PyObject* added_at;              // dict item -> float
  PyObject* started_at;            // dict item -> float
  PyObject* depth_set;             // bound methods of the metric series
  PyObject* adds_inc;
  PyObject* latency_observe;
  PyObject* work_observe;
  PyObject* empty;                 // pop()'s "nothing queued" sentinel
  unsigned long long seq;
  long long adds;
  long long gets;
  char shut;
};

PyTypeObject CoreType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyObject *s_done, *s_set_result;

double now_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<double>(ts.tv_sec) + static_cast<double>(ts.tv_nsec) * 1e-9;
}

int call1(PyObject* fn, PyObject* arg) {
  PyObject* r = PyObject_CallOneArg(fn, arg);
  if (!r) return -1;
  Py_DECREF(r);
  return 0;
}

int call_float(PyObject* fn, double v) {
  PyObject* f = PyFloat_FromDouble(v);
  if (!f) return -1;
  const int rc = call1(fn, f);
  Py_DECREF(f);
  return rc;
}

int set_depth(CoreObject* c) { return call_float(c->depth_set, static_cast<double>(PyDict_GET_SIZE(c->queued))); }

// wake one waiter that is still pending (WorkQueue._push)
int wake_one(CoreObject* c) {
  while (!c->waiters->empty()) {
    PyObject* fut = c->waiters->front();
    c->waiters->pop_front();
    PyObject* d = PyObject_CallMethodNoArgs(fut, s_done);
    if (!d) {
      Py_DECREF(fut);
      return -1;
    }
    const int done = PyObject_IsTrue(d);
    Py_DECREF(d);
    if (done < 0) {
      Py_DECREF(fut);
      return -1;
    }
    if (!done) {
      PyObject* r = PyObject_CallMethodOneArg(fut, s_set_result, Py_None);
      Py_DECREF(fut);
      if (!r) return -1;
      Py_DECREF(r);
      return 0;
    }
    Py_DECREF(fut);
  }
  return 0;
}

int push(CoreObject* c, PyObject* item, long long priority) {
  const long long negp = -priority;
  const unsigned long long seq = c->seq++;
  PyObject* entry = Py_BuildValue("(LK)", negp, seq);
  if (!entry) return -1;
  const int r = PyDict_SetItem(c->queued, item, entry);
  Py_DECREF(entry);
  if (r < 0) return -1;
  Py_INCREF(item);
  c->heap->push_back(Entry{negp, seq, item});
  std::push_heap(c->heap->begin(), c->heap->end(), EntryAfter());
  PyObject* t = PyDict_GetItemWithError(c->added_at, item);
  if (!t) {
    if (PyErr_Occurred()) return -1;
    PyObject* f = PyFloat_FromDouble(now_s());
    if (!f) return -1;
    const int rr = PyDict_SetItem(c->added_at, item, f);
    Py_DECREF(f);
    if (rr < 0) return -1;
  }
  if (set_depth(c) < 0) return -1;
  return wake_one(c);
}

int count_add(CoreObject* c) {
  ++c->adds;
  PyObject* r = PyObject_CallNoArgs(c->adds_inc);
  if (!r) return -1;
  Py_DECREF(r);
  return 0;
}

PyObject* s_priority;

PyObject* core_add(PyObject* self, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
  CoreObject* c = reinterpret_cast<CoreObject*>(self);
  PyObject* prio_obj = nargs == 2 ? args[1] : nullptr;
  const Py_ssize_t nk = kwnames ? PyTuple_GET_SIZE(kwnames) : 0;
  for (Py_ssize_t i = 0; i < nk; ++i) {
    if (PyUnicode_Compare(PyTuple_GET_ITEM(kwnames, i), s_priority) != 0 || prio_obj) {
      PyErr_SetString(PyExc_TypeError, "add(item, priority=0)");
      return nullptr;
    }
    prio_obj = args[nargs + i];
  }
  if (nargs < 1 || nargs > 2) {
    PyErr_SetString(PyExc_TypeError, "add(item, priority=0)");
    return nullptr;
  }
  PyObject* item = args[0];
  long long priority = 0;
  if (prio_obj) {
    priority = PyLong_AsLongLong(prio_obj);
    if (priority == -1 && PyErr_Occurred()) return nullptr;
  }
  if (c->shut) Py_RETURN_NONE;
  PyObject* cur = PyDict_GetItemWithError(c->queued, item);
  if (cur) {
    const long long negp = PyLong_AsLongLong(PyTuple_GET_ITEM(cur, 0));
    if (-negp < priority && push(c, item, priority) < 0) return nullptr;  // raise: a fresher entry
    Py_RETURN_NONE;  // already queued: neither queued nor counted again
  }
  if (PyErr_Occurred()) return nullptr;
  const int busy = PySet_Contains(c->processing, item);
  if (busy < 0) return nullptr;
  if (busy) {
    PyObject* prev = PyDict_GetItemWithError(c->dirty, item);
    if (!prev && PyErr_Occurred()) return nullptr;
    long long best = priority;
    if (prev) {
      const long long p = PyLong_AsLongLong(prev);
      if (p == -1 && PyErr_Occurred()) return nullptr;
      best = std::max(p, priority);
    } else if (count_add(c) < 0) {
      return nullptr;
    }
    PyObject* v = PyLong_FromLongLong(best);
    if (!v) return nullptr;
    const int r = PyDict_SetItem(c->dirty, item, v);
    Py_DECREF(v);
    if (r < 0) return nullptr;
    Py_RETURN_NONE;
  }
  if (count_add(c) < 0 || push(c, item, priority) < 0) return nullptr;
  Py_RETURN_NONE;
}

PyObject* core_pop(PyObject* self, PyObject*) {
  CoreObject* c = reinterpret_cast<CoreObject*>(self);
  auto& h = *c->heap;
  while (!h.empty()) {
    std::pop_heap(h.begin(), h.end(), EntryAfter());
    Entry e = h.back();
    h.pop_back();
    PyObject* item = e.item;  // the heap's reference, now ours
    PyObject* live = PyDict_GetItemWithError(c->queued, item);
    bool stale = true;
    if (live) {
      stale = PyLong_AsLongLong(PyTuple_GET_ITEM(live, 0)) != e.negp ||
              PyLong_AsUnsignedLongLong(PyTuple_GET_ITEM(live, 1)) != e.seq;
    } else if (PyErr_Occurred()) {
      Py_DECREF(item);
      return nullptr;
    }
    if (stale) {
      Py_DECREF(item);
      continue;
    }
    const double now = now_s();
    double t_add = now;
    PyObject* ta = PyDict_GetItemWithError(c->added_at, item);
    if (ta) {
      t_add = PyFloat_AsDouble(ta);
      if (PyDict_DelItem(c->added_at, item) < 0) {
        Py_DECREF(item);
        return nullptr;
      }
    }
    PyObject* st = PyErr_Occurred() ? nullptr : PyFloat_FromDouble(now);
    if (!st || PyDict_DelItem(c->queued, item) < 0 || PySet_Add(c->processing, item) < 0 ||
        call_float(c->latency_observe, now - t_add) < 0 || PyDict_SetItem(c->started_at, item, st) < 0 ||
        set_depth(c) < 0) {
      Py_XDECREF(st);
      Py_DECREF(item);
      return nullptr;
    }
    Py_DECREF(st);
    ++c->gets;
    return item;
  }
  Py_INCREF(c->empty);
  return c->empty;
}

PyObject* core_done(PyObject* self, PyObject* item) {
  CoreObject* c = reinterpret_cast<CoreObject*>(self);
  if (PySet_Discard(c->processing, item) < 0) return nullptr;
  PyObject* t0 = PyDict_GetItemWithError(c->started_at, item);
  if (t0) {
    const double start = PyFloat_AsDouble(t0);
    if (PyDict_DelItem(c->started_at, item) < 0 || call_float(c->work_observe, now_s() - start) < 0) return nullptr;
  } else if (PyErr_Occurred()) {
    return nullptr;
  }
  PyObject* prio = PyDict_GetItemWithError(c->dirty, item);
  if (prio) {
    const long long p = PyLong_AsLongLong(prio);
    if (p == -1 && PyErr_Occurred()) return nullptr;
    if (PyDict_DelItem(c->dirty, item) < 0 || push(c, item, p) < 0) return nullptr;
  } else if (PyErr_Occurred()) {
    return nullptr;
  }
  Py_RETURN_NONE;
}

PyObject* core_add_waiter(PyObject* self, PyObject* fut) {
  Py_INCREF(fut);
  reinterpret_cast<CoreObject*>(self)->waiters->push_back(fut);
  Py_RETURN_NONE;
}

PyObject* core_remove_waiter(PyObject* self, PyObject* fut) {
  auto& w = *reinterpret_cast<CoreObject*>(self)->waiters;
  auto it = std::find(w.begin(), w.end(), fut);
  if (it != w.end()) {
    w.erase(it);
    Py_DECREF(fut);
  }
  Py_RETURN_NONE;
}

PyObject* core_shutdown(PyObject* self, PyObject*) {
  CoreObject* c = reinterpret_cast<CoreObject*>(self);
  c->shut = 1;
  // every waiter resolves (it then sees the queue drained and shut down)
  while (!c->waiters->empty()) {
    PyObject* fut = c->waiters->front();
    c->waiters->pop_front();
    PyObject* d = PyObject_CallMethodNoArgs(fut, s_done);
    int done = d ? PyObject_IsTrue(d) : -1;
    Py_XDECREF(d);
    if (done == 0) {
      PyObject* r = PyObject_CallMethodOneArg(fut, s_set_result, Py_None);
      if (!r) done = -1;
      Py_XDECREF(r);
    }
    Py_DECREF(fut);
    if (done < 0) return nullptr;
  }
  Py_RETURN_NONE;
}

Py_ssize_t core_len(PyObject* self) { return PyDict_GET_SIZE(reinterpret_cast<CoreObject*>(self)->queued); }

PyObject* core_processing(PyObject* self, PyObject*) {
  return PyLong_FromSsize_t(PySet_GET_SIZE(reinterpret_cast<CoreObject*>(self)->processing));
}

PyObject* core_idle(PyObject* self, PyObject*) {
  CoreObject* c = reinterpret_cast<CoreObject*>(self);
  return PyBool_FromLong(PyDict_GET_SIZE(c->queued) == 0 && PySet_GET_SIZE(c->processing) == 0 &&
                         PyDict_GET_SIZE(c->dirty) == 0);
}

PyObject* core_started(PyObject* self, PyObject*) {
  return PyDict_Values(reinterpret_cast<CoreObject*>(self)->started_at);
}

PyObject* core_new(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  static const char* kw[] = {"depth", "adds", "latency", "work", "empty", nullptr};
  PyObject *depth, *adds, *latency, *work, *empty;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "OOOOO", const_cast<char**>(kw), &depth, &adds, &latency, &work,
                                   &empty))
    return nullptr;
  CoreObject* c = reinterpret_cast<CoreObject*>(type->tp_alloc(type, 0));
  if (!c) return nullptr;
  c->heap = new std::vector<Entry>();
  c->waiters = new std::deque<PyObject*>();
  c->queued = PyDict_New();
  c->processing = PySet_New(nullptr);
  c->dirty = PyDict_New();
  c->added_at = PyDict_New();
  c->started_at = PyDict_New();
  c->depth_set = PyObject_GetAttrString(depth, "set");
  c->adds_inc = PyObject_GetAttrString(adds, "inc");
  c->latency_observe = PyObject_GetAttrString(latency, "observe");
  c->work_observe = PyObject_GetAttrString(work, "observe");
  Py_INCREF(empty);
  c->empty = empty;
  if (!c->queued || !c->processing || !c->dirty || !c->added_at || !c->started_at || !c->depth_set || !c->adds_inc ||
      !c->latency_observe || !c->work_observe) {
    Py_DECREF(c);
    return nullptr;
  }
  return reinterpret_cast<PyObject*>(c);
}

int core_traverse(CoreObject* c, visitproc visit, void* arg) {
  if (c->heap)
    for (auto& e : *c->heap) Py_VISIT(e.item);
  if (c->waiters)
    for (PyObject* f : *c->waiters) Py_VISIT(f);
  Py_VISIT(c->queued);
  Py_VISIT(c->processing);
  Py_VISIT(c->dirty);
  Py_VISIT(c->added_at);
  Py_VISIT(c->started_at);
  Py_VISIT(c->depth_set);
  Py_VISIT(c->adds_inc);
  Py_VISIT(c->latency_observe);
  Py_VISIT(c->work_observe);
  Py_VISIT(c->empty);
  return 0;
}

int core_clear(CoreObject* c) {
  if (c->heap) {
    std::vector<Entry> h;
    h.swap(*c->heap);
    for (auto& e : h) Py_DECREF(e.item);
  }
  if (c->waiters) {
    std::deque<PyObject*> w;
    w.swap(*c->waiters);
    for (PyObject* f : w) Py_DECREF(f);
  }
  Py_CLEAR(c->queued);
  Py_CLEAR(c->processing);
  Py_CLEAR(c->dirty);
  Py_CLEAR(c->added_at);
  Py_CLEAR(c->started_at);
  Py_CLEAR(c->depth_set);
  Py_CLEAR(c->adds_inc);
  Py_CLEAR(c->latency_observe);
  Py_CLEAR(c->work_observe);
  Py_CLEAR(c->empty);
  return 0;
}

void core_dealloc(CoreObject* c) {
  PyObject_GC_UnTrack(c);
  core_clear(c);
  delete c->heap;
  delete c->waiters;
  Py_TYPE(c)->tp_free(reinterpret_cast<PyObject*>(c));
}

PyMethodDef core_methods[] = {
    {"add", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(core_add)), METH_FASTCALL | METH_KEYWORDS,
     "add(item, priority=0)"},
    {"pop", core_pop, METH_NOARGS, "the next item (now processing), or the empty sentinel"},
    {"done", core_done, METH_O, "done(item): end of processing; a parked item is re-queued"},
    {"add_waiter", core_add_waiter, METH_O, "add_waiter(future): resolved by the next push or shutdown"},
    {"remove_waiter", core_remove_waiter, METH_O, "remove_waiter(future)"},
    {"shutdown", core_shutdown, METH_NOARGS, "refuse further adds; resolve every waiter"},
    {"processing", core_processing, METH_NOARGS, "items in flight"},
    {"idle", core_idle, METH_NOARGS, "nothing queued, parked or in flight"},
    {"started", core_started, METH_NOARGS, "start times of the items in flight"},
    {nullptr, nullptr, 0, nullptr}};

PyMemberDef core_members[] = {{"adds", T_LONGLONG, offsetof(CoreObject, adds), READONLY, nullptr},
                              {"gets", T_LONGLONG, offsetof(CoreObject, gets), READONLY, nullptr},
                              {"shut", T_BOOL, offsetof(CoreObject, shut), READONLY, nullptr},
                              {nullptr, 0, 0, 0, nullptr}};

PySequenceMethods core_seq = {};

PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_workqueue", "Native work-queue core (dedupe, parking, priorities).",
                      -1, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__workqueue(void) {
  if (!(s_done = PyUnicode_InternFromString("done")) || !(s_set_result = PyUnicode_InternFromString("set_result")) ||
      !(s_priority = PyUnicode_InternFromString("priority")))
    return nullptr;
  core_seq.sq_length = core_len;
  CoreType.tp_name = "_workqueue.Core";
  CoreType.tp_basicsize = sizeof(CoreObject);
  CoreType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  CoreType.tp_doc = "Core(depth, adds, latency, work, empty): the work queue's bookkeeping";
  CoreType.tp_new = core_new;
  CoreType.tp_dealloc = reinterpret_cast<destructor>(core_dealloc);
  CoreType.tp_traverse = reinterpret_cast<traverseproc>(core_traverse);
  CoreType.tp_clear = reinterpret_cast<inquiry>(core_clear);
  CoreType.tp_methods = core_methods;
  CoreType.tp_members = core_members;
  CoreType.tp_as_sequence = &core_seq;
  if (PyType_Ready(&CoreType) < 0) return nullptr;
  PyObject* m = PyModule_Create(&moddef);
  if (!m) return nullptr;
  Py_INCREF(&CoreType);
  if (PyModule_AddObject(m, "Core", reinterpret_cast<PyObject*>(&CoreType)) < 0) {
    Py_DECREF(&CoreType);
    Py_DECREF(m);
    return nullptr;
  }
  return m;
}
