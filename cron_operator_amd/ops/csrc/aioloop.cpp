// Native core of the operator's asyncio event loop (CPython extension `_aioloop`).
//
// The operator is one asyncio process (reference: controller-runtime's manager runs informers
// and 10 reconcile workers as goroutines on the Go scheduler -- /root/reference/cmd/operator/
// start.go:156-209).  Every API response, watch batch and work-queue hand-off wakes a
// task, and CPython 3.10 runs that machinery in Python: `call_soon` builds an `events.Handle`
// (Python __init__), `_run_once` polls the selector through `selectors.EpollSelector.select`,
// dispatches readiness through `_process_events`, and runs each handle through `Handle._run`.
// Counted per fire at 1000 Crons (scripts/opcount.py --bench) that was ~1500 bytecodes, 11.6%
// of the operator's Python work and its largest single layer after the reconciler.
//
// `LoopCore` implements exactly those hot methods natively and is mixed in *before*
// `asyncio.SelectorEventLoop` (runtime/aioloop.py: `class NativeEventLoop(LoopCore,
// SelectorEventLoop)`), so everything else -- run_forever, timers (call_at/call_later and their
// TimerHandles), add_reader/remove_reader, transports, subprocesses, signals, executors,
// shutdown -- stays asyncio's own code working on the same `_ready` deque, `_scheduled` heap and
// selector:
//
//   * `call_soon(cb, *args, context=None)` -> a native `Handle` (same attributes and methods as
//     `events.Handle`: `cancel()`, `cancelled()`, `_run()`, `_callback`, `_args`, `_context`,
//     `_cancelled`) appended to `_ready`;
//   * `_run_once()` -- the same steps in the same order as BaseEventLoop._run_once: drop cancelled
//     timers (or rebuild the heap when more than half of >100 are cancelled), compute the poll
//     timeout, `epoll_wait` on the EpollSelector's own epoll fd (GIL released while blocking),
//     map each fd through the selector's `_fd_to_key` with `selectors`' event-mask rules,
//     queue reader/writer handles like `_process_events` (a cancelled one is removed), move due
//     timers to `_ready`, then run the `len(_ready)` handles present -- native ones directly,
//     asyncio's own (`call_soon_threadsafe`, readers, timers) through their `_run()`;
//   * a callback's exception goes to `loop.call_exception_handler` with the same context keys
//     ('message', 'exception', 'handle') and message format as `Handle._run`; SystemExit and
//     KeyboardInterrupt propagate.
//
// Debug mode (`loop.set_debug(True)`, PYTHONASYNCIODEBUG) and any selector other than
// `selectors.EpollSelector` take asyncio's Python methods unchanged.  The Python loop is the
// oracle of tests/test_aioloop.py (execution-order differential); CRON_OPERATOR_NATIVE_LOOP=python
// turns the native loop off.

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <errno.h>
#include <sys/epoll.h>

#include <climits>
#include <cmath>
#include <vector>

namespace {

// selectors.EVENT_READ / EVENT_WRITE
constexpr long kEventRead = 1;
constexpr long kEventWrite = 2;
// base_events constants
constexpr Py_ssize_t kMinScheduledTimerHandles = 100;
constexpr double kMinCancelledTimerHandlesFraction = 0.5;
constexpr double kMaximumSelectTimeout = 24 * 3600;

PyObject *s_ready, *s_scheduled, *s_stopping, *s_selector, *s_closed, *s_debug, *s_timer_cancelled_count,
    *s_cancelled, *s_when, *s_time, *s_clock_resolution, *s_append, *s_popleft, *s_run, *s_fd_to_key,
    *s_fileno, *s_remove_reader, *s_remove_writer, *s_call_exception_handler, *s_message, *s_exception,
    *s_handle, *s_context_kw, *s_fileobj, *s_events, *s_data;

// set by configure(): selectors.EpollSelector, heapq.heappop, heapq.heapify,
// format_helpers._format_callback_source, BaseEventLoop.call_soon, BaseEventLoop._run_once
PyObject *g_epoll_selector, *g_heappop, *g_heapify, *g_format_cb, *g_py_call_soon, *g_py_run_once;

// ---------------------------------------------------------------------------------------- Handle

struct HandleObject {
  PyObject_HEAD
  PyObject* callback;
  PyObject* args;  // tuple (None once cancelled, like events.Handle)
  PyObject* loop;
  PyObject* context;
  PyObject* repr;
  PyObject* source_traceback;
  PyObject* weakreflist;
  char cancelled;
};

PyTypeObject HandleType = {PyVarObject_HEAD_INIT(nullptr, 0)};

int handle_traverse(HandleObject* h, visitproc visit, void* arg) {
  Py_VISIT(h->callback);
  Py_VISIT(h->args);
  Py_VISIT(h->loop);
  Py_VISIT(h->context);
  Py_VISIT(h->repr);
  Py_VISIT(h->source_traceback);
  return 0;
}

int handle_clear(HandleObject* h) {
  Py_CLEAR(h->callback);
  Py_CLEAR(h->args);
  Py_CLEAR(h->loop);
  Py_CLEAR(h->context);
  Py_CLEAR(h->repr);
  Py_CLEAR(h->source_traceback);
  return 0;
}

void handle_dealloc(HandleObject* h) {
  PyObject_GC_UnTrack(h);
  if (h->weakreflist) PyObject_ClearWeakRefs(reinterpret_cast<PyObject*>(h));
  handle_clear(h);
  Py_TYPE(h)->tp_free(reinterpret_cast<PyObject*>(h));
}

// steals nothing; args must be a tuple, context a contextvars.Context
HandleObject* handle_new(PyObject* callback, PyObject* args, PyObject* loop, PyObject* context) {
  HandleObject* h = PyObject_GC_New(HandleObject, &HandleType);
  if (!h) return nullptr;
  Py_INCREF(callback);
  h->callback = callback;
  Py_INCREF(args);
  h->args = args;
  Py_INCREF(loop);
  h->loop = loop;
  Py_INCREF(context);
  h->context = context;
  Py_INCREF(Py_None);
  h->repr = Py_None;
  Py_INCREF(Py_None);
  h->source_traceback = Py_None;
  h->weakreflist = nullptr;
  h->cancelled = 0;
  PyObject_GC_Track(h);
  return h;
}

// "Exception in callback <source>" as events.Handle._run formats it
PyObject* callback_message(PyObject* cb, PyObject* args) {
  PyObject* src = g_format_cb ? PyObject_CallFunctionObjArgs(g_format_cb, cb, args, nullptr) : nullptr;
  if (!src) {
    PyErr_Clear();
    src = PyObject_Repr(cb);
    if (!src) {
      PyErr_Clear();
      return PyUnicode_FromString("Exception in callback <unprintable>");
    }
  }
  PyObject* msg = PyUnicode_FromFormat("Exception in callback %U", src);
  Py_DECREF(src);
  return msg;
}

// Handle._run: 0 done (a callback exception went to the loop's exception handler), -1 an error
// to propagate (SystemExit, KeyboardInterrupt, or a failing exception handler)
int handle_run(HandleObject* h) {
  // strong references for the duration: the callback may cancel its own handle
  PyObject* cb = h->callback;
  PyObject* args = h->args;
  PyObject* ctx = h->context;
  if (!cb || cb == Py_None || !args || !PyTuple_Check(args) || !ctx) {
    PyErr_SetString(PyExc_RuntimeError, "native Handle run without a callback");
    return -1;
  }
  Py_INCREF(cb);
  Py_INCREF(args);
  Py_INCREF(ctx);
  PyObject* r = nullptr;
  if (PyContext_Enter(ctx) == 0) {
    r = PyObject_Vectorcall(cb, &PyTuple_GET_ITEM(args, 0), PyTuple_GET_SIZE(args), nullptr);
    if (PyContext_Exit(ctx) < 0) Py_CLEAR(r);
  }
  int rc = 0;
  if (r) {
    Py_DECREF(r);
  } else if (PyErr_ExceptionMatches(PyExc_SystemExit) || PyErr_ExceptionMatches(PyExc_KeyboardInterrupt)) {
    rc = -1;
  } else {
    PyObject *et, *ev, *tb;
    PyErr_Fetch(&et, &ev, &tb);
    PyErr_NormalizeException(&et, &ev, &tb);
    if (tb && ev) PyException_SetTraceback(ev, tb);
    PyObject* msg = callback_message(cb, args);
    PyObject* d = msg ? PyDict_New() : nullptr;
    if (d && PyDict_SetItem(d, s_message, msg) == 0 && PyDict_SetItem(d, s_exception, ev ? ev : Py_None) == 0 &&
        PyDict_SetItem(d, s_handle, reinterpret_cast<PyObject*>(h)) == 0) {
      PyObject* loop = h->loop;
      Py_INCREF(loop);
      PyObject* res = PyObject_CallMethodOneArg(loop, s_call_exception_handler, d);
      Py_DECREF(loop);
      if (res)
        Py_DECREF(res);
      else
        rc = -1;
    } else {
      rc = -1;
    }
    Py_XDECREF(d);
    Py_XDECREF(msg);
    Py_XDECREF(et);
    Py_XDECREF(ev);
    Py_XDECREF(tb);
  }
  Py_DECREF(cb);
  Py_DECREF(args);
  Py_DECREF(ctx);
  return rc;
}

PyObject* handle_py_run(PyObject* self, PyObject*) {
  if (handle_run(reinterpret_cast<HandleObject*>(self)) < 0) return nullptr;
  Py_RETURN_NONE;
}

PyObject* handle_cancel(PyObject* self, PyObject*) {
  HandleObject* h = reinterpret_cast<HandleObject*>(self);
  if (!h->cancelled) {
    h->cancelled = 1;
    PyObject* cb = h->callback;
    PyObject* args = h->args;
    Py_INCREF(Py_None);
    h->callback = Py_None;
    Py_INCREF(Py_None);
    h->args = Py_None;
    Py_XDECREF(cb);
    Py_XDECREF(args);
  }
  Py_RETURN_NONE;
}

PyObject* handle_cancelled(PyObject* self, PyObject*) {
  return PyBool_FromLong(reinterpret_cast<HandleObject*>(self)->cancelled);
}

PyObject* handle_repr(PyObject* self) {
  HandleObject* h = reinterpret_cast<HandleObject*>(self);
  if (h->repr && h->repr != Py_None) {
    Py_INCREF(h->repr);
    return h->repr;
  }
  if (h->cancelled) return PyUnicode_FromString("<Handle cancelled>");
  PyObject* src = g_format_cb ? PyObject_CallFunctionObjArgs(g_format_cb, h->callback, h->args, nullptr) : nullptr;
  if (!src) return nullptr;
  PyObject* r = PyUnicode_FromFormat("<Handle %U>", src);
  Py_DECREF(src);
  return r;
}

PyMethodDef handle_methods[] = {
    {"cancel", handle_cancel, METH_NOARGS, "Cancel the call (the callback and its arguments are dropped)."},
    {"cancelled", handle_cancelled, METH_NOARGS, "True once cancel() was called."},
    {"_run", handle_py_run, METH_NOARGS, "Run the callback in its context (events.Handle._run)."},
    {nullptr, nullptr, 0, nullptr}};

PyMemberDef handle_members[] = {
    {"_callback", T_OBJECT, offsetof(HandleObject, callback), 0, nullptr},
    {"_args", T_OBJECT, offsetof(HandleObject, args), 0, nullptr},
    {"_loop", T_OBJECT, offsetof(HandleObject, loop), READONLY, nullptr},
    {"_context", T_OBJECT, offsetof(HandleObject, context), READONLY, nullptr},
    {"_repr", T_OBJECT, offsetof(HandleObject, repr), 0, nullptr},
    {"_source_traceback", T_OBJECT, offsetof(HandleObject, source_traceback), 0, nullptr},
    {"_cancelled", T_BOOL, offsetof(HandleObject, cancelled), READONLY, nullptr},
    {nullptr, 0, 0, 0, nullptr}};

// -------------------------------------------------------------------------------------- LoopCore

struct LoopCore {
  PyObject_HEAD
  PyObject* ready;          // the loop's `_ready` deque (never replaced by asyncio)
  PyObject* ready_append;   // its bound append / popleft
  PyObject* ready_popleft;
  PyObject* fd_to_key;      // the EpollSelector's `_fd_to_key` dict
  PyObject* selector;       // the selector the cache above belongs to
  int epfd;                 // its epoll fd
  char inited;
  char native_select;       // the selector is an EpollSelector
};

int loop_traverse(LoopCore* s, visitproc visit, void* arg) {
  Py_VISIT(s->ready);
  Py_VISIT(s->ready_append);
  Py_VISIT(s->ready_popleft);
  Py_VISIT(s->fd_to_key);
  Py_VISIT(s->selector);
  return 0;
}

int loop_clear(LoopCore* s) {
  Py_CLEAR(s->ready);
  Py_CLEAR(s->ready_append);
  Py_CLEAR(s->ready_popleft);
  Py_CLEAR(s->fd_to_key);
  Py_CLEAR(s->selector);
  s->inited = 0;
  return 0;
}

void loop_dealloc(LoopCore* s) {
  PyObject_GC_UnTrack(s);
  loop_clear(s);
  Py_TYPE(s)->tp_free(reinterpret_cast<PyObject*>(s));
}

// the `_ready` deque and its bound methods, cached on first use
bool ensure_ready(LoopCore* s) {
  if (s->ready) return true;
  PyObject* self = reinterpret_cast<PyObject*>(s);
  PyObject* ready = PyObject_GetAttr(self, s_ready);
  if (!ready) return false;
  PyObject* app = PyObject_GetAttr(ready, s_append);
  PyObject* pop = app ? PyObject_GetAttr(ready, s_popleft) : nullptr;
  if (!pop) {
    Py_XDECREF(app);
    Py_DECREF(ready);
    return false;
  }
  s->ready = ready;
  s->ready_append = app;
  s->ready_popleft = pop;
  return true;
}

// the selector cache: re-checked against `self._selector` on every iteration (cheap identity test)
bool ensure_selector(LoopCore* s, PyObject* sel) {
  if (s->inited && s->selector == sel) return true;
  Py_CLEAR(s->fd_to_key);
  Py_CLEAR(s->selector);
  s->native_select = 0;
  s->epfd = -1;
  s->inited = 1;
  if (!g_epoll_selector || Py_TYPE(sel) != reinterpret_cast<PyTypeObject*>(g_epoll_selector)) {
    Py_INCREF(sel);
    s->selector = sel;
    return true;
  }
  PyObject* fdmap = PyObject_GetAttr(sel, s_fd_to_key);
  if (!fdmap) return false;
  PyObject* fdobj = PyObject_CallMethodNoArgs(sel, s_fileno);
  if (!fdobj) {
    Py_DECREF(fdmap);
    return false;
  }
  const long fd = PyLong_AsLong(fdobj);
  Py_DECREF(fdobj);
  if (fd == -1 && PyErr_Occurred()) {
    Py_DECREF(fdmap);
    return false;
  }
  if (!PyDict_CheckExact(fdmap) || fd < 0) {
    Py_DECREF(fdmap);
    Py_INCREF(sel);
    s->selector = sel;
    return true;
  }
  s->fd_to_key = fdmap;
  Py_INCREF(sel);
  s->selector = sel;
  s->epfd = static_cast<int>(fd);
  s->native_select = 1;
  return true;
}

// truthiness of an attribute; -1 on error
int attr_true(PyObject* o, PyObject* name) {
  PyObject* v = PyObject_GetAttr(o, name);
  if (!v) return -1;
  const int t = PyObject_IsTrue(v);
  Py_DECREF(v);
  return t;
}

// a handle's `_cancelled`: the field for native handles, the attribute otherwise
int handle_is_cancelled(PyObject* h) {
  if (Py_TYPE(h) == &HandleType) return reinterpret_cast<HandleObject*>(h)->cancelled;
  return attr_true(h, s_cancelled);
}

int call_one(PyObject* fn, PyObject* arg) {
  PyObject* r = PyObject_CallOneArg(fn, arg);
  if (!r) return -1;
  Py_DECREF(r);
  return 0;
}

PyObject* loop_call_soon(PyObject* self, PyObject* const* args, Py_ssize_t nargs, PyObject* kwnames) {
  LoopCore* s = reinterpret_cast<LoopCore*>(self);
  PyObject* context = nullptr;
  if (kwnames) {
    const Py_ssize_t nk = PyTuple_GET_SIZE(kwnames);
    for (Py_ssize_t i = 0; i < nk; ++i) {
      PyObject* k = PyTuple_GET_ITEM(kwnames, i);
      if (PyUnicode_Compare(k, s_context_kw) != 0) {
        PyErr_Format(PyExc_TypeError, "call_soon() got an unexpected keyword argument '%U'", k);
        return nullptr;
      }
      context = args[nargs + i];
    }
  }
  if (nargs < 1) {
    PyErr_SetString(PyExc_TypeError, "call_soon() missing 1 required positional argument: 'callback'");
    return nullptr;
  }
  const int closed = attr_true(self, s_closed);
  if (closed < 0) return nullptr;
  if (closed) {
    PyErr_SetString(PyExc_RuntimeError, "Event loop is closed");
    return nullptr;
  }
  const int debug = attr_true(self, s_debug);
  if (debug < 0) return nullptr;
  if (debug) {  // asyncio's own checks and source tracebacks
    std::vector<PyObject*> full(nargs + 1 + (kwnames ? PyTuple_GET_SIZE(kwnames) : 0));
    full[0] = self;
    for (size_t i = 1; i < full.size(); ++i) full[i] = args[i - 1];
    return PyObject_Vectorcall(g_py_call_soon, full.data(), nargs + 1, kwnames);
  }
  if (!ensure_ready(s)) return nullptr;
  PyObject* cargs = PyTuple_New(nargs - 1);
  if (!cargs) return nullptr;
  for (Py_ssize_t i = 1; i < nargs; ++i) {
    Py_INCREF(args[i]);
    PyTuple_SET_ITEM(cargs, i - 1, args[i]);
  }
  PyObject* ctx;
  if (!context || context == Py_None) {
    ctx = PyContext_CopyCurrent();
  } else if (!PyContext_CheckExact(context)) {
    Py_DECREF(cargs);
    PyErr_SetString(PyExc_TypeError, "call_soon(): context must be a contextvars.Context");
    return nullptr;
  } else {
    Py_INCREF(context);
    ctx = context;
  }
  if (!ctx) {
    Py_DECREF(cargs);
    return nullptr;
  }
  HandleObject* h = handle_new(args[0], cargs, self, ctx);
  Py_DECREF(cargs);
  Py_DECREF(ctx);
  if (!h) return nullptr;
  if (call_one(s->ready_append, reinterpret_cast<PyObject*>(h)) < 0) {
    Py_DECREF(h);
    return nullptr;
  }
  return reinterpret_cast<PyObject*>(h);
}

// self._scheduled: drop cancelled timers like BaseEventLoop._run_once (new reference)
PyObject* prune_scheduled(PyObject* self) {
  PyObject* sched = PyObject_GetAttr(self, s_scheduled);
  if (!sched) return nullptr;
  if (!PyList_CheckExact(sched)) {
    Py_DECREF(sched);
    PyErr_SetString(PyExc_TypeError, "loop._scheduled is not a list");
    return nullptr;
  }
  const Py_ssize_t n = PyList_GET_SIZE(sched);
  if (n == 0) return sched;
  PyObject* tcc_obj = PyObject_GetAttr(self, s_timer_cancelled_count);
  if (!tcc_obj) {
    Py_DECREF(sched);
    return nullptr;
  }
  long long tcc = PyLong_AsLongLong(tcc_obj);
  Py_DECREF(tcc_obj);
  if (tcc == -1 && PyErr_Occurred()) {
    Py_DECREF(sched);
    return nullptr;
  }
  if (n > kMinScheduledTimerHandles && static_cast<double>(tcc) / n > kMinCancelledTimerHandlesFraction) {
    PyObject* fresh = PyList_New(0);
    if (!fresh) {
      Py_DECREF(sched);
      return nullptr;
    }
    for (Py_ssize_t i = 0; i < PyList_GET_SIZE(sched); ++i) {
      PyObject* h = PyList_GET_ITEM(sched, i);
      const int c = handle_is_cancelled(h);
      if (c < 0 || (c ? PyObject_SetAttrString(h, "_scheduled", Py_False) : PyList_Append(fresh, h)) < 0) {
        Py_DECREF(fresh);
        Py_DECREF(sched);
        return nullptr;
      }
    }
    Py_DECREF(sched);
    PyObject* zero = PyLong_FromLong(0);
    if (!zero || call_one(g_heapify, fresh) < 0 || PyObject_SetAttr(self, s_scheduled, fresh) < 0 ||
        PyObject_SetAttr(self, s_timer_cancelled_count, zero) < 0) {
      Py_XDECREF(zero);
      Py_DECREF(fresh);
      return nullptr;
    }
    Py_DECREF(zero);
    return fresh;
  }
  bool changed = false;
  while (PyList_GET_SIZE(sched) > 0) {
    const int c = handle_is_cancelled(PyList_GET_ITEM(sched, 0));
    if (c < 0) goto fail;
    if (!c) break;
    --tcc;
    changed = true;
    {
      PyObject* h = PyObject_CallOneArg(g_heappop, sched);
      if (!h) goto fail;
      const int r = PyObject_SetAttrString(h, "_scheduled", Py_False);
      Py_DECREF(h);
      if (r < 0) goto fail;
    }
  }
  if (changed) {
    PyObject* v = PyLong_FromLongLong(tcc);
    if (!v || PyObject_SetAttr(self, s_timer_cancelled_count, v) < 0) {
      Py_XDECREF(v);
      goto fail;
    }
    Py_DECREF(v);
  }
  return sched;
fail:
  Py_DECREF(sched);
  return nullptr;
}

double call_time(PyObject* self) {
  PyObject* t = PyObject_CallMethodNoArgs(self, s_time);
  if (!t) return NAN;
  const double v = PyFloat_AsDouble(t);
  Py_DECREF(t);
  return v;
}

// _process_events for one (key, mask): queue the reader/writer handle or drop a cancelled one
int process_key(LoopCore* s, PyObject* self, PyObject* key, long mask) {
  PyObject *fileobj, *data;
  if (PyTuple_CheckExact(key) || (PyTuple_Check(key) && PyTuple_GET_SIZE(key) == 4)) {
    fileobj = PyTuple_GET_ITEM(key, 0);  // SelectorKey(fileobj, fd, events, data)
    data = PyTuple_GET_ITEM(key, 3);
    Py_INCREF(fileobj);
    Py_INCREF(data);
  } else {
    fileobj = PyObject_GetAttr(key, s_fileobj);
    data = fileobj ? PyObject_GetAttr(key, s_data) : nullptr;
    if (!data) {
      Py_XDECREF(fileobj);
      return -1;
    }
  }
  int rc = 0;
  if (!PyTuple_Check(data) || PyTuple_GET_SIZE(data) != 2) {
    PyErr_SetString(PyExc_TypeError, "selector key data is not a (reader, writer) pair");
    rc = -1;
  } else {
    for (int side = 0; side < 2 && rc == 0; ++side) {
      if (!(mask & (side == 0 ? kEventRead : kEventWrite))) continue;
      PyObject* h = PyTuple_GET_ITEM(data, side);
      if (h == Py_None) continue;
      const int c = handle_is_cancelled(h);
      if (c < 0) {
        rc = -1;
      } else if (c) {
        PyObject* r = PyObject_CallMethodOneArg(self, side == 0 ? s_remove_reader : s_remove_writer, fileobj);
        if (!r) rc = -1;
        Py_XDECREF(r);
      } else {
        rc = call_one(s->ready_append, h);
      }
    }
  }
  Py_DECREF(fileobj);
  Py_DECREF(data);
  return rc;
}

// selector.select(timeout) + _process_events on the EpollSelector's epoll fd.  timeout < 0: block.
int poll_native(LoopCore* s, PyObject* self, double timeout) {
  int ms;
  if (timeout < 0)
    ms = -1;
  else if (timeout <= 0)
    ms = 0;
  else
    ms = static_cast<int>(std::min(std::ceil(timeout * 1e3), static_cast<double>(INT_MAX)));
  Py_ssize_t maxev = PyDict_GET_SIZE(s->fd_to_key);
  if (maxev < 1) maxev = 1;
  if (maxev > 1 << 16) maxev = 1 << 16;
  static thread_local std::vector<struct epoll_event> buf;
  if (static_cast<Py_ssize_t>(buf.size()) < maxev) buf.resize(maxev);
  int n;
  const int epfd = s->epfd;
  if (ms == 0) {
    n = epoll_wait(epfd, buf.data(), static_cast<int>(maxev), 0);
  } else {
    Py_BEGIN_ALLOW_THREADS
    n = epoll_wait(epfd, buf.data(), static_cast<int>(maxev), ms);
    Py_END_ALLOW_THREADS
  }
  if (n < 0) {
    if (errno == EINTR) return PyErr_CheckSignals();  // the loop iterates again; handlers ran
    PyErr_SetFromErrno(PyExc_OSError);
    return -1;
  }
  if (n == 0) return 0;
  // map every fd first (as selectors.select does), then dispatch (as _process_events does)
  std::vector<std::pair<PyObject*, long>> keys;
  keys.reserve(n);
  int rc = 0;
  for (int i = 0; i < n && rc == 0; ++i) {
    const uint32_t ev = buf[i].events;
    long events = 0;
    if (ev & ~static_cast<uint32_t>(EPOLLIN)) events |= kEventWrite;
    if (ev & ~static_cast<uint32_t>(EPOLLOUT)) events |= kEventRead;
    PyObject* fd = PyLong_FromLong(buf[i].data.fd);
    if (!fd) {
      rc = -1;
      break;
    }
    PyObject* key = PyDict_GetItemWithError(s->fd_to_key, fd);
    Py_DECREF(fd);
    if (!key) {
      if (PyErr_Occurred()) rc = -1;
      continue;
    }
    PyObject* kev = PyTuple_Check(key) && PyTuple_GET_SIZE(key) == 4 ? PyTuple_GET_ITEM(key, 2) : nullptr;
    long kmask;
    if (kev) {
      kmask = PyLong_AsLong(kev);
    } else {
      PyObject* e = PyObject_GetAttr(key, s_events);
      kmask = e ? PyLong_AsLong(e) : -1;
      Py_XDECREF(e);
    }
    if (kmask == -1 && PyErr_Occurred()) {
      rc = -1;
      break;
    }
    Py_INCREF(key);
    keys.emplace_back(key, events & kmask);
  }
  for (auto& km : keys) {
    if (rc == 0) rc = process_key(s, self, km.first, km.second);
    Py_DECREF(km.first);
  }
  return rc;
}

PyObject* loop_run_once(PyObject* self, PyObject*) {
  LoopCore* s = reinterpret_cast<LoopCore*>(self);
  const int debug = attr_true(self, s_debug);
  if (debug < 0) return nullptr;
  if (debug) return PyObject_CallOneArg(g_py_run_once, self);
  PyObject* sel = PyObject_GetAttr(self, s_selector);
  if (!sel) return nullptr;
  const bool ok = ensure_selector(s, sel);
  Py_DECREF(sel);
  if (!ok) return nullptr;
  if (!s->native_select) return PyObject_CallOneArg(g_py_run_once, self);
  if (!ensure_ready(s)) return nullptr;

  PyObject* sched = prune_scheduled(self);
  if (!sched) return nullptr;
  double timeout = -1;  // None: block
  const int stopping = attr_true(self, s_stopping);
  if (stopping < 0) {
    Py_DECREF(sched);
    return nullptr;
  }
  const Py_ssize_t nready = PyObject_Size(s->ready);
  if (nready < 0) {
    Py_DECREF(sched);
    return nullptr;
  }
  if (nready > 0 || stopping) {
    timeout = 0;
  } else if (PyList_GET_SIZE(sched) > 0) {
    PyObject* w = PyObject_GetAttr(PyList_GET_ITEM(sched, 0), s_when);
    const double when = w ? PyFloat_AsDouble(w) : -1;
    Py_XDECREF(w);
    if (PyErr_Occurred()) {
      Py_DECREF(sched);
      return nullptr;
    }
    const double now = call_time(self);
    if (std::isnan(now) && PyErr_Occurred()) {
      Py_DECREF(sched);
      return nullptr;
    }
    timeout = std::min(std::max(0.0, when - now), kMaximumSelectTimeout);
  }
  Py_DECREF(sched);
  if (poll_native(s, self, timeout) < 0) return nullptr;

  // timers that are due (asyncio reads self._scheduled afresh here)
  sched = PyObject_GetAttr(self, s_scheduled);
  if (!sched) return nullptr;
  if (PyList_Check(sched) && PyList_GET_SIZE(sched) > 0) {
    PyObject* resolution = PyObject_GetAttr(self, s_clock_resolution);
    const double res = resolution ? PyFloat_AsDouble(resolution) : 0;
    Py_XDECREF(resolution);
    const double end_time = PyErr_Occurred() ? NAN : call_time(self) + res;
    if (PyErr_Occurred()) {
      Py_DECREF(sched);
      return nullptr;
    }
    while (PyList_GET_SIZE(sched) > 0) {
      PyObject* w = PyObject_GetAttr(PyList_GET_ITEM(sched, 0), s_when);
      const double when = w ? PyFloat_AsDouble(w) : 0;
      Py_XDECREF(w);
      if (PyErr_Occurred()) {
        Py_DECREF(sched);
        return nullptr;
      }
      if (when >= end_time) break;
      PyObject* h = PyObject_CallOneArg(g_heappop, sched);
      if (!h || PyObject_SetAttrString(h, "_scheduled", Py_False) < 0 || call_one(s->ready_append, h) < 0) {
        Py_XDECREF(h);
        Py_DECREF(sched);
        return nullptr;
      }
      Py_DECREF(h);
    }
  }
  Py_DECREF(sched);

  // the only place callbacks run: the handles present now, not those they schedule
  const Py_ssize_t ntodo = PyObject_Size(s->ready);
  if (ntodo < 0) return nullptr;
  for (Py_ssize_t i = 0; i < ntodo; ++i) {
    PyObject* h = PyObject_CallNoArgs(s->ready_popleft);
    if (!h) return nullptr;
    int rc;
    if (Py_TYPE(h) == &HandleType) {
      HandleObject* nh = reinterpret_cast<HandleObject*>(h);
      rc = nh->cancelled ? 0 : handle_run(nh);
    } else {
      const int c = attr_true(h, s_cancelled);
      if (c < 0) {
        rc = -1;
      } else if (c) {
        rc = 0;
      } else {
        PyObject* r = PyObject_CallMethodNoArgs(h, s_run);
        rc = r ? 0 : -1;
        Py_XDECREF(r);
      }
    }
    Py_DECREF(h);
    if (rc < 0) return nullptr;
  }
  Py_RETURN_NONE;
}

PyMethodDef loop_methods[] = {
    {"call_soon", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(loop_call_soon)),
     METH_FASTCALL | METH_KEYWORDS,
     "call_soon(callback, *args, context=None): queue a native Handle (BaseEventLoop.call_soon)."},
    {"_run_once", loop_run_once, METH_NOARGS, "One loop iteration (BaseEventLoop._run_once), natively."},
    {nullptr, nullptr, 0, nullptr}};

PyTypeObject LoopCoreType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// configure(EpollSelector, heappop, heapify, format_callback_source, py_call_soon, py_run_once)
PyObject* py_configure(PyObject*, PyObject* args) {
  PyObject *sel, *hp, *hf, *fmt, *cs, *ro;
  if (!PyArg_ParseTuple(args, "OOOOOO", &sel, &hp, &hf, &fmt, &cs, &ro)) return nullptr;
  if (!PyType_Check(sel)) {
    PyErr_SetString(PyExc_TypeError, "configure(): EpollSelector must be a type");
    return nullptr;
  }
  PyObject** slots[] = {&g_epoll_selector, &g_heappop, &g_heapify, &g_format_cb, &g_py_call_soon, &g_py_run_once};
  PyObject* vals[] = {sel, hp, hf, fmt, cs, ro};
  for (int i = 0; i < 6; ++i) {
    Py_INCREF(vals[i]);
    Py_XSETREF(*slots[i], vals[i]);
  }
  Py_RETURN_NONE;
}

PyObject* py_configured(PyObject*, PyObject*) { return PyBool_FromLong(g_py_run_once != nullptr); }

PyMethodDef module_methods[] = {
    {"configure", py_configure, METH_VARARGS,
     "configure(EpollSelector, heappop, heapify, format_callback_source, BaseEventLoop.call_soon, "
     "BaseEventLoop._run_once)"},
    {"configured", py_configured, METH_NOARGS, "True once configure() ran."},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_aioloop",
                      "Native call_soon/_run_once and Handle for the operator's asyncio loop.", -1,
                      module_methods};

bool intern(PyObject** slot, const char* s) { return (*slot = PyUnicode_InternFromString(s)) != nullptr; }

}  // namespace

PyMODINIT_FUNC PyInit__aioloop(void) {
  if (!intern(&s_ready, "_ready") || !intern(&s_scheduled, "_scheduled") || !intern(&s_stopping, "_stopping") ||
      !intern(&s_selector, "_selector") || !intern(&s_closed, "_closed") || !intern(&s_debug, "_debug") ||
      !intern(&s_timer_cancelled_count, "_timer_cancelled_count") || !intern(&s_cancelled, "_cancelled") ||
      !intern(&s_when, "_when") || !intern(&s_time, "time") || !intern(&s_clock_resolution, "_clock_resolution") ||
      !intern(&s_append, "append") || !intern(&s_popleft, "popleft") || !intern(&s_run, "_run") ||
      !intern(&s_fd_to_key, "_fd_to_key") || !intern(&s_fileno, "fileno") ||
      !intern(&s_remove_reader, "_remove_reader") || !intern(&s_remove_writer, "_remove_writer") ||
      !intern(&s_call_exception_handler, "call_exception_handler") || !intern(&s_message, "message") ||
      !intern(&s_exception, "exception") || !intern(&s_handle, "handle") || !intern(&s_context_kw, "context") ||
      !intern(&s_fileobj, "fileobj") || !intern(&s_events, "events") || !intern(&s_data, "data"))
    return nullptr;
  HandleType.tp_name = "_aioloop.Handle";
  HandleType.tp_basicsize = sizeof(HandleObject);
  HandleType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  HandleType.tp_doc = "A callback queued by the native call_soon (the interface of asyncio.Handle).";
  HandleType.tp_dealloc = reinterpret_cast<destructor>(handle_dealloc);
  HandleType.tp_traverse = reinterpret_cast<traverseproc>(handle_traverse);
  HandleType.tp_clear = reinterpret_cast<inquiry>(handle_clear);
  HandleType.tp_repr = handle_repr;
  HandleType.tp_methods = handle_methods;
  HandleType.tp_members = handle_members;
  HandleType.tp_weaklistoffset = offsetof(HandleObject, weakreflist);

  LoopCoreType.tp_name = "_aioloop.LoopCore";
  LoopCoreType.tp_basicsize = sizeof(LoopCore);
  LoopCoreType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_BASETYPE | Py_TPFLAGS_HAVE_GC;
  LoopCoreType.tp_doc = "Mix-in (before asyncio.SelectorEventLoop) with native call_soon and _run_once.";
  LoopCoreType.tp_new = PyType_GenericNew;
  LoopCoreType.tp_dealloc = reinterpret_cast<destructor>(loop_dealloc);
  LoopCoreType.tp_traverse = reinterpret_cast<traverseproc>(loop_traverse);
  LoopCoreType.tp_clear = reinterpret_cast<inquiry>(loop_clear);
  LoopCoreType.tp_methods = loop_methods;
  if (PyType_Ready(&HandleType) < 0 || PyType_Ready(&LoopCoreType) < 0) return nullptr;
  PyObject* m = PyModule_Create(&moddef);
  if (!m) return nullptr;
  Py_INCREF(&HandleType);
  Py_INCREF(&LoopCoreType);
  if (PyModule_AddObject(m, "Handle", reinterpret_cast<PyObject*>(&HandleType)) < 0 ||
      PyModule_AddObject(m, "LoopCore", reinterpret_cast<PyObject*>(&LoopCoreType)) < 0) {
    Py_DECREF(m);
    return nullptr;
  }
  return m;
}
