// Native metric series for runtime/promlite.py (CPython extension `_promlite`).
//
// controller-runtime's metrics (workqueue_*, controller_runtime_reconcile_*, rest_client_*;
// reference: the manager's metrics server, /root/reference/cmd/operator/start.go:118-150) are
// updated ~30 times per Cron fire: each REST request counts itself and observes its latency,
// each work-queue get/done observes queue and work time, each reconcile counts and times
// itself.  In Python each update is a method frame (~20 bytecodes); here it is one C call on a
// series object:
//
//   Counter()            .value (float), inc(amount=1.0) -- ValueError on a negative amount
//   Gauge()              .value, inc(amount=1.0), dec(amount=1.0), set(value)
//   Histogram(bounds)    .bounds (sorted finite upper bounds), .counts (per bucket, last one
//                        above every bound), .sum, .count, observe(v) -- bucket = bisect_left
//                        (le semantics: v <= bound)
//
// Semantics are those of the Python series classes in runtime/promlite.py, which stay the
// fallback and the oracle of tests/test_promlite.py.  The operator is one asyncio thread per
// process, so there is no locking (as in the Python classes).

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <vector>

namespace {

// ---------------------------------------------------------------------------------------- Counter

struct ValueObject {
  PyObject_HEAD
  double value;
};

PyTypeObject CounterType = {PyVarObject_HEAD_INIT(nullptr, 0)};
PyTypeObject GaugeType = {PyVarObject_HEAD_INIT(nullptr, 0)};

// the optional `amount` argument as a double (1.0 when absent); false on error
bool amount_arg(PyObject* const* args, Py_ssize_t nargs, const char* fn, double* out) {
  if (nargs > 1) {
    PyErr_Format(PyExc_TypeError, "%s() takes at most 1 argument (%zd given)", fn, nargs);
    return false;
  }
  if (nargs == 0) {
    *out = 1.0;
    return true;
  }
  *out = PyFloat_AsDouble(args[0]);
  return !(*out == -1.0 && PyErr_Occurred());
}

PyObject* counter_inc(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  double a;
  if (!amount_arg(args, nargs, "inc", &a)) return nullptr;
  if (a < 0) {
    PyErr_SetString(PyExc_ValueError, "counters can only increase");
    return nullptr;
  }
  reinterpret_cast<ValueObject*>(self)->value += a;
  Py_RETURN_NONE;
}

PyObject* value_get(PyObject* self, PyObject*) { return PyFloat_FromDouble(reinterpret_cast<ValueObject*>(self)->value); }

PyObject* gauge_inc(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  double a;
  if (!amount_arg(args, nargs, "inc", &a)) return nullptr;
  reinterpret_cast<ValueObject*>(self)->value += a;
  Py_RETURN_NONE;
}

PyObject* gauge_dec(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  double a;
  if (!amount_arg(args, nargs, "dec", &a)) return nullptr;
  reinterpret_cast<ValueObject*>(self)->value -= a;
  Py_RETURN_NONE;
}

PyObject* gauge_set(PyObject* self, PyObject* v) {
  PyObject* f = PyNumber_Float(v);  // float(value), as the Python class does
  if (!f) return nullptr;
  reinterpret_cast<ValueObject*>(self)->value = PyFloat_AS_DOUBLE(f);
  Py_DECREF(f);
  Py_RETURN_NONE;
}

PyObject* value_new(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  if ((args && PyTuple_GET_SIZE(args)) || (kwds && PyDict_GET_SIZE(kwds))) {
    PyErr_Format(PyExc_TypeError, "%s() takes no arguments", type->tp_name);
    return nullptr;
  }
  ValueObject* o = reinterpret_cast<ValueObject*>(type->tp_alloc(type, 0));
  if (o) o->value = 0.0;
  return reinterpret_cast<PyObject*>(o);
}

PyMethodDef counter_methods[] = {
    {"inc", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(counter_inc)), METH_FASTCALL,
     "inc(amount=1.0): add a non-negative amount"},
    {"get", value_get, METH_NOARGS, "the current value"},
    {nullptr, nullptr, 0, nullptr}};

PyMethodDef gauge_methods[] = {
    {"inc", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(gauge_inc)), METH_FASTCALL,
     "inc(amount=1.0)"},
    {"dec", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(gauge_dec)), METH_FASTCALL,
     "dec(amount=1.0)"},
    {"set", gauge_set, METH_O, "set(value): float(value)"},
    {"get", value_get, METH_NOARGS, "the current value"},
    {nullptr, nullptr, 0, nullptr}};

PyMemberDef value_members[] = {{"value", T_DOUBLE, offsetof(ValueObject, value), 0, nullptr},
                               {nullptr, 0, 0, 0, nullptr}};

// -------------------------------------------------------------------------------------- Histogram

struct HistogramObject {
  PyObject_HEAD
  PyObject* bounds;               // the tuple it was built with
  std::vector<double>* b;         // its values
  std::vector<long long>* counts; // len(bounds) + 1
  double sum;
  long long count;
};

PyTypeObject HistogramType = {PyVarObject_HEAD_INIT(nullptr, 0)};

void hist_dealloc(PyObject* self) {
  HistogramObject* h = reinterpret_cast<HistogramObject*>(self);
  Py_XDECREF(h->bounds);
  delete h->b;
  delete h->counts;
  Py_TYPE(self)->tp_free(self);
}

PyObject* hist_new(PyTypeObject* type, PyObject* args, PyObject* kwds) {
  static const char* kw[] = {"bounds", nullptr};
  PyObject* bounds;
  if (!PyArg_ParseTupleAndKeywords(args, kwds, "O!", const_cast<char**>(kw), &PyTuple_Type, &bounds)) return nullptr;
  std::vector<double> b;
  b.reserve(PyTuple_GET_SIZE(bounds));
  for (Py_ssize_t i = 0; i < PyTuple_GET_SIZE(bounds); ++i) {
    const double d = PyFloat_AsDouble(PyTuple_GET_ITEM(bounds, i));
    if (d == -1.0 && PyErr_Occurred()) return nullptr;
    if (!b.empty() && !(b.back() <= d)) {
      PyErr_SetString(PyExc_ValueError, "histogram bounds must be sorted");
      return nullptr;
    }
    b.push_back(d);
  }
  HistogramObject* h = reinterpret_cast<HistogramObject*>(type->tp_alloc(type, 0));
  if (!h) return nullptr;
  Py_INCREF(bounds);
  h->bounds = bounds;
  h->b = new std::vector<double>(std::move(b));
  h->counts = new std::vector<long long>(h->b->size() + 1, 0);
  h->sum = 0.0;
  h->count = 0;
  return reinterpret_cast<PyObject*>(h);
}

PyObject* hist_observe(PyObject* self, PyObject* arg) {
  HistogramObject* h = reinterpret_cast<HistogramObject*>(self);
  const double v = PyFloat_AsDouble(arg);
  if (v == -1.0 && PyErr_Occurred()) return nullptr;
  // bisect_left(bounds, v): the first bound not below v (a NaN lands in bucket 0, as in Python)
  size_t lo = 0, hi = h->b->size();
  const double* b = h->b->data();
  while (lo < hi) {
    const size_t mid = (lo + hi) / 2;
    if (b[mid] < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  ++(*h->counts)[lo];
  h->sum += v;
  ++h->count;
  Py_RETURN_NONE;
}

PyObject* hist_counts(PyObject* self, void*) {
  const auto& c = *reinterpret_cast<HistogramObject*>(self)->counts;
  PyObject* out = PyList_New(static_cast<Py_ssize_t>(c.size()));
  if (!out) return nullptr;
  for (size_t i = 0; i < c.size(); ++i) {
    PyObject* n = PyLong_FromLongLong(c[i]);
    if (!n) {
      Py_DECREF(out);
      return nullptr;
    }
    PyList_SET_ITEM(out, static_cast<Py_ssize_t>(i), n);
  }
  return out;
}

PyMethodDef hist_methods[] = {{"observe", hist_observe, METH_O, "observe(v): count v in its bucket"},
                              {nullptr, nullptr, 0, nullptr}};

PyMemberDef hist_members[] = {{"bounds", T_OBJECT, offsetof(HistogramObject, bounds), READONLY, nullptr},
                              {"sum", T_DOUBLE, offsetof(HistogramObject, sum), 0, nullptr},
                              {"count", T_LONGLONG, offsetof(HistogramObject, count), 0, nullptr},
                              {nullptr, 0, 0, 0, nullptr}};

PyGetSetDef hist_getset[] = {{"counts", hist_counts, nullptr, "per-bucket counts (a copy)", nullptr},
                             {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_promlite", "Native metric series (Counter, Gauge, Histogram).",
                      -1, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__promlite(void) {
  CounterType.tp_name = "_promlite.Counter";
  CounterType.tp_basicsize = sizeof(ValueObject);
  CounterType.tp_flags = Py_TPFLAGS_DEFAULT;
  CounterType.tp_doc = "A counter series: .value, inc(amount=1.0)";
  CounterType.tp_new = value_new;
  CounterType.tp_methods = counter_methods;
  CounterType.tp_members = value_members;
  GaugeType.tp_name = "_promlite.Gauge";
  GaugeType.tp_basicsize = sizeof(ValueObject);
  GaugeType.tp_flags = Py_TPFLAGS_DEFAULT;
  GaugeType.tp_doc = "A gauge series: .value, inc/dec(amount=1.0), set(value)";
  GaugeType.tp_new = value_new;
  GaugeType.tp_methods = gauge_methods;
  GaugeType.tp_members = value_members;
  HistogramType.tp_name = "_promlite.Histogram";
  HistogramType.tp_basicsize = sizeof(HistogramObject);
  HistogramType.tp_flags = Py_TPFLAGS_DEFAULT;
  HistogramType.tp_doc = "A histogram series: Histogram(bounds); .bounds, .counts, .sum, .count, observe(v)";
  HistogramType.tp_new = hist_new;
  HistogramType.tp_dealloc = hist_dealloc;
  HistogramType.tp_methods = hist_methods;
  HistogramType.tp_members = hist_members;
  HistogramType.tp_getset = hist_getset;
  if (PyType_Ready(&CounterType) < 0 || PyType_Ready(&GaugeType) < 0 || PyType_Ready(&HistogramType) < 0)
    return nullptr;
  PyObject* m = PyModule_Create(&moddef);
  if (!m) return nullptr;
  PyTypeObject* types[] = {&CounterType, &GaugeType, &HistogramType};
  const char* names[] = {"Counter", "Gauge", "Histogram"};
  for (int i = 0; i < 3; ++i) {
    Py_INCREF(types[i]);
    if (PyModule_AddObject(m, names[i], reinterpret_cast<PyObject*>(types[i])) < 0) {
      Py_DECREF(types[i]);
      Py_DECREF(m);
      return nullptr;
    }
  }
  return m;
}
