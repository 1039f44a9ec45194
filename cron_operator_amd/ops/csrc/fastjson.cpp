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

#define PY_SSIZE_T_CLEAN
#include <Python.h>

namespace {

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
    return out;
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
    return out;
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

PyObject* merge_patch_impl(PyObject* old, PyObject* nw, int depth) {
  if (!PyDict_CheckExact(old) || !PyDict_CheckExact(nw)) return deepcopy_impl(nw, depth);
  PyObject* patch = PyDict_New();
  if (!patch) return nullptr;
  Py_ssize_t pos = 0;
  PyObject *k, *v;
  while (PyDict_Next(nw, &pos, &k, &v)) {
    PyObject* ov = PyDict_GetItemWithError(old, k);
    PyObject* entry = nullptr;
    if (!ov) {
      if (PyErr_Occurred()) goto fail;
      entry = deepcopy_impl(v, depth + 1);
      if (!entry) goto fail;
    } else if (PyDict_CheckExact(ov) && PyDict_CheckExact(v)) {
      PyObject* sub = merge_patch_impl(ov, v, depth + 1);
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
      entry = deepcopy_impl(v, depth + 1);
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
  if (nargs != 2) {
    PyErr_SetString(PyExc_TypeError, "create_merge_patch(old, new)");
    return nullptr;
  }
  return merge_patch_impl(args[0], args[1], 0);
}

PyMethodDef methods[] = {
    {"deepcopy", py_deepcopy, METH_O, "copy a JSON tree"},
    {"json_equal", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(py_json_equal)), METH_FASTCALL,
     "structural JSON equality"},
    {"create_merge_patch", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(py_merge_patch)),
     METH_FASTCALL, "RFC 7386 merge patch from old to new"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_fastjson", "Native JSON-tree helpers", -1, methods,
                      nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__fastjson(void) { return PyModule_Create(&moddef); }
