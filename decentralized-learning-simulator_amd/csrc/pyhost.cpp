// pyhost.cpp — CPython helpers of the per-task module path (host code, no GPU).
//
// functions.aggregate -> FedAvg.aggregate (fedavg.py:12-26) touches every
// parameter of every model each task: the reference iterates
// `zip(center.parameters(), m.parameters())`; the GPU path needs the same
// parameter lists, checked against models[0]'s layout, and their data
// pointers. For the reference's default model (GNLeNet, 14 tensors, fan-in 7)
// that is ~100 tensor visits per task, which in Python cost more than the
// kernel. These three helpers do the visits in C:
//
//   module_params(module)          == list(module.parameters()): modules in
//                                      named_modules() pre-order, each once,
//                                      then each module's _parameters in
//                                      order, skipping None and parameters
//                                      already seen (by identity)
//   matches(params, signature)     len and every (shape, dtype) equal to the
//                                      signature [(torch.Size, dtype), ...]
//   data_ptrs(rows, idx)           [rows[i][k].data_ptr() for i, k], or None
//                                      if one of them is not contiguous
//
// Built by __graft_entry__.build() as dasklearn_amd/_pyhost*.so.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <unordered_set>

namespace {

PyObject* s_parameters = nullptr;
PyObject* s_modules = nullptr;
PyObject* s_shape = nullptr;
PyObject* s_dtype = nullptr;
PyObject* s_data_ptr = nullptr;
PyObject* s_is_contiguous = nullptr;

int visit(PyObject* m, PyObject* out, std::unordered_set<PyObject*>& seen, int depth) {
  if (depth > 10000) {
    PyErr_SetString(PyExc_RecursionError, "module tree too deep");
    return -1;
  }
  PyObject* params = PyObject_GetAttr(m, s_parameters);
  if (!params) return -1;
  if (!PyDict_Check(params)) {
    Py_DECREF(params);
    PyErr_SetString(PyExc_TypeError, "_parameters is not a dict");
    return -1;
  }
  Py_ssize_t pos = 0;
  PyObject *key, *val;
  while (PyDict_Next(params, &pos, &key, &val)) {
    if (val == Py_None || !seen.insert(val).second) continue;
    if (PyList_Append(out, val) < 0) {
      Py_DECREF(params);
      return -1;
    }
  }
  Py_DECREF(params);
  PyObject* mods = PyObject_GetAttr(m, s_modules);
  if (!mods) return -1;
  if (!PyDict_Check(mods)) {
    Py_DECREF(mods);
    PyErr_SetString(PyExc_TypeError, "_modules is not a dict");
    return -1;
  }
  pos = 0;
  // _modules may not change while we walk it (no Python code runs between
  // PyDict_Next calls except attribute lookups on plain instance dicts)
  while (PyDict_Next(mods, &pos, &key, &val)) {
    if (val == Py_None || !seen.insert(val).second) continue;
    Py_INCREF(val);
    const int rc = visit(val, out, seen, depth + 1);
    Py_DECREF(val);
    if (rc < 0) {
      Py_DECREF(mods);
      return -1;
    }
  }
  Py_DECREF(mods);
  return 0;
}

PyObject* py_module_params(PyObject*, PyObject* module) {
  PyObject* out = PyList_New(0);
  if (!out) return nullptr;
  std::unordered_set<PyObject*> seen;
  seen.insert(module);
  if (visit(module, out, seen, 0) < 0) {
    Py_DECREF(out);
    return nullptr;
  }
  return out;
}

PyObject* py_matches(PyObject*, PyObject* args) {
  PyObject *params, *sig;
  if (!PyArg_ParseTuple(args, "OO", &params, &sig)) return nullptr;
  PyObject* ps = PySequence_Fast(params, "params must be a sequence");
  if (!ps) return nullptr;
  PyObject* ss = PySequence_Fast(sig, "signature must be a sequence");
  if (!ss) {
    Py_DECREF(ps);
    return nullptr;
  }
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(ps);
  int ok = n == PySequence_Fast_GET_SIZE(ss);
  for (Py_ssize_t k = 0; ok && k < n; ++k) {
    PyObject* p = PySequence_Fast_GET_ITEM(ps, k);
    PyObject* entry = PySequence_Fast_GET_ITEM(ss, k);  // (shape, dtype)
    if (!PyTuple_Check(entry) || PyTuple_GET_SIZE(entry) != 2) {
      PyErr_SetString(PyExc_TypeError, "signature entries are (shape, dtype)");
      ok = -1;
      break;
    }
    PyObject* dt = PyObject_GetAttr(p, s_dtype);
    if (!dt) {
      ok = -1;
      break;
    }
    ok = dt == PyTuple_GET_ITEM(entry, 1);
    Py_DECREF(dt);
    if (!ok) break;
    PyObject* sh = PyObject_GetAttr(p, s_shape);
    if (!sh) {
      ok = -1;
      break;
    }
    ok = PyObject_RichCompareBool(sh, PyTuple_GET_ITEM(entry, 0), Py_EQ);
    Py_DECREF(sh);
  }
  Py_DECREF(ps);
  Py_DECREF(ss);
  if (ok < 0) return nullptr;
  return PyBool_FromLong(ok);
}

PyObject* py_data_ptrs(PyObject*, PyObject* args) {
  PyObject *rows, *idx;
  if (!PyArg_ParseTuple(args, "OO", &rows, &idx)) return nullptr;
  PyObject* rs = PySequence_Fast(rows, "rows must be a sequence");
  if (!rs) return nullptr;
  PyObject* ks = PySequence_Fast(idx, "idx must be a sequence");
  if (!ks) {
    Py_DECREF(rs);
    return nullptr;
  }
  const Py_ssize_t nr = PySequence_Fast_GET_SIZE(rs), nk = PySequence_Fast_GET_SIZE(ks);
  PyObject* out = PyList_New(nr * nk);
  bool contiguous = true;
  for (Py_ssize_t i = 0; out && contiguous && i < nr; ++i) {
    PyObject* row = PySequence_Fast_GET_ITEM(rs, i);
    for (Py_ssize_t j = 0; j < nk; ++j) {
      PyObject* t = PyObject_GetItem(row, PySequence_Fast_GET_ITEM(ks, j));
      if (!t) {
        Py_CLEAR(out);
        break;
      }
      PyObject* c = PyObject_CallMethodNoArgs(t, s_is_contiguous);
      if (!c) {
        Py_DECREF(t);
        Py_CLEAR(out);
        break;
      }
      const int isc = PyObject_IsTrue(c);
      Py_DECREF(c);
      if (isc != 1) {
        Py_DECREF(t);
        if (isc < 0) Py_CLEAR(out);
        contiguous = false;
        break;
      }
      PyObject* ptr = PyObject_CallMethodNoArgs(t, s_data_ptr);
      Py_DECREF(t);
      if (!ptr) {
        Py_CLEAR(out);
        break;
      }
      PyList_SET_ITEM(out, i * nk + j, ptr);  // steals the reference
    }
  }
  Py_DECREF(rs);
  Py_DECREF(ks);
  if (!out) return nullptr;
  if (!contiguous) {
    Py_DECREF(out);
    Py_RETURN_NONE;
  }
  return out;
}

PyMethodDef kMethods[] = {
    {"module_params", py_module_params, METH_O, "list(module.parameters()), in C"},
    {"matches", py_matches, METH_VARARGS, "params match a [(shape, dtype)] signature"},
    {"data_ptrs", py_data_ptrs, METH_VARARGS, "data pointers of rows[i][k] for k in idx, None if not contiguous"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_pyhost", "CPython helpers of the per-task module path", -1,
                       kMethods, nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__pyhost(void) {
  s_parameters = PyUnicode_InternFromString("_parameters");
  s_modules = PyUnicode_InternFromString("_modules");
  s_shape = PyUnicode_InternFromString("shape");
  s_dtype = PyUnicode_InternFromString("dtype");
  s_data_ptr = PyUnicode_InternFromString("data_ptr");
  s_is_contiguous = PyUnicode_InternFromString("is_contiguous");
  if (!s_parameters || !s_modules || !s_shape || !s_dtype || !s_data_ptr || !s_is_contiguous) return nullptr;
  return PyModule_Create(&kModule);
}
