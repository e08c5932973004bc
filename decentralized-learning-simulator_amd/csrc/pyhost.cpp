// pyhost.cpp — CPython helpers of the per-task module path (host code, no GPU).
//
// functions.aggregate -> FedAvg.aggregate (fedavg.py:12-26) touches every
// parameter of every model each task: the reference iterates
// `zip(center.parameters(), m.parameters())`; the GPU path needs the same
// parameter lists, checked against models[0]'s layout, and their data
// pointers. For the reference's default model (GNLeNet, 14 tensors, fan-in 7)
// that is ~100 tensor visits per task, which in Python cost more than the
// kernel. These helpers do the visits in C:
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
//   clone_module(module, memo)     arena._clone_module_py: copy.deepcopy of
//                                      models[0] with parameters from the memo
//   checked_params(module, sig)    module_params + matches in one call
//   fill_param_views(...)          the output module's Parameters as views of
//                                      the reduced arena, into the clone's memo
//   flat_run(params, idx, offs, n) the dtype group already is one flat arena
//   wreduce_rows(...)              the data pointers of a task's parameter
//                                      tensors straight into one
//                                      dlsim_wreduce_tensors call
//   wreduce_rows_multi(...)        the same for many tasks, one
//                                      dlsim_wreduce_batched call
//   shm_keys(rows, idx)            per model, the identity of its tensors'
//                                      torch.multiprocessing file_system
//                                      storages (device_cache.py), or None
//
// Tensor fields (shape, dtype, contiguity, device, data pointer) are read from
// the at::Tensor itself (libtorch headers; the extension links torch's
// libraries), not through Python attribute calls.
//
// Built by __graft_entry__.build() as dasklearn_amd/_pyhost*.so.
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <libshm.h>
#include <torch/csrc/Dtype.h>
#include <torch/csrc/autograd/python_variable.h>

#include <cstdint>
#include <algorithm>
#include <cstring>
#include <unordered_set>
#include <vector>

namespace {

PyObject* s_parameters = nullptr;
PyObject* s_modules = nullptr;

// Identity set of the objects a walk has visited: open addressing over a
// power-of-two table (a std::unordered_set allocated a node per insert, ~30
// per GNLeNet model and per task).
class PtrSet {
 public:
  explicit PtrSet(size_t cap = 128) : slots_(cap, nullptr) {}
  // true if p was not in the set (and is now)
  bool insert(PyObject* p) {
    if (2 * (count_ + 1) > slots_.size()) grow();
    if (!place(slots_, p)) return false;
    ++count_;
    return true;
  }

 private:
  static bool place(std::vector<PyObject*>& t, PyObject* p) {
    const size_t mask = t.size() - 1;
    size_t h = (static_cast<size_t>(reinterpret_cast<uintptr_t>(p)) >> 4) * 0x9E3779B97F4A7C15ull;
    for (size_t i = (h >> 20) & mask;; i = (i + 1) & mask) {
      if (t[i] == p) return false;
      if (!t[i]) {
        t[i] = p;
        return true;
      }
    }
  }
  void grow() {
    std::vector<PyObject*> t(slots_.size() * 2, nullptr);
    for (PyObject* p : slots_)
      if (p) place(t, p);
    slots_.swap(t);
  }
  std::vector<PyObject*> slots_;
  size_t count_ = 0;
};

// m.<name> as a new reference: the instance dict first (where nn.Module keeps
// _parameters and _modules; one dict lookup instead of the attribute protocol
// of a class with __getattr__), the full attribute lookup otherwise
PyObject* module_attr(PyObject* m, PyObject* name) {
  PyObject** dp = _PyObject_GetDictPtr(m);
  if (dp && *dp) {
    PyObject* v = PyDict_GetItemWithError(*dp, name);
    if (v) {
      Py_INCREF(v);
      return v;
    }
    if (PyErr_Occurred()) return nullptr;
  }
  return PyObject_GetAttr(m, name);
}

int visit(PyObject* m, PyObject* out, PtrSet& seen, int depth) {
  if (depth > 10000) {
    PyErr_SetString(PyExc_RecursionError, "module tree too deep");
    return -1;
  }
  PyObject* params = module_attr(m, s_parameters);
  if (!params) return -1;
  if (!PyDict_Check(params)) {
    Py_DECREF(params);
    PyErr_SetString(PyExc_TypeError, "_parameters is not a dict");
    return -1;
  }
  Py_ssize_t pos = 0;
  PyObject *key, *val;
  while (PyDict_Next(params, &pos, &key, &val)) {
    if (val == Py_None || !seen.insert(val)) continue;
    if (PyList_Append(out, val) < 0) {
      Py_DECREF(params);
      return -1;
    }
  }
  Py_DECREF(params);
  PyObject* mods = module_attr(m, s_modules);
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
    if (val == Py_None || !seen.insert(val)) continue;
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
  PtrSet seen;
  seen.insert(module);
  if (visit(module, out, seen, 0) < 0) {
    Py_DECREF(out);
    return nullptr;
  }
  return out;
}

// ---- tensor fields read in C++ ---------------------------------------------
//
// THPVariable_Unpack gives the at::Tensor behind a torch.Tensor/nn.Parameter
// object, so shape, dtype, contiguity, device and data pointer are field reads
// instead of Python attribute and method calls (about 100 tensors per task).

// The tensor behind `o`, or nullptr (TypeError set) for anything else.
const at::Tensor* tensor_of(PyObject* o) {
  if (!THPVariable_Check(o)) {
    PyErr_Format(PyExc_TypeError, "expected a tensor, got %.200s", Py_TYPE(o)->tp_name);
    return nullptr;
  }
  return &THPVariable_Unpack(o);
}

// A layout signature ((torch.Size, torch.dtype), ...) as C++ values, cached by
// the identity of the tuple (ParamLayout.rebind shares it across tasks). The
// cache holds a reference to each key, so a cached address cannot be reused
// by another object while its entry exists.
struct Sig {
  std::vector<std::vector<int64_t>> shapes;
  std::vector<at::ScalarType> dtypes;
};
constexpr size_t kSigCache = 16;
std::vector<std::pair<PyObject*, Sig>> g_sigs;

const Sig* sig_of(PyObject* sig) {
  for (auto& e : g_sigs)
    if (e.first == sig) return &e.second;
  PyObject* ss = PySequence_Fast(sig, "signature must be a sequence");
  if (!ss) return nullptr;
  Sig s;
  bool ok = true;
  for (Py_ssize_t k = 0; ok && k < PySequence_Fast_GET_SIZE(ss); ++k) {
    PyObject* entry = PySequence_Fast_GET_ITEM(ss, k);
    if (!PyTuple_Check(entry) || PyTuple_GET_SIZE(entry) != 2 || !THPDtype_Check(PyTuple_GET_ITEM(entry, 1))) {
      PyErr_SetString(PyExc_TypeError, "signature entries are (shape, dtype)");
      ok = false;
      break;
    }
    PyObject* sh = PySequence_Fast(PyTuple_GET_ITEM(entry, 0), "shape must be a sequence");
    if (!sh) {
      ok = false;
      break;
    }
    std::vector<int64_t> dims;
    for (Py_ssize_t d = 0; d < PySequence_Fast_GET_SIZE(sh); ++d)
      dims.push_back(PyLong_AsLongLong(PySequence_Fast_GET_ITEM(sh, d)));
    Py_DECREF(sh);
    if (PyErr_Occurred()) {
      ok = false;
      break;
    }
    s.shapes.push_back(std::move(dims));
    s.dtypes.push_back(reinterpret_cast<THPDtype*>(PyTuple_GET_ITEM(entry, 1))->scalar_type);
  }
  Py_DECREF(ss);
  if (!ok) return nullptr;
  if (g_sigs.size() == kSigCache) {
    Py_DECREF(g_sigs.front().first);
    g_sigs.erase(g_sigs.begin());
  }
  Py_INCREF(sig);
  g_sigs.emplace_back(sig, std::move(s));
  return &g_sigs.back().second;
}

// 1 if the tensors in `ps` (a PySequence_Fast) have the signature's count,
// shapes and dtypes, 0 if not, -1 on error
int matches_sig(PyObject* ps, const Sig& s) {
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(ps);
  if (static_cast<size_t>(n) != s.shapes.size()) return 0;
  for (Py_ssize_t k = 0; k < n; ++k) {
    const at::Tensor* t = tensor_of(PySequence_Fast_GET_ITEM(ps, k));
    if (!t) return -1;
    if (t->scalar_type() != s.dtypes[k] || !t->sizes().equals(s.shapes[k])) return 0;
  }
  return 1;
}

PyObject* py_matches(PyObject*, PyObject* args) {
  PyObject *params, *sig;
  if (!PyArg_ParseTuple(args, "OO", &params, &sig)) return nullptr;
  const Sig* s = sig_of(sig);
  if (!s) return nullptr;
  PyObject* ps = PySequence_Fast(params, "params must be a sequence");
  if (!ps) return nullptr;
  const int ok = matches_sig(ps, *s);
  Py_DECREF(ps);
  if (ok < 0) return nullptr;
  return PyBool_FromLong(ok);
}

// rows[i][idx[j]] for every i, j (model-major) as tensors; false (error set)
// if an item is missing or not a tensor
bool row_tensors(PyObject* rows, PyObject* idx, std::vector<const at::Tensor*>& out, Py_ssize_t* n_out,
                 Py_ssize_t* t_out) {
  PyObject* rs = PySequence_Fast(rows, "rows must be a sequence");
  if (!rs) return false;
  PyObject* ks = PySequence_Fast(idx, "idx must be a sequence");
  if (!ks) {
    Py_DECREF(rs);
    return false;
  }
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(rs), t = PySequence_Fast_GET_SIZE(ks);
  out.resize(static_cast<size_t>(n * t));
  bool ok = true;
  for (Py_ssize_t i = 0; ok && i < n; ++i) {
    PyObject* row = PySequence_Fast(PySequence_Fast_GET_ITEM(rs, i), "each row must be a sequence");
    if (!row) {
      ok = false;
      break;
    }
    const Py_ssize_t len = PySequence_Fast_GET_SIZE(row);
    for (Py_ssize_t j = 0; j < t; ++j) {
      const Py_ssize_t k = PyLong_AsSsize_t(PySequence_Fast_GET_ITEM(ks, j));
      if (k < 0 || k >= len) {
        if (!PyErr_Occurred()) PyErr_SetString(PyExc_IndexError, "parameter index out of range");
        ok = false;
        break;
      }
      // the rows (and so the tensors) outlive this call: borrowed pointers
      const at::Tensor* tt = tensor_of(PySequence_Fast_GET_ITEM(row, k));
      if (!tt) {
        ok = false;
        break;
      }
      out[static_cast<size_t>(i * t + j)] = tt;
    }
    Py_DECREF(row);
  }
  Py_DECREF(ks);
  Py_DECREF(rs);
  *n_out = n;
  *t_out = t;
  return ok;
}

PyObject* py_data_ptrs(PyObject*, PyObject* args) {
  PyObject *rows, *idx;
  if (!PyArg_ParseTuple(args, "OO", &rows, &idx)) return nullptr;
  std::vector<const at::Tensor*> ts;
  Py_ssize_t n, t;
  if (!row_tensors(rows, idx, ts, &n, &t)) return nullptr;
  for (const at::Tensor* x : ts)
    if (!x->is_contiguous()) Py_RETURN_NONE;
  PyObject* out = PyList_New(static_cast<Py_ssize_t>(ts.size()));
  if (!out) return nullptr;
  for (size_t q = 0; q < ts.size(); ++q) {
    PyObject* p = PyLong_FromVoidPtr(const_cast<void*>(ts[q]->const_data_ptr()));
    if (!p) {
      Py_DECREF(out);
      return nullptr;
    }
    PyList_SET_ITEM(out, static_cast<Py_ssize_t>(q), p);
  }
  return out;
}

// shm_keys(rows, idx) -> [key_i or None]: for model i, the identity of
// tensors rows[i][k] (k in idx) when every one is a CPU tensor whose storage
// is a torch.multiprocessing file_system shared-memory file (what a worker of
// the reference receives, worker.py:6): (the first tensor's shm file name,
// a 64-bit FNV-style hash over every tensor's file name, storage offset,
// numel, dtype and strides). A file name names one storage allocation for the run, so a key
// seen again by this process is the same model's memory (device_cache.py);
// None for a model with any tensor elsewhere. No Python attribute calls.
// The storages of freshly received models are cold in the CPU caches, and
// each tensor's file name sits four dependent loads away (tensor -> storage ->
// allocator context -> name): the walk goes level by level over all tensors,
// so the loads of one level overlap, and the hash mixes 8 bytes a step.
PyObject* shm_keys_of(const std::vector<const at::Tensor*>& ts, Py_ssize_t n, Py_ssize_t t) {
  const size_t m = ts.size();
  std::vector<const c10::DataPtr*> dps(m, nullptr);
  std::vector<const char*> names(m, nullptr);
  std::vector<char> model_ok(static_cast<size_t>(n), t > 0);
  for (size_t q = 0; q < m; ++q) {
    const at::Tensor* x = ts[q];
    if (x->device().type() == c10::DeviceType::CPU && x->has_storage()) dps[q] = &x->storage().data_ptr();
  }
  for (size_t q = 0; q < m; ++q) {
    THManagedMapAllocator* ctx = dps[q] ? THManagedMapAllocator::fromDataPtr(*dps[q]) : nullptr;
    if (ctx) names[q] = ctx->filename();
  }
  for (size_t q = 0; q < m; ++q)
    if (!names[q]) model_ok[q / static_cast<size_t>(t)] = 0;
  PyObject* out = PyList_New(n);
  if (!out) return nullptr;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* key;
    if (model_ok[static_cast<size_t>(i)]) {
      uint64_t h = 1469598103934665603ull;
      auto mix = [&h](uint64_t w) {
        h = (h ^ w) * 1099511628211ull;
        h ^= h >> 29;
      };
      for (Py_ssize_t j = 0; j < t; ++j) {
        const size_t q = static_cast<size_t>(i * t + j);
        const char* fn = names[q];
        const size_t len = std::strlen(fn);
        for (size_t o = 0; o < len; o += 8) {
          uint64_t w = 0;
          std::memcpy(&w, fn + o, std::min<size_t>(8, len - o));
          mix(w);
        }
        mix(len);
        const at::Tensor* x = ts[q];
        mix(static_cast<uint64_t>(x->storage_offset()));
        mix(static_cast<uint64_t>(x->numel()));
        mix(static_cast<uint64_t>(x->scalar_type()));
        for (const int64_t st : x->strides()) mix(static_cast<uint64_t>(st));  // a view's layout too
      }
      key = Py_BuildValue("(yK)", names[static_cast<size_t>(i * t)], static_cast<unsigned long long>(h));
      if (!key) {
        Py_DECREF(out);
        return nullptr;
      }
    } else {
      key = Py_None;
      Py_INCREF(key);
    }
    PyList_SET_ITEM(out, i, key);
  }
  return out;
}

PyObject* py_shm_keys(PyObject*, PyObject* args) {
  PyObject *rows, *idx;
  if (!PyArg_ParseTuple(args, "OO", &rows, &idx)) return nullptr;
  std::vector<const at::Tensor*> ts;
  Py_ssize_t n, t;
  if (!row_tensors(rows, idx, ts, &n, &t)) return nullptr;
  return shm_keys_of(ts, n, t);
}

// Content fingerprint of model i's tensors [i*t, (i+1)*t) for the device
// cache's stale-hit check: EVERY tensor of
// the model contributes words spread evenly along its bytes -- the first and
// the last word, plus one more per MiB up to kFpMaxWords -- mixed with the
// tensor's index and each word's offset. A model written in place after it
// was cached (the reference trains its input model in place,
// functions.py:57) changes essentially every element, so a changed word
// shows it; a partial update (one layer fine-tuned, a frozen backbone) still
// rewrites whole tensors, and every tensor is sampled. What it cannot see is
// an update that leaves every sampled word as it was.
// A strided view is sampled at its first element only (its other offsets
// need not be inside its storage).
constexpr size_t kFpMaxWords = 16;
inline void fp_mix(uint64_t& h, uint64_t w, uint64_t where) {
  h = (h ^ (w + where)) * 0x100000001b3ull;
  h ^= h >> 31;
}
uint64_t content_fingerprint(const std::vector<const at::Tensor*>& ts, Py_ssize_t i, Py_ssize_t t) {
  uint64_t h = 0x9e3779b97f4a7c15ull;
  for (Py_ssize_t j = 0; j < t; ++j) {
    const at::Tensor* x = ts[static_cast<size_t>(i * t + j)];
    const int64_t ne = x->numel();
    if (ne <= 0) {
      fp_mix(h, 0, static_cast<uint64_t>(j) << 32);
      continue;
    }
    const char* base = static_cast<const char*>(x->const_data_ptr());
    const size_t bytes = x->is_contiguous() ? static_cast<size_t>(ne) * x->element_size() : x->element_size();
    const size_t words = bytes <= 8 ? 1 : std::min(kFpMaxWords, 2 + bytes / (size_t{1} << 20));
    for (size_t q = 0; q < words; ++q) {
      // word q at an 8-byte-granular offset from 0 to the last full word
      const size_t last = bytes >= 8 ? bytes - 8 : 0;
      const size_t off = words > 1 ? (last * q / (words - 1)) & ~size_t{7} : 0;
      uint64_t w = 0;
      std::memcpy(&w, base + off, std::min<size_t>(8, bytes - off));
      fp_mix(h, w, (static_cast<uint64_t>(j) << 32) ^ off);
    }
  }
  return h;
}

// shm_rows(rows, idx) -> (shm_keys(rows, idx), data_ptrs(rows, idx),
// fingerprints): one pass over the tensors of freshly received models, whose
// first touch is most of the cost (device cache path,
// arena._cached_host_reduce); fingerprints[i] is content_fingerprint of
// model i, or None where keys[i] is None.
PyObject* py_shm_rows(PyObject*, PyObject* args) {
  PyObject *rows, *idx;
  if (!PyArg_ParseTuple(args, "OO", &rows, &idx)) return nullptr;
  std::vector<const at::Tensor*> ts;
  Py_ssize_t n, t;
  if (!row_tensors(rows, idx, ts, &n, &t)) return nullptr;
  PyObject* keys = shm_keys_of(ts, n, t);
  if (!keys) return nullptr;
  PyObject* fps = PyList_New(n);
  if (!fps) {
    Py_DECREF(keys);
    return nullptr;
  }
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* f;
    if (PyList_GET_ITEM(keys, i) == Py_None) {
      f = Py_None;
      Py_INCREF(f);
    } else {
      f = PyLong_FromUnsignedLongLong(content_fingerprint(ts, i, t));
      if (!f) {
        Py_DECREF(keys);
        Py_DECREF(fps);
        return nullptr;
      }
    }
    PyList_SET_ITEM(fps, i, f);
  }
  bool contiguous = true;
  for (const at::Tensor* x : ts) contiguous = contiguous && x->is_contiguous();
  PyObject* ptrs;
  if (contiguous) {
    ptrs = PyList_New(static_cast<Py_ssize_t>(ts.size()));
    for (size_t q = 0; ptrs && q < ts.size(); ++q) {
      PyObject* p = PyLong_FromVoidPtr(const_cast<void*>(ts[q]->const_data_ptr()));
      if (!p) {
        Py_CLEAR(ptrs);
        break;
      }
      PyList_SET_ITEM(ptrs, static_cast<Py_ssize_t>(q), p);
    }
  } else {
    ptrs = Py_None;
    Py_INCREF(ptrs);
  }
  if (!ptrs) {
    Py_DECREF(keys);
    Py_DECREF(fps);
    return nullptr;
  }
  PyObject* res = PyTuple_Pack(3, keys, ptrs, fps);
  Py_DECREF(keys);
  Py_DECREF(ptrs);
  Py_DECREF(fps);
  return res;
}

// chunk_scan(chunks) -> (same_dtype, place, device_index, numels, fans, ptrs)
// for ChunkManager.mean_chunk_indices (chunk_manager.py:38-40 semantics):
// chunks[i] is the list of contributors of chunk index i. Raises
// RuntimeError("stack expects each tensor to be equal size") as torch.stack
// does when one index's tensors differ in shape or dtype. same_dtype: every
// index has the dtype of chunks[0][0]; place: 1 all on the host, 2 all on one
// GPU (device_index), 0 otherwise; numels / fans per index; ptrs the data
// pointers index by index, or None when a tensor is not contiguous. One pass
// in C instead of several Python loops over every contributor.
PyObject* py_chunk_scan(PyObject*, PyObject* chunks) {
  PyObject* cs_all = PySequence_Fast(chunks, "chunks must be a sequence");
  if (!cs_all) return nullptr;
  const Py_ssize_t k = PySequence_Fast_GET_SIZE(cs_all);
  std::vector<const at::Tensor*> ts;
  std::vector<Py_ssize_t> fans(static_cast<size_t>(k));
  std::vector<int64_t> numels(static_cast<size_t>(k));
  bool ok = true, same_dtype = true, all_cpu = true, all_cuda = true, contiguous = true;
  int dev_index = -2;
  c10::ScalarType dt0 = c10::ScalarType::Undefined;
  for (Py_ssize_t i = 0; ok && i < k; ++i) {
    PyObject* cs = PySequence_Fast(PySequence_Fast_GET_ITEM(cs_all, i), "each index must be a sequence");
    if (!cs) {
      ok = false;
      break;
    }
    const Py_ssize_t m = PySequence_Fast_GET_SIZE(cs);
    if (m < 1) {
      PyErr_SetString(PyExc_RuntimeError, "stack expects a non-empty TensorList");
      ok = false;
    }
    const at::Tensor* first = nullptr;
    for (Py_ssize_t j = 0; ok && j < m; ++j) {
      const at::Tensor* x = tensor_of(PySequence_Fast_GET_ITEM(cs, j));
      if (!x) {
        ok = false;
        break;
      }
      if (!first) {
        first = x;
        if (dt0 == c10::ScalarType::Undefined) dt0 = x->scalar_type();
        same_dtype = same_dtype && x->scalar_type() == dt0;
      } else if (x->sizes() != first->sizes() || x->scalar_type() != first->scalar_type()) {
        PyErr_SetString(PyExc_RuntimeError, "stack expects each tensor to be equal size");
        ok = false;
        break;
      }
      const c10::Device d = x->device();
      if (d.is_cpu()) {
        all_cuda = false;
      } else {
        all_cpu = false;
        const int di = d.is_cuda() ? static_cast<int>(d.index()) : -3;
        if (dev_index == -2) dev_index = di;
        if (!d.is_cuda() || di != dev_index) all_cuda = false;
      }
      contiguous = contiguous && x->is_contiguous();
      ts.push_back(x);
    }
    if (ok) {
      fans[static_cast<size_t>(i)] = m;
      numels[static_cast<size_t>(i)] = first ? first->numel() : 0;
    }
    Py_DECREF(cs);
  }
  Py_DECREF(cs_all);
  if (!ok) return nullptr;
  const int place = k > 0 && all_cpu ? 1 : (k > 0 && all_cuda ? 2 : 0);
  PyObject* n_list = PyList_New(k);
  PyObject* f_list = PyList_New(k);
  PyObject* p_list = contiguous ? PyList_New(static_cast<Py_ssize_t>(ts.size())) : nullptr;
  bool built = n_list && f_list && (!contiguous || p_list);
  for (Py_ssize_t i = 0; built && i < k; ++i) {
    PyObject* a = PyLong_FromLongLong(numels[static_cast<size_t>(i)]);
    PyObject* b = PyLong_FromSsize_t(fans[static_cast<size_t>(i)]);
    if (!a || !b) {
      Py_XDECREF(a);
      Py_XDECREF(b);
      built = false;
      break;
    }
    PyList_SET_ITEM(n_list, i, a);
    PyList_SET_ITEM(f_list, i, b);
  }
  for (size_t q = 0; built && contiguous && q < ts.size(); ++q) {
    PyObject* v = PyLong_FromVoidPtr(const_cast<void*>(ts[q]->const_data_ptr()));
    if (!v) {
      built = false;
      break;
    }
    PyList_SET_ITEM(p_list, static_cast<Py_ssize_t>(q), v);
  }
  if (!built) {
    Py_XDECREF(n_list);
    Py_XDECREF(f_list);
    Py_XDECREF(p_list);
    return nullptr;
  }
  PyObject* ptrs = p_list;
  if (!ptrs) {
    ptrs = Py_None;
    Py_INCREF(ptrs);
  }
  return Py_BuildValue("(NiiNNN)", PyBool_FromLong(same_dtype), place, place == 2 ? dev_index : -1, n_list,
                       f_list, ptrs);
}

// checked_params(module, signature) -> module_params(module) if it matches the
// signature, else None
PyObject* py_checked_params(PyObject*, PyObject* args) {
  PyObject *module, *sig;
  if (!PyArg_ParseTuple(args, "OO", &module, &sig)) return nullptr;
  const Sig* s = sig_of(sig);
  if (!s) return nullptr;
  PyObject* ps = py_module_params(nullptr, module);
  if (!ps) return nullptr;
  const int ok = matches_sig(ps, *s);  // a list is its own PySequence_Fast
  if (ok == 1) return ps;
  Py_DECREF(ps);
  if (ok < 0) return nullptr;
  Py_RETURN_NONE;
}

// flat_run(params, idx, byte_offsets, total_elems) -> True iff the dtype group
// params[idx] already is one flat arena: every tensor contiguous and
// byte_offsets[j] bytes after params[idx[0]], and total_elems elements from
// the first one still inside its storage (adjacent separate allocations are
// not an arena)
PyObject* py_flat_run(PyObject*, PyObject* args) {
  PyObject *params, *idx, *offs;
  unsigned long long total;
  if (!PyArg_ParseTuple(args, "OOOK", &params, &idx, &offs, &total)) return nullptr;
  PyObject* row = PyTuple_Pack(1, params);
  if (!row) return nullptr;
  std::vector<const at::Tensor*> ts;
  Py_ssize_t n, t;
  const bool got = row_tensors(row, idx, ts, &n, &t);
  Py_DECREF(row);
  if (!got) return nullptr;
  PyObject* os = PySequence_Fast(offs, "byte_offsets must be a sequence");
  if (!os) return nullptr;
  if (PySequence_Fast_GET_SIZE(os) != t) {
    Py_DECREF(os);
    PyErr_SetString(PyExc_ValueError, "idx and byte_offsets differ in length");
    return nullptr;
  }
  bool flat = t > 0;
  try {
    const auto base = reinterpret_cast<uintptr_t>(flat ? ts[0]->const_data_ptr() : nullptr);
    for (Py_ssize_t j = 0; flat && j < t; ++j) {
      const size_t off = PyLong_AsSize_t(PySequence_Fast_GET_ITEM(os, j));
      if (PyErr_Occurred()) {
        Py_DECREF(os);
        return nullptr;
      }
      flat = reinterpret_cast<uintptr_t>(ts[j]->const_data_ptr()) - base == off && ts[j]->is_contiguous();
    }
    if (flat) {
      const at::Tensor& first = *ts[0];
      flat = first.has_storage() &&
             first.storage().nbytes() >= (static_cast<size_t>(first.storage_offset()) + total) * first.element_size();
    }
  } catch (const std::exception&) {  // tensors without a plain storage (sparse, nested, ...)
    flat = false;
  }
  Py_DECREF(os);
  return PyBool_FromLong(flat);
}

// ---- the output module's parameters: views of the reduced arena --------------
//
int memo_set(PyObject* memo, PyObject* v, PyObject* value);  // memo[id(v)] = value (below)
//
// A layout's view specs [(shape, strides, element offset), ...] as C++
// values, cached by the identity of the list like signatures above.
struct ViewSpecs {
  std::vector<std::vector<int64_t>> shapes, strides;
  std::vector<int64_t> offsets;
};
std::vector<std::pair<PyObject*, ViewSpecs>> g_specs;

bool int_seq(PyObject* o, std::vector<int64_t>& out) {
  PyObject* f = PySequence_Fast(o, "expected a sequence of ints");
  if (!f) return false;
  for (Py_ssize_t d = 0; d < PySequence_Fast_GET_SIZE(f); ++d)
    out.push_back(PyLong_AsLongLong(PySequence_Fast_GET_ITEM(f, d)));
  Py_DECREF(f);
  return !PyErr_Occurred();
}

const ViewSpecs* specs_of(PyObject* specs) {
  for (auto& e : g_specs)
    if (e.first == specs) return &e.second;
  PyObject* ss = PySequence_Fast(specs, "view specs must be a sequence");
  if (!ss) return nullptr;
  ViewSpecs v;
  bool ok = true;
  for (Py_ssize_t k = 0; ok && k < PySequence_Fast_GET_SIZE(ss); ++k) {
    PyObject* e = PySequence_Fast_GET_ITEM(ss, k);
    if (!PyTuple_Check(e) || PyTuple_GET_SIZE(e) != 3) {
      PyErr_SetString(PyExc_TypeError, "view specs are (shape, strides, offset)");
      ok = false;
      break;
    }
    v.shapes.emplace_back();
    v.strides.emplace_back();
    ok = int_seq(PyTuple_GET_ITEM(e, 0), v.shapes.back()) && int_seq(PyTuple_GET_ITEM(e, 1), v.strides.back());
    if (ok) {
      v.offsets.push_back(PyLong_AsLongLong(PyTuple_GET_ITEM(e, 2)));
      ok = !PyErr_Occurred();
    }
  }
  Py_DECREF(ss);
  if (!ok) return nullptr;
  if (g_specs.size() == kSigCache) {
    Py_DECREF(g_specs.front().first);
    g_specs.erase(g_specs.begin());
  }
  Py_INCREF(specs);
  g_specs.emplace_back(specs, std::move(v));
  return &g_specs.back().second;
}

// fill_param_views(memo, arena, specs, params, idx): for each j, memo[id(p)]
// = nn.Parameter(arena.as_strided(*specs[j]) + offset, p.requires_grad) with
// p = params[idx[j]] -- what torch.Tensor._make_subclass(nn.Parameter, view,
// requires_grad) builds (detach, metadata changes allowed, requires_grad set,
// wrapped as the Parameter class), without a Python call per parameter.
PyObject* py_fill_param_views(PyObject*, PyObject* args) {
  PyObject *memo, *arena, *specs, *params, *idx;
  if (!PyArg_ParseTuple(args, "O!OOOO", &PyDict_Type, &memo, &arena, &specs, &params, &idx)) return nullptr;
  const at::Tensor* a = tensor_of(arena);
  if (!a) return nullptr;
  const ViewSpecs* v = specs_of(specs);
  if (!v) return nullptr;
  PyObject* row = PyTuple_Pack(1, params);
  if (!row) return nullptr;
  std::vector<const at::Tensor*> ps;
  Py_ssize_t n, t;
  const bool got = row_tensors(row, idx, ps, &n, &t);
  if (!got) {
    Py_DECREF(row);
    return nullptr;
  }
  if (static_cast<size_t>(t) != v->offsets.size()) {
    Py_DECREF(row);
    PyErr_SetString(PyExc_ValueError, "idx and view specs differ in length");
    return nullptr;
  }
  PyObject* rs = PySequence_Fast(params, "params must be a sequence");
  PyObject* ks = rs ? PySequence_Fast(idx, "idx must be a sequence") : nullptr;
  bool ok = ks != nullptr;
  try {
    const int64_t base = a->storage_offset();
    for (Py_ssize_t j = 0; ok && j < t; ++j) {
      // the detached view built directly (what as_strided(...).detach()
      // yields, minus two dispatcher round trips): a TensorImpl on the
      // arena's storage with its key set and dtype, then this parameter's
      // sizes, strides and offset. Its own version counter, like the
      // reference's separately allocated deepcopy parameters.
      c10::intrusive_ptr<c10::TensorImpl> impl =
          a->unsafeGetTensorImpl()->shallow_copy_and_detach(c10::VariableVersion(0), true);
      impl->set_sizes_and_strides(v->shapes[j], v->strides[j], base + v->offsets[j]);
      at::Tensor data(std::move(impl));
      data.set_requires_grad(ps[j]->requires_grad());
      PyObject* q = THPVariable_Wrap(data, reinterpret_cast<PyTypeObject*>(ParameterClass));
      PyObject* p = q ? PySequence_Fast_GET_ITEM(rs, PyLong_AsSsize_t(PySequence_Fast_GET_ITEM(ks, j))) : nullptr;
      ok = q && p && memo_set(memo, p, q) == 0;
      Py_XDECREF(q);
    }
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    ok = false;
  }
  Py_XDECREF(ks);
  Py_XDECREF(rs);
  Py_DECREF(row);
  if (!ok) return nullptr;
  Py_RETURN_NONE;
}

// ---- one device task's reduce: pointers collected and the library called ----
//
// dlsim_wreduce_tensors (include/dlsim.h) bound by address from _native.py, so
// a task whose models keep their parameters in separate device tensors makes
// one call from Python: the data pointers of rows[i][k] for k in idx go
// straight into the C arrays (no list of ints, no ctypes marshalling).
using WreduceTensorsFn = int (*)(const void* const*, int, int, const size_t*, const float*, void* const*, int, int,
                                 void*);
WreduceTensorsFn g_wreduce_tensors = nullptr;

PyObject* py_bind_wreduce_tensors(PyObject*, PyObject* addr) {
  void* p = PyLong_AsVoidPtr(addr);
  if (!p && PyErr_Occurred()) return nullptr;
  g_wreduce_tensors = reinterpret_cast<WreduceTensorsFn>(p);
  Py_RETURN_NONE;
}

// wreduce_rows(rows, idx, numels, weights_f32, out_base, out_offsets, dtype,
//              mode, stream, device) -> rc, or None (nothing launched) if a
// tensor is not contiguous or not on CUDA device `device`. rows[i][idx[j]] is
// tensor j of model i; numels[j] its element count; out_offsets[j] its byte
// offset from out_base; weights_f32 a C-contiguous buffer of len(rows) floats.
PyObject* py_wreduce_rows(PyObject*, PyObject* args) {
  PyObject *rows, *idx, *numels, *weights, *offsets;
  unsigned long long out_base, stream;
  int dtype, mode, device;
  if (!PyArg_ParseTuple(args, "OOOOKOiiKi", &rows, &idx, &numels, &weights, &out_base, &offsets, &dtype, &mode,
                        &stream, &device))
    return nullptr;
  if (!g_wreduce_tensors) {
    PyErr_SetString(PyExc_RuntimeError, "bind_wreduce_tensors was not called");
    return nullptr;
  }
  std::vector<const at::Tensor*> ts;
  Py_ssize_t n, t;
  if (!row_tensors(rows, idx, ts, &n, &t)) return nullptr;
  PyObject* ns = PySequence_Fast(numels, "numels must be a sequence");
  PyObject* os = ns ? PySequence_Fast(offsets, "out_offsets must be a sequence") : nullptr;
  PyObject* result = nullptr;
  Py_buffer wb{};
  bool have_wb = false;
  do {
    if (!os) break;
    if (PySequence_Fast_GET_SIZE(ns) != t || PySequence_Fast_GET_SIZE(os) != t) {
      PyErr_SetString(PyExc_ValueError, "idx, numels and out_offsets differ in length");
      break;
    }
    if (PyObject_GetBuffer(weights, &wb, PyBUF_C_CONTIGUOUS) < 0) break;
    have_wb = true;
    if (wb.len != static_cast<Py_ssize_t>(n * sizeof(float))) {
      PyErr_SetString(PyExc_ValueError, "weights_f32 must hold one float per model");
      break;
    }
    std::vector<const void*> ins(ts.size());
    std::vector<size_t> ne(static_cast<size_t>(t));
    std::vector<void*> outs(static_cast<size_t>(t));
    for (Py_ssize_t j = 0; j < t; ++j) {
      ne[j] = PyLong_AsSize_t(PySequence_Fast_GET_ITEM(ns, j));
      outs[j] = reinterpret_cast<void*>(
          static_cast<uintptr_t>(out_base + PyLong_AsSize_t(PySequence_Fast_GET_ITEM(os, j))));
    }
    if (PyErr_Occurred()) break;
    bool here = true;
    for (size_t q = 0; here && q < ts.size(); ++q) {
      const at::Tensor& x = *ts[q];
      here = x.is_cuda() && x.get_device() == device && x.is_contiguous();
      ins[q] = x.const_data_ptr();
    }
    if (!here) {
      Py_INCREF(Py_None);
      result = Py_None;
      break;
    }
    int rc;
    const float* w = static_cast<const float*>(wb.buf);
    Py_BEGIN_ALLOW_THREADS
    rc = g_wreduce_tensors(ins.data(), static_cast<int>(n), static_cast<int>(t), ne.data(), w, outs.data(), dtype,
                           mode, reinterpret_cast<void*>(static_cast<uintptr_t>(stream)));
    Py_END_ALLOW_THREADS
    result = PyLong_FromLong(rc);
  } while (false);
  if (have_wb) PyBuffer_Release(&wb);
  Py_XDECREF(os);
  Py_XDECREF(ns);
  return result;
}

// ---- a small host task's zero-copy reduce in one call (round 6) -------------
//
// dlsim_host_wreduce_zc (include/dlsim.h) bound by address from _native.py:
// arena._host_zc_aggregate hands over the models' parameter lists, and the
// data pointers, element counts and weights go to the library from here --
// no Python list of pointers, no ctypes arrays.
using HostZcFn = int (*)(int, int, const void* const*, const size_t*, const float*, void*, size_t, void*, int, int,
                         int, void*);
HostZcFn g_host_zc = nullptr;

PyObject* py_bind_host_zc(PyObject*, PyObject* addr) {
  void* p = PyLong_AsVoidPtr(addr);
  if (!p && PyErr_Occurred()) return nullptr;
  g_host_zc = reinterpret_cast<HostZcFn>(p);
  Py_RETURN_NONE;
}

// host_zc(rows, idx, numels, weights_f32, staging, host_out, dtype, mode,
//         threads, stream) -> rc, or None (nothing launched) if a tensor is
// not a contiguous host tensor. rows[i][idx[j]] is tensor j of model i;
// numels[j] its element count; weights_f32 a C-contiguous buffer of len(rows)
// floats; staging a page-locked 2-D [>= n, stride] tensor; host_out a
// page-locked tensor of sum(numels) elements.
PyObject* py_host_zc(PyObject*, PyObject* args) {
  PyObject *rows, *idx, *numels, *weights, *staging, *host;
  int dtype, mode, threads;
  unsigned long long stream;
  if (!PyArg_ParseTuple(args, "OOOOOOiiiK", &rows, &idx, &numels, &weights, &staging, &host, &dtype, &mode, &threads,
                        &stream))
    return nullptr;
  if (!g_host_zc) {
    PyErr_SetString(PyExc_RuntimeError, "bind_host_zc was not called");
    return nullptr;
  }
  std::vector<const at::Tensor*> ts;
  Py_ssize_t n, t;
  if (!row_tensors(rows, idx, ts, &n, &t)) return nullptr;
  for (const at::Tensor* x : ts)
    if (!x->is_contiguous() || !x->is_cpu()) Py_RETURN_NONE;
  const at::Tensor* st = tensor_of(staging);
  const at::Tensor* ho = st ? tensor_of(host) : nullptr;
  if (!ho) return nullptr;
  if (st->dim() != 2 || !st->is_cpu() || !ho->is_cpu()) {
    PyErr_SetString(PyExc_ValueError, "staging: a page-locked [n, stride] host tensor; host_out: a host tensor");
    return nullptr;
  }
  PyObject* ns = PySequence_Fast(numels, "numels must be a sequence");
  if (!ns) return nullptr;
  PyObject* result = nullptr;
  Py_buffer wb{};
  bool have_wb = false;
  do {
    if (PySequence_Fast_GET_SIZE(ns) != t) {
      PyErr_SetString(PyExc_ValueError, "idx and numels differ in length");
      break;
    }
    if (PyObject_GetBuffer(weights, &wb, PyBUF_C_CONTIGUOUS) < 0) break;
    have_wb = true;
    if (wb.len != static_cast<Py_ssize_t>(n * sizeof(float))) {
      PyErr_SetString(PyExc_ValueError, "weights_f32 must hold one float per model");
      break;
    }
    std::vector<size_t> ne(static_cast<size_t>(t));
    bool ok = true;
    for (Py_ssize_t j = 0; ok && j < t; ++j) {
      ne[static_cast<size_t>(j)] = PyLong_AsSize_t(PySequence_Fast_GET_ITEM(ns, j));
      ok = !PyErr_Occurred();
    }
    if (!ok) break;
    std::vector<const void*> ptrs(ts.size());
    for (size_t q = 0; q < ts.size(); ++q) ptrs[q] = ts[q]->const_data_ptr();
    const float* w = static_cast<const float*>(wb.buf);
    void* sp = st->data_ptr();
    const size_t stride = static_cast<size_t>(st->stride(0));
    void* hp = ho->data_ptr();
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = g_host_zc(static_cast<int>(n), static_cast<int>(t), ptrs.data(), ne.data(), w, sp, stride, hp, dtype, mode,
                   threads, reinterpret_cast<void*>(static_cast<uintptr_t>(stream)));
    Py_END_ALLOW_THREADS
    result = PyLong_FromLong(rc);
  } while (false);
  if (have_wb) PyBuffer_Release(&wb);
  Py_DECREF(ns);
  return result;
}

// ---- many device tasks' reduces in one library call ------------------------
//
// RoundExecutor's wave (dasklearn_amd/batch.py): every task whose models keep
// their parameters in separate device tensors becomes one sub-task per
// tensor, all of them through one dlsim_wreduce_batched call (its
// kernel-argument batches), instead of one wreduce_rows call per task.
using WreduceBatchedFn = int (*)(int, const int*, const void* const*, const float*, void* const*, const size_t*, int,
                                 int, void*);
WreduceBatchedFn g_wreduce_batched = nullptr;

PyObject* py_bind_wreduce_batched(PyObject*, PyObject* addr) {
  void* p = PyLong_AsVoidPtr(addr);
  if (!p && PyErr_Occurred()) return nullptr;
  g_wreduce_batched = reinterpret_cast<WreduceBatchedFn>(p);
  Py_RETURN_NONE;
}

// wreduce_rows_multi(tasks, dtype, mode, stream, device) -> rc, or None
// (nothing launched) if a tensor is not contiguous or not on CUDA device
// `device`. tasks: [(rows, idx, numels, weights_f32, out_base, out_offsets)],
// each as wreduce_rows takes them. Sub-tasks of zero elements are skipped.
PyObject* py_wreduce_rows_multi(PyObject*, PyObject* args) {
  PyObject* tasks;
  unsigned long long stream;
  int dtype, mode, device;
  if (!PyArg_ParseTuple(args, "OiiKi", &tasks, &dtype, &mode, &stream, &device)) return nullptr;
  if (!g_wreduce_batched) {
    PyErr_SetString(PyExc_RuntimeError, "bind_wreduce_batched was not called");
    return nullptr;
  }
  PyObject* tl = PySequence_Fast(tasks, "tasks must be a sequence");
  if (!tl) return nullptr;
  std::vector<int> fan;
  std::vector<const void*> ins;
  std::vector<float> ws;
  std::vector<void*> outs;
  std::vector<size_t> ne;
  bool ok = true, here = true;
  std::vector<const at::Tensor*> ts;
  for (Py_ssize_t q = 0; ok && here && q < PySequence_Fast_GET_SIZE(tl); ++q) {
    PyObject *rows, *idx, *numels, *weights, *offsets;
    unsigned long long out_base;
    if (!PyArg_ParseTuple(PySequence_Fast_GET_ITEM(tl, q), "OOOOKO", &rows, &idx, &numels, &weights, &out_base,
                          &offsets)) {
      ok = false;
      break;
    }
    Py_ssize_t n, t;
    if (!row_tensors(rows, idx, ts, &n, &t)) {
      ok = false;
      break;
    }
    PyObject* ns = PySequence_Fast(numels, "numels must be a sequence");
    PyObject* os = ns ? PySequence_Fast(offsets, "out_offsets must be a sequence") : nullptr;
    Py_buffer wb{};
    bool have_wb = false;
    do {
      if (!os) {
        ok = false;
        break;
      }
      if (PySequence_Fast_GET_SIZE(ns) != t || PySequence_Fast_GET_SIZE(os) != t) {
        PyErr_SetString(PyExc_ValueError, "idx, numels and out_offsets differ in length");
        ok = false;
        break;
      }
      if (PyObject_GetBuffer(weights, &wb, PyBUF_C_CONTIGUOUS) < 0) {
        ok = false;
        break;
      }
      have_wb = true;
      if (wb.len != static_cast<Py_ssize_t>(n * sizeof(float))) {
        PyErr_SetString(PyExc_ValueError, "weights_f32 must hold one float per model");
        ok = false;
        break;
      }
      const float* w = static_cast<const float*>(wb.buf);
      for (Py_ssize_t j = 0; here && j < t; ++j) {
        const size_t e = PyLong_AsSize_t(PySequence_Fast_GET_ITEM(ns, j));
        const size_t o = PyLong_AsSize_t(PySequence_Fast_GET_ITEM(os, j));
        if (PyErr_Occurred()) {
          ok = false;
          break;
        }
        for (Py_ssize_t i = 0; i < n; ++i) {
          const at::Tensor& x = *ts[static_cast<size_t>(i * t + j)];
          here = here && x.is_cuda() && x.get_device() == device && x.is_contiguous();
        }
        if (!here || e == 0) continue;
        fan.push_back(static_cast<int>(n));
        for (Py_ssize_t i = 0; i < n; ++i) {
          ins.push_back(ts[static_cast<size_t>(i * t + j)]->const_data_ptr());
          ws.push_back(w[i]);
        }
        outs.push_back(reinterpret_cast<void*>(static_cast<uintptr_t>(out_base + o)));
        ne.push_back(e);
      }
    } while (false);
    if (have_wb) PyBuffer_Release(&wb);
    Py_XDECREF(os);
    Py_XDECREF(ns);
  }
  Py_DECREF(tl);
  if (!ok) return nullptr;
  if (!here) Py_RETURN_NONE;
  if (fan.empty()) return PyLong_FromLong(0);
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = g_wreduce_batched(static_cast<int>(fan.size()), fan.data(), ins.data(), ws.data(), outs.data(), ne.data(),
                         dtype, mode, reinterpret_cast<void*>(static_cast<uintptr_t>(stream)));
  Py_END_ALLOW_THREADS
  return PyLong_FromLong(rc);
}

// ---- module clone (arena._clone_module restated; see its docstring) --------
//
// copy.deepcopy(models[0]) with the parameters taken from the memo: for the
// reference's GNLeNet (16 modules, ~20 attributes each) this walk is the
// largest host cost of one aggregate task. The Python version in arena.py is
// the specification; tests/test_host_logic.py compares the two.
struct CloneCtx {
  PyObject* plain_cache = nullptr;    // {cls: kind}
  PyObject* plain_fn = nullptr;       // cls -> kind 0/1/2 (fills plain_cache)
  PyObject* atomic = nullptr;         // frozenset of atomic types
  PyObject* setstate_keys = nullptr;  // frozenset of attribute names
  PyObject* deepcopy = nullptr;       // copy.deepcopy
  PyObject* odict = nullptr;          // collections.OrderedDict
} g_clone;

PyObject* s_modules_key = nullptr;
PyObject* s_params_key = nullptr;
PyObject* s_compiled_key = nullptr;
PyObject* s_new = nullptr;
PyObject* s_setstate = nullptr;

bool key_is(PyObject* k, PyObject* s) {
  return k == s || (PyUnicode_CheckExact(k) && PyUnicode_Compare(k, s) == 0);
}

int is_atomic(PyObject* v) { return PySet_Contains(g_clone.atomic, reinterpret_cast<PyObject*>(Py_TYPE(v))); }

int all_atomic(PyObject* seq) {  // tuple or list
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  PyObject** items = PySequence_Fast_ITEMS(seq);
  for (Py_ssize_t i = 0; i < n; ++i) {
    const int a = is_atomic(items[i]);
    if (a != 1) return a;
  }
  return 1;
}

PyObject* deepcopy(PyObject* v, PyObject* memo) { return PyObject_CallFunctionObjArgs(g_clone.deepcopy, v, memo, nullptr); }

// new reference to memo[id(v)] or nullptr (no error) / nullptr (error set)
PyObject* memo_get(PyObject* memo, PyObject* v) {
  PyObject* key = PyLong_FromVoidPtr(v);
  if (!key) return nullptr;
  PyObject* got = PyDict_GetItemWithError(memo, key);
  Py_DECREF(key);
  Py_XINCREF(got);
  return got;
}

int memo_set(PyObject* memo, PyObject* v, PyObject* value) {
  PyObject* key = PyLong_FromVoidPtr(v);
  if (!key) return -1;
  const int rc = PyDict_SetItem(memo, key, value);
  Py_DECREF(key);
  return rc;
}

PyObject* clone(PyObject* m, PyObject* memo, int depth);

// the mapping `src` (dict or OrderedDict of name -> value) with each value
// passed through `f` (None kept), as an object of src's type
template <class F>
PyObject* map_values(PyObject* src, F&& f) {
  PyObject* d = PyDict_New();
  if (!d) return nullptr;
  Py_ssize_t pos = 0;
  PyObject *name, *v;
  while (PyDict_Next(src, &pos, &name, &v)) {
    PyObject* nv = v == Py_None ? (Py_INCREF(Py_None), Py_None) : f(v);
    if (!nv || PyDict_SetItem(d, name, nv) < 0) {
      Py_XDECREF(nv);
      Py_DECREF(d);
      return nullptr;
    }
    Py_DECREF(nv);
  }
  if (PyDict_CheckExact(src)) return d;
  PyObject* r = PyObject_CallOneArg(reinterpret_cast<PyObject*>(Py_TYPE(src)), d);
  Py_DECREF(d);
  return r;
}

// state[k] for one attribute v of a plain module; returns a new reference,
// Py_None-borrowed sentinel `keep` (leave state[k] as is) or nullptr (error)
PyObject* const kKeep = reinterpret_cast<PyObject*>(1);

PyObject* clone_attr(PyObject* k, PyObject* v, PyObject* memo, int depth) {
  const int at = is_atomic(v);
  if (at < 0) return nullptr;
  if (at) return kKeep;
  if (key_is(k, s_modules_key) && PyDict_Check(v))
    return map_values(v, [&](PyObject* c) { return clone(c, memo, depth + 1); });
  if (key_is(k, s_params_key) && PyDict_Check(v))
    return map_values(v, [&](PyObject* q) -> PyObject* {
      PyObject* got = memo_get(memo, q);
      if (got || PyErr_Occurred()) return got;
      return deepcopy(q, memo);
    });
  if (PyTuple_CheckExact(v)) {
    const int a = all_atomic(v);
    if (a < 0) return nullptr;
    if (a) return kKeep;
  } else if (PyDict_CheckExact(v) || Py_IS_TYPE(v, reinterpret_cast<PyTypeObject*>(g_clone.odict)) ||
             PySet_CheckExact(v)) {
    const Py_ssize_t len = PyObject_Length(v);
    if (len < 0) return nullptr;
    if (len == 0) {
      // exact types through their C constructors (PyODict_New skips the
      // type call and OrderedDict.__init__: 11 hook registries per module)
      PyObject* e = Py_IS_TYPE(v, reinterpret_cast<PyTypeObject*>(g_clone.odict)) &&
                            g_clone.odict == reinterpret_cast<PyObject*>(&PyODict_Type)
                        ? PyODict_New()
                    : PyDict_CheckExact(v) ? PyDict_New()
                    : PySet_CheckExact(v)  ? PySet_New(nullptr)
                                           : PyObject_CallNoArgs(reinterpret_cast<PyObject*>(Py_TYPE(v)));
      // An empty OrderedDict (the hook registries, 11 per module) holds
      // nothing a cycle could pass through; like the empty plain dicts
      // CPython creates untracked, it is re-tracked by the dict insert path
      // (MAINTAIN_TRACKING) the moment a trackable object is put in it. Left
      // tracked, the clones of a 16-module tree add ~180 objects to every
      // collection the process runs.
      if (e && Py_IS_TYPE(e, reinterpret_cast<PyTypeObject*>(g_clone.odict)) && PyObject_GC_IsTracked(e))
        PyObject_GC_UnTrack(e);
      return e;
    }
  } else if (PyList_CheckExact(v)) {
    const int a = all_atomic(v);
    if (a < 0) return nullptr;
    if (a) {
      PyObject* got = memo_get(memo, v);
      if (got || PyErr_Occurred()) return got;
      PyObject* c = PyList_GetSlice(v, 0, PyList_GET_SIZE(v));
      if (!c || memo_set(memo, v, c) < 0) {
        Py_XDECREF(c);
        return nullptr;
      }
      return c;
    }
  }
  return deepcopy(v, memo);
}

// arena._plain_module_class: 0 deepcopy, 1 Module's setstate, 2 own setstate
int plain_class(PyObject* cls) {
  PyObject* kind = PyDict_GetItemWithError(g_clone.plain_cache, cls);
  if (kind) return static_cast<int>(PyLong_AsLong(kind));
  if (PyErr_Occurred()) return -1;
  PyObject* r = PyObject_CallOneArg(g_clone.plain_fn, cls);
  if (!r) return -1;
  const long t = PyLong_AsLong(r);
  Py_DECREF(r);
  return static_cast<int>(t);
}

PyObject* clone(PyObject* m, PyObject* memo, int depth) {
  if (depth > 10000) {
    PyErr_SetString(PyExc_RecursionError, "module tree too deep");
    return nullptr;
  }
  PyObject* got = memo_get(memo, m);
  if (got || PyErr_Occurred()) return got;
  PyObject* cls = reinterpret_cast<PyObject*>(Py_TYPE(m));
  const int plain = plain_class(cls);
  if (plain < 0) return nullptr;
  if (!plain) return deepcopy(m, memo);
  PyObject* newobj = PyObject_CallMethodOneArg(cls, s_new, cls);
  if (!newobj) return nullptr;
  PyObject* state = nullptr;
  PyObject* d = nullptr;
  int ok = -1;
  do {
    if (memo_set(memo, m, newobj) < 0) break;
    d = PyObject_GenericGetDict(m, nullptr);
    if (!d) break;
    state = PyDict_Copy(d);
    if (!state) break;
    // Walk the entries of `state`, this function's private copy of the
    // module's dict: clone_attr runs arbitrary Python (copy.deepcopy,
    // __setstate__) that may mutate the module's dict, but cannot reach
    // `state`, and replacing a value of an existing key keeps PyDict_Next
    // valid (the walk used to hold borrowed references into the
    // module's own dict). k and v are held across the call; a size change of
    // the module's dict raises as the Python specification's
    // `for k, v in d.items()` does; the compiled-call key goes after the walk.
    const Py_ssize_t n0 = PyDict_Size(d);
    Py_ssize_t pos = 0;
    PyObject *k, *v;
    bool drop_compiled = false;
    ok = 0;
    while (ok == 0 && PyDict_Next(state, &pos, &k, &v)) {
      if (key_is(k, s_compiled_key)) {
        drop_compiled = true;
        continue;
      }
      Py_INCREF(k);
      Py_INCREF(v);
      PyObject* nv = clone_attr(k, v, memo, depth);
      if (!nv) ok = -1;
      else if (nv != kKeep) {
        ok = PyDict_SetItem(state, k, nv);
        Py_DECREF(nv);
      }
      Py_DECREF(v);
      Py_DECREF(k);
      if (ok == 0 && PyDict_Size(d) != n0) {
        PyErr_SetString(PyExc_RuntimeError, "dictionary changed size during iteration");
        ok = -1;
      }
    }
    if (ok == 0 && drop_compiled) ok = PyDict_DelItem(state, s_compiled_key);
    if (ok < 0) break;
    // Module.__setstate__ is __dict__.update(state) when the state already has
    // every attribute it would add; a class's own __setstate__ is called
    int complete = plain == 1;
    if (complete) {
      PyObject* it = PyObject_GetIter(g_clone.setstate_keys);
      if (!it) {
        ok = -1;
        break;
      }
      PyObject* key;
      while (complete == 1 && (key = PyIter_Next(it))) {
        complete = PyDict_Contains(state, key);
        Py_DECREF(key);
      }
      Py_DECREF(it);
    }
    if (complete < 0 || PyErr_Occurred()) {
      ok = -1;
      break;
    }
    if (complete) {
      PyObject* nd = PyObject_GenericGetDict(newobj, nullptr);
      ok = nd ? PyDict_Update(nd, state) : -1;
      Py_XDECREF(nd);
    } else {
      PyObject* r = PyObject_CallMethodOneArg(newobj, s_setstate, state);
      ok = r ? 0 : -1;
      Py_XDECREF(r);
    }
  } while (false);
  Py_XDECREF(d);
  Py_XDECREF(state);
  if (ok < 0) {
    Py_DECREF(newobj);
    return nullptr;
  }
  return newobj;
}

PyObject* py_clone_init(PyObject*, PyObject* args) {
  CloneCtx c;
  if (!PyArg_ParseTuple(args, "O!OO!O!OO", &PyDict_Type, &c.plain_cache, &c.plain_fn, &PyFrozenSet_Type, &c.atomic,
                        &PyFrozenSet_Type, &c.setstate_keys, &c.deepcopy, &c.odict))
    return nullptr;
  if (!PyType_Check(c.odict)) {
    PyErr_SetString(PyExc_TypeError, "odict must be a type");
    return nullptr;
  }
  for (PyObject* o : {c.plain_cache, c.plain_fn, c.atomic, c.setstate_keys, c.deepcopy, c.odict}) Py_INCREF(o);
  for (PyObject* o : {g_clone.plain_cache, g_clone.plain_fn, g_clone.atomic, g_clone.setstate_keys, g_clone.deepcopy,
                      g_clone.odict})
    Py_XDECREF(o);
  g_clone = c;
  Py_RETURN_NONE;
}

PyObject* py_clone_module(PyObject*, PyObject* args) {
  PyObject *m, *memo;
  if (!PyArg_ParseTuple(args, "OO!", &m, &PyDict_Type, &memo)) return nullptr;
  if (!g_clone.atomic) {
    PyErr_SetString(PyExc_RuntimeError, "clone_init was not called");
    return nullptr;
  }
  return clone(m, memo, 0);
}

PyMethodDef kMethods[] = {
    {"module_params", py_module_params, METH_O, "list(module.parameters()), in C"},
    {"matches", py_matches, METH_VARARGS, "params match a [(shape, dtype)] signature"},
    {"data_ptrs", py_data_ptrs, METH_VARARGS, "data pointers of rows[i][k] for k in idx, None if not contiguous"},
    {"shm_keys", py_shm_keys, METH_VARARGS, "per model, the identity of its file_system shm storages, or None"},
    {"shm_rows", py_shm_rows, METH_VARARGS,
     "(shm_keys(rows, idx), data_ptrs(rows, idx), content fingerprints) in one pass"},
    {"chunk_scan", py_chunk_scan, METH_O,
     "chunk_scan(chunks) -> (same_dtype, place, device_index, numels, fans, ptrs or None)"},
    {"clone_init", py_clone_init, METH_VARARGS,
     "clone_init(plain_cache, plain_fn, atomic_types, setstate_keys, deepcopy, OrderedDict)"},
    {"clone_module", py_clone_module, METH_VARARGS, "clone_module(module, memo): arena._clone_module in C"},
    {"bind_wreduce_tensors", py_bind_wreduce_tensors, METH_O, "bind dlsim_wreduce_tensors by address"},
    {"bind_wreduce_batched", py_bind_wreduce_batched, METH_O, "bind dlsim_wreduce_batched by address"},
    {"bind_host_zc", py_bind_host_zc, METH_O, "bind dlsim_host_wreduce_zc by address"},
    {"host_zc", py_host_zc, METH_VARARGS,
     "host_zc(rows, idx, numels, weights_f32, staging, host_out, dtype, mode, threads, stream): "
     "dlsim_host_wreduce_zc on the models' data pointers; None if a tensor is not a contiguous host tensor"},
    {"wreduce_rows_multi", py_wreduce_rows_multi, METH_VARARGS,
     "wreduce_rows_multi(tasks, dtype, mode, stream, device): many tasks' tensor rows in one dlsim_wreduce_batched"},
    {"fill_param_views", py_fill_param_views, METH_VARARGS,
     "fill_param_views(memo, arena, specs, params, idx): memo[id(p)] = Parameter view of the arena"},
    {"checked_params", py_checked_params, METH_VARARGS, "module_params(module) if it matches signature, else None"},
    {"flat_run", py_flat_run, METH_VARARGS, "flat_run(params, idx, byte_offsets, total): the group is one arena"},
    {"wreduce_rows", py_wreduce_rows, METH_VARARGS,
     "wreduce_rows(rows, idx, numels, weights_f32, out_base, out_offsets, dtype, mode, stream, device) -> rc or None"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_pyhost", "CPython helpers of the per-task module path", -1,
                       kMethods, nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__pyhost(void) {
  s_parameters = PyUnicode_InternFromString("_parameters");
  s_modules = PyUnicode_InternFromString("_modules");
  s_modules_key = s_modules;
  s_params_key = s_parameters;
  s_compiled_key = PyUnicode_InternFromString("_compiled_call_impl");
  s_new = PyUnicode_InternFromString("__new__");
  s_setstate = PyUnicode_InternFromString("__setstate__");
  if (!s_parameters || !s_modules || !s_compiled_key || !s_new || !s_setstate)
    return nullptr;
  PyObject* mod = PyModule_Create(&kModule);
  if (!mod) return nullptr;
  // The torch build this file was compiled against (torch.__version__ at
  // build time): it reads at::Tensor fields and restates deepcopy against
  // that torch's internals, so arena.py refuses to use it under another.
#ifndef DLSIM_TORCH_VERSION
#error "build with -DDLSIM_TORCH_VERSION=\"<torch.__version__>\" (__graft_entry__.build())"
#endif
  if (PyModule_AddStringConstant(mod, "BUILT_FOR_TORCH", DLSIM_TORCH_VERSION) < 0) {
    Py_DECREF(mod);
    return nullptr;
  }
  return mod;
}
