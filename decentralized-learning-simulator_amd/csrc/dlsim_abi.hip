// dlsim_abi.hip — the C ABI of include/dlsim.h over the gfx950 kernels of
// wreduce_kernels.hpp. Host-side dispatch only: argument checks, choice of
// vector vs scalar kernel, launch shape, kernarg or device-table fan-in, batching
// and its hazard checks, host staging pipelines. The RCCL entry points are in
// sharded_abi.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "abi_common.hpp"
#include "dispatch.hpp"

// Every DLSIM_* switch named below is an A/B switch, read through
// dlsim::ab_getenv: only when DLSIM_AB=1 is set as well (ab_env.hpp).
#include "host_pack.hpp"

namespace dlsim_host __attribute__((visibility("hidden"))) {

// f(Op{}) with the element policy of (dtype, mode). Callers check both first.
template <class F>
int with_policy(int dtype, int mode, F&& f) {
  const bool fast = mode == DLSIM_FAST;
  if (dtype == DLSIM_F32) return fast ? f(dlsim::F32Fast{}) : f(dlsim::F32Exact{});
  if (dtype == DLSIM_BF16) return fast ? f(dlsim::BF16Fast{}) : f(dlsim::BF16Exact{});
  return fast ? f(dlsim::F16Fast{}) : f(dlsim::F16Exact{});
}

// f(Op{}) with the mean policy (element format) of dtype.
template <class F>
int with_mean_policy(int dtype, F&& f) {
  if (dtype == DLSIM_F32) return f(dlsim::F32Mean{});
  if (dtype == DLSIM_BF16) return f(dlsim::BF16Mean{});
  return f(dlsim::F16Mean{});
}

// The chunk mean's policies: the mean ones plus fp64 (chunk_mean_kernels.hpp).
template <class F>
int with_chunk_policy(int dtype, F&& f) {
  if (dtype == DLSIM_F64) return f(dlsim::F64Mean{});
  return with_mean_policy(dtype, f);
}

int dispatch(const void* const* in, int n, const float* w, void* out, size_t nelem, int dtype,
             int mode, hipStream_t st) {
  return with_policy(dtype, mode, [&](auto op) { return run<decltype(op)>(in, n, w, out, nelem, st); });
}

// ---- host staging pipelines (dlsim_host_wreduce, dlsim_host_chunk_mean) -------
// Cross-stream ordering by events. Destroying a recorded event is deferred by
// the runtime until it completes, so the destructor may run right away.
struct StreamLinks {
  std::vector<hipEvent_t> evs;
  int rc = DLSIM_OK;
  void link(hipStream_t from, hipStream_t to, const char* what) {
    if (rc != DLSIM_OK || from == to) return;
    hipEvent_t ev;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      rc = hip_fail(e, what);
      return;
    }
    evs.push_back(ev);
    e = hipEventRecord(ev, from);
    if (e == hipSuccess) e = hipStreamWaitEvent(to, ev, 0);
    if (e != hipSuccess) rc = hip_fail(e, what);
  }
  ~StreamLinks() {
    for (hipEvent_t ev : evs) (void)hipEventDestroy(ev);
  }
};

// Pack `job` on `threads` host threads (the caller's included) and call
// on_units(u, v) on this thread for each run [u, v) of units that completed,
// in order (u = 0 first; a run is every unit already packed when the
// dispatcher looks, so a fast pack hands over long runs the caller can copy
// with one DMA each). Below DLSIM_PACK_HELPERS_MIN_KB of input (read per
// call, A/B probes) the helpers stay asleep: their wake-up costs more than
// they save on sources already in the CPU caches.
constexpr long kPackHelpersMinKB = 1024;
size_t pack_helpers_min_bytes() {
  const char* e = dlsim::ab_getenv("DLSIM_PACK_HELPERS_MIN_KB");
  const long kb = e ? std::strtol(e, nullptr, 10) : kPackHelpersMinKB;
  return static_cast<size_t>(kb > 0 ? kb : 0) << 10;
}

// DLSIM_PACK_THREADS=k (read per call; deployment A/B runs): pack on k
// threads whatever the caller asked for.
int pack_threads(int threads) {
  const char* e = dlsim::ab_getenv("DLSIM_PACK_THREADS");
  const long k = e ? std::strtol(e, nullptr, 10) : 0;
  return k > 0 ? static_cast<int>(std::min<long>(k, 64)) : threads;
}

template <class F>
void pack_and_dispatch(dlsim::PackJob& job, int threads, size_t in_bytes, F&& on_units) {
  threads = pack_threads(threads);
  const int helpers = in_bytes < pack_helpers_min_bytes() ? 0 : std::min(std::max(threads, 1), 64) - 1;
  dlsim::PackPool& pool = dlsim::PackPool::get();
  std::lock_guard<std::mutex> lk(pool.call_mutex());
  if (helpers > 0) pool.start(&job, helpers);
  for (size_t u = 0; u < job.units;) {
    if (job.unit_done(u)) {
      size_t v = u + 1;
      while (v < job.units && job.unit_done(v)) ++v;
      on_units(u, v);
      u = v;
    } else if (!job.run_one()) {
      std::this_thread::yield();
    }
  }
  if (helpers > 0) pool.join();
}

// Smallest H2D run of a one-chunk dlsim_host_wreduce (DLSIM_H2D_MIN_KB, read
// per call: A/B probes; default 1 MiB).
size_t h2d_min_bytes() {
  const char* e = dlsim::ab_getenv("DLSIM_H2D_MIN_KB");
  const long kb = e ? std::strtol(e, nullptr, 10) : 1024;
  return static_cast<size_t>(kb > 0 ? kb : 0) << 10;
}

// dlsim_host_chunk_mean jobs below this many staged bytes take the one-DMA
// path (pack all, one H2D, one batched launch, one D2H).
constexpr size_t kSmallHostJobBytes = size_t{4} << 20;

// Staging layout of dlsim_host_chunk_mean: input rows back to back, each at
// a 256-B aligned offset.
size_t staged_row_elems(size_t n, size_t esz) {
  const size_t al = 256 / esz;
  return (n + al - 1) / al * al;
}

// The results of a small host chunk job in ONE D2H, when that is exact: the
// non-empty outputs, sorted by device address, lie back to back (each starts
// where the previous one ends) and every host output sits at the same offset
// from the first as its device output. Returns DLSIM_OK after queueing the
// one copy, 1 when the layout does not qualify (the caller copies per task),
// or a HIP error code.
int d2h_one_span(int b, void* const* d_outs, void* const* h_outs, const size_t* n_elems, size_t esz,
                 hipStream_t st) {
  struct Part {
    uintptr_t d, h;
    size_t bytes;
  };
  std::vector<Part> parts;
  for (int t = 0; t < b; ++t) {
    if (n_elems[t] == 0) continue;
    if (!h_outs[t]) return 1;
    parts.push_back({reinterpret_cast<uintptr_t>(d_outs[t]), reinterpret_cast<uintptr_t>(h_outs[t]),
                     n_elems[t] * esz});
  }
  if (parts.empty()) return DLSIM_OK;
  std::sort(parts.begin(), parts.end(), [](const Part& x, const Part& y) { return x.d < y.d; });
  const uintptr_t d0 = parts[0].d, h0 = parts[0].h;
  size_t span = 0;
  for (const Part& q : parts) {
    if (q.d - d0 != span || q.h - h0 != span) return 1;  // a gap, an overlap or a different host offset
    span += q.bytes;
  }
  const hipError_t e = hipMemcpyAsync(reinterpret_cast<void*>(h0), reinterpret_cast<const void*>(d0), span,
                                      hipMemcpyDeviceToHost, st);
  return e == hipSuccess ? DLSIM_OK : hip_fail(e, "result D2H");
}

const char* with_mean_policy_name(int dtype, int n, size_t n_elems) {
  const char* name = "";
  with_mean_policy(dtype, [&](auto op) {
    name = kernel_name<decltype(op)>(n, n_elems);
    return 0;
  });
  return name;
}

// CUs of the current device, for the deferred-store grid (dispatch.hpp).
// Read once per device; 256 (MI355X) if the query fails.
int device_cus() {
  constexpr int kMaxDev = 64;
  static int cus[kMaxDev] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return 256;
  int c = __atomic_load_n(&cus[dev], __ATOMIC_RELAXED);
  if (c > 0) return c;
  if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
  __atomic_store_n(&cus[dev], c, __ATOMIC_RELAXED);
  return c;
}

}  // namespace dlsim_host

// the per-policy entries live in the inst_*.hip units
#define DLSIM_EXTERN extern template
DLSIM_ALL_ENTRIES(DLSIM_EXTERN)
#undef DLSIM_EXTERN

using namespace dlsim_host;

extern "C" {

int dlsim_wreduce(const void* const* d_inputs, int n, const float* h_weights, void* d_out,
                  size_t n_elems, int dtype, int mode, void* stream) {
  g_err.clear();
  int rc = check_args(d_inputs, n, h_weights, d_out, n_elems, dtype, mode);
  if (rc != DLSIM_OK) return rc;
  return dispatch(d_inputs, n, h_weights, d_out, n_elems, dtype, mode,
                  static_cast<hipStream_t>(stream));
}

int dlsim_wreduce_f64(const void* const* d_inputs, int n, const double* h_weights, void* d_out, size_t n_elems,
                      int mode, void* stream) {
  g_err.clear();
  int rc = check_args(d_inputs, n, h_weights, d_out, n_elems, DLSIM_F64, mode, true, true);
  if (rc != DLSIM_OK) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (mode == DLSIM_FAST) return run<dlsim::F64Fast>(d_inputs, n, h_weights, d_out, n_elems, st);
  return run<dlsim::F64Exact>(d_inputs, n, h_weights, d_out, n_elems, st);
}

int dlsim_wreduce_tensors(const void* const* d_inputs, int n, int t, const size_t* numels,
                          const float* h_weights, void* const* d_outs, int dtype, int mode,
                          void* stream) {
  g_err.clear();
  if (t < 0) return fail(DLSIM_E_ARG, "t must be >= 0 (got %d)", t);
  if (t > 0 && (!d_inputs || !numels || !d_outs)) return fail(DLSIM_E_ARG, "null array argument");
  if (n < 1) return fail(DLSIM_E_ARG, "n must be >= 1 (got %d)", n);
  if (!h_weights) return fail(DLSIM_E_ARG, "null weights array");
  // Tensor k of every model is one task of fan-in n; the T tasks run as a
  // batch (a handful of launches instead of one per tensor).
  std::vector<const void*> ins(static_cast<size_t>(n) * t);
  std::vector<float> ws(static_cast<size_t>(n) * t);
  std::vector<int> fan(static_cast<size_t>(t), n);
  for (int k = 0; k < t; ++k) {
    for (int i = 0; i < n; ++i) {
      ins[static_cast<size_t>(k) * n + i] = d_inputs[static_cast<size_t>(i) * t + k];
      ws[static_cast<size_t>(k) * n + i] = h_weights[i];
    }
    int rc = check_args(&ins[static_cast<size_t>(k) * n], n, h_weights, d_outs[k], numels[k], dtype, mode);
    if (rc != DLSIM_OK) return fail(rc, "tensor %d: %s", k, g_err.c_str());
  }
  if (t == 0) return DLSIM_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  return with_policy(dtype, mode, [&](auto op) {
    return run_batched<decltype(op)>(t, fan.data(), ins.data(), ws.data(), d_outs, numels, st);
  });
}

int dlsim_wreduce_batched(int b, const int* fan_in, const void* const* d_inputs,
                          const float* h_weights, void* const* d_outs, const size_t* n_elems,
                          int dtype, int mode, void* stream) {
  g_err.clear();
  if (b < 0) return fail(DLSIM_E_ARG, "b must be >= 0 (got %d)", b);
  if (b == 0) return DLSIM_OK;
  if (!fan_in || !d_inputs || !h_weights || !d_outs || !n_elems) return fail(DLSIM_E_ARG, "null array argument");
  size_t off = 0;
  for (int t = 0; t < b; ++t) {
    int rc = check_args(d_inputs + off, fan_in[t], h_weights + off, d_outs[t], n_elems[t], dtype, mode);
    if (rc != DLSIM_OK) return fail(rc, "task %d: %s", t, g_err.c_str());
    off += static_cast<size_t>(fan_in[t]);
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  return with_policy(dtype, mode, [&](auto op) {
    return run_batched<decltype(op)>(b, fan_in, d_inputs, h_weights, d_outs, n_elems, st);
  });
}

int dlsim_batch_table_bytes(int b, const int* fan_in, const size_t* n_elems, int dtype, size_t* bytes) {
  g_err.clear();
  if (b < 0 || (b > 0 && (!fan_in || !n_elems)) || !bytes) return fail(DLSIM_E_ARG, "bad arguments");
  if (!known_dtype(dtype)) return dtype_fail(dtype);
  for (int t = 0; t < b; ++t)
    if (fan_in[t] < 1) return fail(DLSIM_E_ARG, "task %d: fan-in must be >= 1", t);
  TableLayout L;
  const bool ok = with_policy(dtype, DLSIM_EXACT, [&](auto op) {
    return table_layout<decltype(op)>(b, fan_in, n_elems, &L) ? 1 : 0;
  }) != 0;
  if (!ok) return fail(DLSIM_E_ARG, "batch too large");
  *bytes = L.bytes;
  return DLSIM_OK;
}

int dlsim_batch_table_fill(int b, const int* fan_in, const void* const* d_inputs, const float* h_weights,
                           void* const* d_outs, const size_t* n_elems, int dtype, void* h_table,
                           size_t table_bytes) {
  g_err.clear();
  if (b < 0 || !h_table) return fail(DLSIM_E_ARG, "bad arguments");
  if (b > 0 && (!fan_in || !d_inputs || !h_weights || !d_outs || !n_elems))
    return fail(DLSIM_E_ARG, "null array argument");
  size_t off = 0;
  for (int t = 0; t < b; ++t) {
    int rc = check_args(d_inputs + off, fan_in[t], h_weights + off, d_outs[t], n_elems[t], dtype, DLSIM_EXACT);
    if (rc != DLSIM_OK) return fail(rc, "task %d: %s", t, g_err.c_str());
    off += static_cast<size_t>(fan_in[t]);
  }
  return with_policy(dtype, DLSIM_EXACT, [&](auto op) {
    return table_fill<decltype(op)>(b, fan_in, d_inputs, h_weights, d_outs, n_elems, h_table, table_bytes);
  });
}

int dlsim_batch_table_launch(const void* h_table, const void* d_table, int dtype, int mode, void* stream) {
  g_err.clear();
  if (!h_table || !d_table) return fail(DLSIM_E_ARG, "null table");
  if (!known_dtype(dtype)) return dtype_fail(dtype);
  if (mode != DLSIM_EXACT && mode != DLSIM_FAST) return fail(DLSIM_E_MODE, "unsupported mode %d", mode);
  hipStream_t st = static_cast<hipStream_t>(stream);
  return with_policy(dtype, mode, [&](auto op) { return table_launch<decltype(op)>(h_table, d_table, st); });
}

int dlsim_mean(const void* const* d_inputs, int n, void* d_out, size_t n_elems, int dtype,
               void* stream) {
  g_err.clear();
  int rc = check_args(d_inputs, n, nullptr, d_out, n_elems, dtype, DLSIM_EXACT, false);
  if (rc != DLSIM_OK) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const float div = static_cast<float>(n);
  return with_mean_policy(dtype, [&](auto op) {
    return run<decltype(op)>(d_inputs, n, nullptr, d_out, n_elems, st, div);
  });
}

int dlsim_mean_batched(int b, const int* fan_in, const void* const* d_inputs, void* const* d_outs,
                       const size_t* n_elems, int dtype, void* stream) {
  g_err.clear();
  if (b < 0) return fail(DLSIM_E_ARG, "b must be >= 0 (got %d)", b);
  if (b == 0) return DLSIM_OK;
  if (!fan_in || !d_inputs || !d_outs || !n_elems) return fail(DLSIM_E_ARG, "null array argument");
  size_t off = 0;
  std::vector<float> divs(static_cast<size_t>(b));
  for (int t = 0; t < b; ++t) {
    int rc = check_args(d_inputs + off, fan_in[t], nullptr, d_outs[t], n_elems[t], dtype, DLSIM_EXACT, false);
    if (rc != DLSIM_OK) return fail(rc, "task %d: %s", t, g_err.c_str());
    off += static_cast<size_t>(fan_in[t]);
    divs[t] = static_cast<float>(fan_in[t]);
  }
  const std::vector<float> ones(off, 1.0f);  // unused by the mean policies
  hipStream_t st = static_cast<hipStream_t>(stream);
  return with_mean_policy(dtype, [&](auto op) {
    return run_batched<decltype(op)>(b, fan_in, d_inputs, ones.data(), d_outs, n_elems, st, divs.data());
  });
}

size_t dlsim_chunk_mean_ilp_begin(int m, size_t n_elems, int cpu_threads) {
  return chunk_mean_ilp_begin(m, n_elems, cpu_threads);
}

int dlsim_chunk_mean_batched(int b, const int* fan_in, const void* const* d_inputs, void* const* d_outs,
                             const size_t* n_elems, int dtype, int cpu_threads, void* stream) {
  g_err.clear();
  if (b < 0) return fail(DLSIM_E_ARG, "b must be >= 0 (got %d)", b);
  if (b == 0) return DLSIM_OK;
  if (!fan_in || !d_inputs || !d_outs || !n_elems) return fail(DLSIM_E_ARG, "null array argument");
  if (cpu_threads < 1) return fail(DLSIM_E_ARG, "cpu_threads must be >= 1 (got %d)", cpu_threads);
  size_t off = 0;
  for (int t = 0; t < b; ++t) {
    int rc = check_args(d_inputs + off, fan_in[t], nullptr, d_outs[t], n_elems[t], dtype, DLSIM_EXACT, false, true);
    if (rc != DLSIM_OK) return fail(rc, "task %d: %s", t, g_err.c_str());
    if (fan_in[t] > 65535) return fail(DLSIM_E_ARG, "task %d: fan-in %d > 65535", t, fan_in[t]);
    if (n_elems[t] * elem_bytes(dtype) >= kMaxLaunchOutBytes)
      return fail(DLSIM_E_ARG, "task %d: chunk of %zu elements is >= 2 GiB", t, n_elems[t]);
    off += static_cast<size_t>(fan_in[t]);
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  return with_chunk_policy(dtype, [&](auto op) {
    return run_chunk_mean<decltype(op)>(b, fan_in, d_inputs, d_outs, n_elems, cpu_threads, st);
  });
}

int dlsim_host_wreduce(int n, int t, const void* const* h_srcs, const size_t* numels,
                       const float* h_weights, void* h_staging, void* d_rows, size_t row_stride,
                       void* d_out, void* h_out, int dtype, int mode, size_t chunk_elems, int threads,
                       void* stream, void* h2d_stream, void* d2h_stream) {
  g_err.clear();
  if (!known_dtype(dtype)) return dtype_fail(dtype);
  if (mode != DLSIM_EXACT && mode != DLSIM_FAST) return fail(DLSIM_E_MODE, "unsupported mode %d", mode);
  if (n < 1 || t < 0) return fail(DLSIM_E_ARG, "need n >= 1 and t >= 0 (got %d, %d)", n, t);
  if (!h_weights || (t > 0 && (!h_srcs || !numels))) return fail(DLSIM_E_ARG, "null array argument");
  const size_t esz = elem_bytes(dtype);
  size_t total = 0;
  for (int k = 0; k < t; ++k) total += numels[k];
  if (total == 0) return DLSIM_OK;
  if (!h_staging || !d_rows || !d_out) return fail(DLSIM_E_ARG, "null staging, rows or output");
  if (!aligned16(h_staging) || !aligned16(d_rows) || row_stride % 8 != 0)
    return fail(DLSIM_E_ARG, "staging rows must be 16-B aligned with a stride that is a multiple of 8");
  if (row_stride < total) return fail(DLSIM_E_ARG, "row_stride %zu < %zu elements", row_stride, total);
  {
    const uintptr_t r0 = reinterpret_cast<uintptr_t>(d_rows), r1 = r0 + static_cast<size_t>(n) * row_stride * esz;
    const uintptr_t o0 = reinterpret_cast<uintptr_t>(d_out), o1 = o0 + total * esz;
    if (o0 < r1 && r0 < o1) return fail(DLSIM_E_ARG, "d_out overlaps the device staging rows");
  }
  for (size_t j = 0; j < static_cast<size_t>(n) * t; ++j)
    if (!h_srcs[j] && numels[j % t] > 0) return fail(DLSIM_E_ARG, "null source pointer at index %zu", j);
  const size_t chunk = chunk_elems == 0 || chunk_elems >= total ? total : (chunk_elems + 1023) / 1024 * 1024;
  const size_t n_chunks = (total + chunk - 1) / chunk;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // One chunk has nothing to overlap (its H2D, reduce and D2H are serial):
  // everything on `stream`, without the cross-stream event waits, whose
  // signalling latency a small task would pay several times.
  const bool side = n_chunks > 1;
  hipStream_t h2d = side && h2d_stream ? static_cast<hipStream_t>(h2d_stream) : st;
  hipStream_t d2h = side && d2h_stream ? static_cast<hipStream_t>(d2h_stream) : st;
  char* stage = static_cast<char*>(h_staging);
  char* rows = static_cast<char*>(d_rows);
  char* out = static_cast<char*>(d_out);
  const size_t row_bytes = row_stride * esz;

  // Units u = c * n + i (chunk c of model i), slices in that order.
  dlsim::PackJob job;
  {
    std::vector<size_t> off(static_cast<size_t>(t) + 1, 0);
    for (int k = 0; k < t; ++k) off[k + 1] = off[k] + numels[k];
    for (size_t c = 0; c < n_chunks; ++c) {
      const size_t c0 = c * chunk, c1 = std::min(total, c0 + chunk);
      const int k0 = static_cast<int>(std::upper_bound(off.begin(), off.end(), c0) - off.begin()) - 1;
      for (int i = 0; i < n; ++i) {
        const uint32_t u = static_cast<uint32_t>(c * n + i);
        for (int k = k0; k < t && off[k] < c1; ++k) {
          const size_t a = std::max(c0, off[k]), b = std::min(c1, off[k + 1]);
          if (a >= b) continue;
          const char* src = static_cast<const char*>(h_srcs[static_cast<size_t>(i) * t + k]);
          job.add(u, src + (a - off[k]) * esz, stage + i * row_bytes + a * esz, (b - a) * esz);
        }
      }
    }
    job.seal(n_chunks * n);
  }

  // `stream` -> copy streams before the first copy (earlier work on the
  // rows); per chunk, H2D -> reduce and reduce -> D2H; D2H -> `stream` at the
  // end (every H2D is already ordered before its chunk's reduce).
  StreamLinks ln;
  ln.link(st, h2d, "order H2D after stream");
  if (h_out) ln.link(st, d2h, "order D2H after stream");
  std::vector<const void*> ins(static_cast<size_t>(n));
  // Once every model's share of chunk c is on the device: reduce it, D2H it.
  auto finish_chunk = [&](size_t c) {
    const size_t c0 = c * chunk, c1 = std::min(total, c0 + chunk);
    ln.link(h2d, st, "order reduce after H2D");
    if (ln.rc != DLSIM_OK) return;
    for (int r = 0; r < n; ++r) ins[r] = rows + r * row_bytes + c0 * esz;
    ln.rc = dispatch(ins.data(), n, h_weights, out + c0 * esz, c1 - c0, dtype, mode, st);
    if (ln.rc != DLSIM_OK || !h_out) return;
    ln.link(st, d2h, "order D2H after reduce");
    if (ln.rc != DLSIM_OK) return;
    const hipError_t e = hipMemcpyAsync(static_cast<char*>(h_out) + c0 * esz, out + c0 * esz, (c1 - c0) * esz,
                                        hipMemcpyDeviceToHost, d2h);
    if (e != hipSuccess) ln.rc = hip_fail(e, "result D2H");
  };
  // One chunk: packed rows go H2D in runs of at least min_dma bytes (the last
  // run whatever is left). A DMA costs ~8 us of copy-engine time beyond its
  // bytes, so one per 341 KB GNLeNet row made the copies, not the pack, the
  // task's critical path (7 rows: ~105 us against 50 us for one 2.4 MB DMA);
  // two runs overlap the first one's copy with the rest of the pack
  // (DLSIM_H2D_MIN_KB overrides the 1 MiB, for A/B runs).
  const size_t min_dma = h2d_min_bytes();
  size_t pending = 0;  // first row not yet sent (one chunk)
  pack_and_dispatch(job, threads, total * esz * n, [&](size_t u0, size_t u1) {
    if (n_chunks == 1) {
      if (ln.rc != DLSIM_OK) return;
      const size_t j = u1;  // rows [pending, j) are packed
      if (j < static_cast<size_t>(n) && (j - pending) * row_bytes < min_dma) return;
      const size_t o = pending * row_bytes;
      const size_t bytes = (j - pending - 1) * row_bytes + total * esz;
      const hipError_t e = hipMemcpyAsync(rows + o, stage + o, bytes, hipMemcpyHostToDevice, h2d);
      if (e != hipSuccess) {
        ln.rc = hip_fail(e, "staging H2D");
        return;
      }
      pending = j;
      if (j == static_cast<size_t>(n)) finish_chunk(0);
      return;
    }
    for (size_t u = u0; u < u1 && ln.rc == DLSIM_OK; ++u) {
      // several chunks: one DMA per unit (model i's share of chunk c, ~8 MiB)
      const size_t c = u / n, i = u % n;
      const size_t c0 = c * chunk, c1 = std::min(total, c0 + chunk);
      const size_t o = i * row_bytes + c0 * esz;
      const hipError_t e = hipMemcpyAsync(rows + o, stage + o, (c1 - c0) * esz, hipMemcpyHostToDevice, h2d);
      if (e != hipSuccess) {
        ln.rc = hip_fail(e, "staging H2D");
        return;
      }
      if (i + 1 == static_cast<size_t>(n)) finish_chunk(c);
    }
  });
  if (h_out) ln.link(d2h, st, "order stream after D2H");
  return ln.rc;
}

// Smallest chunk per model of a zero-copy task's pipeline (bytes):
// DLSIM_ZC_CHUNK_KB, read per call (A/B runs); default 128 KiB.
static size_t zc_chunk_bytes() {
  const char* e = dlsim::ab_getenv("DLSIM_ZC_CHUNK_KB");
  const long kb = e ? std::strtol(e, nullptr, 10) : 128;
  return static_cast<size_t>(kb > 0 ? kb : 0) << 10;
}

int dlsim_host_wreduce_zc(int n, int t, const void* const* h_srcs, const size_t* numels, const float* h_weights,
                          void* h_staging, size_t row_stride, void* h_out, int dtype, int mode, int threads,
                          void* stream) {
  g_err.clear();
  if (!known_dtype(dtype)) return dtype_fail(dtype);
  if (mode != DLSIM_EXACT && mode != DLSIM_FAST) return fail(DLSIM_E_MODE, "unsupported mode %d", mode);
  if (n < 1 || t < 0) return fail(DLSIM_E_ARG, "need n >= 1 and t >= 0 (got %d, %d)", n, t);
  if (!h_weights || (t > 0 && (!h_srcs || !numels))) return fail(DLSIM_E_ARG, "null array argument");
  const size_t esz = elem_bytes(dtype);
  size_t total = 0;
  for (int k = 0; k < t; ++k) total += numels[k];
  if (total == 0) return DLSIM_OK;
  if (!h_staging || !h_out) return fail(DLSIM_E_ARG, "null staging or output");
  if (!aligned16(h_staging) || row_stride % 8 != 0)
    return fail(DLSIM_E_ARG, "staging rows must be 16-B aligned with a stride that is a multiple of 8");
  if (row_stride < total) return fail(DLSIM_E_ARG, "row_stride %zu < %zu elements", row_stride, total);
  const size_t row_bytes = row_stride * esz;
  {
    const uintptr_t r0 = reinterpret_cast<uintptr_t>(h_staging), r1 = r0 + static_cast<size_t>(n) * row_bytes;
    const uintptr_t o0 = reinterpret_cast<uintptr_t>(h_out), o1 = o0 + total * esz;
    if (o0 < r1 && r0 < o1) return fail(DLSIM_E_ARG, "h_out overlaps the staging rows");
  }
  for (size_t j = 0; j < static_cast<size_t>(n) * t; ++j)
    if (!h_srcs[j] && numels[j % t] > 0) return fail(DLSIM_E_ARG, "null source pointer at index %zu", j);
  // The kernel reads the rows and writes the result over PCIe: both must be
  // page-locked memory the device maps. Anything else would fault the GPU,
  // so it is refused here, before any launch.
  void* d_stage = nullptr;
  void* d_res = nullptr;
  if (hipHostGetDevicePointer(&d_stage, h_staging, 0) != hipSuccess || !d_stage) {
    (void)hipGetLastError();
    return fail(DLSIM_E_ARG, "h_staging is not page-locked host memory the device maps (hipHostMalloc)");
  }
  if (hipHostGetDevicePointer(&d_res, h_out, 0) != hipSuccess || !d_res) {
    (void)hipGetLastError();
    return fail(DLSIM_E_ARG, "h_out is not page-locked host memory the device maps (hipHostMalloc)");
  }
  char* stage = static_cast<char*>(h_staging);
  // The element axis in K chunks, each a pack unit (every model's part of it,
  // in chunk order): once chunk c is packed its reduce is launched, and it
  // reads its rows over PCIe while the pack goes on with chunk c + 1.
  // Chunks of >= zc_chunk_bytes() per model, a multiple of 1024 elements (16-B
  // aligned ranges), for tasks of >= 1 MiB of rows (the 100-peer fan-in-7
  // GNLeNet round: 229-243 -> 200-208 us per task, batched 139-145 -> 106-110;
  // cfg1's 2 x 341 KB even or slower chunked, profiles/r05be_ab/);
  // DLSIM_ZC_CHUNK_KB (read per call) sets it, 0 = one chunk.
  const size_t min_chunk = zc_chunk_bytes() / esz;
  size_t L = total;
  if (min_chunk > 0 && total > 2 * min_chunk && total * esz * static_cast<size_t>(n) >= (size_t{1} << 20)) {
    const size_t k = std::min<size_t>(8, total / min_chunk);
    L = ((total + k - 1) / k + 1023) / 1024 * 1024;
  }
  const size_t K = (total + L - 1) / L;
  dlsim::PackJob job;
  job.streaming = dlsim::pack_streaming(true);  // rows read over PCIe next: leave them in the CPU caches
  for (size_t c = 0; c < K; ++c) {
    const size_t c0 = c * L, c1 = std::min(total, c0 + L);
    for (int i = 0; i < n; ++i) {
      size_t off = 0;
      for (int k = 0; k < t; ++k) {
        const size_t b = std::max(off, c0), e = std::min(off + numels[k], c1);
        if (b < e)
          job.add(static_cast<uint32_t>(c),
                  static_cast<const char*>(h_srcs[static_cast<size_t>(i) * t + k]) + (b - off) * esz,
                  stage + i * row_bytes + b * esz, (e - b) * esz);
        off += numels[k];
      }
    }
  }
  job.seal(K);
  int rc = DLSIM_OK;
  std::vector<const void*> ins(static_cast<size_t>(n));
  hipStream_t st = static_cast<hipStream_t>(stream);
  pack_and_dispatch(job, threads, total * esz * n, [&](size_t u0, size_t u1) {
    for (size_t c = u0; c < u1 && rc == DLSIM_OK; ++c) {
      const size_t c0 = c * L, len = std::min(total, c0 + L) - c0;
      for (int r = 0; r < n; ++r) ins[r] = static_cast<const char*>(d_stage) + r * row_bytes + c0 * esz;
      rc = dispatch(ins.data(), n, h_weights, static_cast<char*>(d_res) + c0 * esz, len, dtype, mode, st);
    }
  });
  return rc;
}

int dlsim_host_wreduce_resident(int n, int t, const void* const* h_srcs, const size_t* numels,
                                const float* h_weights, const int* resident, void* const* d_rows, void* h_staging,
                                size_t staging_stride, void* d_out, void* h_out, int dtype, int mode, int threads,
                                void* stream) {
  g_err.clear();
  if (!known_dtype(dtype)) return dtype_fail(dtype);
  if (mode != DLSIM_EXACT && mode != DLSIM_FAST) return fail(DLSIM_E_MODE, "unsupported mode %d", mode);
  if (n < 1 || t < 0) return fail(DLSIM_E_ARG, "need n >= 1 and t >= 0 (got %d, %d)", n, t);
  if (!h_weights || !resident || !d_rows || (t > 0 && (!h_srcs || !numels)))
    return fail(DLSIM_E_ARG, "null array argument");
  const size_t esz = elem_bytes(dtype);
  size_t total = 0;
  for (int k = 0; k < t; ++k) total += numels[k];
  if (total == 0) return DLSIM_OK;
  if (!d_out) return fail(DLSIM_E_ARG, "null output");
  int misses = 0;
  for (int i = 0; i < n; ++i) {
    if (!d_rows[i]) return fail(DLSIM_E_ARG, "null device row %d", i);
    if (!aligned16(d_rows[i])) return fail(DLSIM_E_ARG, "device row %d is not 16-B aligned", i);
    const uintptr_t r0 = reinterpret_cast<uintptr_t>(d_rows[i]), r1 = r0 + total * esz;
    const uintptr_t o0 = reinterpret_cast<uintptr_t>(d_out), o1 = o0 + total * esz;
    if (o0 < r1 && r0 < o1) return fail(DLSIM_E_ARG, "d_out overlaps device row %d", i);
    if (resident[i]) continue;
    ++misses;
    for (int k = 0; k < t; ++k)
      if (!h_srcs[static_cast<size_t>(i) * t + k] && numels[k] > 0)
        return fail(DLSIM_E_ARG, "null source pointer (model %d, tensor %d)", i, k);
  }
  if (misses > 0) {
    if (!h_staging || !aligned16(h_staging) || staging_stride % 8 != 0 || staging_stride < total)
      return fail(DLSIM_E_ARG, "staging: 16-B aligned rows of >= %zu elements, stride a multiple of 8", total);
    // A row the call writes (a miss) must not overlap any other row; resident
    // rows may alias each other (the same model twice in one task). Rows are
    // all total*esz long, so sorted by address an overlap involving a miss
    // shows between neighbours.
    std::vector<std::pair<uintptr_t, int>> span(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) span[i] = {reinterpret_cast<uintptr_t>(d_rows[i]), i};
    std::sort(span.begin(), span.end());
    for (size_t k = 1; k < span.size(); ++k) {
      const int a = span[k - 1].second, b = span[k].second;
      if (span[k].first < span[k - 1].first + total * esz && (!resident[a] || !resident[b]))
        return fail(DLSIM_E_ARG, "device rows %d and %d overlap and one of them is written (not resident)",
                    std::min(a, b), std::max(a, b));
    }
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  char* stage = static_cast<char*>(h_staging);
  const size_t row_bytes = staging_stride * esz;
  // The models not resident: model miss[j] is packed into staging row j, then
  // sent to d_rows[miss[j]]; consecutive misses whose device rows are one
  // staging stride apart go in one DMA (a cache fills them that way).
  std::vector<int> miss;
  dlsim::PackJob job;
  for (int i = 0; i < n; ++i) {
    if (resident[i]) continue;
    const uint32_t j = static_cast<uint32_t>(miss.size());
    miss.push_back(i);
    size_t o = 0;
    for (int k = 0; k < t; ++k) {
      if (numels[k] > 0)
        job.add(j, static_cast<const char*>(h_srcs[static_cast<size_t>(i) * t + k]), stage + j * row_bytes + o * esz,
                numels[k] * esz);
      o += numels[k];
    }
  }
  job.seal(miss.size());
  int rc = DLSIM_OK;
  size_t sent = 0;  // first packed row not yet sent
  auto send = [&](size_t j1) {  // rows [sent, j1) are packed: DMA them in device-contiguous runs
    while (sent < j1 && rc == DLSIM_OK) {
      size_t e = sent + 1;
      while (e < j1 && static_cast<const char*>(d_rows[miss[e]]) ==
                           static_cast<const char*>(d_rows[miss[e - 1]]) + row_bytes)
        ++e;
      const size_t bytes = (e - sent - 1) * row_bytes + total * esz;
      const hipError_t err = hipMemcpyAsync(d_rows[miss[sent]], stage + sent * row_bytes, bytes,
                                            hipMemcpyHostToDevice, st);
      if (err != hipSuccess) rc = hip_fail(err, "staging H2D");
      sent = e;
    }
  };
  if (!miss.empty()) {
    const size_t min_dma = h2d_min_bytes();
    pack_and_dispatch(job, threads, total * esz * miss.size(), [&](size_t, size_t u1) {
      if (u1 < miss.size() && (u1 - sent) * row_bytes < min_dma) return;
      send(u1);
    });
    send(miss.size());
    if (rc != DLSIM_OK) return rc;
  }
  std::vector<const void*> ins(d_rows, d_rows + n);
  rc = dispatch(ins.data(), n, h_weights, d_out, total, dtype, mode, st);
  if (rc != DLSIM_OK || !h_out) return rc;
  const hipError_t e = hipMemcpyAsync(h_out, d_out, total * esz, hipMemcpyDeviceToHost, st);
  return e == hipSuccess ? DLSIM_OK : hip_fail(e, "result D2H");
}

int dlsim_host_chunk_mean(int b, const int* fan_in, const void* const* h_inputs, const size_t* n_elems,
                          void* h_staging, void* d_staging, size_t staging_elems, void* const* d_outs,
                          void* const* h_outs, int dtype, int cpu_threads, int threads, void* stream,
                          void* h2d_stream, void* d2h_stream) {
  g_err.clear();
  if (b < 0) return fail(DLSIM_E_ARG, "b must be >= 0 (got %d)", b);
  if (b == 0) return DLSIM_OK;
  if (!fan_in || !h_inputs || !d_outs || !n_elems) return fail(DLSIM_E_ARG, "null array argument");
  if (!known_dtype(dtype) && dtype != DLSIM_F64) return dtype_fail(dtype);
  if (cpu_threads < 1) return fail(DLSIM_E_ARG, "cpu_threads must be >= 1 (got %d)", cpu_threads);
  const size_t esz = elem_bytes(dtype);
  size_t need = 0, rows_total = 0;
  for (int t = 0; t < b; ++t) {
    if (fan_in[t] < 1 || fan_in[t] > 65535) return fail(DLSIM_E_ARG, "task %d: fan-in %d not in [1, 65535]", t, fan_in[t]);
    if (n_elems[t] * esz >= kMaxLaunchOutBytes)
      return fail(DLSIM_E_ARG, "task %d: chunk of %zu elements is >= 2 GiB", t, n_elems[t]);
    if (n_elems[t] > 0 && !d_outs[t]) return fail(DLSIM_E_ARG, "task %d: null output", t);
    for (int i = 0; i < fan_in[t]; ++i)
      if (n_elems[t] > 0 && !h_inputs[rows_total + i]) return fail(DLSIM_E_ARG, "task %d: null input %d", t, i);
    need += static_cast<size_t>(fan_in[t]) * staged_row_elems(n_elems[t], esz);
    rows_total += static_cast<size_t>(fan_in[t]);
  }
  if (need == 0) return DLSIM_OK;
  if (!h_staging || !d_staging) return fail(DLSIM_E_ARG, "null staging");
  if (!aligned16(h_staging) || !aligned16(d_staging)) return fail(DLSIM_E_ARG, "staging must be 16-B aligned");
  if (staging_elems < need) return fail(DLSIM_E_ARG, "staging of %zu elements < %zu needed", staging_elems, need);
  {
    const uintptr_t s0 = reinterpret_cast<uintptr_t>(d_staging), s1 = s0 + need * esz;
    for (int t = 0; t < b; ++t) {
      const uintptr_t o0 = reinterpret_cast<uintptr_t>(d_outs[t]), o1 = o0 + n_elems[t] * esz;
      if (n_elems[t] > 0 && o0 < s1 && s0 < o1) return fail(DLSIM_E_ARG, "task %d: output overlaps the device staging", t);
    }
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  // one task: nothing to overlap, everything on `stream` (see dlsim_host_wreduce)
  hipStream_t h2d = b > 1 && h2d_stream ? static_cast<hipStream_t>(h2d_stream) : st;
  hipStream_t d2h = b > 1 && d2h_stream ? static_cast<hipStream_t>(d2h_stream) : st;
  char* hs = static_cast<char*>(h_staging);
  char* ds = static_cast<char*>(d_staging);

  // One unit per input row, in task order; row r sits at row_off[r].
  std::vector<size_t> row_off(rows_total), row_task(rows_total);
  dlsim::PackJob job;
  {
    size_t r = 0, o = 0;
    for (int t = 0; t < b; ++t)
      for (int i = 0; i < fan_in[t]; ++i, ++r) {
        row_off[r] = o;
        row_task[r] = static_cast<size_t>(t);
        job.add(static_cast<uint32_t>(r), static_cast<const char*>(h_inputs[r]), hs + o * esz, n_elems[t] * esz);
        o += staged_row_elems(n_elems[t], esz);
      }
    job.seal(rows_total);
  }
  if (need * esz < kSmallHostJobBytes) {
    // Small job (GNLeNet's Conflux reconstruct: ~1.4 MB):
    // a DMA costs ~15 us of copy-engine time whatever its size, so pack every
    // row first, then ONE H2D of the staging, ONE batched launch of every
    // task's mean and, when the outputs lie back to back at the same offsets
    // on both sides (the ChunkManager's layout), ONE D2H; all on `stream`.
    pack_and_dispatch(job, threads, need * esz, [](size_t, size_t) {});
    hipError_t e = hipMemcpyAsync(ds, hs, need * esz, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return hip_fail(e, "staging H2D");
    std::vector<const void*> ins_all(rows_total);
    for (size_t r = 0; r < rows_total; ++r) ins_all[r] = ds + row_off[r] * esz;
    int rc = with_chunk_policy(dtype, [&](auto op) {
      return run_chunk_mean<decltype(op)>(b, fan_in, ins_all.data(), d_outs, n_elems, cpu_threads, st);
    });
    if (rc != DLSIM_OK || !h_outs) return rc;
    // One D2H when the non-empty outputs tile one span back to back (sorted
    // by offset, each starting where the previous one ends) at the same
    // offsets on both sides; else one per task. Equal offsets alone are not
    // enough: host bytes between outputs must not be overwritten, and the
    // copy must not read past the device outputs.
    if (const int rc1 = d2h_one_span(b, d_outs, h_outs, n_elems, esz, st); rc1 != 1) return rc1;
    for (int t = 0; t < b; ++t) {
      if (n_elems[t] == 0 || !h_outs[t]) continue;
      e = hipMemcpyAsync(h_outs[t], d_outs[t], n_elems[t] * esz, hipMemcpyDeviceToHost, st);
      if (e != hipSuccess) return hip_fail(e, "result D2H");
    }
    return DLSIM_OK;
  }
  StreamLinks ln;
  ln.link(st, h2d, "order H2D after stream");
  if (h_outs) ln.link(st, d2h, "order D2H after stream");
  std::vector<const void*> ins;
  size_t task_first = 0;  // first row of the current task
  // Row r is on the device: if it completes its task, that task's mean and D2H.
  auto row_done = [&](size_t r) {
    if (ln.rc != DLSIM_OK) return;
    const int t = static_cast<int>(row_task[r]);
    const size_t n = n_elems[t];
    if (r + 1 - task_first < static_cast<size_t>(fan_in[t])) return;
    const size_t first = task_first;
    task_first = r + 1;
    if (n == 0) return;
    // every row of task t is queued: its mean, then its D2H
    ln.link(h2d, st, "order chunk mean after H2D");
    if (ln.rc != DLSIM_OK) return;
    ins.assign(static_cast<size_t>(fan_in[t]), nullptr);
    for (int i = 0; i < fan_in[t]; ++i) ins[i] = ds + row_off[first + i] * esz;
    void* out = d_outs[t];
    ln.rc = with_chunk_policy(dtype, [&](auto op) {
      return run_chunk_mean<decltype(op)>(1, &fan_in[t], ins.data(), &out, &n_elems[t], cpu_threads, st);
    });
    if (ln.rc != DLSIM_OK || !h_outs || !h_outs[t]) return;
    ln.link(st, d2h, "order D2H after chunk mean");
    if (ln.rc != DLSIM_OK) return;
    hipError_t e = hipMemcpyAsync(h_outs[t], out, n * esz, hipMemcpyDeviceToHost, d2h);
    if (e != hipSuccess) ln.rc = hip_fail(e, "result D2H");
  };
  pack_and_dispatch(job, threads, need * esz, [&](size_t r0, size_t r1) {
    if (ln.rc != DLSIM_OK) return;
    // the run's rows lie back to back in staging (256-B aligned offsets, the
    // gaps are copied too): one DMA for all of them
    const size_t b = row_off[r0] * esz, e1 = (row_off[r1 - 1] + n_elems[row_task[r1 - 1]]) * esz;
    if (e1 > b) {
      const hipError_t e = hipMemcpyAsync(ds + b, hs + b, e1 - b, hipMemcpyHostToDevice, h2d);
      if (e != hipSuccess) {
        ln.rc = hip_fail(e, "staging H2D");
        return;
      }
    }
    for (size_t r = r0; r < r1; ++r) row_done(r);
  });
  if (h_outs) ln.link(d2h, st, "order stream after D2H");
  return ln.rc;
}

int dlsim_host_pack(int t, const void* const* h_srcs, const size_t* nbytes, const size_t* dst_off, void* h_dst,
                    int threads) {
  g_err.clear();
  if (t < 0) return fail(DLSIM_E_ARG, "t must be >= 0 (got %d)", t);
  if (t == 0) return DLSIM_OK;
  if (!h_srcs || !nbytes || !dst_off || !h_dst) return fail(DLSIM_E_ARG, "null argument");
  dlsim::PackJob job;
  size_t total = 0;
  char* dst = static_cast<char*>(h_dst);
  for (int j = 0; j < t; ++j) {
    if (nbytes[j] == 0) continue;
    if (!h_srcs[j]) return fail(DLSIM_E_ARG, "null source pointer at index %d", j);
    job.add(0, static_cast<const char*>(h_srcs[j]), dst + dst_off[j], nbytes[j]);
    total += nbytes[j];
  }
  job.seal(1);
  pack_and_dispatch(job, threads, total, [](size_t, size_t) {});
  return DLSIM_OK;
}

int dlsim_shard_range(size_t n_elems, int world, int rank, size_t align_elems, size_t* begin,
                      size_t* end) {
  g_err.clear();
  if (world < 1 || rank < 0 || rank >= world) return fail(DLSIM_E_ARG, "bad world/rank %d/%d", world, rank);
  if (!begin || !end) return fail(DLSIM_E_ARG, "null begin/end");
  if (align_elems == 0) align_elems = 1;
  // Whole aligned units are dealt out as evenly as possible; the last rank
  // also takes the ragged remainder.
  const size_t units = n_elems / align_elems;
  const size_t q = units / static_cast<size_t>(world), r = units % static_cast<size_t>(world);
  const size_t rk = static_cast<size_t>(rank);
  const size_t u0 = rk * q + std::min(rk, r);
  const size_t u1 = u0 + q + (rk < r ? 1 : 0);
  *begin = u0 * align_elems;
  *end = (rank == world - 1) ? n_elems : u1 * align_elems;
  return DLSIM_OK;
}

int dlsim_probe_pattern(const void* const* d_inputs, int n, void* d_out, size_t n_elems, int dtype,
                        void* stream) {
  g_err.clear();
  int rc = check_args(d_inputs, n, nullptr, d_out, n_elems, dtype, DLSIM_EXACT, false);
  if (rc != DLSIM_OK) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (dtype == DLSIM_F32) return run<dlsim::XorProbe<4>>(d_inputs, n, nullptr, d_out, n_elems, st);
  return run<dlsim::XorProbe<2>>(d_inputs, n, nullptr, d_out, n_elems, st);
}

int dlsim_wreduce_mixed(const void* const* d_inputs, const int* dtypes, int n, const double* h_weights,
                        void* d_out, int out_dtype, size_t n_elems, void* stream) {
  g_err.clear();
  if (n < 1) return fail(DLSIM_E_ARG, "n must be >= 1 (got %d)", n);
  if (!d_inputs || !dtypes || !h_weights) return fail(DLSIM_E_ARG, "null inputs, dtypes or weights array");
  if (out_dtype < DLSIM_F32 || out_dtype > DLSIM_F64) return fail(DLSIM_E_DTYPE, "unsupported dtype %d", out_dtype);
  for (int i = 0; i < n; ++i)
    if (dtypes[i] < DLSIM_F32 || dtypes[i] > DLSIM_F64)
      return fail(DLSIM_E_DTYPE, "unsupported dtype %d at index %d", dtypes[i], i);
  if (dtypes[0] != out_dtype)
    return fail(DLSIM_E_ARG, "input 0 (models[0]'s parameter) must have the output's dtype");
  if (n_elems == 0) return DLSIM_OK;
  if (!d_out) return fail(DLSIM_E_ARG, "null output pointer");
  const uintptr_t o0 = reinterpret_cast<uintptr_t>(d_out), o1 = o0 + n_elems * elem_bytes(out_dtype);
  for (int i = 0; i < n; ++i) {
    if (!d_inputs[i]) return fail(DLSIM_E_ARG, "null input pointer at index %d", i);
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(d_inputs[i]), a1 = a0 + n_elems * elem_bytes(dtypes[i]);
    // later passes (n > 32) read the output back: no input may share its bytes
    if (a0 < o1 && o0 < a1) return fail(DLSIM_E_ARG, "output overlaps input %d", i);
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t blocks = std::min<size_t>((n_elems + dlsim::kBlock - 1) / dlsim::kBlock, 2048);
  for (int i0 = 0; i0 < n; i0 += dlsim::kMixedMaxInputs) {
    dlsim::MixedSlots s;
    std::memset(&s, 0, sizeof(s));
    s.n = std::min(n - i0, dlsim::kMixedMaxInputs);
    s.out_dt = out_dtype;
    s.seed = i0 == 0;
    for (int k = 0; k < s.n; ++k) {
      s.p[k] = d_inputs[i0 + k];
      s.w[k] = h_weights[i0 + k];
      s.dt[k] = dtypes[i0 + k];
    }
    hipLaunchKernelGGL(dlsim::k_wreduce_mixed<dlsim::MixedSlots>, dim3(static_cast<unsigned>(blocks)),
                       dim3(dlsim::kBlock), 0, st, s, d_out, n_elems);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_wreduce_mixed launch");
  }
  return DLSIM_OK;
}

int dlsim_device_alloc(size_t nbytes, int flags, void** d_out, int* contiguous) {
  g_err.clear();
  if (!d_out) return fail(DLSIM_E_ARG, "null d_out");
  *d_out = nullptr;
  if (contiguous) *contiguous = 0;
  if (nbytes == 0) return fail(DLSIM_E_ARG, "zero-byte allocation");
  if (flags & ~DLSIM_ALLOC_CONTIGUOUS) return fail(DLSIM_E_ARG, "unknown flags 0x%x", flags);
  if (flags & DLSIM_ALLOC_CONTIGUOUS) {
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, nbytes, hipDeviceMallocContiguous) == hipSuccess && p) {
      *d_out = p;
      if (contiguous) *contiguous = 1;
      return DLSIM_OK;
    }
    (void)hipGetLastError();  // best effort: the plain allocation below decides
  }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, nbytes);
  if (e != hipSuccess) return hip_fail(e, "hipMalloc");
  *d_out = p;
  return DLSIM_OK;
}

int dlsim_device_free(void* d_ptr) {
  g_err.clear();
  if (!d_ptr) return DLSIM_OK;
  hipError_t e = hipFree(d_ptr);
  return e == hipSuccess ? DLSIM_OK : hip_fail(e, "hipFree");
}

}  // extern "C"

// ---- torch pluggable allocator over contiguous blocks (dlsim_pool_*) -----------
// Segments come from hipExtMallocWithFlags(hipDeviceMallocContiguous), else
// hipMalloc. A segment whose base is not 2 MiB-aligned is re-made 2 MiB larger
// and handed out from its first aligned byte; `realigned` maps that address
// back to the driver's for the free. Called under torch's allocator lock.
namespace dlsim_host __attribute__((visibility("hidden"))) {
constexpr size_t kPoolAlign = size_t(2) << 20;
std::mutex g_pool_mu;
std::vector<std::pair<void*, void*>> g_realigned;  // (handed out, driver's base); rare
unsigned long long g_pool_contig = 0, g_pool_fallback = 0, g_pool_live = 0;

void* pool_raw(size_t nbytes, bool* contiguous) {
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, nbytes, hipDeviceMallocContiguous) == hipSuccess && p) {
    *contiguous = true;
    return p;
  }
  (void)hipGetLastError();
  p = nullptr;
  if (hipMalloc(&p, nbytes) != hipSuccess) {
    (void)hipGetLastError();  // torch sees NULL and runs its own out-of-memory path
    return nullptr;
  }
  *contiguous = false;
  return p;
}
}  // namespace dlsim_host

extern "C" {

void* dlsim_pool_alloc(size_t nbytes, int device, void* /*stream*/) {
  if (nbytes == 0) return nullptr;
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != device) (void)hipSetDevice(device);
  bool contig = false;
  void* p = pool_raw(nbytes, &contig);
  void* out = p;
  if (p && reinterpret_cast<uintptr_t>(p) % kPoolAlign) {
    (void)hipFree(p);
    p = pool_raw(nbytes + kPoolAlign, &contig);
    out = p ? reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(p) + kPoolAlign - 1) & ~(kPoolAlign - 1))
            : nullptr;
  }
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  if (!out) return nullptr;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (out != p) g_realigned.emplace_back(out, p);
  (contig ? g_pool_contig : g_pool_fallback) += 1;
  g_pool_live += nbytes;
  return out;
}

void dlsim_pool_free(void* d_ptr, size_t nbytes, int device, void* /*stream*/) {
  if (!d_ptr) return;
  void* base = d_ptr;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_realigned.size(); ++i) {
      if (g_realigned[i].first == d_ptr) {
        base = g_realigned[i].second;
        g_realigned.erase(g_realigned.begin() + static_cast<long>(i));
        break;
      }
    }
    g_pool_live -= std::min<unsigned long long>(g_pool_live, nbytes);
  }
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != device) (void)hipSetDevice(device);
  (void)hipFree(base);
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
}

void dlsim_pool_stats(unsigned long long* contiguous, unsigned long long* fallback, unsigned long long* live_bytes) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (contiguous) *contiguous = g_pool_contig;
  if (fallback) *fallback = g_pool_fallback;
  if (live_bytes) *live_bytes = g_pool_live;
}

const char* dlsim_last_error(void) { return g_err.c_str(); }

const char* dlsim_kernel_name(int n, size_t n_elems, int dtype, int mode) {
  if (dtype != DLSIM_F32 && dtype != DLSIM_BF16 && dtype != DLSIM_F16) return "";
  if (mode == -1) return with_mean_policy_name(dtype, n, n_elems);
  if (mode != DLSIM_EXACT && mode != DLSIM_FAST) return "";
  const char* name = "";
  with_policy(dtype, mode, [&](auto op) {
    name = kernel_name<decltype(op)>(n, n_elems);
    return 0;
  });
  return name;
}

int dlsim_version(void) { return (1 << 16) | 1; }

}  // extern "C"
