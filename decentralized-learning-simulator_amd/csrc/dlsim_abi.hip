// dlsim_abi.hip — the C ABI of include/dlsim.h over the gfx950 kernels of
// wreduce_kernels.hpp. Host-side dispatch only: argument checks, choice of
// vector vs scalar kernel, launch shape, kernarg or device-table fan-in, batching
// and its hazard checks, host staging pipelines.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "dlsim.h"
#include "wreduce_kernels.hpp"
#include "chunk_mean_kernels.hpp"
#include "host_pack.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(DLSIM_E_HIP - static_cast<int>(e), "%s: %s", what, hipGetErrorString(e));
}

// Launch shape (tuned on MI355X with csrc/tune_wreduce.hip):
// 4 vectors of 16 B per lane (a 16 KiB tile per stream per block), one tile
// per block, non-temporal loads and stores. Small fan-in runs a kernel
// specialised on n (all n*4 loads issued back to back, fewer VGPRs than the
// grouped loop); larger n folds groups of G inputs. The specialised kernels
// are used only while they fit in 256 VGPRs (two waves per SIMD): past that
// the measured rate drops by up to 20% (profiles/r01_sweep_fanin_*.jsonl).
constexpr int kVpt = 4;
constexpr bool kNT = true;
// Output stores are buffer_store_dwordx4 with sc1 (write-through): no dirty
// output lines are left in L2 for the kernel-boundary writeback, which was
// worth 3-4% per launch on the north star (profiles/r01_tune_store_*.log).
// The buffer's 32-bit byte offsets cap one launch's output at 2 GiB; longer
// outputs are split into independent launches over element ranges.
constexpr int kStore = 16;  // sc1
// Per element type (profiles/r01_tune_*): fp32 takes sc1 write-through stores
// and the wave-contiguous lane map (each wave sweeps 4 KiB per stream, +1.3%
// on the north star); bf16, whose output is a third of the traffic in the
// 2-way merge, keeps non-temporal stores (+2% there) and the block map.
// These are the policies of the grouped (runtime fan-in) kernel and of the
// batched kernels.
template <class Op> constexpr int store_policy() { return Op::kBytes == 4 ? kStore : dlsim::kStNT; }
template <class Op> constexpr bool wave_map() { return Op::kBytes == 4; }
constexpr size_t kMaxLaunchOutBytes = (size_t{1} << 31) - (size_t{1} << 20);
template <class Op> constexpr int max_fixed_fan_in() { return Op::kBytes == 4 ? 14 : 9; }
template <class Op> constexpr int group_size() { return Op::kBytes == 4 ? 8 : 4; }

// Launch shape of the fixed fan-in kernels, chosen by the per-stream size
// class (size sweeps with arena rows as in bench.py and >= 1 GiB of rotating
// inputs: profiles/r01_tune_shape_sweep.log, profiles/r02_tune_slices/):
//   fp32  < 2 M elements   : VPT 2, block map, sc1 (+7% at the 8-rank slice
//                            of the north star, 1.4 M: 9.85 vs 10.57 us)
//   fp32  2 M .. 5 M       : VPT 4, block map, sc1 (1-4% over the wave map)
//   fp32 >= 5 M            : VPT 4, wave map,  sc1 (~1% at 6-11 M)
//   bf16  < 48 M elements  : VPT 1, wave map, sc1  (+7-12% at 4-33 M for n = 2)
//   bf16 >= 48 M           : VPT 4, block map, nt  (+1.5-2.5% at 64-125 M)
struct Shape {
  int vpt;
  int store;
  bool wave;
};
template <class Op, int C> constexpr Shape fixed_shape() {
  if constexpr (Op::kBytes == 4) {
    if constexpr (C == 0) return Shape{2, kStore, false};
    else if constexpr (C == 1) return Shape{4, kStore, false};
    else return Shape{4, kStore, true};
  } else {
    if constexpr (C < 2) return Shape{1, kStore, true};
    else return Shape{4, dlsim::kStNT, false};
  }
}
template <class Op> int size_class(size_t nelem) {
  if constexpr (Op::kBytes == 4) return nelem < 2000000 ? 0 : nelem < 5000000 ? 1 : 2;
  else return nelem < 48000000 ? 0 : 2;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <class Op, class S, int NF, int VPT, int STP, bool WAVE>
hipError_t launch_shape(const S& s, int n, void* out, size_t nelem, hipStream_t st) {
  const size_t nvec = nelem / Op::E;
  const size_t tile = static_cast<size_t>(dlsim::kBlock) * VPT;
  const size_t blocks = nvec / tile + 1;  // full tiles + one block for the ragged end
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  hipLaunchKernelGGL((dlsim::k_wreduce_tiles<Op, S, NF, group_size<Op>(), VPT, kNT, STP, WAVE>),
                     dim3(static_cast<unsigned>(blocks)), dim3(dlsim::kBlock), 0, st, s, n, out, nvec, nelem);
  return hipGetLastError();
}

template <class Op, class S, int NF, int C>
hipError_t launch_class(const S& s, int n, void* out, size_t nelem, hipStream_t st) {
  constexpr Shape k = fixed_shape<Op, C>();
  return launch_shape<Op, S, NF, k.vpt, k.store, k.wave>(s, n, out, nelem, st);
}

template <class Op, class S, int NF>
hipError_t launch_tiles(const S& s, int n, void* out, size_t nelem, hipStream_t st) {
  if constexpr (NF > 0) {
    switch (size_class<Op>(nelem)) {
      case 0: return launch_class<Op, S, NF, 0>(s, n, out, nelem, st);
      case 1: return launch_class<Op, S, NF, 1>(s, n, out, nelem, st);
      default: return launch_class<Op, S, NF, 2>(s, n, out, nelem, st);
    }
  } else {
    return launch_shape<Op, S, 0, kVpt, store_policy<Op>(), wave_map<Op>()>(s, n, out, nelem, st);
  }
}

template <class Op, int K>
hipError_t launch_fixed_k(const dlsim::Slots<16>& s, int n, void* out, size_t nelem, hipStream_t st) {
  if constexpr (K > max_fixed_fan_in<Op>()) {
    return hipErrorInvalidValue;
  } else {
    if (n == K) return launch_tiles<Op, dlsim::Slots<16>, K>(s, n, out, nelem, st);
    return launch_fixed_k<Op, K + 1>(s, n, out, nelem, st);
  }
}

template <class Op, class S>
hipError_t launch_any(const S& s, int n, void* out, size_t nelem, bool vec, hipStream_t st) {
  if (vec) {
    if constexpr (std::is_same<S, dlsim::Slots<16>>::value) {
      if (n <= max_fixed_fan_in<Op>()) return launch_fixed_k<Op, 1>(s, n, out, nelem, st);
    }
    return launch_tiles<Op, S, 0>(s, n, out, nelem, st);
  }
  const size_t blocks = (nelem + dlsim::kBlock - 1) / dlsim::kBlock;
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  hipLaunchKernelGGL((dlsim::k_wreduce_scalar<Op, S>), dim3(static_cast<unsigned>(blocks)), dim3(dlsim::kBlock), 0,
                     st, s, n, out, nelem);
  return hipGetLastError();
}

template <int NB>
void fill_slots(dlsim::Slots<NB>& s, const void* const* in, const float* w, int n, float div) {
  std::memset(&s, 0, sizeof(s));
  for (int i = 0; i < n; ++i) {
    s.p[i] = in[i];
    s.w[i] = w ? w[i] : 1.0f;
  }
  s.div = div;
}

// One launch over [0, nelem) of n inputs: every output element is written
// once, after all n of its terms are folded in input order. Up to
// DLSIM_MAX_FUSED_INPUTS inputs travel as kernel arguments; above that the
// pointer/weight table goes to a stream-ordered device buffer (the pageable
// host copy is staged by the runtime before hipMemcpyAsync returns).
// div: final divisor (the mean policies; 1 for the weighted reduce).
template <class Op>
int run_range(const void* const* in, int n, const float* w, void* out, size_t nelem, bool vec, float div,
              hipStream_t st) {
  hipError_t e;
  if (n <= 16) {
    dlsim::Slots<16> s;
    fill_slots(s, in, w, n, div);
    e = launch_any<Op>(s, n, out, nelem, vec, st);
  } else if (n <= DLSIM_MAX_FUSED_INPUTS) {
    dlsim::Slots<DLSIM_MAX_FUSED_INPUTS> s;
    fill_slots(s, in, w, n, div);
    e = launch_any<Op>(s, n, out, nelem, vec, st);
  } else {
    const size_t pbytes = static_cast<size_t>(n) * sizeof(void*);
    std::vector<unsigned char> h(pbytes + static_cast<size_t>(n) * sizeof(float));
    std::memcpy(h.data(), in, pbytes);
    for (int i = 0; i < n; ++i) {
      const float wi = w ? w[i] : 1.0f;
      std::memcpy(h.data() + pbytes + static_cast<size_t>(i) * sizeof(float), &wi, sizeof(float));
    }
    void* d = nullptr;
    e = hipMallocAsync(&d, h.size(), st);
    if (e != hipSuccess) return hip_fail(e, "fan-in table alloc");
    e = hipMemcpyAsync(d, h.data(), h.size(), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
      const dlsim::DevSlots s{static_cast<const void* const*>(d),
                              reinterpret_cast<const float*>(static_cast<unsigned char*>(d) + pbytes), div};
      e = launch_any<Op>(s, n, out, nelem, vec, st);
    }
    const hipError_t e2 = hipFreeAsync(d, st);
    if (e == hipSuccess) e = e2;
  }
  if (e != hipSuccess) return hip_fail(e, "kernel launch");
  return DLSIM_OK;
}

// Elements are independent: an output longer than one launch's 2 GiB store
// window is reduced as consecutive ranges (pointers offset by the range start).
template <class Op>
int run(const void* const* in, int n, const float* w, void* out, size_t nelem, hipStream_t st,
        float div = 1.0f) {
  if (nelem == 0) return DLSIM_OK;
  bool vec = aligned16(out);
  for (int i = 0; i < n && vec; ++i) vec = aligned16(in[i]);
  const size_t chunk = kMaxLaunchOutBytes / Op::kBytes;  // multiple of every tile size
  if (!vec || nelem <= chunk) return run_range<Op>(in, n, w, out, nelem, vec, div, st);
  std::vector<const void*> sub(static_cast<size_t>(n));
  for (size_t b = 0; b < nelem; b += chunk) {
    const size_t len = std::min(chunk, nelem - b);
    for (int i = 0; i < n; ++i) sub[i] = static_cast<const char*>(in[i]) + b * Op::kBytes;
    int rc = run_range<Op>(sub.data(), n, w, static_cast<char*>(out) + b * Op::kBytes, len, vec, div, st);
    if (rc != DLSIM_OK) return rc;
  }
  return DLSIM_OK;
}

// ---- cross-task hazards of the batched entry points ---------------------------
// A batched launch runs its tasks concurrently; b separate calls run them in
// order. They agree unless one task writes bytes another task reads or
// writes. Detected in O((inputs + b) log b): the output spans are sorted (any
// overlap among them shows between neighbours), then each input span is
// looked up among them. A task's exact in-place alias of its own input is
// fine (one lane reads every term of an element before writing it).
struct Span {
  uintptr_t a, b;
  int task;
};

bool cross_task_overlap(int nt, const int* fan_in, const void* const* in, void* const* outs, const size_t* nelem,
                        size_t esz) {
  std::vector<Span> wr;
  wr.reserve(static_cast<size_t>(nt));
  for (int t = 0; t < nt; ++t) {
    if (nelem[t] == 0) continue;
    const uintptr_t a = reinterpret_cast<uintptr_t>(outs[t]);
    wr.push_back({a, a + nelem[t] * esz, t});
  }
  std::sort(wr.begin(), wr.end(), [](const Span& x, const Span& y) { return x.a < y.a; });
  for (size_t k = 1; k < wr.size(); ++k)
    if (wr[k].a < wr[k - 1].b) return true;  // two outputs overlap (disjoint otherwise: ends sorted too)
  size_t off = 0;
  for (int t = 0; t < nt; ++t) {
    const size_t bytes = nelem[t] * esz;
    for (int i = 0; i < fan_in[t]; ++i) {
      if (bytes == 0) continue;
      const uintptr_t a = reinterpret_cast<uintptr_t>(in[off + i]), b = a + bytes;
      auto it = std::upper_bound(wr.begin(), wr.end(), a, [](uintptr_t v, const Span& x) { return v < x.b; });
      for (; it != wr.end() && it->a < b; ++it)
        if (it->task != t) return true;
    }
    off += static_cast<size_t>(fan_in[t]);
  }
  return false;
}

// ---- batched launches ---------------------------------------------------------
template <class Op, int NF>
hipError_t launch_batch_nf(const dlsim::BatchSlots& s, unsigned blocks, hipStream_t st) {
  hipLaunchKernelGGL((dlsim::k_wreduce_batch<Op, NF, group_size<Op>(), kVpt, kNT, store_policy<Op>()>), dim3(blocks),
                     dim3(dlsim::kBlock), 0, st, s);
  return hipGetLastError();
}

template <class Op, int K>
hipError_t launch_batch_fixed(const dlsim::BatchSlots& s, int n, unsigned blocks, hipStream_t st) {
  if constexpr (K > max_fixed_fan_in<Op>()) {
    return launch_batch_nf<Op, 0>(s, blocks, st);
  } else {
    if (n == K) return launch_batch_nf<Op, K>(s, blocks, st);
    return launch_batch_fixed<Op, K + 1>(s, n, blocks, st);
  }
}

// Fill and launch BatchSlots with tasks [t0, t1); all tasks vector-eligible.
// divs: per-task final divisor (the mean policies), nullptr = 1.
template <class Op>
hipError_t launch_batch(const int* fan_in, const size_t* in_off, const void* const* in, const float* w,
                        const float* divs, void* const* outs, const size_t* nelem, int t0, int t1,
                        hipStream_t st) {
  dlsim::BatchSlots s;
  std::memset(&s, 0, sizeof(s));
  const size_t tile = static_cast<size_t>(dlsim::kBlock) * kVpt;
  uint32_t blocks = 0;
  int ptrs = 0;
  bool uniform = true;
  for (int t = t0; t < t1; ++t) {
    const int k = t - t0;
    const size_t nvec = nelem[t] / Op::E;
    s.out[k] = outs[t];
    s.nvec[k] = nvec;
    s.nelem[k] = nelem[t];
    s.block_start[k] = blocks;
    s.ptr_off[k] = static_cast<uint16_t>(ptrs);
    s.fan_in[k] = static_cast<uint16_t>(fan_in[t]);
    s.div[k] = divs ? divs[t] : 1.0f;
    for (int i = 0; i < fan_in[t]; ++i) {
      s.p[ptrs + i] = in[in_off[t] + i];
      s.w[ptrs + i] = w[in_off[t] + i];
    }
    ptrs += fan_in[t];
    blocks += static_cast<uint32_t>(nvec / tile + 1);
    uniform = uniform && fan_in[t] == fan_in[t0];
  }
  s.ntasks = t1 - t0;
  s.block_start[t1 - t0] = blocks;
  if (uniform) return launch_batch_fixed<Op, 1>(s, fan_in[t0], blocks, st);
  return launch_batch_nf<Op, 0>(s, blocks, st);
}

template <class Op>
int run_batched(int b, const int* fan_in, const void* const* in, const float* w, void* const* outs,
                const size_t* nelem, hipStream_t st, const float* divs = nullptr) {
  std::vector<size_t> off(static_cast<size_t>(b) + 1, 0);
  for (int t = 0; t < b; ++t) off[t + 1] = off[t] + static_cast<size_t>(fan_in[t]);
  if (cross_task_overlap(b, fan_in, in, outs, nelem, Op::kBytes)) {
    // A task reads or writes another task's output: keep the semantics of b
    // separate calls by running the tasks one launch each, in order.
    for (int t = 0; t < b; ++t) {
      int rc = run<Op>(in + off[t], fan_in[t], w + off[t], outs[t], nelem[t], st, divs ? divs[t] : 1.0f);
      if (rc != DLSIM_OK) return rc;
    }
    return DLSIM_OK;
  }
  const size_t tile = static_cast<size_t>(dlsim::kBlock) * kVpt;
  auto batchable = [&](int t) {
    if (nelem[t] == 0 || fan_in[t] > 16) return false;
    if (nelem[t] * Op::kBytes > kMaxLaunchOutBytes) return false;
    if (!aligned16(outs[t])) return false;
    for (int i = 0; i < fan_in[t]; ++i)
      if (!aligned16(in[off[t] + i])) return false;
    return true;
  };
  // Tasks that cannot ride in a batch (large fan-in, misaligned, > 2 GiB) go
  // alone (no task touches another's output, so the order is free).
  std::vector<int> group;
  for (int t = 0; t < b; ++t) {
    if (batchable(t)) {
      group.push_back(t);
      continue;
    }
    if (nelem[t] == 0) continue;
    int rc = run<Op>(in + off[t], fan_in[t], w + off[t], outs[t], nelem[t], st, divs ? divs[t] : 1.0f);
    if (rc != DLSIM_OK) return rc;
  }
  // Pack the rest greedily into kernel-argument batches, in task order.
  std::vector<const void*> ins;
  std::vector<float> ws, dv;
  std::vector<void*> os;
  std::vector<size_t> ne, ioff;
  std::vector<int> fi;
  for (int t : group) {
    ioff.push_back(ins.size());
    for (int i = 0; i < fan_in[t]; ++i) {
      ins.push_back(in[off[t] + i]);
      ws.push_back(w[off[t] + i]);
    }
    os.push_back(outs[t]);
    ne.push_back(nelem[t]);
    fi.push_back(fan_in[t]);
    dv.push_back(divs ? divs[t] : 1.0f);
  }
  const int g = static_cast<int>(group.size());
  int t0 = 0;
  while (t0 < g) {
    int t1 = t0, ptrs = 0;
    uint64_t blocks = 0;
    while (t1 < g && t1 - t0 < dlsim::kBatchMaxTasks && ptrs + fi[t1] <= dlsim::kBatchMaxPtrs &&
           blocks + ne[t1] / Op::E / tile + 1 < 0x7fffffffull) {
      ptrs += fi[t1];
      blocks += ne[t1] / Op::E / tile + 1;
      ++t1;
    }
    hipError_t e = launch_batch<Op>(fi.data(), ioff.data(), ins.data(), ws.data(), dv.data(), os.data(),
                                    ne.data(), t0, t1, st);
    if (e != hipSuccess) return hip_fail(e, "batched kernel launch");
    t0 = t1;
  }
  return DLSIM_OK;
}

// ---- descriptor-table batches ---------------------------------------------------
struct TableLayout {
  size_t tasks_off, map_off, ptrs_off, w_off, bytes;
  uint32_t nblocks;
};

size_t round8(size_t x) { return (x + 7) / 8 * 8; }

template <class Op>
uint32_t task_blocks(size_t nelem) {
  const size_t tile = static_cast<size_t>(dlsim::kBlock) * kVpt;
  return static_cast<uint32_t>(nelem / Op::E / tile + 1);
}

template <class Op>
bool table_layout(int b, const int* fan_in, const size_t* nelem, TableLayout* L) {
  uint64_t blocks = 0, ptrs = 0;
  for (int t = 0; t < b; ++t) {
    blocks += task_blocks<Op>(nelem[t]);
    ptrs += static_cast<uint64_t>(fan_in[t]);
  }
  if (blocks >= 0x7fffffffull) return false;
  L->nblocks = static_cast<uint32_t>(blocks);
  L->tasks_off = round8(sizeof(dlsim::BatchTableHeader));
  L->map_off = round8(L->tasks_off + sizeof(dlsim::BatchTaskDesc) * static_cast<size_t>(b));
  L->ptrs_off = round8(L->map_off + sizeof(uint32_t) * static_cast<size_t>(blocks));
  L->w_off = round8(L->ptrs_off + sizeof(void*) * static_cast<size_t>(ptrs));
  L->bytes = round8(L->w_off + sizeof(float) * static_cast<size_t>(ptrs));
  return true;
}

template <class Op>
int table_fill(int b, const int* fan_in, const void* const* in, const float* w, void* const* outs,
               const size_t* nelem, void* h_table, size_t bytes) {
  TableLayout L;
  if (!table_layout<Op>(b, fan_in, nelem, &L)) return fail(DLSIM_E_ARG, "batch too large");
  if (bytes < L.bytes) return fail(DLSIM_E_ARG, "table buffer too small (%zu < %zu)", bytes, L.bytes);
  if (cross_task_overlap(b, fan_in, in, outs, nelem, Op::kBytes))
    return fail(DLSIM_E_ARG,
                "a task's output overlaps another task's input or output: one table launch runs all tasks "
                "concurrently (use separate calls, or dlsim_wreduce_batched, which orders them)");
  unsigned char* base = static_cast<unsigned char*>(h_table);
  std::memset(base, 0, L.bytes);
  auto* h = reinterpret_cast<dlsim::BatchTableHeader*>(base);
  auto* tasks = reinterpret_cast<dlsim::BatchTaskDesc*>(base + L.tasks_off);
  auto* map = reinterpret_cast<uint32_t*>(base + L.map_off);
  auto* ptrs = reinterpret_cast<const void**>(base + L.ptrs_off);
  auto* ws = reinterpret_cast<float*>(base + L.w_off);
  h->ntasks = static_cast<uint32_t>(b);
  h->nblocks = L.nblocks;
  h->tasks_off = L.tasks_off;
  h->map_off = L.map_off;
  h->ptrs_off = L.ptrs_off;
  h->w_off = L.w_off;
  uint32_t blk = 0, off = 0;
  bool uniform = true;
  for (int t = 0; t < b; ++t) {
    const size_t total = nelem[t] * Op::kBytes;
    if (fan_in[t] > DLSIM_MAX_FUSED_INPUTS || total > kMaxLaunchOutBytes || !aligned16(outs[t]))
      return fail(DLSIM_E_ARG, "task %d cannot be table-batched (fan-in <= %d, 16-B aligned, < 2 GiB)", t,
                  DLSIM_MAX_FUSED_INPUTS);
    const uint32_t nb = task_blocks<Op>(nelem[t]);
    tasks[t].out = outs[t];
    tasks[t].nvec = nelem[t] / Op::E;
    tasks[t].nelem = nelem[t];
    tasks[t].block_start = blk;
    tasks[t].ptr_off = off;
    tasks[t].fan_in = static_cast<uint32_t>(fan_in[t]);
    for (uint32_t k = 0; k < nb; ++k) map[blk + k] = static_cast<uint32_t>(t);
    for (int i = 0; i < fan_in[t]; ++i) {
      if (!aligned16(in[off + i]))
        return fail(DLSIM_E_ARG, "task %d input %d is not 16-byte aligned", t, i);
      ptrs[off + i] = in[off + i];
      ws[off + i] = w[off + i];
    }
    blk += nb;
    off += static_cast<uint32_t>(fan_in[t]);
    uniform = uniform && fan_in[t] == fan_in[0];
  }
  h->uniform_fan_in = uniform ? static_cast<uint32_t>(fan_in[0]) : 0u;
  return DLSIM_OK;
}

template <class Op, int NF>
hipError_t launch_table_nf(const void* d_table, uint32_t blocks, hipStream_t st) {
  hipLaunchKernelGGL((dlsim::k_wreduce_batch_table<Op, NF, group_size<Op>(), kVpt, kNT, store_policy<Op>()>),
                     dim3(blocks), dim3(dlsim::kBlock), 0, st, static_cast<const unsigned char*>(d_table));
  return hipGetLastError();
}

template <class Op, int K>
hipError_t launch_table_fixed(const void* d_table, int n, uint32_t blocks, hipStream_t st) {
  if constexpr (K > max_fixed_fan_in<Op>()) {
    return launch_table_nf<Op, 0>(d_table, blocks, st);
  } else {
    if (n == K) return launch_table_nf<Op, K>(d_table, blocks, st);
    return launch_table_fixed<Op, K + 1>(d_table, n, blocks, st);
  }
}

template <class Op>
int table_launch(const void* h_table, const void* d_table, hipStream_t st) {
  const auto* h = static_cast<const dlsim::BatchTableHeader*>(h_table);
  if (h->ntasks == 0) return DLSIM_OK;
  hipError_t e = h->uniform_fan_in ? launch_table_fixed<Op, 1>(d_table, static_cast<int>(h->uniform_fan_in),
                                                               h->nblocks, st)
                                   : launch_table_nf<Op, 0>(d_table, h->nblocks, st);
  if (e != hipSuccess) return hip_fail(e, "table batch launch");
  return DLSIM_OK;
}

size_t elem_bytes(int dtype) { return dtype == DLSIM_F32 ? 4 : 2; }

bool known_dtype(int dtype) { return dtype == DLSIM_F32 || dtype == DLSIM_BF16 || dtype == DLSIM_F16; }

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

int check_args(const void* const* in, int n, const float* w, const void* out, size_t nelem,
               int dtype, int mode, bool need_w = true) {
  if (!known_dtype(dtype)) return fail(DLSIM_E_DTYPE, "unsupported dtype %d", dtype);
  if (mode != DLSIM_EXACT && mode != DLSIM_FAST) return fail(DLSIM_E_MODE, "unsupported mode %d", mode);
  if (n < 1) return fail(DLSIM_E_ARG, "n must be >= 1 (got %d)", n);
  if (!in || (need_w && !w)) return fail(DLSIM_E_ARG, "null inputs or weights array");
  if (nelem == 0) return DLSIM_OK;
  if (!out) return fail(DLSIM_E_ARG, "null output pointer");
  const size_t bytes = nelem * elem_bytes(dtype);
  const uintptr_t o0 = reinterpret_cast<uintptr_t>(out), o1 = o0 + bytes;
  for (int i = 0; i < n; ++i) {
    if (!in[i]) return fail(DLSIM_E_ARG, "null input pointer at index %d", i);
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(in[i]), a1 = a0 + bytes;
    // Exact aliasing (out == in[i]) is safe for every i: the reduce is one
    // pass, and a lane reads all n terms of an element before writing it.
    // Partial overlap is not.
    if (a0 != o0 && a0 < o1 && o0 < a1)
      return fail(DLSIM_E_ARG, "output partially overlaps input %d", i);
  }
  return DLSIM_OK;
}

int dispatch(const void* const* in, int n, const float* w, void* out, size_t nelem, int dtype,
             int mode, hipStream_t st) {
  return with_policy(dtype, mode, [&](auto op) { return run<decltype(op)>(in, n, w, out, nelem, st); });
}

// ---- chunk mean in PyTorch's CPU order (chunk_mean_kernels.hpp) --------------
// First column that ATen's cascade_sum folds in row_sum (ilp) order, for an
// [m, n] fp32 reduction over dim 0 at `threads` intra-op threads
// (parallel_dim_reduction's column split, 32-column rounding; the 8-wide
// vectorized_outer_sum blocks of 32 columns; scalar_outer_sum's groups of 4
// under 8 columns). n == 1 is the inner reduction (all "ilp"/inner).
size_t chunk_mean_ilp_begin(int m, size_t n, int threads) {
  if (n <= 1) return 0;
  size_t b = 0, e = n;
  if (!(static_cast<unsigned long long>(m) * n < 32768ULL || threads <= 1)) {
    const size_t tp = static_cast<size_t>(threads) < n ? static_cast<size_t>(threads) : n;
    const size_t cs = (n + tp - 1) / tp;
    for (size_t t = 0; t < tp; ++t) {
      size_t tb = t * cs;
      if (tb >= n) break;
      size_t te = tb + cs < n ? tb + cs : n;
      tb -= tb % 32;
      if (te != n) te -= te % 32;
      if (tb < te) {
        b = tb;
        e = te;
      }
    }
  }
  const size_t s1 = e - b;
  return b + (s1 >= 8 ? s1 / 32 * 32 : s1 / 4 * 4);
}

// Chunk mean tiles: VPT 4, wave map, 8 rows per load group. Block and wave
// maps, VPT 2/4 and 8/16 rows in flight measured within +-3% of each other
// (profiles/r01_tune_chunk_mean_shapes.log); the wave map matches the fp32
// reduce's shape.
using CmDefault = dlsim::CmShape<4, true, 8>;

template <class Op>
int run_chunk_mean(int b, const int* fan_in, const void* const* in, void* const* outs, const size_t* nelem,
                   int threads, hipStream_t st) {
  constexpr size_t tile = static_cast<size_t>(dlsim::kBlock) * CmDefault::VPT;
  std::vector<size_t> off(static_cast<size_t>(b) + 1, 0);
  for (int t = 0; t < b; ++t) off[t + 1] = off[t] + static_cast<size_t>(fan_in[t]);
  if (b > 1 && cross_task_overlap(b, fan_in, in, outs, nelem, Op::kBytes)) {
    // tasks touch each other's outputs: one launch per task, in order
    for (int t = 0; t < b; ++t) {
      int rc = run_chunk_mean<Op>(1, fan_in + t, in + off[t], outs + t, nelem + t, threads, st);
      if (rc != DLSIM_OK) return rc;
    }
    return DLSIM_OK;
  }
  auto task_flags = [&](int t) {
    bool vec = aligned16(outs[t]);
    for (int i = 0; i < fan_in[t] && vec; ++i) vec = aligned16(in[off[t] + i]);
    uint8_t f = vec ? dlsim::kCmVec : 0;
    if (nelem[t] == 1 && fan_in[t] >= 8) f |= dlsim::kCmInner;
    return f;
  };
  auto task_blocks = [&](int t, size_t ib) { return ib / Op::E / tile + 1; };
  dlsim::ChunkMeanSlots s;
  std::memset(&s, 0, sizeof(s));
  int nt = 0, np = 0;
  size_t blocks = 0;
  auto flush = [&]() -> int {
    if (nt == 0) return DLSIM_OK;
    s.ntasks = nt;
    s.block_start[nt] = static_cast<uint32_t>(blocks);
    hipLaunchKernelGGL((dlsim::k_chunk_mean_batch<Op, CmDefault>), dim3(static_cast<unsigned>(blocks)),
                       dim3(dlsim::kBlock), 0, st, s);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "chunk mean batch launch");
    std::memset(&s, 0, sizeof(s));
    nt = np = 0;
    blocks = 0;
    return DLSIM_OK;
  };
  for (int t = 0; t < b; ++t) {
    const size_t n = nelem[t];
    if (n == 0) continue;
    const int m = fan_in[t];
    const size_t ib = chunk_mean_ilp_begin(m, n, threads);
    const uint8_t flags = task_flags(t);
    const size_t tb = task_blocks(t, ib);
    if (m > dlsim::kCmMaxPtrs) {
      // input pointers through a stream-ordered device array (any m)
      void* d = nullptr;
      const size_t bytes = static_cast<size_t>(m) * sizeof(void*);
      hipError_t e = hipMallocAsync(&d, bytes, st);
      if (e != hipSuccess) return hip_fail(e, "chunk mean pointer table alloc");
      // pageable source: the copy is staged before the call returns
      e = hipMemcpyAsync(d, in + off[t], bytes, hipMemcpyHostToDevice, st);
      if (e == hipSuccess) {
        hipLaunchKernelGGL((dlsim::k_chunk_mean_table<Op, CmDefault>), dim3(static_cast<unsigned>(tb)),
                           dim3(dlsim::kBlock), 0, st, static_cast<const void* const*>(d), m, outs[t], n, ib,
                           flags);
        e = hipGetLastError();
      }
      hipError_t e2 = hipFreeAsync(d, st);
      if (e != hipSuccess) return hip_fail(e, "chunk mean table launch");
      if (e2 != hipSuccess) return hip_fail(e2, "chunk mean pointer table free");
      continue;
    }
    if (nt == dlsim::kCmMaxTasks || np + m > dlsim::kCmMaxPtrs || blocks + tb > 0x7fffffffu) {
      int rc = flush();
      if (rc != DLSIM_OK) return rc;
    }
    s.block_start[nt] = static_cast<uint32_t>(blocks);
    s.ptr_off[nt] = static_cast<uint16_t>(np);
    s.m[nt] = static_cast<uint16_t>(m);
    s.out[nt] = outs[t];
    s.nelem[nt] = n;
    s.ilp_begin[nt] = ib;
    s.flags[nt] = flags;
    for (int i = 0; i < m; ++i) s.p[np + i] = in[off[t] + i];
    np += m;
    blocks += tb;
    ++nt;
  }
  return flush();
}

// ---- RCCL, bound at run time --------------------------------------------------
// The sharded entry point drives collectives on a caller's RCCL communicator.
// The library does not link RCCL: dlsim_rccl_bind() dlopens the copy the
// caller already uses (for a PyTorch process, the librccl.so next to
// libtorch_hip.so, whose communicator ProcessGroupNCCL._comm_ptr() returns),
// so one RCCL instance owns the communicator and its calls.
typedef int rccl_result_t;  // ncclResult_t
struct Rccl {
  void* lib = nullptr;
  rccl_result_t (*bcast)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
  rccl_result_t (*group_start)() = nullptr;
  rccl_result_t (*group_end)() = nullptr;
  rccl_result_t (*count)(void*, int*) = nullptr;
  rccl_result_t (*user_rank)(void*, int*) = nullptr;
  const char* (*err)(rccl_result_t) = nullptr;
};
Rccl g_rccl;
constexpr int kRcclFloat16 = 6, kRcclFloat32 = 7, kRcclBfloat16 = 9;  // ncclDataType_t (rccl.h)

int rccl_fail(rccl_result_t r, const char* what) {
  return fail(DLSIM_E_RCCL, "%s: %s (ncclResult %d)", what, g_rccl.err ? g_rccl.err(r) : "?", r);
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
// on_unit(u) for u = 0, 1, ... as each unit completes, in order, on this
// thread. Below ~1 MiB of input the helpers stay asleep: their wake-up costs
// more than they save.
template <class F>
void pack_and_dispatch(dlsim::PackJob& job, int threads, size_t in_bytes, F&& on_unit) {
  const int helpers = in_bytes < (size_t{1} << 20) ? 0 : std::min(std::max(threads, 1), 64) - 1;
  dlsim::PackPool& pool = dlsim::PackPool::get();
  std::lock_guard<std::mutex> lk(pool.call_mutex());
  if (helpers > 0) pool.start(&job, helpers);
  for (size_t u = 0; u < job.units;) {
    if (job.unit_done(u)) {
      on_unit(u++);
    } else if (!job.run_one()) {
      std::this_thread::yield();
    }
  }
  if (helpers > 0) pool.join();
}

// Staging layout of dlsim_host_chunk_mean: input rows back to back, each at
// a 256-B aligned offset.
size_t staged_row_elems(size_t n, size_t esz) {
  const size_t al = 256 / esz;
  return (n + al - 1) / al * al;
}

}  // namespace

extern "C" {

int dlsim_wreduce(const void* const* d_inputs, int n, const float* h_weights, void* d_out,
                  size_t n_elems, int dtype, int mode, void* stream) {
  g_err.clear();
  int rc = check_args(d_inputs, n, h_weights, d_out, n_elems, dtype, mode);
  if (rc != DLSIM_OK) return rc;
  return dispatch(d_inputs, n, h_weights, d_out, n_elems, dtype, mode,
                  static_cast<hipStream_t>(stream));
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
  if (!known_dtype(dtype)) return fail(DLSIM_E_DTYPE, "unsupported dtype %d", dtype);
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
  if (!known_dtype(dtype)) return fail(DLSIM_E_DTYPE, "unsupported dtype %d", dtype);
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
    int rc = check_args(d_inputs + off, fan_in[t], nullptr, d_outs[t], n_elems[t], dtype, DLSIM_EXACT, false);
    if (rc != DLSIM_OK) return fail(rc, "task %d: %s", t, g_err.c_str());
    if (fan_in[t] > 65535) return fail(DLSIM_E_ARG, "task %d: fan-in %d > 65535", t, fan_in[t]);
    if (n_elems[t] * elem_bytes(dtype) >= kMaxLaunchOutBytes)
      return fail(DLSIM_E_ARG, "task %d: chunk of %zu elements is >= 2 GiB", t, n_elems[t]);
    off += static_cast<size_t>(fan_in[t]);
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  return with_mean_policy(dtype, [&](auto op) {
    return run_chunk_mean<decltype(op)>(b, fan_in, d_inputs, d_outs, n_elems, cpu_threads, st);
  });
}

int dlsim_rccl_bind(const char* librccl_path) {
  g_err.clear();
  if (!librccl_path || !*librccl_path) return fail(DLSIM_E_ARG, "null/empty librccl path");
  void* h = dlopen(librccl_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return fail(DLSIM_E_RCCL, "dlopen(%s): %s", librccl_path, dlerror());
  Rccl r;
  r.lib = h;
  r.bcast = reinterpret_cast<decltype(r.bcast)>(dlsym(h, "ncclBroadcast"));
  r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
  r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
  r.count = reinterpret_cast<decltype(r.count)>(dlsym(h, "ncclCommCount"));
  r.user_rank = reinterpret_cast<decltype(r.user_rank)>(dlsym(h, "ncclCommUserRank"));
  r.err = reinterpret_cast<decltype(r.err)>(dlsym(h, "ncclGetErrorString"));
  if (!r.bcast || !r.group_start || !r.group_end || !r.count || !r.user_rank || !r.err)
    return fail(DLSIM_E_RCCL, "%s lacks an RCCL symbol", librccl_path);
  g_rccl = r;
  return DLSIM_OK;
}

int dlsim_wreduce_sharded(const void* const* d_slices, size_t slice_elems, int n, const float* h_weights,
                          void* d_out, size_t n_elems, int dtype, int mode, void* rccl_comm, int gather,
                          void* stream) {
  g_err.clear();
  if (!g_rccl.lib) return fail(DLSIM_E_RCCL, "RCCL not bound (call dlsim_rccl_bind first)");
  if (!rccl_comm) return fail(DLSIM_E_ARG, "null RCCL communicator");
  int world = 0, rank = 0;
  rccl_result_t rr = g_rccl.count(rccl_comm, &world);
  if (rr != 0) return rccl_fail(rr, "ncclCommCount");
  rr = g_rccl.user_rank(rccl_comm, &rank);
  if (rr != 0) return rccl_fail(rr, "ncclCommUserRank");
  if (n_elems > 0 && !d_out) return fail(DLSIM_E_ARG, "null output pointer");
  size_t b = 0, e = 0;
  int rc = dlsim_shard_range(n_elems, world, rank, 64, &b, &e);
  if (rc != DLSIM_OK) return rc;
  if (slice_elems != e - b)
    return fail(DLSIM_E_ARG, "rank %d of %d: slices have %zu elements, its shard [%zu, %zu) has %zu", rank, world,
                slice_elems, b, e, e - b);
  const size_t esz = elem_bytes(dtype);
  char* out = static_cast<char*>(d_out);
  // this rank's slice of every model -> this rank's slice of the output
  if (e > b) {
    rc = dlsim_wreduce(d_slices, n, h_weights, out + b * esz, e - b, dtype, mode, stream);
    if (rc != DLSIM_OK) return rc;
  } else {
    rc = check_args(d_slices, n, h_weights, nullptr, 0, dtype, mode);
    if (rc != DLSIM_OK) return rc;
  }
  if (!gather || world == 1 || n_elems == 0) return DLSIM_OK;
  // variable-size all-gather: every rank broadcasts its slice in place
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int dt = dtype == DLSIM_BF16 ? kRcclBfloat16 : dtype == DLSIM_F16 ? kRcclFloat16 : kRcclFloat32;
  rr = g_rccl.group_start();
  if (rr != 0) return rccl_fail(rr, "ncclGroupStart");
  for (int r = 0; r < world; ++r) {
    size_t rb = 0, re = 0;
    dlsim_shard_range(n_elems, world, r, 64, &rb, &re);
    if (re == rb) continue;
    rr = g_rccl.bcast(out + rb * esz, out + rb * esz, re - rb, dt, r, rccl_comm, st);
    if (rr != 0) {
      g_rccl.group_end();
      return rccl_fail(rr, "ncclBroadcast");
    }
  }
  rr = g_rccl.group_end();
  if (rr != 0) return rccl_fail(rr, "ncclGroupEnd");
  return DLSIM_OK;
}

int dlsim_host_wreduce(int n, int t, const void* const* h_srcs, const size_t* numels,
                       const float* h_weights, void* h_staging, void* d_rows, size_t row_stride,
                       void* d_out, void* h_out, int dtype, int mode, size_t chunk_elems, int threads,
                       void* stream, void* h2d_stream, void* d2h_stream) {
  g_err.clear();
  if (!known_dtype(dtype)) return fail(DLSIM_E_DTYPE, "unsupported dtype %d", dtype);
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
  hipStream_t h2d = h2d_stream ? static_cast<hipStream_t>(h2d_stream) : st;
  hipStream_t d2h = d2h_stream ? static_cast<hipStream_t>(d2h_stream) : st;
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
  pack_and_dispatch(job, threads, total * esz * n, [&](size_t u) {
    if (ln.rc != DLSIM_OK) return;
    const size_t c = u / n, i = u % n;
    const size_t c0 = c * chunk, c1 = std::min(total, c0 + chunk);
    const size_t o = i * row_bytes + c0 * esz;
    hipError_t e = hipMemcpyAsync(rows + o, stage + o, (c1 - c0) * esz, hipMemcpyHostToDevice, h2d);
    if (e != hipSuccess) {
      ln.rc = hip_fail(e, "staging H2D");
      return;
    }
    if (i + 1 < static_cast<size_t>(n)) return;
    ln.link(h2d, st, "order reduce after H2D");
    if (ln.rc != DLSIM_OK) return;
    for (int r = 0; r < n; ++r) ins[r] = rows + r * row_bytes + c0 * esz;
    ln.rc = dispatch(ins.data(), n, h_weights, out + c0 * esz, c1 - c0, dtype, mode, st);
    if (ln.rc != DLSIM_OK || !h_out) return;
    ln.link(st, d2h, "order D2H after reduce");
    if (ln.rc != DLSIM_OK) return;
    e = hipMemcpyAsync(static_cast<char*>(h_out) + c0 * esz, out + c0 * esz, (c1 - c0) * esz,
                       hipMemcpyDeviceToHost, d2h);
    if (e != hipSuccess) ln.rc = hip_fail(e, "result D2H");
  });
  if (h_out) ln.link(d2h, st, "order stream after D2H");
  return ln.rc;
}

int dlsim_host_chunk_mean(int b, const int* fan_in, const void* const* h_inputs, const size_t* n_elems,
                          void* h_staging, void* d_staging, size_t staging_elems, void* const* d_outs,
                          void* const* h_outs, int dtype, int cpu_threads, int threads, void* stream,
                          void* h2d_stream, void* d2h_stream) {
  g_err.clear();
  if (b < 0) return fail(DLSIM_E_ARG, "b must be >= 0 (got %d)", b);
  if (b == 0) return DLSIM_OK;
  if (!fan_in || !h_inputs || !d_outs || !n_elems) return fail(DLSIM_E_ARG, "null array argument");
  if (!known_dtype(dtype)) return fail(DLSIM_E_DTYPE, "unsupported dtype %d", dtype);
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
  hipStream_t h2d = h2d_stream ? static_cast<hipStream_t>(h2d_stream) : st;
  hipStream_t d2h = d2h_stream ? static_cast<hipStream_t>(d2h_stream) : st;
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
  StreamLinks ln;
  ln.link(st, h2d, "order H2D after stream");
  if (h_outs) ln.link(st, d2h, "order D2H after stream");
  std::vector<const void*> ins;
  size_t task_first = 0;  // first row of the current task
  pack_and_dispatch(job, threads, need * esz, [&](size_t r) {
    if (ln.rc != DLSIM_OK) return;
    const int t = static_cast<int>(row_task[r]);
    const size_t n = n_elems[t];
    if (n > 0) {
      hipError_t e = hipMemcpyAsync(ds + row_off[r] * esz, hs + row_off[r] * esz, n * esz, hipMemcpyHostToDevice, h2d);
      if (e != hipSuccess) {
        ln.rc = hip_fail(e, "staging H2D");
        return;
      }
    }
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
    ln.rc = with_mean_policy(dtype, [&](auto op) {
      return run_chunk_mean<decltype(op)>(1, &fan_in[t], ins.data(), &out, &n_elems[t], cpu_threads, st);
    });
    if (ln.rc != DLSIM_OK || !h_outs || !h_outs[t]) return;
    ln.link(st, d2h, "order D2H after chunk mean");
    if (ln.rc != DLSIM_OK) return;
    hipError_t e = hipMemcpyAsync(h_outs[t], out, n * esz, hipMemcpyDeviceToHost, d2h);
    if (e != hipSuccess) ln.rc = hip_fail(e, "result D2H");
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
  pack_and_dispatch(job, threads, total, [](size_t) {});
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

int dlsim_probe_copy(const void* d_src, void* d_dst, size_t bytes, void* stream) {
  g_err.clear();
  if (!d_src || !d_dst) return fail(DLSIM_E_ARG, "null pointer");
  if (bytes % 16 != 0 || !aligned16(d_src) || !aligned16(d_dst))
    return fail(DLSIM_E_ARG, "probe_copy needs 16-byte aligned sizes and pointers");
  const size_t nvec = bytes / 16;
  if (nvec == 0) return DLSIM_OK;
  dlsim::Slots<16> s;
  std::memset(&s, 0, sizeof(s));
  s.p[0] = d_src;
  s.w[0] = 1.0f;
  s.div = 1.0f;
  if (bytes > kMaxLaunchOutBytes) return fail(DLSIM_E_ARG, "probe_copy is limited to < 2 GiB");
  hipError_t e =
      launch_tiles<dlsim::CopyProbe, dlsim::Slots<16>, 1>(s, 1, d_dst, nvec * 4, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "probe_copy launch");
  return DLSIM_OK;
}

const char* dlsim_last_error(void) { return g_err.c_str(); }

int dlsim_version(void) { return (1 << 16) | 0; }

}  // extern "C"
