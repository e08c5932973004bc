// dlsim_abi.hip — the C ABI of include/dlsim.h over the gfx950 kernels of
// wreduce_kernels.hpp. Host-side dispatch only: argument checks, choice of
// vector vs scalar kernel, kernarg packing, multi-pass for n > 128.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "dlsim.h"
#include "wreduce_kernels.hpp"

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
constexpr size_t kMaxLaunchOutBytes = (size_t{1} << 31) - (size_t{1} << 20);
template <class Op> constexpr int max_fixed_fan_in() { return Op::kBytes == 4 ? 14 : 9; }
template <class Op> constexpr int group_size() { return Op::kBytes == 4 ? 8 : 4; }

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

template <class Op, int NB, int NF>
hipError_t launch_tiles(const dlsim::Slots<NB>& s, int n, const void* acc_in, void* out, size_t nelem,
                        hipStream_t st) {
  const size_t nvec = nelem / Op::E;
  const size_t tile = static_cast<size_t>(dlsim::kBlock) * kVpt;
  const size_t blocks = nvec / tile + 1;  // full tiles + one block for the ragged end
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  hipLaunchKernelGGL((dlsim::k_wreduce_tiles<Op, NB, NF, group_size<Op>(), kVpt, kNT, kStore>),
                     dim3(static_cast<unsigned>(blocks)), dim3(dlsim::kBlock), 0, st, s, n, acc_in, out,
                     nvec, nelem);
  return hipGetLastError();
}

template <class Op, int K>
hipError_t launch_fixed_k(const dlsim::Slots<16>& s, int n, void* out, size_t nelem, hipStream_t st) {
  if constexpr (K > max_fixed_fan_in<Op>()) {
    return hipErrorInvalidValue;
  } else {
    if (n == K) return launch_tiles<Op, 16, K>(s, n, nullptr, out, nelem, st);
    return launch_fixed_k<Op, K + 1>(s, n, out, nelem, st);
  }
}

template <class Op>
hipError_t launch_fixed(const dlsim::Slots<16>& s, int n, void* out, size_t nelem, hipStream_t st) {
  return launch_fixed_k<Op, 1>(s, n, out, nelem, st);
}

template <class Op, int NB>
hipError_t launch_pass(const dlsim::Slots<NB>& s, int n, const void* acc_in, void* out,
                       size_t nelem, bool vec, hipStream_t st) {
  if (vec) {
    if constexpr (NB == 16) {
      if (!acc_in && n <= max_fixed_fan_in<Op>()) return launch_fixed<Op>(s, n, out, nelem, st);
    }
    return launch_tiles<Op, NB, 0>(s, n, acc_in, out, nelem, st);
  }
  const size_t blocks = (nelem + dlsim::kBlock - 1) / dlsim::kBlock;
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  hipLaunchKernelGGL((dlsim::k_wreduce_scalar<Op, NB>), dim3(static_cast<unsigned>(blocks)),
                     dim3(dlsim::kBlock), 0, st, s, n, acc_in, out, nelem);
  return hipGetLastError();
}

// Packs up to NB inputs into kernel arguments and launches one pass.
template <class Op, int NB>
hipError_t pass_nb(const void* const* in, const float* w, int cnt, const void* acc_in, void* out,
                   size_t nelem, bool vec, hipStream_t st) {
  dlsim::Slots<NB> s;
  std::memset(&s, 0, sizeof(s));
  for (int i = 0; i < cnt; ++i) {
    s.p[i] = in[i];
    s.w[i] = w[i];
  }
  return launch_pass<Op, NB>(s, cnt, acc_in, out, nelem, vec, st);
}

template <class Op>
int run_range(const void* const* in, int n, const float* w, void* out, size_t nelem, bool vec,
              hipStream_t st);

// Elements are independent: an output longer than one launch's 2 GiB store
// window is reduced as consecutive ranges (pointers offset by the range start).
template <class Op>
int run(const void* const* in, int n, const float* w, void* out, size_t nelem, hipStream_t st) {
  if (nelem == 0) return DLSIM_OK;
  bool vec = aligned16(out);
  for (int i = 0; i < n && vec; ++i) vec = aligned16(in[i]);
  const size_t chunk = kMaxLaunchOutBytes / Op::kBytes;  // multiple of every tile size
  if (!vec || nelem <= chunk) return run_range<Op>(in, n, w, out, nelem, vec, st);
  std::vector<const void*> sub(static_cast<size_t>(n));
  for (size_t b = 0; b < nelem; b += chunk) {
    const size_t len = std::min(chunk, nelem - b);
    for (int i = 0; i < n; ++i) sub[i] = static_cast<const char*>(in[i]) + b * Op::kBytes;
    int rc = run_range<Op>(sub.data(), n, w, static_cast<char*>(out) + b * Op::kBytes, len, vec, st);
    if (rc != DLSIM_OK) return rc;
  }
  return DLSIM_OK;
}

template <class Op>
int run_range(const void* const* in, int n, const float* w, void* out, size_t nelem, bool vec,
              hipStream_t st) {
  // Passes of <= DLSIM_MAX_FUSED_INPUTS inputs; pass k > 0 continues the sum
  // held in `out` (stored exactly: fp32, or bf16-valued in EXACT bf16).
  for (int i0 = 0; i0 < n; i0 += DLSIM_MAX_FUSED_INPUTS) {
    const int cnt = std::min(DLSIM_MAX_FUSED_INPUTS, n - i0);
    const void* acc_in = (i0 == 0) ? nullptr : out;
    hipError_t e = (cnt <= 16)
                       ? pass_nb<Op, 16>(in + i0, w + i0, cnt, acc_in, out, nelem, vec, st)
                       : pass_nb<Op, DLSIM_MAX_FUSED_INPUTS>(in + i0, w + i0, cnt, acc_in, out,
                                                             nelem, vec, st);
    if (e != hipSuccess) return hip_fail(e, "kernel launch");
  }
  return DLSIM_OK;
}

size_t elem_bytes(int dtype) { return dtype == DLSIM_BF16 ? 2 : 4; }

int check_args(const void* const* in, int n, const float* w, const void* out, size_t nelem,
               int dtype, int mode) {
  if (dtype != DLSIM_F32 && dtype != DLSIM_BF16) return fail(DLSIM_E_DTYPE, "unsupported dtype %d", dtype);
  if (mode != DLSIM_EXACT && mode != DLSIM_FAST) return fail(DLSIM_E_MODE, "unsupported mode %d", mode);
  if (n < 1) return fail(DLSIM_E_ARG, "n must be >= 1 (got %d)", n);
  if (!in || !w) return fail(DLSIM_E_ARG, "null inputs or weights array");
  if (nelem == 0) return DLSIM_OK;
  if (!out) return fail(DLSIM_E_ARG, "null output pointer");
  const size_t bytes = nelem * elem_bytes(dtype);
  const uintptr_t o0 = reinterpret_cast<uintptr_t>(out), o1 = o0 + bytes;
  for (int i = 0; i < n; ++i) {
    if (!in[i]) return fail(DLSIM_E_ARG, "null input pointer at index %d", i);
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(in[i]), a1 = a0 + bytes;
    // Exact aliasing (out == in[i]) is safe: a lane reads every input of an
    // element before it writes that element. Partial overlap is not.
    if (a0 != o0 && a0 < o1 && o0 < a1)
      return fail(DLSIM_E_ARG, "output partially overlaps input %d", i);
  }
  return DLSIM_OK;
}

int dispatch(const void* const* in, int n, const float* w, void* out, size_t nelem, int dtype,
             int mode, hipStream_t st) {
  if (dtype == DLSIM_F32)
    return mode == DLSIM_EXACT ? run<dlsim::F32Exact>(in, n, w, out, nelem, st)
                               : run<dlsim::F32Fast>(in, n, w, out, nelem, st);
  return mode == DLSIM_EXACT ? run<dlsim::BF16Exact>(in, n, w, out, nelem, st)
                             : run<dlsim::BF16Fast>(in, n, w, out, nelem, st);
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
  const void* col[DLSIM_MAX_FUSED_INPUTS];
  for (int k = 0; k < t; ++k) {
    // Gather tensor k of every model; n may exceed the stack column, so go
    // in slices that continue the sum like the flat path's passes.
    for (int i0 = 0; i0 < n; i0 += DLSIM_MAX_FUSED_INPUTS) {
      const int cnt = std::min(DLSIM_MAX_FUSED_INPUTS, n - i0);
      for (int i = 0; i < cnt; ++i) col[i] = d_inputs[static_cast<size_t>(i0 + i) * t + k];
      int rc = check_args(col, cnt, h_weights + i0, d_outs[k], numels[k], dtype, mode);
      if (rc != DLSIM_OK) return rc;
    }
  }
  for (int k = 0; k < t; ++k) {
    if (numels[k] == 0) continue;
    if (n <= DLSIM_MAX_FUSED_INPUTS) {
      for (int i = 0; i < n; ++i) col[i] = d_inputs[static_cast<size_t>(i) * t + k];
      int rc = dispatch(col, n, h_weights, d_outs[k], numels[k], dtype, mode,
                        static_cast<hipStream_t>(stream));
      if (rc != DLSIM_OK) return rc;
    } else {
      std::vector<const void*> full(static_cast<size_t>(n));
      for (int i = 0; i < n; ++i) full[i] = d_inputs[static_cast<size_t>(i) * t + k];
      int rc = dispatch(full.data(), n, h_weights, d_outs[k], numels[k], dtype, mode,
                        static_cast<hipStream_t>(stream));
      if (rc != DLSIM_OK) return rc;
    }
  }
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
  constexpr int VPT = 4;
  const size_t blocks = (nvec + dlsim::kBlock * VPT - 1) / (dlsim::kBlock * VPT);
  hipLaunchKernelGGL((dlsim::k_copy16<VPT>), dim3(static_cast<unsigned>(blocks)), dim3(dlsim::kBlock), 0,
                     static_cast<hipStream_t>(stream), static_cast<const dlsim::u32x4*>(d_src),
                     static_cast<dlsim::u32x4*>(d_dst), nvec);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(e, "probe_copy launch");
  return DLSIM_OK;
}

const char* dlsim_last_error(void) { return g_err.c_str(); }

int dlsim_version(void) { return (1 << 16) | 0; }

}  // extern "C"
