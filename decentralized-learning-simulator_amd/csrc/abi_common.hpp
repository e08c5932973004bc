// abi_common.hpp — what the C ABI's translation units share (dlsim_abi.hip:
// the single-GPU and host entry points; sharded_abi.hip: the RCCL ones):
// the thread-local error string, argument checks, and the RCCL entry points
// bound at run time. Host code only; everything here has hidden visibility.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "dlsim.h"

namespace dlsim_host __attribute__((visibility("hidden"))) {

inline thread_local std::string g_err;

inline int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

inline int hip_fail(hipError_t e, const char* what) {
  return fail(DLSIM_E_HIP - static_cast<int>(e), "%s: %s", what, hipGetErrorString(e));
}

inline size_t elem_bytes(int dtype) { return dtype == DLSIM_F64 ? 8 : dtype == DLSIM_F32 ? 4 : 2; }

// dtypes of the float-weight entry points (fp64 buffers take dlsim_wreduce_f64)
inline bool known_dtype(int dtype) { return dtype == DLSIM_F32 || dtype == DLSIM_BF16 || dtype == DLSIM_F16; }

inline int dtype_fail(int dtype) {
  if (dtype == DLSIM_F64)
    return fail(DLSIM_E_DTYPE, "DLSIM_F64 buffers go through dlsim_wreduce_f64 (double weights)");
  return fail(DLSIM_E_DTYPE, "unsupported dtype %d", dtype);
}

inline int check_args(const void* const* in, int n, const void* w, const void* out, size_t nelem, int dtype,
                      int mode, bool need_w = true, bool f64_ok = false) {
  if (!known_dtype(dtype) && !(f64_ok && dtype == DLSIM_F64)) return dtype_fail(dtype);
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
    if (a0 != o0 && a0 < o1 && o0 < a1) return fail(DLSIM_E_ARG, "output partially overlaps input %d", i);
  }
  return DLSIM_OK;
}

// ---- RCCL, bound at run time --------------------------------------------------
// The sharded entry points drive collectives on a caller's RCCL communicator.
// The library does not link RCCL: dlsim_rccl_bind() dlopens the copy the
// caller already uses (for a PyTorch process, the librccl.so next to
// libtorch_hip.so, whose communicator ProcessGroupNCCL._comm_ptr() returns),
// so one RCCL instance owns the communicator and its calls.
typedef int rccl_result_t;  // ncclResult_t
struct Rccl {
  void* lib = nullptr;
  rccl_result_t (*bcast)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
  rccl_result_t (*allreduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
  rccl_result_t (*allgather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
  rccl_result_t (*group_start)() = nullptr;
  rccl_result_t (*group_end)() = nullptr;
  rccl_result_t (*count)(void*, int*) = nullptr;
  rccl_result_t (*user_rank)(void*, int*) = nullptr;
  const char* (*err)(rccl_result_t) = nullptr;
};
inline Rccl g_rccl;
constexpr int kRcclFloat16 = 6, kRcclFloat32 = 7, kRcclFloat64 = 8, kRcclBfloat16 = 9;  // ncclDataType_t (rccl.h)
constexpr int kRcclInt64 = 4, kRcclMax = 2;                                            // ncclInt64, ncclMax

inline int rccl_fail(rccl_result_t r, const char* what) {
  return fail(DLSIM_E_RCCL, "%s: %s (ncclResult %d)", what, g_rccl.err ? g_rccl.err(r) : "?", r);
}

inline int rccl_dtype(int dtype) {
  return dtype == DLSIM_BF16 ? kRcclBfloat16 : dtype == DLSIM_F16 ? kRcclFloat16 : dtype == DLSIM_F64 ? kRcclFloat64
                                                                                                     : kRcclFloat32;
}

}  // namespace dlsim_host
