// sharded_abi.hip — the parameter-sharded aggregate on a caller's RCCL
// communicator (include/dlsim.h: dlsim_rccl_bind, dlsim_wreduce_sharded[_f64],
// dlsim_sharded_plan_*). One process per GPU; rank r of W reduces its
// contiguous slice [b_r, e_r) = dlsim_shard_range(n_elems, W, r, 64) of every
// model with the single-GPU kernels (dlsim_wreduce / dlsim_wreduce_f64), so
// every element's N terms are still folded in input order on one GPU and the
// result is bit-identical to one GPU (the reference is
// single-process CPU, fedavg.py:12-26). The gather that materialises the whole
// output on every rank is one of
//   DLSIM_GATHER_BCAST      every rank broadcasts its slice in place in d_out,
//                           W ncclBroadcast in one group (variable-size slices,
//                           no padding, no extra copy);
//   DLSIM_GATHER_ALLGATHER  one in-place ncclAllGather of equal-width padded
//                           segments in a scratch buffer (the local reduce
//                           writes straight into this rank's segment), then
//                           one unpad kernel that moves the W segments to
//                           their offsets in d_out.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <type_traits>
#include <vector>

#include "abi_common.hpp"

// The opaque plan of dlsim_sharded_plan_create: everything that shapes the
// collectives, agreed by every rank once.
struct dlsim_sharded_plan {
  void* comm;
  int world, rank;
  size_t n_elems;
  int n, dtype, gather;
  size_t b, e;      // this rank's slice
  size_t width;     // ALLGATHER: elements per padded segment (a multiple of 64)
  void* scratch;    // ALLGATHER, W > 1: world * width elements
};

namespace dlsim_host __attribute__((visibility("hidden"))) {

constexpr size_t kShardAlign = 64;   // elements: every slice but the last is a multiple (256 B of fp32)
constexpr int kMaxUnpadRanks = 64;   // ALLGATHER: ranks the unpad kernel's arguments hold

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct UnpadArgs {
  const char* src;
  char* dst;
  uint64_t seg_bytes;
  uint64_t dst_off[kMaxUnpadRanks];
  uint64_t len[kMaxUnpadRanks];
};

// Segment r (blockIdx.y) of the gathered padded buffer -> its slice of the
// output: 16-B vectors when both sides are 16-B aligned, bytes for the tail
// (the last rank's ragged end) or a misaligned output.
__global__ __launch_bounds__(256) void k_unpad(const UnpadArgs a) {
  const int r = static_cast<int>(blockIdx.y);
  const char* s = a.src + static_cast<uint64_t>(r) * a.seg_bytes;
  char* d = a.dst + a.dst_off[r];
  const uint64_t len = a.len[r];
  const bool vec = (reinterpret_cast<uintptr_t>(s) % 16 == 0) && (reinterpret_cast<uintptr_t>(d) % 16 == 0);
  const uint64_t nv = vec ? len / 16 : 0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (uint64_t v = tid; v < nv; v += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s) + v),
                                reinterpret_cast<u32x4*>(d) + v);
  for (uint64_t i = nv * 16 + tid; i < len; i += stride) d[i] = s[i];
}

struct Geometry {
  size_t b = 0, e = 0, width = 0;
  std::vector<size_t> begins, ends;
};

Geometry geometry(size_t n_elems, int world, int rank) {
  Geometry g;
  g.begins.resize(static_cast<size_t>(world));
  g.ends.resize(static_cast<size_t>(world));
  for (int r = 0; r < world; ++r) {
    dlsim_shard_range(n_elems, world, r, kShardAlign, &g.begins[r], &g.ends[r]);
    g.width = std::max(g.width, g.ends[r] - g.begins[r]);
  }
  g.width = (g.width + kShardAlign - 1) / kShardAlign * kShardAlign;
  g.b = g.begins[static_cast<size_t>(rank)];
  g.e = g.ends[static_cast<size_t>(rank)];
  return g;
}

// The agreement step: one int64 MAX all-reduce of
// [a failure slot per rank | a_0, -a_0, a_1, -a_1, ...] on the caller's
// stream, read back by the host. Every rank learns which ranks failed their
// local checks (or their local reduce's launch) and whether all ranks agree
// on the arguments that shape the collectives, so either every rank enters
// them or none does.
int sharded_agree(void* comm, int world, int rank, bool local_fail, const std::vector<int64_t>& args, hipStream_t st,
                  std::vector<int>* failed, bool* mismatch) {
  const size_t nw = static_cast<size_t>(world) + 2 * args.size();
  std::vector<int64_t> w(nw, 0);
  w[static_cast<size_t>(rank)] = local_fail ? 1 : 0;
  for (size_t k = 0; k < args.size(); ++k) {
    w[world + 2 * k] = args[k];
    w[world + 2 * k + 1] = -args[k];
  }
  void* d = nullptr;
  const size_t bytes = sizeof(int64_t) * nw;
  hipError_t e = hipMallocAsync(&d, bytes, st);
  if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(agreement)");
  int rc = DLSIM_OK;
  e = hipMemcpyAsync(d, w.data(), bytes, hipMemcpyHostToDevice, st);
  if (e != hipSuccess) rc = hip_fail(e, "hipMemcpyAsync(agreement H2D)");
  if (rc == DLSIM_OK) {
    const rccl_result_t rr = g_rccl.allreduce(d, d, nw, kRcclInt64, kRcclMax, comm, st);
    if (rr != 0) rc = rccl_fail(rr, "ncclAllReduce(agreement)");
  }
  if (rc == DLSIM_OK) {
    e = hipMemcpyAsync(w.data(), d, bytes, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) rc = hip_fail(e, "agreement D2H");
  }
  (void)hipFreeAsync(d, st);
  if (rc != DLSIM_OK) return rc;
  failed->clear();
  for (int r = 0; r < world; ++r)
    if (w[static_cast<size_t>(r)] != 0) failed->push_back(r);
  *mismatch = false;
  for (size_t k = 0; k < args.size(); ++k) *mismatch |= w[world + 2 * k] != -w[world + 2 * k + 1];
  return DLSIM_OK;
}

// What every rank returns after the agreement: its own error, DLSIM_E_PEER
// naming the failed ranks, or DLSIM_E_DISAGREE.
int agreement_verdict(int rc, const std::string& local_err, const std::vector<int>& failed, bool mismatch,
                      int world, const char* what) {
  if (rc != DLSIM_OK) {
    g_err = local_err;
    return rc;
  }
  if (!failed.empty()) {
    std::string who;
    for (int r : failed) who += (who.empty() ? "" : ",") + std::to_string(r);
    return fail(DLSIM_E_PEER, "rank(s) %s of %d failed their checks; no rank %s", who.c_str(), world, what);
  }
  if (mismatch) return fail(DLSIM_E_DISAGREE, "ranks disagree on the collective's arguments; no rank %s", what);
  return DLSIM_OK;
}

// DLSIM_GATHER_BCAST: every rank broadcasts its slice of `out` in place, one group.
int gather_bcast(char* out, const Geometry& g, int world, size_t esz, int dt, void* comm, hipStream_t st) {
  rccl_result_t rr = g_rccl.group_start();
  if (rr != 0) return rccl_fail(rr, "ncclGroupStart");
  for (int r = 0; r < world; ++r) {
    const size_t rb = g.begins[r], re = g.ends[r];
    if (re == rb) continue;
    rr = g_rccl.bcast(out + rb * esz, out + rb * esz, re - rb, dt, r, comm, st);
    if (rr != 0) {
      g_rccl.group_end();
      return rccl_fail(rr, "ncclBroadcast");
    }
  }
  rr = g_rccl.group_end();
  if (rr != 0) return rccl_fail(rr, "ncclGroupEnd");
  return DLSIM_OK;
}

// DLSIM_GATHER_ALLGATHER: one in-place all-gather of the equal-width segments
// of `scratch` (this rank's is at rank * width), then (out != nullptr) one
// unpad launch that moves every segment's slice to its offset in `out`.
int gather_allgather(char* scratch, char* out, const Geometry& g, int world, int rank, size_t esz, int dt, void* comm,
                     hipStream_t st) {
  const size_t seg = g.width * esz;
  const rccl_result_t rr = g_rccl.allgather(scratch + static_cast<size_t>(rank) * seg, scratch, g.width, dt, comm, st);
  if (rr != 0) return rccl_fail(rr, "ncclAllGather");
  if (!out) return DLSIM_OK;
  UnpadArgs a{};
  a.src = scratch;
  a.dst = out;
  a.seg_bytes = seg;
  size_t longest = 0;
  for (int r = 0; r < world; ++r) {
    a.dst_off[r] = g.begins[r] * esz;
    a.len[r] = (g.ends[r] - g.begins[r]) * esz;
    longest = std::max<size_t>(longest, a.len[r]);
  }
  const size_t blocks = std::min<size_t>(std::max<size_t>((longest / 16 + 255) / 256, 1), 1024);
  hipLaunchKernelGGL(k_unpad, dim3(static_cast<unsigned>(blocks), static_cast<unsigned>(world)), dim3(256), 0, st, a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? DLSIM_OK : hip_fail(e, "k_unpad launch");
}

int comm_shape(void* comm, int* world, int* rank) {
  if (!g_rccl.lib) return fail(DLSIM_E_RCCL, "RCCL not bound (call dlsim_rccl_bind first)");
  if (!comm) return fail(DLSIM_E_ARG, "null RCCL communicator");
  rccl_result_t rr = g_rccl.count(comm, world);
  if (rr != 0) return rccl_fail(rr, "ncclCommCount");
  rr = g_rccl.user_rank(comm, rank);
  if (rr != 0) return rccl_fail(rr, "ncclCommUserRank");
  return DLSIM_OK;
}

bool gather_ok(int gather) {
  return gather == DLSIM_GATHER_NONE || gather == DLSIM_GATHER_BCAST || gather == DLSIM_GATHER_ALLGATHER;
}

// The local reduce of this rank's slices into `target` (float or double
// weights), or only the argument checks when the slice is empty.
template <class W>
int local_reduce(const void* const* d_slices, int n, const W* h_weights, void* target, size_t len, int dtype,
                 int mode, void* stream) {
  if constexpr (std::is_same<W, double>::value) {
    if (len > 0) return dlsim_wreduce_f64(d_slices, n, h_weights, target, len, mode, stream);
    return check_args(d_slices, n, h_weights, nullptr, 0, dtype, mode, true, true);
  } else {
    if (len > 0) return dlsim_wreduce(d_slices, n, h_weights, target, len, dtype, mode, stream);
    return check_args(d_slices, n, h_weights, nullptr, 0, dtype, mode);
  }
}

// The body of dlsim_wreduce_sharded / _f64 (one call, agreement included).
template <class W>
int wreduce_sharded(const void* const* d_slices, size_t slice_elems, int n, const W* h_weights, void* d_out,
                    size_t n_elems, int dtype, int mode, void* rccl_comm, int gather, void* stream) {
  g_err.clear();
  int world = 0, rank = 0;
  if (const int rc0 = comm_shape(rccl_comm, &world, &rank); rc0 != DLSIM_OK) return rc0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  constexpr bool kF64 = std::is_same<W, double>::value;
  // Rank-local checks and the local reduce: a failure here is not returned
  // before the other ranks have heard of it (sharded_agree), so no rank is
  // left waiting inside a collective.
  int rc = DLSIM_OK;
  if (!gather_ok(gather)) rc = fail(DLSIM_E_ARG, "gather must be DLSIM_GATHER_NONE, _BCAST or _ALLGATHER (got %d)", gather);
  if (rc == DLSIM_OK && gather == DLSIM_GATHER_ALLGATHER && world > kMaxUnpadRanks)
    rc = fail(DLSIM_E_ARG, "DLSIM_GATHER_ALLGATHER takes at most %d ranks (got %d)", kMaxUnpadRanks, world);
  if (rc == DLSIM_OK && n_elems > 0 && !d_out) rc = fail(DLSIM_E_ARG, "null output pointer");
  const Geometry g = geometry(n_elems, world, rank);
  if (rc == DLSIM_OK && slice_elems != g.e - g.b)
    rc = fail(DLSIM_E_ARG, "rank %d of %d: slices have %zu elements, its shard [%zu, %zu) has %zu", rank, world,
              slice_elems, g.b, g.e, g.e - g.b);
  const bool dtype_ok = kF64 ? dtype == DLSIM_F64 : known_dtype(dtype);
  const size_t esz = dtype_ok ? elem_bytes(dtype) : 0;
  const bool padded = rc == DLSIM_OK && dtype_ok && gather == DLSIM_GATHER_ALLGATHER && world > 1 && n_elems > 0;
  char* out = static_cast<char*>(d_out);
  char* scratch = nullptr;
  if (padded) {
    const hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&scratch), static_cast<size_t>(world) * g.width * esz, st);
    if (e != hipSuccess) rc = hip_fail(e, "hipMallocAsync(all-gather segments)");
  }
  if (rc == DLSIM_OK) {
    void* target = padded ? static_cast<void*>(scratch + static_cast<size_t>(rank) * g.width * esz)
                          : static_cast<void*>(out + g.b * esz);
    rc = local_reduce(d_slices, n, h_weights, target, g.e - g.b, dtype, mode, stream);
  }
  if (world > 1) {
    const std::string local_err = g_err;
    std::vector<int> failed;
    bool mismatch = false;
    const int arc = sharded_agree(rccl_comm, world, rank, rc != DLSIM_OK,
                                  {static_cast<int64_t>(n_elems), dtype, gather}, st, &failed, &mismatch);
    int vrc = arc != DLSIM_OK ? arc : agreement_verdict(rc, local_err, failed, mismatch, world, "entered the gather");
    if (vrc == DLSIM_OK && gather != DLSIM_GATHER_NONE && n_elems > 0) {
      const int dt = rccl_dtype(dtype);
      vrc = padded ? gather_allgather(scratch, out, g, world, rank, esz, dt, rccl_comm, st)
                   : gather_bcast(out, g, world, esz, dt, rccl_comm, st);
    }
    if (scratch) (void)hipFreeAsync(scratch, st);
    return vrc;
  }
  if (scratch) (void)hipFreeAsync(scratch, st);
  return rc;
}

// The body of dlsim_sharded_plan_run / _f64: no agreement. A rank whose
// local checks or launch fail still enters the plan's gather (so no peer is
// left waiting in it) and then returns its error. Its peers get no error
// code, but its slice arrives as NaN everywhere: the rank fills its share
// with all-ones bytes, a NaN in every supported format, before the gather.
// A stale or partial slice would otherwise reach them as plausible numbers.
template <class W>
int plan_run(dlsim_sharded_plan* p, const void* const* d_slices, size_t slice_elems, const W* h_weights, void* d_out,
             int mode, void* stream) {
  g_err.clear();
  if (!p) return fail(DLSIM_E_ARG, "null plan");
  constexpr bool kF64 = std::is_same<W, double>::value;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t esz = elem_bytes(p->dtype);
  const bool padded = p->scratch != nullptr;
  char* out = static_cast<char*>(d_out);
  int rc = DLSIM_OK;
  if (kF64 != (p->dtype == DLSIM_F64))
    rc = fail(DLSIM_E_DTYPE, kF64 ? "plan is not DLSIM_F64: use dlsim_sharded_plan_run"
                                  : "DLSIM_F64 plan: use dlsim_sharded_plan_run_f64");
  if (rc == DLSIM_OK && p->n_elems > 0 && !d_out) rc = fail(DLSIM_E_ARG, "null output pointer");
  if (rc == DLSIM_OK && slice_elems != p->e - p->b)
    rc = fail(DLSIM_E_ARG, "rank %d of %d: slices have %zu elements, the plan's shard [%zu, %zu) has %zu", p->rank,
              p->world, slice_elems, p->b, p->e, p->e - p->b);
  if (rc == DLSIM_OK) {
    void* target = padded ? static_cast<void*>(static_cast<char*>(p->scratch) + static_cast<size_t>(p->rank) * p->width * esz)
                          : static_cast<void*>(out + p->b * esz);
    rc = local_reduce(d_slices, p->n, h_weights, target, p->e - p->b, p->dtype, mode, stream);
  }
  if (p->world == 1 || p->gather == DLSIM_GATHER_NONE || p->n_elems == 0) return rc;
  const std::string local_err = g_err;
  const Geometry g = geometry(p->n_elems, p->world, p->rank);
  const int dt = rccl_dtype(p->dtype);
  int crc;
  const size_t share = (p->e - p->b) * esz;
  if (padded) {
    if (rc != DLSIM_OK && share > 0)
      (void)hipMemsetAsync(static_cast<char*>(p->scratch) + static_cast<size_t>(p->rank) * p->width * esz, 0xff,
                           share, st);
    crc = gather_allgather(static_cast<char*>(p->scratch), out, g, p->world, p->rank, esz, dt, p->comm, st);
  } else {
    char* buf = out;
    if (!buf) {  // a failed rank without an output still sends and receives its share
      const hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&buf), p->n_elems * esz, st);
      if (e != hipSuccess) return hip_fail(e, "hipMallocAsync(stand-in output)");
    }
    if (rc != DLSIM_OK && share > 0) (void)hipMemsetAsync(buf + p->b * esz, 0xff, share, st);
    crc = gather_bcast(buf, g, p->world, esz, dt, p->comm, st);
    if (buf != out) (void)hipFreeAsync(buf, st);
  }
  if (rc != DLSIM_OK) {
    g_err = local_err;
    return rc;
  }
  return crc;
}

}  // namespace dlsim_host

using namespace dlsim_host;

extern "C" {

int dlsim_rccl_bind(const char* librccl_path) {
  g_err.clear();
  if (!librccl_path || !*librccl_path) return fail(DLSIM_E_ARG, "null/empty librccl path");
  void* h = dlopen(librccl_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return fail(DLSIM_E_RCCL, "dlopen(%s): %s", librccl_path, dlerror());
  Rccl r;
  r.lib = h;
  r.bcast = reinterpret_cast<decltype(r.bcast)>(dlsym(h, "ncclBroadcast"));
  r.allreduce = reinterpret_cast<decltype(r.allreduce)>(dlsym(h, "ncclAllReduce"));
  r.allgather = reinterpret_cast<decltype(r.allgather)>(dlsym(h, "ncclAllGather"));
  r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
  r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
  r.count = reinterpret_cast<decltype(r.count)>(dlsym(h, "ncclCommCount"));
  r.user_rank = reinterpret_cast<decltype(r.user_rank)>(dlsym(h, "ncclCommUserRank"));
  r.err = reinterpret_cast<decltype(r.err)>(dlsym(h, "ncclGetErrorString"));
  if (!r.bcast || !r.allreduce || !r.allgather || !r.group_start || !r.group_end || !r.count || !r.user_rank ||
      !r.err)
    return fail(DLSIM_E_RCCL, "%s lacks an RCCL symbol", librccl_path);
  g_rccl = r;
  return DLSIM_OK;
}

int dlsim_wreduce_sharded(const void* const* d_slices, size_t slice_elems, int n, const float* h_weights,
                          void* d_out, size_t n_elems, int dtype, int mode, void* rccl_comm, int gather,
                          void* stream) {
  return wreduce_sharded(d_slices, slice_elems, n, h_weights, d_out, n_elems, dtype, mode, rccl_comm, gather,
                         stream);
}

int dlsim_wreduce_sharded_f64(const void* const* d_slices, size_t slice_elems, int n, const double* h_weights,
                              void* d_out, size_t n_elems, int mode, void* rccl_comm, int gather, void* stream) {
  return wreduce_sharded(d_slices, slice_elems, n, h_weights, d_out, n_elems, DLSIM_F64, mode, rccl_comm, gather,
                         stream);
}

int dlsim_sharded_plan_create(void* rccl_comm, size_t n_elems, int n, int dtype, int gather, void* stream,
                              dlsim_sharded_plan** plan) {
  g_err.clear();
  if (!plan) return fail(DLSIM_E_ARG, "null plan pointer");
  *plan = nullptr;
  int world = 0, rank = 0;
  if (const int rc0 = comm_shape(rccl_comm, &world, &rank); rc0 != DLSIM_OK) return rc0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  int rc = DLSIM_OK;
  if (n < 1) rc = fail(DLSIM_E_ARG, "n must be >= 1 (got %d)", n);
  if (rc == DLSIM_OK && !known_dtype(dtype) && dtype != DLSIM_F64) rc = fail(DLSIM_E_DTYPE, "unsupported dtype %d", dtype);
  if (rc == DLSIM_OK && !gather_ok(gather))
    rc = fail(DLSIM_E_ARG, "gather must be DLSIM_GATHER_NONE, _BCAST or _ALLGATHER (got %d)", gather);
  if (rc == DLSIM_OK && gather == DLSIM_GATHER_ALLGATHER && world > kMaxUnpadRanks)
    rc = fail(DLSIM_E_ARG, "DLSIM_GATHER_ALLGATHER takes at most %d ranks (got %d)", kMaxUnpadRanks, world);
  const Geometry g = geometry(n_elems, world, rank);
  void* scratch = nullptr;
  if (rc == DLSIM_OK && gather == DLSIM_GATHER_ALLGATHER && world > 1 && n_elems > 0) {
    const hipError_t e = hipMalloc(&scratch, static_cast<size_t>(world) * g.width * elem_bytes(dtype));
    if (e != hipSuccess) {
      scratch = nullptr;
      rc = hip_fail(e, "hipMalloc(all-gather segments)");
    }
  }
  if (world > 1) {
    const std::string local_err = g_err;
    std::vector<int> failed;
    bool mismatch = false;
    const int arc = sharded_agree(rccl_comm, world, rank, rc != DLSIM_OK,
                                  {static_cast<int64_t>(n_elems), n, dtype, gather}, st, &failed, &mismatch);
    rc = arc != DLSIM_OK ? arc : agreement_verdict(rc, local_err, failed, mismatch, world, "created the plan");
  }
  if (rc != DLSIM_OK) {
    if (scratch) (void)hipFree(scratch);
    return rc;
  }
  *plan = new dlsim_sharded_plan{rccl_comm, world, rank, n_elems, n, dtype, gather, g.b, g.e, g.width, scratch};
  return DLSIM_OK;
}

int dlsim_sharded_plan_run(dlsim_sharded_plan* plan, const void* const* d_slices, size_t slice_elems,
                           const float* h_weights, void* d_out, int mode, void* stream) {
  return plan_run(plan, d_slices, slice_elems, h_weights, d_out, mode, stream);
}

int dlsim_sharded_plan_run_f64(dlsim_sharded_plan* plan, const void* const* d_slices, size_t slice_elems,
                               const double* h_weights, void* d_out, int mode, void* stream) {
  return plan_run(plan, d_slices, slice_elems, h_weights, d_out, mode, stream);
}

int dlsim_sharded_plan_destroy(dlsim_sharded_plan* plan) {
  g_err.clear();
  if (!plan) return DLSIM_OK;
  int rc = DLSIM_OK;
  if (plan->scratch) {
    const hipError_t e = hipFree(plan->scratch);
    if (e != hipSuccess) rc = hip_fail(e, "hipFree(all-gather segments)");
  }
  delete plan;
  return rc;
}

}  // extern "C"
