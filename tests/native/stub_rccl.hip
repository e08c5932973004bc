// stub_rccl.hip — TEST INFRASTRUCTURE: a stand-in for the RCCL entry points
// dlsim_wreduce_sharded binds (dlsim_rccl_bind dlopens this file), so its
// agreement step and gather path run with W > 1 ranks on ONE GPU.
//
// A stub communicator names a world size W, this rank r, this rank's full
// output buffer and the full output buffers the other W - 1 ranks would hold
// (pre-filled by the test). ncclBroadcast(root) of an in-place slice copies
// that slice from root's buffer (hipMemcpyAsync on the caller's stream) and
// logs (root, byte offset, count), which is exactly what the real grouped
// broadcasts deliver when every rank runs the call. ncclAllGather (in place)
// fills every other rank's padded segment from the sources the test set.
// Host code only.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

namespace {

struct StubComm {
  int world;
  int rank;
  char* own_out;
  size_t own_bytes = 0;  // 0 = not set (then any in-place slice at or past own_out is taken as own_out's)
  std::vector<char*> peer_out;
  struct Call {
    int root;
    size_t offset_bytes;
    size_t count;
    int dtype;
  };
  std::vector<Call> calls;
  // the other ranks' contributions to an int64 MAX all-reduce (already
  // max-combined), set by the test; empty = they contribute this rank's words
  std::vector<int64_t> peer_words;
  int allreduces = 0;
  // ncclAllGather: segment q comes from gather_src[q] (set by the test)
  std::vector<char*> gather_src;
  struct Gather {
    size_t count;
    int dtype;
    size_t send_offset_bytes;  // sendbuff - recvbuff
  };
  std::vector<Gather> gathers;
  int group_depth = 0;
  int max_group_depth = 0;
};

size_t nccl_bytes(int dtype) {
  switch (dtype) {
    case 6:  // ncclFloat16
    case 9:  // ncclBfloat16
      return 2;
    case 7:  // ncclFloat32
      return 4;
    case 8:  // ncclFloat64
      return 8;
    default:
      return 0;
  }
}

int g_depth = 0;

}  // namespace

extern "C" {

int ncclGroupStart() {
  ++g_depth;
  return 0;
}

int ncclGroupEnd() {
  if (g_depth <= 0) return 5;  // ncclInvalidUsage
  --g_depth;
  return 0;
}

int ncclCommCount(void* comm, int* count) {
  if (!comm || !count) return 4;  // ncclInvalidArgument
  *count = static_cast<StubComm*>(comm)->world;
  return 0;
}

int ncclCommUserRank(void* comm, int* rank) {
  if (!comm || !rank) return 4;
  *rank = static_cast<StubComm*>(comm)->rank;
  return 0;
}

const char* ncclGetErrorString(int) { return "stub RCCL error"; }

int ncclBroadcast(const void* sendbuff, void* recvbuff, size_t count, int datatype, int root, void* comm,
                  hipStream_t stream) {
  StubComm* c = static_cast<StubComm*>(comm);
  const size_t esz = nccl_bytes(datatype);
  if (!c || esz == 0 || root < 0 || root >= c->world) return 4;
  if (sendbuff != recvbuff) return 4;  // dlsim broadcasts in place
  char* dst = static_cast<char*>(recvbuff);
  if (g_depth > c->max_group_depth) c->max_group_depth = g_depth;
  if (c->own_bytes > 0 && (dst < c->own_out || dst + count * esz > c->own_out + c->own_bytes)) {
    // a buffer other than own_out (a failed rank's stand-in): logged, not filled
    c->calls.push_back({root, static_cast<size_t>(-1), count, datatype});
    return 0;
  }
  if (dst < c->own_out) return 4;
  const size_t off = static_cast<size_t>(dst - c->own_out);
  c->calls.push_back({root, off, count, datatype});
  if (root == c->rank || count == 0) return 0;
  const hipError_t e = hipMemcpyAsync(dst, c->peer_out[root] + off, count * esz, hipMemcpyDeviceToDevice, stream);
  return e == hipSuccess ? 0 : 1;  // ncclUnhandledCudaError
}

// int64 MAX only (the agreement step): this rank's words, max-combined with
// the peers' words the test set. Host-synchronous (test infrastructure).
int ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, int datatype, int op, void* comm,
                  hipStream_t stream) {
  StubComm* c = static_cast<StubComm*>(comm);
  if (!c || datatype != 4 || op != 2) return 4;  // ncclInt64, ncclMax
  if (g_depth > 0) return 5;                     // not inside the broadcast group
  std::vector<int64_t> w(count);
  if (hipMemcpyAsync(w.data(), sendbuff, count * 8, hipMemcpyDeviceToHost, stream) != hipSuccess) return 1;
  if (hipStreamSynchronize(stream) != hipSuccess) return 1;
  for (size_t k = 0; k < count && k < c->peer_words.size(); ++k)
    if (c->peer_words[k] > w[k]) w[k] = c->peer_words[k];
  ++c->allreduces;
  if (hipMemcpyAsync(recvbuff, w.data(), count * 8, hipMemcpyHostToDevice, stream) != hipSuccess) return 1;
  return hipStreamSynchronize(stream) == hipSuccess ? 0 : 1;
}

// In place only (sendbuff = recvbuff + rank * count elements): segment q of
// recvbuff is copied from the source the test set for rank q.
int ncclAllGather(const void* sendbuff, void* recvbuff, size_t count, int datatype, void* comm, hipStream_t stream) {
  StubComm* c = static_cast<StubComm*>(comm);
  const size_t esz = nccl_bytes(datatype);
  if (!c || esz == 0) return 4;
  const size_t seg = count * esz;
  char* recv = static_cast<char*>(recvbuff);
  const char* send = static_cast<const char*>(sendbuff);
  if (send != recv + static_cast<size_t>(c->rank) * seg) return 4;  // dlsim gathers in place
  if (g_depth > 0) return 5;
  c->gathers.push_back({count, datatype, static_cast<size_t>(send - recv)});
  if (c->gather_src.size() != static_cast<size_t>(c->world)) return 4;
  for (int q = 0; q < c->world; ++q) {
    if (q == c->rank || seg == 0) continue;
    if (hipMemcpyAsync(recv + static_cast<size_t>(q) * seg, c->gather_src[q], seg, hipMemcpyDeviceToDevice,
                       stream) != hipSuccess)
      return 1;
  }
  return 0;
}

// ---- test helpers ------------------------------------------------------------
void* stub_comm_create(int world, int rank, void* own_out, void* const* peer_out) {
  StubComm* c = new StubComm;
  c->world = world;
  c->rank = rank;
  c->own_out = static_cast<char*>(own_out);
  for (int q = 0; q < world; ++q) c->peer_out.push_back(static_cast<char*>(peer_out[q]));
  return c;
}

void stub_comm_destroy(void* comm) { delete static_cast<StubComm*>(comm); }

// Size of own_out: broadcasts into any other buffer are then logged, not filled.
void stub_comm_set_out_bytes(void* comm, size_t bytes) { static_cast<StubComm*>(comm)->own_bytes = bytes; }

// Broadcast calls logged so far (at most max written); returns their number.
int stub_comm_calls(void* comm, int* roots, size_t* offsets, size_t* counts, int max) {
  StubComm* c = static_cast<StubComm*>(comm);
  const int n = static_cast<int>(c->calls.size());
  for (int k = 0; k < n && k < max; ++k) {
    roots[k] = c->calls[k].root;
    offsets[k] = c->calls[k].offset_bytes;
    counts[k] = c->calls[k].count;
  }
  return n;
}

int stub_comm_max_group_depth(void* comm) { return static_cast<StubComm*>(comm)->max_group_depth; }

void stub_comm_set_peer_words(void* comm, const int64_t* w, int n) {
  static_cast<StubComm*>(comm)->peer_words.assign(w, w + n);
}

int stub_comm_allreduces(void* comm) { return static_cast<StubComm*>(comm)->allreduces; }

void stub_comm_set_gather_sources(void* comm, void* const* src) {
  StubComm* c = static_cast<StubComm*>(comm);
  c->gather_src.clear();
  for (int q = 0; q < c->world; ++q) c->gather_src.push_back(static_cast<char*>(src[q]));
}

// ncclAllGather calls so far; the first one's count (elements per segment)
// and in-place send offset (bytes) go to *count / *send_off when non-null.
int stub_comm_gathers(void* comm, size_t* count, size_t* send_off) {
  StubComm* c = static_cast<StubComm*>(comm);
  if (!c->gathers.empty()) {
    if (count) *count = c->gathers[0].count;
    if (send_off) *send_off = c->gathers[0].send_offset_bytes;
  }
  return static_cast<int>(c->gathers.size());
}

}  // extern "C"
