// tune_wreduce.hip — standalone tuning harness for the reduce kernels.
// Times launch-shape variants of k_wreduce_vec on rotating input sets (so
// the 256 MiB Infinity Cache cannot serve re-reads) with hipEvents around
// each launch, checks every variant bit-for-bit against the shipped shape,
// and prints one line per variant. Not part of the product library.
//
//   tune_wreduce [n] [P] [dtype f32|bf16] [mode exact|fast] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "wreduce_kernels.hpp"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

using namespace dlsim;

__global__ void k_fill(uint32_t* p, size_t nwords, uint32_t seed, int bf16) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < nwords; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    // finite values of moderate magnitude: exponent 120..127, random mantissa/sign
    uint32_t f = (h & 0x807fffffu) | ((120u + (h >> 28) % 8u) << 23);
    if (bf16) {
      const uint32_t lo = (h & 0x807fu) | ((120u + ((h >> 8) & 7u)) << 7);
      const uint32_t hi = ((h >> 16) & 0x807fu) | ((120u + ((h >> 24) & 7u)) << 7);
      f = lo | (hi << 16);
    }
    p[i] = f;
  }
}

struct Variant {
  const char* name;
  void (*launch)(const Slots<128>&, int, void*, size_t, size_t, hipStream_t);
};

template <class Op, int G, int VPT, bool NT>
void launch_v(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st) {
  const size_t per = (size_t)kBlock * VPT;
  size_t blocks = std::max<size_t>(1, (nvec + per - 1) / per);
  hipLaunchKernelGGL((k_wreduce_vec<Op, 128, G, VPT, NT>), dim3((unsigned)blocks), dim3(kBlock), 0,
                     st, s, n, nullptr, out, nvec, nelem);
}

template <class Op>
std::vector<Variant> variants() {
  return {
      {"G8_V1_nt", launch_v<Op, 8, 1, true>},   {"G8_V2_nt", launch_v<Op, 8, 2, true>},
      {"G8_V4_nt", launch_v<Op, 8, 4, true>},   {"G8_V1", launch_v<Op, 8, 1, false>},
      {"G8_V2", launch_v<Op, 8, 2, false>},     {"G8_V4", launch_v<Op, 8, 4, false>},
      {"G4_V2_nt", launch_v<Op, 4, 2, true>},   {"G16_V1_nt", launch_v<Op, 16, 1, true>},
      {"G16_V2_nt", launch_v<Op, 16, 2, true>},
  };
}

template <class Op>
int run(int n, size_t P, int reps, double peak_gbs) {
  const int sets = 3;
  const size_t bytes = P * Op::kBytes;
  const size_t nvec = P / Op::E;
  std::vector<void*> in((size_t)sets * n);
  std::vector<void*> out(sets);
  for (auto& p : in) CK(hipMalloc(&p, bytes + 256));
  for (auto& p : out) CK(hipMalloc(&p, bytes + 256));
  for (size_t k = 0; k < in.size(); ++k)
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, (uint32_t*)in[k], bytes / 4,
                       (uint32_t)(k * 7919 + 1), Op::kBytes == 2);
  CK(hipDeviceSynchronize());
  std::vector<Slots<128>> slots(sets);
  for (int s = 0; s < sets; ++s) {
    memset(&slots[s], 0, sizeof(Slots<128>));
    for (int i = 0; i < n; ++i) {
      slots[s].p[i] = in[(size_t)s * n + i];
      slots[s].w[i] = 1.0f / n + 0.001f * i;
    }
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::vector<hipEvent_t> ev(2 * reps);
  for (auto& e : ev) CK(hipEventCreate(&e));
  const double alg_bytes = (double)(n + 1) * bytes;

  auto vs = variants<Op>();
  // reference output of the first (shipped-like) variant on set 0
  std::vector<char> ref(bytes), got(bytes);
  vs[1].launch(slots[0], n, out[0], nvec, P, st);
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(ref.data(), out[0], bytes, hipMemcpyDeviceToHost));

  // interleaved rounds (one process, same device) — rule 24 of the guide
  const int rounds = 3;
  std::vector<std::vector<double>> med(vs.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t v = 0; v < vs.size(); ++v) {
      for (int w = 0; w < 10; ++w) vs[v].launch(slots[w % sets], n, out[w % sets], nvec, P, st);
      for (int k = 0; k < reps; ++k) {
        CK(hipEventRecord(ev[2 * k], st));
        vs[v].launch(slots[k % sets], n, out[k % sets], nvec, P, st);
        CK(hipEventRecord(ev[2 * k + 1], st));
      }
      CK(hipStreamSynchronize(st));
      std::vector<double> t(reps);
      for (int k = 0; k < reps; ++k) {
        float ms;
        CK(hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]));
        t[k] = ms * 1e3;
      }
      std::sort(t.begin(), t.end());
      med[v].push_back(t[reps / 2]);
    }
  }
  for (size_t v = 0; v < vs.size(); ++v) {
    vs[v].launch(slots[0], n, out[0], nvec, P, st);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(got.data(), out[0], bytes, hipMemcpyDeviceToHost));
    // compare only the vector part (tail elements are folded by every variant identically)
    const bool same = memcmp(ref.data(), got.data(), nvec * 16) == 0;
    std::sort(med[v].begin(), med[v].end());
    const double us = med[v][rounds / 2];
    const double gbs = alg_bytes / (us * 1e-6) / 1e9;
    printf("variant=%-10s n=%d P=%zu bytes=%.1fMB median_us=%.2f GBps=%.0f frac=%.3f same=%d\n", vs[v].name, n,
           P, alg_bytes / 1e6, us, gbs, gbs / peak_gbs, (int)same);
  }
  // copy ceiling on the same footprint
  {
    const size_t cbytes = (size_t)(alg_bytes / 2) & ~(size_t)15;
    void *a, *b;
    CK(hipMalloc(&a, cbytes));
    CK(hipMalloc(&b, cbytes));
    CK(hipMemset(a, 1, cbytes));
    std::vector<double> t;
    for (int k = 0; k < reps; ++k) {
      CK(hipEventRecord(ev[0], st));
      const size_t nv = cbytes / 16;
      hipLaunchKernelGGL((k_copy16<4>), dim3((unsigned)((nv + 1023) / 1024)), dim3(256), 0, st,
                         (const u32x4*)a, (u32x4*)b, nv);
      CK(hipEventRecord(ev[1], st));
      CK(hipEventSynchronize(ev[1]));
      float ms;
      CK(hipEventElapsedTime(&ms, ev[0], ev[1]));
      t.push_back(ms * 1e3);
    }
    std::sort(t.begin(), t.end());
    const double us = t[t.size() / 2];
    printf("copy16 bytes_moved=%.1fMB median_us=%.2f GBps=%.0f frac=%.3f\n", 2.0 * cbytes / 1e6, us,
           2.0 * cbytes / (us * 1e-6) / 1e9, 2.0 * cbytes / (us * 1e-6) / 1e9 / peak_gbs);
    CK(hipFree(a));
    CK(hipFree(b));
  }
  for (auto& p : in) CK(hipFree(p));
  for (auto& p : out) CK(hipFree(p));
  return 0;
}

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 8;
  size_t P = argc > 2 ? strtoull(argv[2], nullptr, 10) : 11181642ull;
  std::string dt = argc > 3 ? argv[3] : "f32";
  std::string mode = argc > 4 ? argv[4] : "exact";
  int reps = argc > 5 ? atoi(argv[5]) : 50;
  if (n < 1 || n > 128 || reps < 1 || reps > 10000) {
    fprintf(stderr, "bad args\n");
    return 1;
  }
  const double peak = 8000.0;  // GB/s, MI355X HBM3E spec
  if (dt == "f32")
    return mode == "exact" ? run<F32Exact>(n, P, reps, peak) : run<F32Fast>(n, P, reps, peak);
  return mode == "exact" ? run<BF16Exact>(n, P, reps, peak) : run<BF16Fast>(n, P, reps, peak);
}
