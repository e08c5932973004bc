// Probe (round 6, session 4): do a D-PSGD round's overlapping inputs get
// served by the Infinity Cache if the reduce loads them with ordinary
// (temporal) loads instead of non-temporal ones? In a ring of P peers with
// fan-in 7 (peer i aggregates models i-3..i+3), consecutive aggregates share
// 6 of their 7 inputs. The first-set study showed
// non-temporal streams leave the cache's contents alone; here the same
// 7-input weighted sum over 100 ResNet-18-sized fp32 models (4.5 GB) is timed
// per aggregate with non-temporal and with ordinary loads, peers in ring
// order (maximal reuse) and in a shuffled order (little reuse), HIP events
// around three passes over the round. One JSON line per (order, loads).
//
//   hipcc --offload-arch=gfx950 -O3 scripts/probes/ring_reuse_probe.hip -o ring_reuse_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int F = 7;
struct Rows {
  const f4* p[F];
  float w[F];
};

template <bool NT>
__global__ __launch_bounds__(512) void k_sum(const Rows r, f4* out, size_t nvec) {
  const size_t base = static_cast<size_t>(blockIdx.x) * 1024 + threadIdx.x;
  f4 x[F][2];
#pragma unroll
  for (int i = 0; i < F; ++i)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const size_t v = base + u * 512;
      if (v < nvec) x[i][u] = NT ? __builtin_nontemporal_load(r.p[i] + v) : r.p[i][v];
      else x[i][u] = f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < F; ++i) a += r.w[i] * x[i][u];
    const size_t v = base + u * 512;
    if (v < nvec) __builtin_nontemporal_store(a, out + v);
  }
}

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 100;
  const size_t elems = argc > 2 ? strtoull(argv[2], nullptr, 10) : 11181642;
  const size_t nvec = elems / 4;
  f4* models;
  f4* outs;
  CHECK(hipMalloc(&models, static_cast<size_t>(P) * nvec * 16));
  CHECK(hipMalloc(&outs, static_cast<size_t>(P) * nvec * 16));
  CHECK(hipMemset(models, 0, static_cast<size_t>(P) * nvec * 16));
  std::vector<Rows> rows(P);
  for (int i = 0; i < P; ++i)
    for (int k = 0; k < F; ++k) {
      rows[i].p[k] = models + static_cast<size_t>((i + k - F / 2 + P) % P) * nvec;
      rows[i].w[k] = 1.0f / F;
    }
  std::vector<int> ring(P), shuffled(P);
  std::iota(ring.begin(), ring.end(), 0);
  shuffled = ring;
  std::shuffle(shuffled.begin(), shuffled.end(), std::mt19937(7));
  const unsigned grid = static_cast<unsigned>((nvec + 1023) / 1024);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // an ordinary 2 GiB copy evicts the caches between legs
  f4* flush;
  const size_t fl = (size_t{1} << 31) / 16;
  CHECK(hipMalloc(&flush, 2 * fl * 16));
  for (int rep = 0; rep < 2; ++rep)
    for (int ord = 0; ord < 2; ++ord)
      for (int nt = 1; nt >= 0; --nt) {
        const std::vector<int>& order = ord ? shuffled : ring;
        CHECK(hipMemcpy(flush + fl, flush, fl * 16, hipMemcpyDeviceToDevice));
        auto launch = [&](int i) {
          if (nt) hipLaunchKernelGGL(k_sum<true>, dim3(grid), dim3(512), 0, 0, rows[i], outs + static_cast<size_t>(i) * nvec, nvec);
          else hipLaunchKernelGGL(k_sum<false>, dim3(grid), dim3(512), 0, 0, rows[i], outs + static_cast<size_t>(i) * nvec, nvec);
        };
        for (int i : order) launch(i);  // warm-up pass
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        for (int pass = 0; pass < 3; ++pass)
          for (int i : order) launch(i);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / (3.0 * P);
        printf("{\"rep\": %d, \"order\": \"%s\", \"loads\": \"%s\", \"peers\": %d, \"elems\": %zu, "
               "\"us_per_aggregate\": %.3f, \"algorithmic_GBps\": %.1f}\n",
               rep, ord ? "shuffled" : "ring", nt ? "nt" : "plain", P, elems, us, (F + 1.0) * nvec * 16 / us / 1e3);
        fflush(stdout);
      }
  CHECK(hipFree(models));
  CHECK(hipFree(outs));
  CHECK(hipFree(flush));
  return 0;
}
