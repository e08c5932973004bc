// Probe (round 6, session 4): how fast can a kernel read page-locked host rows
// over PCIe, by launch shape? The zero-copy host task (dlsim_host_wreduce_zc)
// runs the device-tuned reduce on mapped host rows: cfg1's 2 x 341 KB took
// ~30 us in round 5 (~22 GB/s). Here the same weighted sum of n host rows
// into a host result, shapes: lanes per block x float4 per lane, grid =
// every element once; plus hipMemcpyAsync H2D of the same bytes for scale.
// HIP events around K launches of each, one JSON line per (n, shape).
//
//   hipcc --offload-arch=gfx950 -O3 scripts/probes/zc_shape_probe.hip -o zc_shape_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
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

struct Rows {
  const f4* p[8];
  float w[8];
};

template <int VPT>
__global__ void k_sum(const Rows r, int n, f4* out, size_t nvec) {
  const size_t base = (static_cast<size_t>(blockIdx.x) * blockDim.x) * VPT + threadIdx.x;
  f4 x[8][VPT];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i < n)
#pragma unroll
      for (int u = 0; u < VPT; ++u) {
        const size_t v = base + static_cast<size_t>(u) * blockDim.x;
        x[i][u] = v < nvec ? __builtin_nontemporal_load(r.p[i] + v) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < n) a += r.w[i] * x[i][u];
    const size_t v = base + static_cast<size_t>(u) * blockDim.x;
    if (v < nvec) out[v] = a;
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 200;
  const size_t elems = 85354;  // GNLeNet
  const size_t nvec = (elems + 3) / 4;
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int n : {2, 7}) {
    std::vector<f4*> h(n), d(n);
    for (int i = 0; i < n; ++i) {
      CHECK(hipHostMalloc(&h[i], nvec * 16, hipHostMallocDefault));
      for (size_t v = 0; v < nvec; ++v) h[i][v] = f4{1.f, 2.f, 3.f, 4.f};
      CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d[i]), h[i], 0));
    }
    f4 *hout, *dout, *dev_rows;
    CHECK(hipHostMalloc(&hout, nvec * 16, hipHostMallocDefault));
    CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dout), hout, 0));
    CHECK(hipMalloc(&dev_rows, nvec * 16 * n));
    Rows r{};
    for (int i = 0; i < n; ++i) {
      r.p[i] = d[i];
      r.w[i] = 1.0f / n;
    }
    const int lanes[] = {64, 128, 256, 512, 1024};
    for (int vpt : {1, 2, 4}) {
      for (int L : lanes) {
        const unsigned grid = static_cast<unsigned>((nvec + static_cast<size_t>(L) * vpt - 1) / (static_cast<size_t>(L) * vpt));
        auto launch = [&]() {
          if (vpt == 1) hipLaunchKernelGGL(k_sum<1>, dim3(grid), dim3(L), 0, st, r, n, dout, nvec);
          else if (vpt == 2) hipLaunchKernelGGL(k_sum<2>, dim3(grid), dim3(L), 0, st, r, n, dout, nvec);
          else hipLaunchKernelGGL(k_sum<4>, dim3(grid), dim3(L), 0, st, r, n, dout, nvec);
        };
        for (int k = 0; k < 10; ++k) launch();
        CHECK(hipStreamSynchronize(st));
        CHECK(hipEventRecord(e0, st));
        for (int k = 0; k < K; ++k) launch();
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / K;
        printf("{\"n\": %d, \"form\": \"zero_copy\", \"lanes\": %d, \"vpt\": %d, \"blocks\": %u, \"us\": %.3f, "
               "\"read_GBps\": %.1f}\n",
               n, L, vpt, grid, us, n * nvec * 16 / us / 1e3);
        fflush(stdout);
      }
    }
    // the DMA path's copy of the same rows, for scale
    CHECK(hipStreamSynchronize(st));
    CHECK(hipEventRecord(e0, st));
    for (int k = 0; k < K; ++k)
      for (int i = 0; i < n; ++i)
        CHECK(hipMemcpyAsync(dev_rows + i * nvec, h[i], nvec * 16, hipMemcpyHostToDevice, st));
    CHECK(hipEventRecord(e1, st));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"n\": %d, \"form\": \"h2d_memcpy_per_row\", \"us\": %.3f, \"read_GBps\": %.1f}\n", n, ms * 1e3 / K,
           n * nvec * 16 / (ms * 1e3 / K) / 1e3);
    fflush(stdout);
    for (int i = 0; i < n; ++i) CHECK(hipHostFree(h[i]));
    CHECK(hipHostFree(hout));
    CHECK(hipFree(dev_rows));
  }
  return 0;
}
