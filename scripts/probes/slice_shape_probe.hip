// Probe (round 6, session 4): the small slices' launch shape, again. At the
// 8-rank slice (8 x 1,397,760 fp32) the shipped grid is 342 blocks of 512
// lanes x 2 float4 on 256 CUs, all resident at once, so 86 CUs fetch two
// tiles and the rest one: the launch runs at the pace of the two-tile CUs.
// Smaller blocks spread the tiles more evenly (64-lane blocks: 21-22 per CU).
// Here the 8-input weighted sum (one fp32 fma chain per element, the reduce's
// traffic) for every (lanes, float4 per lane), over rotating inputs and
// outputs (>= 1 GiB each, a decoy set read first), HIP events around K
// launches; one JSON line per (size, shape).
//
//   hipcc --offload-arch=gfx950 -O3 scripts/probes/slice_shape_probe.hip -o slice_shape_probe
#include <hip/hip_runtime.h>

#include <algorithm>
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
__global__ void k_sum(const Rows r, f4* out, size_t nvec) {
  const size_t base = (static_cast<size_t>(blockIdx.x) * blockDim.x) * VPT + threadIdx.x;
  f4 x[8][VPT];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int u = 0; u < VPT; ++u) {
      const size_t v = base + static_cast<size_t>(u) * blockDim.x;
      x[i][u] = v < nvec ? __builtin_nontemporal_load(r.p[i] + v) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
  for (int u = 0; u < VPT; ++u) {
    f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i) a += r.w[i] * x[i][u];
    const size_t v = base + static_cast<size_t>(u) * blockDim.x;
    if (v < nvec) __builtin_nontemporal_store(a, out + v);
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 400;
  const size_t sizes[] = {1397760, 1048576, 2795456};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (size_t n : sizes) {
    const size_t nvec = n / 4;
    const size_t set_bytes = 8 * nvec * 16;
    const int sets = static_cast<int>(std::max<size_t>(3, ((size_t{1} << 30) + set_bytes - 1) / set_bytes)) + 1;
    const int outs = static_cast<int>(((size_t{1} << 30) + nvec * 16 - 1) / (nvec * 16)) + 1;
    std::vector<f4*> in(static_cast<size_t>(sets) * 8), out(static_cast<size_t>(outs));
    for (auto& b : in) {
      CHECK(hipMalloc(&b, nvec * 16));
      CHECK(hipMemset(b, 0, nvec * 16));
    }
    for (auto& b : out) CHECK(hipMalloc(&b, nvec * 16));
    std::vector<Rows> rows(static_cast<size_t>(sets));
    for (int s = 0; s < sets; ++s)
      for (int i = 0; i < 8; ++i) {
        rows[s].p[i] = in[static_cast<size_t>(s) * 8 + i];
        rows[s].w[i] = 0.125f;
      }
    const int T = sets - 1;  // set T is the decoy
    const int lanes[] = {64, 128, 256, 512};
    for (int rep = 0; rep < 2; ++rep)
      for (int vpt : {1, 2, 4})
        for (int L : lanes) {
          const unsigned grid =
              static_cast<unsigned>((nvec + static_cast<size_t>(L) * vpt - 1) / (static_cast<size_t>(L) * vpt));
          auto launch = [&](int s, int o) {
            if (vpt == 1) hipLaunchKernelGGL(k_sum<1>, dim3(grid), dim3(L), 0, 0, rows[s], out[o], nvec);
            else if (vpt == 2) hipLaunchKernelGGL(k_sum<2>, dim3(grid), dim3(L), 0, 0, rows[s], out[o], nvec);
            else hipLaunchKernelGGL(k_sum<4>, dim3(grid), dim3(L), 0, 0, rows[s], out[o], nvec);
          };
          for (int k = 0; k < 8; ++k) launch(T, outs - 1);
          for (int k = 0; k < 20; ++k) launch(k % T, k % (outs - 1));
          CHECK(hipDeviceSynchronize());
          CHECK(hipEventRecord(e0, 0));
          for (int k = 0; k < K; ++k) launch(k % T, k % (outs - 1));
          CHECK(hipEventRecord(e1, 0));
          CHECK(hipEventSynchronize(e1));
          float ms = 0;
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          const double us = ms * 1e3 / K;
          printf("{\"n\": %zu, \"rep\": %d, \"lanes\": %d, \"vpt\": %d, \"blocks\": %u, \"us\": %.3f, \"frac\": %.4f}\n",
                 n, rep, L, vpt, grid, us, 9.0 * nvec * 16 / us / 1e3 / 8000.0);
          fflush(stdout);
        }
    for (auto b : in) CHECK(hipFree(b));
    for (auto b : out) CHECK(hipFree(b));
  }
  return 0;
}
