// Probe (round 6): does the kernel-argument load before a block's first input
// load cost a streaming reduce measurable time? The same 8-input fp32 sum
// (one tile of 256 lanes x 2 f4 per block, like the 8-rank slice's
// shape) launched back to back with its pointers (a) in a struct argument
// (scalar loads from the kernarg segment, then the input loads) and (b) as
// leading pointer arguments that the hardware preloads into SGPRs at wave
// launch (built with -mllvm -amdgpu-kernarg-preload-count=16; what does not
// fit is loaded as usual). HIP events around K launches over rotating
// inputs/outputs (>= 1 GiB), several sizes; one JSON line per (size, form).
//
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-kernarg-preload-count=16 \
//         scripts/probes/kernarg_preload_probe.hip -o kernarg_preload_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

struct Ptrs8 {
  const f4* p[8];
  float w[8];
};

__device__ __forceinline__ f4 ld(const f4* p, size_t i) { return __builtin_nontemporal_load(p + i); }

__device__ __forceinline__ void body(const f4* const (&p)[8], const float (&w)[8], f4* out, size_t nvec) {
  const size_t base = static_cast<size_t>(blockIdx.x) * 512 + threadIdx.x;
  f4 x[8][2];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const size_t v = base + u * 256;
      x[i][u] = v < nvec ? ld(p[i], v) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      a.x = a.x + w[i] * x[i][u].x;
      a.y = a.y + w[i] * x[i][u].y;
      a.z = a.z + w[i] * x[i][u].z;
      a.w = a.w + w[i] * x[i][u].w;
    }
    const size_t v = base + u * 256;
    if (v < nvec) __builtin_nontemporal_store(a, out + v);
  }
}

__global__ __launch_bounds__(256) void k_struct(const Ptrs8 s, f4* out, size_t nvec) {
  const f4* const p[8] = {s.p[0], s.p[1], s.p[2], s.p[3], s.p[4], s.p[5], s.p[6], s.p[7]};
  const float w[8] = {s.w[0], s.w[1], s.w[2], s.w[3], s.w[4], s.w[5], s.w[6], s.w[7]};
  body(p, w, out, nvec);
}

// nvec first: the full-tile test needs it before the first load; then as many
// pointers as the preload fits (16 SGPRs: nvec and p0..p6)
__global__ __launch_bounds__(256) void k_leading(size_t nvec, const f4* p0, const f4* p1, const f4* p2,
                                                 const f4* p3, const f4* p4, const f4* p5,
                                                 const f4* p6, const f4* p7, f4* out,
                                                 const Ptrs8 s) {
  const f4* const p[8] = {p0, p1, p2, p3, p4, p5, p6, p7};
  const float w[8] = {s.w[0], s.w[1], s.w[2], s.w[3], s.w[4], s.w[5], s.w[6], s.w[7]};
  body(p, w, out, nvec);
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 400;
  const size_t sizes[] = {1397760, 2795456, 11181642};
  for (size_t n : sizes) {
    const size_t nvec = n / 4;
    const size_t set_bytes = 9 * nvec * 16;
    const int sets = static_cast<int>(std::max<size_t>(3, ((size_t{1} << 30) + set_bytes - 1) / set_bytes));
    std::vector<f4*> bufs(static_cast<size_t>(sets) * 9);
    for (auto& b : bufs) {
      CHECK(hipMalloc(&b, nvec * 16));
      CHECK(hipMemset(b, 0, nvec * 16));
    }
    std::vector<Ptrs8> args(static_cast<size_t>(sets));
    for (int s = 0; s < sets; ++s)
      for (int i = 0; i < 8; ++i) {
        args[s].p[i] = bufs[static_cast<size_t>(s) * 9 + i];
        args[s].w[i] = 0.125f;
      }
    const unsigned grid = static_cast<unsigned>((nvec + 511) / 512);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
      for (int form = 0; form < 2; ++form) {
        auto launch = [&](int k) {
          const int s = k % sets;
          f4* out = bufs[static_cast<size_t>(s) * 9 + 8];
          const Ptrs8& a = args[static_cast<size_t>(s)];
          if (form == 0)
            hipLaunchKernelGGL(k_struct, dim3(grid), dim3(256), 0, 0, a, out, nvec);
          else
            hipLaunchKernelGGL(k_leading, dim3(grid), dim3(256), 0, 0, nvec, a.p[0], a.p[1], a.p[2], a.p[3],
                               a.p[4], a.p[5], a.p[6], a.p[7], out, a);
        };
        for (int k = 0; k < 20; ++k) launch(k);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0, 0));
        for (int k = 0; k < K; ++k) launch(k);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / K;
        printf("{\"n\": %zu, \"form\": \"%s\", \"rep\": %d, \"us_per_launch\": %.3f, \"GBps\": %.1f}\n", n,
               form ? "leading_preloaded" : "struct", rep, us, set_bytes / us / 1e3);
        fflush(stdout);
      }
    }
    for (auto b : bufs) CHECK(hipFree(b));
  }
  return 0;
}
