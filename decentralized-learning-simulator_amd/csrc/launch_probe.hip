// launch_probe.hip — host-side cost of one small launch on gfx950 (measurement
// only; built by scripts/gpu_launch_probe.sh, not part of the library).
//
// 1. An empty kernel whose by-value argument is 16 B, 256 B, 1 KiB, 2 KiB or
//    3.5 KiB (the batched reduce's BatchSlots): median host time of the
//    launch call alone, and of launch + hipStreamSynchronize.
// 2. dlsim_wreduce_tensors for one D-PSGD task of GNLeNet tensors (14 tensors,
//    fan-in 7) through the library: launch-only and + sync, with the time of
//    the argument checks alone (the library called with t = 0 tensors).
//
// Prints one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#include "dlsim.h"

template <int BYTES>
struct Blob {
  unsigned char b[BYTES];
};

template <int BYTES>
__global__ void k_empty(Blob<BYTES> a, int* sink) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.b[BYTES - 1] == 0xAB) sink[0] = 1;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double median_us(F&& f, int reps) {
  std::vector<double> t;
  for (int i = 0; i < 50; ++i) f();
  for (int i = 0; i < reps; ++i) {
    const double t0 = now_us();
    f();
    t.push_back(now_us() - t0);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      return 1;                                                                \
    }                                                                          \
  } while (0)

template <int BYTES>
static void empty_case(hipStream_t st, int* sink, const char* name, bool first) {
  Blob<BYTES> a{};
  auto launch = [&] { hipLaunchKernelGGL(k_empty<BYTES>, dim3(1), dim3(64), 0, st, a, sink); };
  const double lo = median_us(launch, 2000);
  hipStreamSynchronize(st);
  const double ls = median_us([&] { launch(); hipStreamSynchronize(st); }, 2000);
  std::printf("%s\"empty_%s\": {\"launch_us\": %.2f, \"launch_sync_us\": %.2f}", first ? "" : ", ", name, lo, ls);
}

int main() {
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int* sink;
  CHECK(hipMalloc(&sink, 4));
  std::printf("{");
  empty_case<16>(st, sink, "16B", true);
  empty_case<256>(st, sink, "256B", false);
  empty_case<1024>(st, sink, "1KiB", false);
  empty_case<2048>(st, sink, "2KiB", false);
  empty_case<3584>(st, sink, "3.5KiB", false);

  // GNLeNet's 14 tensors, fan-in 7
  const size_t shapes[14] = {2400, 32, 32, 32, 25600, 32, 32, 32, 51200, 64, 64, 64, 5760, 10};
  const int n = 7, t = 14;
  size_t total = 0;
  for (size_t s : shapes) total += s;
  float* buf;
  CHECK(hipMalloc(&buf, (n + 1) * total * sizeof(float) + 4096));
  CHECK(hipMemset(buf, 0, (n + 1) * total * sizeof(float)));
  std::vector<const void*> ins(static_cast<size_t>(n) * t);
  std::vector<void*> outs(t);
  std::vector<size_t> ne(shapes, shapes + t);
  std::vector<float> w(n, 1.0f / n);
  size_t off = 0;
  for (int k = 0; k < t; ++k) {
    for (int i = 0; i < n; ++i) ins[static_cast<size_t>(i) * t + k] = buf + i * total + off;
    outs[k] = buf + n * total + off;
    off += shapes[k];
  }
  auto call = [&] {
    dlsim_wreduce_tensors(ins.data(), n, t, ne.data(), w.data(), outs.data(), DLSIM_F32, DLSIM_EXACT, st);
  };
  if (dlsim_wreduce_tensors(ins.data(), n, t, ne.data(), w.data(), outs.data(), DLSIM_F32, DLSIM_EXACT, st) !=
      DLSIM_OK) {
    std::fprintf(stderr, "dlsim_wreduce_tensors: %s\n", dlsim_last_error());
    return 1;
  }
  CHECK(hipStreamSynchronize(st));
  const double lo = median_us(call, 2000);
  CHECK(hipStreamSynchronize(st));
  const double ls = median_us([&] { call(); hipStreamSynchronize(st); }, 2000);
  const double checks = median_us([&] {
    dlsim_wreduce_tensors(ins.data(), n, 0, ne.data(), w.data(), outs.data(), DLSIM_F32, DLSIM_EXACT, st);
  }, 2000);
  // the same bytes as one flat reduce (one stream per model)
  std::vector<const void*> flat(n);
  for (int i = 0; i < n; ++i) flat[i] = buf + i * total;
  auto flat_call = [&] { dlsim_wreduce(flat.data(), n, w.data(), buf + n * total, total, DLSIM_F32, DLSIM_EXACT, st); };
  const double fl = median_us(flat_call, 2000);
  CHECK(hipStreamSynchronize(st));
  const double fs = median_us([&] { flat_call(); hipStreamSynchronize(st); }, 2000);
  std::printf(", \"gnlenet_tensors\": {\"launch_us\": %.2f, \"launch_sync_us\": %.2f, \"t0_call_us\": %.2f}", lo, ls,
              checks);
  std::printf(", \"gnlenet_flat\": {\"launch_us\": %.2f, \"launch_sync_us\": %.2f}}\n", fl, fs);
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  CHECK(hipStreamDestroy(st));
  return 0;
}
