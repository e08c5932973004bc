/*
 * c_host_check.c — the C ABI (include/dlsim.h) driven from a plain C host,
 * with no Python and no PyTorch: what a non-Python binding of the reference's
 * aggregate does. Device memory and streams come from
 * the HIP runtime; every result is compared bit for bit with the C oracle
 * (oracle/fedavg_oracle.c, the checker: test infrastructure only).
 *
 * Cases: dlsim_wreduce fp32 (n = 8, ragged size, and in place) and bf16
 * (n = 2), dlsim_wreduce_f64, dlsim_wreduce_tensors (7 models x 3 tensors),
 * dlsim_wreduce_batched (tasks of several fan-ins), dlsim_chunk_mean_batched
 * (k = 10 chunks of a flat model, chunks off 128-B lines), dlsim_host_wreduce
 * (host models, pinned staging, pipelined chunks), dlsim_host_wreduce_resident
 * (some models already on the device), a descriptor-table batch
 * (dlsim_batch_table_*), dlsim_host_chunk_mean (host chunks), the error
 * codes, and dlsim_version / dlsim_shard_range.
 *
 * Built by __graft_entry__.build(); run by tests/test_gpu_c_host.py. Prints
 * one line per case and "c_host_check OK"; exits non-zero on the first
 * mismatch.
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dlsim.h"

/* the oracle's entry points (oracle/fedavg_oracle.c) */
int oracle_wreduce_f32(const float* const* in, int n, const float* w, float* out, size_t p);
int oracle_wreduce_f64(const double* const* in, int n, const double* w, double* out, size_t p);
int oracle_wreduce_bf16(const uint16_t* const* in, int n, const float* w, uint16_t* out, size_t p);
int oracle_chunk_mean_f32(const float* const* in, int m, float* out, size_t n, int threads);
uint16_t oracle_f32_to_bf16(float f);

#define HIPCK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                        \
    }                                                                                 \
  } while (0)
#define DLCK(x)                                                                          \
  do {                                                                                   \
    int r_ = (x);                                                                        \
    if (r_ != DLSIM_OK) {                                                                \
      fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, r_, dlsim_last_error()); \
      exit(3);                                                                           \
    }                                                                                    \
  } while (0)

static uint64_t g_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
  g_state ^= g_state << 13;
  g_state ^= g_state >> 7;
  g_state ^= g_state << 17;
  return (uint32_t)(g_state >> 11);
}
/* finite values over many binades, with +-0 and subnormals sprinkled in */
static float rnd_f32(void) {
  const uint32_t r = rnd();
  if (r % 97 == 0) return (r & 256) ? -0.0f : 0.0f;
  if (r % 89 == 0) return ldexpf((float)(r % 1000) + 1.0f, -140); /* subnormal */
  const float u = (float)(rnd() % 2000001) / 1000000.0f - 1.0f;
  return ldexpf(u, (int)(r % 24) - 12);
}
static void fill_f32(float* x, size_t n) {
  for (size_t j = 0; j < n; ++j) x[j] = rnd_f32();
}
static void weights(float* w, int n) { /* positive, summing to ~1, not representable exactly */
  double s = 0.0, t[256];
  for (int i = 0; i < n; ++i) s += (t[i] = 0.05 + (double)(rnd() % 1000) / 997.0);
  for (int i = 0; i < n; ++i) w[i] = (float)(t[i] / s);
}
static void* dev_copy(const void* h, size_t bytes) {
  void* d = NULL;
  HIPCK(hipMalloc(&d, bytes ? bytes : 1));
  if (bytes) HIPCK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
  return d;
}
static void expect_same(const char* what, const void* got, const void* exp, size_t bytes) {
  if (memcmp(got, exp, bytes) != 0) {
    const unsigned char* a = (const unsigned char*)got;
    const unsigned char* b = (const unsigned char*)exp;
    size_t k = 0;
    while (k < bytes && a[k] == b[k]) ++k;
    fprintf(stderr, "%s: MISMATCH at byte %zu of %zu\n", what, k, bytes);
    exit(1);
  }
  printf("%-46s bit-identical (%zu bytes)\n", what, bytes);
}

static void case_wreduce_f32(hipStream_t st) {
  const int n = 8;
  const size_t p = 1000003; /* ragged: not a whole number of tiles or vectors */
  float* h[8];
  void* d[8];
  float w[8];
  weights(w, n);
  for (int i = 0; i < n; ++i) {
    h[i] = (float*)malloc(p * sizeof(float));
    fill_f32(h[i], p);
    d[i] = dev_copy(h[i], p * sizeof(float));
  }
  float* exp = (float*)malloc(p * sizeof(float));
  float* got = (float*)malloc(p * sizeof(float));
  oracle_wreduce_f32((const float* const*)h, n, w, exp, p);
  void* dout = NULL;
  HIPCK(hipMalloc(&dout, p * sizeof(float)));
  DLCK(dlsim_wreduce((const void* const*)d, n, w, dout, p, DLSIM_F32, DLSIM_EXACT, st));
  HIPCK(hipStreamSynchronize(st));
  HIPCK(hipMemcpy(got, dout, p * sizeof(float), hipMemcpyDeviceToHost));
  expect_same("dlsim_wreduce f32 n=8 p=1000003", got, exp, p * sizeof(float));
  /* in place: the output is input 3 */
  DLCK(dlsim_wreduce((const void* const*)d, n, w, d[3], p, DLSIM_F32, DLSIM_EXACT, st));
  HIPCK(hipStreamSynchronize(st));
  HIPCK(hipMemcpy(got, d[3], p * sizeof(float), hipMemcpyDeviceToHost));
  expect_same("dlsim_wreduce f32 in place (out = input 3)", got, exp, p * sizeof(float));
  for (int i = 0; i < n; ++i) {
    free(h[i]);
    HIPCK(hipFree(d[i]));
  }
  HIPCK(hipFree(dout));
  free(exp);
  free(got);
}

static void case_wreduce_bf16(hipStream_t st) {
  const int n = 2;
  const size_t p = 100001;
  uint16_t* h[2];
  void* d[2];
  const float w[2] = {3.0f / 8.0f, 5.0f / 8.0f}; /* gossip age weights */
  for (int i = 0; i < n; ++i) {
    h[i] = (uint16_t*)malloc(p * 2);
    for (size_t j = 0; j < p; ++j) h[i][j] = oracle_f32_to_bf16(rnd_f32());
    d[i] = dev_copy(h[i], p * 2);
  }
  uint16_t* exp = (uint16_t*)malloc(p * 2);
  uint16_t* got = (uint16_t*)malloc(p * 2);
  oracle_wreduce_bf16((const uint16_t* const*)h, n, w, exp, p);
  void* dout = NULL;
  HIPCK(hipMalloc(&dout, p * 2));
  DLCK(dlsim_wreduce((const void* const*)d, n, w, dout, p, DLSIM_BF16, DLSIM_EXACT, st));
  HIPCK(hipStreamSynchronize(st));
  HIPCK(hipMemcpy(got, dout, p * 2, hipMemcpyDeviceToHost));
  expect_same("dlsim_wreduce bf16 n=2 p=100001", got, exp, p * 2);
  for (int i = 0; i < n; ++i) {
    free(h[i]);
    HIPCK(hipFree(d[i]));
  }
  HIPCK(hipFree(dout));
  free(exp);
  free(got);
}

static void case_wreduce_f64(hipStream_t st) {
  const int n = 5;
  const size_t p = 65539;
  double* h[5];
  void* d[5];
  double w[5];
  for (int i = 0; i < n; ++i) w[i] = 0.1 + 0.0123456789 * i; /* Python floats: kept exact */
  for (int i = 0; i < n; ++i) {
    h[i] = (double*)malloc(p * 8);
    for (size_t j = 0; j < p; ++j) h[i][j] = (double)rnd_f32() * (1.0 + 1e-9 * (double)(rnd() % 1000));
    d[i] = dev_copy(h[i], p * 8);
  }
  double* exp = (double*)malloc(p * 8);
  double* got = (double*)malloc(p * 8);
  oracle_wreduce_f64((const double* const*)h, n, w, exp, p);
  void* dout = NULL;
  HIPCK(hipMalloc(&dout, p * 8));
  DLCK(dlsim_wreduce_f64((const void* const*)d, n, w, dout, p, DLSIM_EXACT, st));
  HIPCK(hipStreamSynchronize(st));
  HIPCK(hipMemcpy(got, dout, p * 8, hipMemcpyDeviceToHost));
  expect_same("dlsim_wreduce_f64 n=5 p=65539", got, exp, p * 8);
  for (int i = 0; i < n; ++i) {
    free(h[i]);
    HIPCK(hipFree(d[i]));
  }
  HIPCK(hipFree(dout));
  free(exp);
  free(got);
}

static void case_tensors_and_batched(hipStream_t st) {
  /* 7 models x 3 tensors (a bias, a ragged tensor, a weight matrix) */
  enum { N = 7, T = 3 };
  const size_t numels[T] = {10, 4099, 65536};
  float* h[N * T];
  void* d[N * T];
  void* douts[T];
  float w[N];
  weights(w, N);
  for (int i = 0; i < N; ++i)
    for (int k = 0; k < T; ++k) {
      h[i * T + k] = (float*)malloc(numels[k] * 4);
      fill_f32(h[i * T + k], numels[k]);
      d[i * T + k] = dev_copy(h[i * T + k], numels[k] * 4);
    }
  for (int k = 0; k < T; ++k) HIPCK(hipMalloc(&douts[k], numels[k] * 4));
  DLCK(dlsim_wreduce_tensors((const void* const*)d, N, T, numels, w, douts, DLSIM_F32, DLSIM_EXACT, st));
  HIPCK(hipStreamSynchronize(st));
  for (int k = 0; k < T; ++k) {
    const float* in[N];
    for (int i = 0; i < N; ++i) in[i] = h[i * T + k];
    float* exp = (float*)malloc(numels[k] * 4);
    float* got = (float*)malloc(numels[k] * 4);
    oracle_wreduce_f32(in, N, w, exp, numels[k]);
    HIPCK(hipMemcpy(got, douts[k], numels[k] * 4, hipMemcpyDeviceToHost));
    char what[64];
    snprintf(what, sizeof what, "dlsim_wreduce_tensors tensor %d (%zu)", k, numels[k]);
    expect_same(what, got, exp, numels[k] * 4);
    free(exp);
    free(got);
  }
  /* batched: task k reduces tensor k of the first fan[k] models */
  const int fan[T] = {1, 3, 7};
  const void* bin[1 + 3 + 7];
  float bw[1 + 3 + 7];
  size_t bn[T];
  int o = 0;
  for (int k = 0; k < T; ++k) {
    for (int i = 0; i < fan[k]; ++i) {
      bin[o] = d[i * T + k];
      bw[o] = w[i];
      ++o;
    }
    bn[k] = numels[k];
  }
  DLCK(dlsim_wreduce_batched(T, fan, bin, bw, douts, bn, DLSIM_F32, DLSIM_EXACT, st));
  HIPCK(hipStreamSynchronize(st));
  o = 0;
  for (int k = 0; k < T; ++k) {
    const float* in[N];
    for (int i = 0; i < fan[k]; ++i) in[i] = h[i * T + k];
    float* exp = (float*)malloc(numels[k] * 4);
    float* got = (float*)malloc(numels[k] * 4);
    oracle_wreduce_f32(in, fan[k], bw + o, exp, numels[k]);
    o += fan[k];
    HIPCK(hipMemcpy(got, douts[k], numels[k] * 4, hipMemcpyDeviceToHost));
    char what[64];
    snprintf(what, sizeof what, "dlsim_wreduce_batched task %d (fan-in %d)", k, fan[k]);
    expect_same(what, got, exp, numels[k] * 4);
    free(exp);
    free(got);
  }
  for (int j = 0; j < N * T; ++j) {
    free(h[j]);
    HIPCK(hipFree(d[j]));
  }
  for (int k = 0; k < T; ++k) HIPCK(hipFree(douts[k]));
}

static void case_chunk_means(hipStream_t st) {
  /* Conflux: m = 4 contributors' flat models, k = 10 chunks of P / k
   * elements (the last takes the rest), each chunk a slice of its model */
  enum { M = 4, K = 10 };
  const size_t p = 1000003, c = p / K;
  float* h[M];
  void* d[M];
  for (int i = 0; i < M; ++i) {
    h[i] = (float*)malloc(p * 4);
    fill_f32(h[i], p);
    d[i] = dev_copy(h[i], p * 4);
  }
  void* dout = NULL;
  HIPCK(hipMalloc(&dout, p * 4));
  int fan[K];
  const void* in[K * M];
  void* outs[K];
  size_t ns[K];
  for (int k = 0; k < K; ++k) {
    const size_t b = k * c, e = k == K - 1 ? p : b + c;
    fan[k] = M;
    ns[k] = e - b;
    outs[k] = (float*)dout + b;
    for (int i = 0; i < M; ++i) in[k * M + i] = (const float*)d[i] + b;
  }
  DLCK(dlsim_chunk_mean_batched(K, fan, in, outs, ns, DLSIM_F32, 4, st));
  HIPCK(hipStreamSynchronize(st));
  float* got = (float*)malloc(p * 4);
  float* exp = (float*)malloc(p * 4);
  HIPCK(hipMemcpy(got, dout, p * 4, hipMemcpyDeviceToHost));
  for (int k = 0; k < K; ++k) {
    const size_t b = k * c;
    const float* hin[M];
    for (int i = 0; i < M; ++i) hin[i] = h[i] + b;
    oracle_chunk_mean_f32(hin, M, exp + b, ns[k], 4);
  }
  expect_same("dlsim_chunk_mean_batched k=10 m=4 (4 threads)", got, exp, p * 4);
  for (int i = 0; i < M; ++i) {
    free(h[i]);
    HIPCK(hipFree(d[i]));
  }
  HIPCK(hipFree(dout));
  free(got);
  free(exp);
}

static void case_host_wreduce(hipStream_t st) {
  /* 7 host models of 2 tensors (the reference's CPU modules), pinned
   * staging, chunked pipeline with separate copy streams, host result */
  enum { N = 7, T = 2 };
  const size_t numels[T] = {300007, 123};
  const size_t total = numels[0] + numels[1];
  const size_t stride = (total + 63) / 64 * 64;
  float* h[N * T];
  float w[N];
  weights(w, N);
  for (int j = 0; j < N * T; ++j) {
    h[j] = (float*)malloc(numels[j % T] * 4 + 4);
    fill_f32(h[j], numels[j % T]);
  }
  void *staging = NULL, *rows = NULL, *dout = NULL, *hout = NULL;
  HIPCK(hipHostMalloc(&staging, N * stride * 4, 0));
  HIPCK(hipHostMalloc(&hout, total * 4, 0));
  HIPCK(hipMalloc(&rows, N * stride * 4));
  HIPCK(hipMalloc(&dout, total * 4));
  hipStream_t h2d, d2h;
  HIPCK(hipStreamCreate(&h2d));
  HIPCK(hipStreamCreate(&d2h));
  DLCK(dlsim_host_wreduce(N, T, (const void* const*)h, numels, w, staging, rows, stride, dout, hout, DLSIM_F32,
                          DLSIM_EXACT, 65536, 4, st, h2d, d2h));
  HIPCK(hipStreamSynchronize(st));
  /* expected: the reduce of the concatenated models */
  float* cat[N];
  for (int i = 0; i < N; ++i) {
    cat[i] = (float*)malloc(total * 4);
    memcpy(cat[i], h[i * T], numels[0] * 4);
    memcpy(cat[i] + numels[0], h[i * T + 1], numels[1] * 4);
  }
  float* exp = (float*)malloc(total * 4);
  oracle_wreduce_f32((const float* const*)cat, N, w, exp, total);
  expect_same("dlsim_host_wreduce 7 host models, h_out", hout, exp, total * 4);
  float* got = (float*)malloc(total * 4);
  HIPCK(hipMemcpy(got, dout, total * 4, hipMemcpyDeviceToHost));
  expect_same("dlsim_host_wreduce 7 host models, d_out", got, exp, total * 4);
  for (int i = 0; i < N; ++i) free(cat[i]);
  for (int j = 0; j < N * T; ++j) free(h[j]);
  free(exp);
  free(got);
  HIPCK(hipHostFree(staging));
  HIPCK(hipHostFree(hout));
  HIPCK(hipFree(rows));
  HIPCK(hipFree(dout));
  HIPCK(hipStreamDestroy(h2d));
  HIPCK(hipStreamDestroy(d2h));
}

static void case_host_wreduce_resident(hipStream_t st) {
  /* 5 host models of 2 tensors; models 1 and 3 already on the device (a
   * worker's cache), the other three packed and sent to their device rows,
   * which keep them: a second call with every model resident gives the same */
  enum { N = 5, T = 2 };
  const size_t numels[T] = {70001, 33};
  const size_t total = numels[0] + numels[1];
  const size_t stride = (total + 63) / 64 * 64;
  float* h[N * T];
  float w[N];
  weights(w, N);
  float* cat[N];
  for (int i = 0; i < N; ++i) {
    cat[i] = (float*)malloc(total * 4);
    for (int k = 0; k < T; ++k) {
      h[i * T + k] = (float*)malloc(numels[k] * 4);
      fill_f32(h[i * T + k], numels[k]);
    }
    memcpy(cat[i], h[i * T], numels[0] * 4);
    memcpy(cat[i] + numels[0], h[i * T + 1], numels[1] * 4);
  }
  void *staging = NULL, *block = NULL, *dout = NULL, *hout = NULL;
  HIPCK(hipHostMalloc(&staging, N * stride * 4, 0));
  HIPCK(hipHostMalloc(&hout, total * 4, 0));
  HIPCK(hipMalloc(&block, N * stride * 4));
  HIPCK(hipMalloc(&dout, total * 4));
  void* rows[N];
  for (int i = 0; i < N; ++i) rows[i] = (char*)block + (size_t)i * stride * 4;
  int resident[N] = {0, 1, 0, 1, 0};
  HIPCK(hipMemcpy(rows[1], cat[1], total * 4, hipMemcpyHostToDevice));
  HIPCK(hipMemcpy(rows[3], cat[3], total * 4, hipMemcpyHostToDevice));
  const void* srcs[N * T];
  for (int j = 0; j < N * T; ++j) srcs[j] = resident[j / T] ? NULL : h[j];
  float* exp = (float*)malloc(total * 4);
  oracle_wreduce_f32((const float* const*)cat, N, w, exp, total);
  DLCK(dlsim_host_wreduce_resident(N, T, srcs, numels, w, resident, rows, staging, stride, dout, hout, DLSIM_F32,
                                   DLSIM_EXACT, 4, st));
  HIPCK(hipStreamSynchronize(st));
  expect_same("dlsim_host_wreduce_resident 2 of 5 resident", hout, exp, total * 4);
  int all[N] = {1, 1, 1, 1, 1};
  memset(hout, 0, total * 4);
  DLCK(dlsim_host_wreduce_resident(N, T, srcs, numels, w, all, rows, NULL, 0, dout, hout, DLSIM_F32, DLSIM_EXACT, 4,
                                   st));
  HIPCK(hipStreamSynchronize(st));
  expect_same("dlsim_host_wreduce_resident all resident (rows kept)", hout, exp, total * 4);
  for (int i = 0; i < N; ++i) free(cat[i]);
  for (int j = 0; j < N * T; ++j) free(h[j]);
  free(exp);
  HIPCK(hipHostFree(staging));
  HIPCK(hipHostFree(hout));
  HIPCK(hipFree(block));
  HIPCK(hipFree(dout));
}

static void case_table_batch(hipStream_t st) {
  /* a prepared round: 5 tasks of several sizes and fan-ins in one caller-owned
   * descriptor table, launched twice (graph-capturable: no allocation) */
  enum { B = 5 };
  const int fan[B] = {2, 7, 3, 7, 1};
  const size_t ns[B] = {85354, 4096, 333333, 17, 70000};
  int tot = 0;
  for (int t = 0; t < B; ++t) tot += fan[t];
  float* h[2 + 7 + 3 + 7 + 1];
  const void* din[2 + 7 + 3 + 7 + 1];
  float w[2 + 7 + 3 + 7 + 1];
  void* douts[B];
  int o = 0;
  for (int t = 0; t < B; ++t) {
    weights(w + o, fan[t]);
    for (int i = 0; i < fan[t]; ++i, ++o) {
      h[o] = (float*)malloc(ns[t] * 4);
      fill_f32(h[o], ns[t]);
      din[o] = dev_copy(h[o], ns[t] * 4);
    }
    HIPCK(hipMalloc(&douts[t], ns[t] * 4));
  }
  size_t bytes = 0;
  DLCK(dlsim_batch_table_bytes(B, fan, ns, DLSIM_F32, &bytes));
  void *htab = NULL, *dtab = NULL;
  HIPCK(hipHostMalloc(&htab, bytes, 0));
  HIPCK(hipMalloc(&dtab, bytes));
  DLCK(dlsim_batch_table_fill(B, fan, din, w, douts, ns, DLSIM_F32, htab, bytes));
  HIPCK(hipMemcpyAsync(dtab, htab, bytes, hipMemcpyHostToDevice, st));
  for (int rep = 0; rep < 2; ++rep) DLCK(dlsim_batch_table_launch(htab, dtab, DLSIM_F32, DLSIM_EXACT, st));
  HIPCK(hipStreamSynchronize(st));
  o = 0;
  for (int t = 0; t < B; ++t) {
    float* exp = (float*)malloc(ns[t] * 4);
    float* got = (float*)malloc(ns[t] * 4);
    oracle_wreduce_f32((const float* const*)(h + o), fan[t], w + o, exp, ns[t]);
    HIPCK(hipMemcpy(got, douts[t], ns[t] * 4, hipMemcpyDeviceToHost));
    char what[64];
    snprintf(what, sizeof what, "dlsim_batch_table task %d (fan-in %d, %zu)", t, fan[t], ns[t]);
    expect_same(what, got, exp, ns[t] * 4);
    free(exp);
    free(got);
    o += fan[t];
  }
  for (int j = 0; j < tot; ++j) {
    free(h[j]);
    HIPCK(hipFree((void*)din[j]));
  }
  for (int t = 0; t < B; ++t) HIPCK(hipFree(douts[t]));
  HIPCK(hipHostFree(htab));
  HIPCK(hipFree(dtab));
}

static void case_host_chunk_mean(hipStream_t st) {
  /* Conflux from host chunks: k = 6 indices, 3-5 contributors each, pinned
   * staging, means back on the device and in page-locked host memory */
  enum { K = 6 };
  const int fan[K] = {3, 4, 5, 3, 4, 5};
  const size_t ns[K] = {14226, 14226, 14226, 14226, 14226, 14224};
  float* h[3 + 4 + 5 + 3 + 4 + 5];
  const void* hin[3 + 4 + 5 + 3 + 4 + 5];
  void *douts[K], *houts[K];
  size_t need = 0;
  int o = 0;
  for (int t = 0; t < K; ++t) {
    for (int i = 0; i < fan[t]; ++i, ++o) {
      h[o] = (float*)malloc(ns[t] * 4 + 4);
      fill_f32(h[o], ns[t]);
      hin[o] = h[o];
    }
    need += (size_t)fan[t] * ((ns[t] + 63) / 64 * 64);
    HIPCK(hipMalloc(&douts[t], ns[t] * 4));
    HIPCK(hipHostMalloc(&houts[t], ns[t] * 4, 0));
  }
  void *stage = NULL, *dstage = NULL;
  HIPCK(hipHostMalloc(&stage, need * 4, 0));
  HIPCK(hipMalloc(&dstage, need * 4));
  DLCK(dlsim_host_chunk_mean(K, fan, hin, ns, stage, dstage, need, douts, houts, DLSIM_F32, 4, 2, st, NULL, NULL));
  HIPCK(hipStreamSynchronize(st));
  o = 0;
  for (int t = 0; t < K; ++t) {
    float* exp = (float*)malloc(ns[t] * 4);
    float* got = (float*)malloc(ns[t] * 4);
    oracle_chunk_mean_f32((const float* const*)(h + o), fan[t], exp, ns[t], 4);
    HIPCK(hipMemcpy(got, douts[t], ns[t] * 4, hipMemcpyDeviceToHost));
    char what[64];
    snprintf(what, sizeof what, "dlsim_host_chunk_mean index %d (m=%d)", t, fan[t]);
    expect_same(what, got, exp, ns[t] * 4);
    if (memcmp(houts[t], exp, ns[t] * 4) != 0) {
      fprintf(stderr, "dlsim_host_chunk_mean index %d: host copy differs\n", t);
      exit(1);
    }
    free(exp);
    free(got);
    o += fan[t];
  }
  for (int j = 0; j < o; ++j) free(h[j]);
  for (int t = 0; t < K; ++t) {
    HIPCK(hipFree(douts[t]));
    HIPCK(hipHostFree(houts[t]));
  }
  HIPCK(hipHostFree(stage));
  HIPCK(hipFree(dstage));
}

static void case_errors(hipStream_t st) {
  void* d = NULL;
  HIPCK(hipMalloc(&d, 256));
  const void* in[1] = {d};
  const float w[1] = {1.0f};
  int rc = dlsim_wreduce(in, 0, w, d, 16, DLSIM_F32, DLSIM_EXACT, st);
  if (rc != DLSIM_E_ARG || !dlsim_last_error() || !*dlsim_last_error()) {
    fprintf(stderr, "n = 0: expected DLSIM_E_ARG with a message, got %d\n", rc);
    exit(1);
  }
  rc = dlsim_wreduce(in, 1, w, d, 16, 9, DLSIM_EXACT, st);
  if (rc != DLSIM_E_DTYPE) {
    fprintf(stderr, "dtype 9: expected DLSIM_E_DTYPE, got %d\n", rc);
    exit(1);
  }
  rc = dlsim_wreduce(in, 1, w, d, 16, DLSIM_F32, 7, st);
  if (rc != DLSIM_E_MODE) {
    fprintf(stderr, "mode 7: expected DLSIM_E_MODE, got %d\n", rc);
    exit(1);
  }
  HIPCK(hipFree(d));
  printf("%-46s DLSIM_E_ARG / _DTYPE / _MODE with messages\n", "error codes");
}

/* dlsim_device_alloc: a contiguous block holds the rows and the output of
 * a reduce (the arena placement of DESIGN.md §5c), then dlsim_device_free. */
static void case_device_block(hipStream_t st) {
  const int n = 4;
  const size_t p = 3000017, stride = (p + 63) / 64 * 64;
  float* h[4];
  const void* d[4];
  float w[4];
  weights(w, n);
  void* blk = NULL;
  int contiguous = -1;
  DLCK(dlsim_device_alloc((n + 1) * stride * sizeof(float), DLSIM_ALLOC_CONTIGUOUS, &blk, &contiguous));
  if (!blk || (contiguous != 0 && contiguous != 1)) {
    fprintf(stderr, "dlsim_device_alloc: block %p contiguous %d\n", blk, contiguous);
    exit(1);
  }
  for (int i = 0; i < n; ++i) {
    h[i] = (float*)malloc(p * sizeof(float));
    fill_f32(h[i], p);
    d[i] = (const float*)blk + i * stride;
    HIPCK(hipMemcpy((void*)d[i], h[i], p * sizeof(float), hipMemcpyHostToDevice));
  }
  float* exp = (float*)malloc(p * sizeof(float));
  float* got = (float*)malloc(p * sizeof(float));
  oracle_wreduce_f32((const float* const*)h, n, w, exp, p);
  void* dout = (float*)blk + n * stride;
  DLCK(dlsim_wreduce(d, n, w, dout, p, DLSIM_F32, DLSIM_EXACT, st));
  HIPCK(hipStreamSynchronize(st));
  HIPCK(hipMemcpy(got, dout, p * sizeof(float), hipMemcpyDeviceToHost));
  expect_same(contiguous ? "dlsim_device_alloc (contiguous) rows + output" : "dlsim_device_alloc (hipMalloc) rows + output",
              got, exp, p * sizeof(float));
  DLCK(dlsim_device_free(blk));
  DLCK(dlsim_device_free(NULL));
  void* none = NULL;
  if (dlsim_device_alloc(0, DLSIM_ALLOC_CONTIGUOUS, &none, NULL) != DLSIM_E_ARG || none) {
    fprintf(stderr, "dlsim_device_alloc(0): expected DLSIM_E_ARG\n");
    exit(1);
  }
  for (int i = 0; i < n; ++i) free(h[i]);
  free(exp);
  free(got);
}

int main(void) {
  if ((dlsim_version() >> 16) != 1) {
    fprintf(stderr, "unexpected ABI major version %d\n", dlsim_version() >> 16);
    return 1;
  }
  size_t b = 0, e = 0, prev = 0;
  for (int r = 0; r < 8; ++r) {
    DLCK(dlsim_shard_range(11181642, 8, r, 64, &b, &e));
    if (b != prev || (r < 7 && b % 64 != 0)) {
      fprintf(stderr, "shard_range: rank %d [%zu, %zu)\n", r, b, e);
      return 1;
    }
    prev = e;
  }
  if (prev != 11181642) return 1;
  hipStream_t st;
  HIPCK(hipStreamCreate(&st));
  case_wreduce_f32(st);
  case_wreduce_bf16(st);
  case_wreduce_f64(st);
  case_tensors_and_batched(st);
  case_chunk_means(st);
  case_host_wreduce(st);
  case_host_wreduce_resident(st);
  case_table_batch(st);
  case_host_chunk_mean(st);
  case_device_block(st);
  case_errors(st);
  HIPCK(hipStreamDestroy(st));
  printf("c_host_check OK\n");
  return 0;
}
