/*
 * fedavg_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C CPU restatement of the reference's aggregation arithmetic,
 *   dasklearn/gradient_aggregation/fedavg.py:12-26  FedAvg.aggregate
 * on flat parameter arenas. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library.
 *
 * Reference semantics restated (per element j of every parameters() tensor):
 *   fedavg.py:14-15   weights None/[] -> float(1./N) each (caller's job here)
 *   fedavg.py:20-22   center = deepcopy(models[0]); p.mul_(0)   => acc = x0*0
 *   fedavg.py:23-25   for (m, w): c1.add_(w * p1)               => acc = acc + fl(w*x)
 * `w * p1` is a tensor-times-Python-float: PyTorch converts w to the tensor's
 * opmath type (fp32 for fp32 and bf16 tensors, RNE from double), computes the
 * product in fp32 and rounds it to the tensor dtype; add_ then adds in fp32
 * and rounds to the tensor dtype. So:
 *   fp32: two separately rounded binary32 operations per term (no FMA);
 *   bf16: product and sum each rounded to bf16 (round-to-nearest-even).
 * Parity is pinned by the tests/golden fixtures, produced by running the reference's
 * own FedAvg.aggregate (tests/golden/make_golden.py).
 *
 * Build (oracle/Makefile): gcc -O2 -ffp-contract=off, no -ffast-math, so the
 * compiler may neither fuse nor flush subnormals (x86-64 SSE arithmetic is
 * IEEE binary32 without excess precision).
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* fp32 -> bf16 bits, round-to-nearest-even; NaN -> 0x7FC0 (c10 scalar rule). */
uint16_t oracle_f32_to_bf16(float f) {
  uint32_t u = f2u(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0u;
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

float oracle_bf16_to_f32(uint16_t h) { return u2f((uint32_t)h << 16); }

static float bf16r(float f) { return oracle_bf16_to_f32(oracle_f32_to_bf16(f)); }

/* out[j] = fold over i of fl(w[i] * in[i][j]), starting from in[0][j] * 0. */
int oracle_wreduce_f32(const float* const* in, int n, const float* w, float* out, size_t p) {
  if (n < 1 || !in || !w || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    float acc = in[0][j] * 0.0f;
    for (int i = 0; i < n; ++i) {
      float prod = w[i] * in[i][j];
      acc = acc + prod;
    }
    out[j] = acc;
  }
  return 0;
}

/* Same fold, element-major over a (n, p) row-major block: faster restatement
 * used for full-size checks (identical arithmetic, loop order swapped: every
 * element's terms are still added in input order). */
int oracle_wreduce_f32_rows(const float* x, int n, const float* w, float* out, size_t p) {
  if (n < 1 || !x || !w || !out) return -1;
  for (size_t j = 0; j < p; ++j) out[j] = x[j] * 0.0f;
  for (int i = 0; i < n; ++i) {
    const float* xi = x + (size_t)i * p;
    const float wi = w[i];
    for (size_t j = 0; j < p; ++j) {
      float prod = wi * xi[j];
      out[j] = out[j] + prod;
    }
  }
  return 0;
}

int oracle_wreduce_bf16(const uint16_t* const* in, int n, const float* w, uint16_t* out,
                        size_t p) {
  if (n < 1 || !in || !w || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    float acc = bf16r(oracle_bf16_to_f32(in[0][j]) * 0.0f);
    for (int i = 0; i < n; ++i) {
      float prod = bf16r(w[i] * oracle_bf16_to_f32(in[i][j]));
      acc = bf16r(acc + prod);
    }
    out[j] = oracle_f32_to_bf16(acc);
  }
  return 0;
}

/* FAST-mode reference: fp32 fma chain (bf16: fp32 accumulation, one final
 * rounding). Not the reference's rounding — used only to bound the FAST
 * mode's error in tests. */
int oracle_wreduce_fast_f32(const float* const* in, int n, const float* w, float* out, size_t p) {
  if (n < 1 || !in || !w || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    float acc = in[0][j] * 0.0f;
    for (int i = 0; i < n; ++i) acc = fmaf(w[i], in[i][j], acc);
    out[j] = acc;
  }
  return 0;
}

int oracle_wreduce_fast_bf16(const uint16_t* const* in, int n, const float* w, uint16_t* out,
                             size_t p) {
  if (n < 1 || !in || !w || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    float acc = oracle_bf16_to_f32(in[0][j]) * 0.0f;
    for (int i = 0; i < n; ++i) acc = fmaf(w[i], oracle_bf16_to_f32(in[i][j]), acc);
    out[j] = oracle_f32_to_bf16(acc);
  }
  return 0;
}

/* Mean of n rows, as PyTorch's CPU `torch.mean(torch.stack(xs), 0)` computes
 * it while its dim-0 reduction is sequential (n <= 4): acc = +0, acc += x_i
 * in order, then one IEEE division by n (sum followed by div_).
 * Restates simulation/conflux/chunk_manager.py:38-40 for the chunked path.
 * bf16: the fp32 sum is rounded to bf16, then divided and rounded again. */
int oracle_mean_f32(const float* const* in, int n, float* out, size_t p) {
  if (n < 1 || !in || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    float acc = 0.0f;
    for (int i = 0; i < n; ++i) acc = acc + in[i][j];
    out[j] = acc / (float)n;
  }
  return 0;
}

int oracle_mean_bf16(const uint16_t* const* in, int n, uint16_t* out, size_t p) {
  if (n < 1 || !in || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    float acc = 0.0f;
    for (int i = 0; i < n; ++i) acc = acc + oracle_bf16_to_f32(in[i][j]);
    out[j] = oracle_f32_to_bf16(bf16r(acc) / (float)n);
  }
  return 0;
}
