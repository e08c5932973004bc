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
#include <stdlib.h>
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


/* fp32 -> IEEE binary16 bits, round-to-nearest-even, subnormals kept,
 * overflow to inf; NaN stays NaN (quiet). */
uint16_t oracle_f32_to_f16(float f) {
  const uint32_t x = f2u(f);
  const uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
  const uint32_t ax = x & 0x7fffffffu;
  if (ax > 0x7f800000u) return (uint16_t)(sign | 0x7e00u | ((ax >> 13) & 0x3ffu));
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* >= 65520: inf (ties to even) */
  if (ax < 0x38800000u) {                                    /* below 2^-14: subnormal or zero */
    if (ax < 0x33000000u) return sign;                       /* <= 2^-25 rounds to zero */
    const uint32_t e = ax >> 23, m = (ax & 0x7fffffu) | 0x800000u;
    const uint32_t shift = 126u - e; /* value / 2^-24 = m >> shift */
    uint32_t q = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1u), half = 1u << (shift - 1u);
    if (rem > half || (rem == half && (q & 1u))) ++q;
    return (uint16_t)(sign | q);
  }
  uint32_t r = ax - (112u << 23);
  r += 0xfffu + ((r >> 13) & 1u);
  return (uint16_t)(sign | (r >> 13));
}

float oracle_f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  if (e == 0) {
    const float v = ldexpf((float)m, -24);
    return sign ? -v : v;
  }
  if (e == 31) return u2f(sign | 0x7f800000u | (m << 13));
  return u2f(sign | ((e + 112u) << 23) | (m << 13));
}

/* 16-bit element formats: bf16 and IEEE f16 share every routine below
 * through these conversions. */
typedef float (*h2f_fn)(uint16_t);
typedef uint16_t (*f2h_fn)(float);

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
/* fp64 (fedavg.py:20-25 on a double model): `w * p1` keeps the Python-float
 * weight exact as a double scalar, and every product and partial sum is a
 * double rounding (PyTorch's CPU opmath for double is double). */
int oracle_wreduce_f64(const double* const* in, int n, const double* w, double* out, size_t p) {
  if (n < 1 || !in || !w || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    double acc = in[0][j] * 0.0;
    for (int i = 0; i < n; ++i) {
      double prod = w[i] * in[i][j];
      acc = acc + prod;
    }
    out[j] = acc;
  }
  return 0;
}

int oracle_wreduce_fast_f64(const double* const* in, int n, const double* w, double* out, size_t p) {
  if (n < 1 || !in || !w || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    double acc = in[0][j] * 0.0;
    for (int i = 0; i < n; ++i) acc = fma(w[i], in[i][j], acc);
    out[j] = acc;
  }
  return 0;
}

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

static int wreduce_h16(const uint16_t* const* in, int n, const float* w, uint16_t* out, size_t p,
                       h2f_fn h2f, f2h_fn f2h) {
  if (n < 1 || !in || !w || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    float acc = h2f(f2h(h2f(in[0][j]) * 0.0f));
    for (int i = 0; i < n; ++i) {
      float prod = h2f(f2h(w[i] * h2f(in[i][j])));
      acc = h2f(f2h(acc + prod));
    }
    out[j] = f2h(acc);
  }
  return 0;
}

int oracle_wreduce_bf16(const uint16_t* const* in, int n, const float* w, uint16_t* out, size_t p) {
  return wreduce_h16(in, n, w, out, p, oracle_bf16_to_f32, oracle_f32_to_bf16);
}

/* fp16 (torch.float16 models): the same opmath as bf16 — fp32 products and
 * sums, each rounded to binary16 (checked against torch's CPU Half ops). */
int oracle_wreduce_f16(const uint16_t* const* in, int n, const float* w, uint16_t* out, size_t p) {
  return wreduce_h16(in, n, w, out, p, oracle_f16_to_f32, oracle_f32_to_f16);
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

static int wreduce_fast_h16(const uint16_t* const* in, int n, const float* w, uint16_t* out, size_t p,
                            h2f_fn h2f, f2h_fn f2h) {
  if (n < 1 || !in || !w || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    float acc = h2f(in[0][j]) * 0.0f;
    for (int i = 0; i < n; ++i) acc = fmaf(w[i], h2f(in[i][j]), acc);
    out[j] = f2h(acc);
  }
  return 0;
}

int oracle_wreduce_fast_bf16(const uint16_t* const* in, int n, const float* w, uint16_t* out, size_t p) {
  return wreduce_fast_h16(in, n, w, out, p, oracle_bf16_to_f32, oracle_f32_to_bf16);
}

int oracle_wreduce_fast_f16(const uint16_t* const* in, int n, const float* w, uint16_t* out, size_t p) {
  return wreduce_fast_h16(in, n, w, out, p, oracle_f16_to_f32, oracle_f32_to_f16);
}

/* Mean of n rows, as PyTorch's CPU `torch.mean(torch.stack(xs), 0)` computes
 * it while its dim-0 reduction is sequential (n <= 4): acc = +0, acc += x_i
 * in order, then one IEEE division by n (sum followed by div_).
 * Restates simulation/conflux/chunk_manager.py:38-40 for the chunked path.
 * bf16: the fp32 sum is divided in fp32 and rounded to bf16 once (mean_out
 * on CPU sums a bf16 input in fp32, divides, then casts back). */
int oracle_mean_f32(const float* const* in, int n, float* out, size_t p) {
  if (n < 1 || !in || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    float acc = 0.0f;
    for (int i = 0; i < n; ++i) acc = acc + in[i][j];
    out[j] = acc / (float)n;
  }
  return 0;
}

static int mean_h16(const uint16_t* const* in, int n, uint16_t* out, size_t p, h2f_fn h2f, f2h_fn f2h) {
  if (n < 1 || !in || !out) return -1;
  for (size_t j = 0; j < p; ++j) {
    float acc = 0.0f;
    for (int i = 0; i < n; ++i) acc = acc + h2f(in[i][j]);
    out[j] = f2h(acc / (float)n);
  }
  return 0;
}

int oracle_mean_bf16(const uint16_t* const* in, int n, uint16_t* out, size_t p) {
  return mean_h16(in, n, out, p, oracle_bf16_to_f32, oracle_f32_to_bf16);
}

int oracle_mean_f16(const uint16_t* const* in, int n, uint16_t* out, size_t p) {
  return mean_h16(in, n, out, p, oracle_f16_to_f32, oracle_f32_to_f16);
}

/* ---- torch.mean(torch.stack(rows), 0) in PyTorch's own CPU order ----------
 *
 * The reference's chunk mean (simulation/conflux/chunk_manager.py:40) runs on
 * the worker's CPU at settings.torch_threads intra-op threads (broker.py:31,
 * session_settings.py:52). On CPU, mean = sum over dim 0 then div_ (fp32; a
 * bf16 input is summed in fp32, divided, and rounded once). The sum is ATen's
 * cascade_sum (SumKernel.cpp), whose order per output column is:
 *
 *  - columns are split over T threads by parallel_dim_reduction
 *    (TensorIteratorReduce.cpp): only when m*n >= 32768 (GRAIN_SIZE) and
 *    T > 1; T' = min(T, n) ranges of ceil(n/T') columns, both ends rounded
 *    down to 32 columns (128 B), the final end kept;
 *  - within a range of s1 columns, vectorized_outer_sum (s1 >= 8, the float
 *    vector width of the AVX2 kernel, which AVX512 machines also run for sum)
 *    folds whole 32-column blocks with multi_row_sum ("cascade" below) and the
 *    rest with row_sum ("ilp"); for s1 < 8, scalar_outer_sum folds groups of
 *    4 columns with multi_row_sum and the rest with row_sum;
 *  - n == 1 (a one-element chunk) is an inner reduction: vectorized_inner_sum
 *    ("inner") for m >= 8, row_sum otherwise.
 *
 * Every rule above was checked against torch.mean on this image for
 * T in {1,2,3,4,8}, m in 1..513, n in 1..1,118,166 (tests/test_chunk_mean_order.py).
 * All chunk-internal ranges have 32-multiple lengths, so the only non-cascade
 * columns are the last < 32 columns of the final range: ilp_begin below. */

static int ceil_log2_i64(long long x) {
  if (x <= 2) return 1;
  int b = 0;
  unsigned long long v = (unsigned long long)(x - 1);
  while (v) { ++b; v >>= 1; }
  return b;
}

/* multi_row_sum over S values x[0], x[st], x[2 st], ...: 4 accumulator levels,
 * 2^lp values per level-0 block. */
static float cascade_sum(const float* x, long long S, long long st) {
  int lp = ceil_log2_i64(S) / 4;
  if (lp < 4) lp = 4;
  const long long step = 1LL << lp, mask = step - 1;
  float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  long long i = 0;
  while (i + step <= S) {
    for (long long j = 0; j < step; ++j, ++i) a[0] = a[0] + x[i * st];
    for (int l = 1; l < 4; ++l) {
      a[l] = a[l] + a[l - 1];
      a[l - 1] = 0.0f;
      if ((i & (mask << (l * lp))) != 0) break;
    }
  }
  for (; i < S; ++i) a[0] = a[0] + x[i * st];
  for (int l = 1; l < 4; ++l) a[0] = a[0] + a[l];
  return a[0];
}

/* row_sum: 4 interleaved cascades (ILP), the remainder into the first, then
 * ((p0 + p1) + p2) + p3. */
static float ilp_sum(const float* x, long long len, long long st) {
  const long long s = len / 4;
  float p[4];
  for (int k = 0; k < 4; ++k) p[k] = cascade_sum(x + k * st, s, 4 * st);
  for (long long i = 4 * s; i < len; ++i) p[0] = p[0] + x[i * st];
  return ((p[0] + p[1]) + p[2]) + p[3];
}

/* vectorized_inner_sum over a contiguous run of m values (8 lanes). */
static float inner_sum(const float* x, long long m) {
  const long long vs = m / 8;
  float fin = 0.0f;
  for (long long k = vs * 8; k < m; ++k) fin = fin + x[k];
  for (int l = 0; l < 8; ++l) fin = fin + ilp_sum(x + l, vs, 8);
  return fin;
}

/* The column split for an element of `esz` bytes whose Vectorized<acc> has
 * `vw` lanes (fp32: 4 B, 8 lanes; fp64: 8 B, 4 lanes): ranges rounded to
 * 128 B of columns, whole blocks of 4 vectors (nrows = 4 of
 * vectorized_outer_sum) in the cascade order, the vectorized path from vw
 * columns up, scalar_outer_sum's 4-column groups below. */
static size_t ilp_begin_gen(int m, size_t n, int threads, size_t esz, size_t vw) {
  if (n <= 1) return 0;
  const size_t rnd = 128 / esz;
  size_t b = 0, e = n;
  if (!((unsigned long long)m * n < 32768ULL || threads <= 1)) {
    const size_t tp = (size_t)threads < n ? (size_t)threads : n;
    const size_t cs = (n + tp - 1) / tp;
    for (size_t t = 0; t < tp; ++t) {
      size_t tb = t * cs;
      if (tb >= n) break;
      size_t te = tb + cs < n ? tb + cs : n;
      tb -= tb % rnd;
      if (te != n) te -= te % rnd;
      if (tb < te) { b = tb; e = te; }
    }
  }
  const size_t s1 = e - b;
  const size_t main = s1 >= vw ? s1 / (4 * vw) * (4 * vw) : s1 / 4 * 4;
  return b + main;
}

/* fp64 (chunk_manager.py:40 on a double model): the same orders in double,
 * with SumKernel's Vectorized<double> (4 lanes) and 16-column (128 B)
 * rounding; restated per function from the fp32 ones above. */
static double cascade_sum_f64(const double* x, long long S, long long st) {
  int lp = ceil_log2_i64(S) / 4;
  if (lp < 4) lp = 4;
  const long long step = 1LL << lp, mask = step - 1;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  long long i = 0;
  while (i + step <= S) {
    for (long long j = 0; j < step; ++j, ++i) a[0] = a[0] + x[i * st];
    for (int l = 1; l < 4; ++l) {
      a[l] = a[l] + a[l - 1];
      a[l - 1] = 0.0;
      if ((i & (mask << (l * lp))) != 0) break;
    }
  }
  for (; i < S; ++i) a[0] = a[0] + x[i * st];
  for (int l = 1; l < 4; ++l) a[0] = a[0] + a[l];
  return a[0];
}

static double ilp_sum_f64(const double* x, long long len, long long st) {
  const long long s = len / 4;
  double p[4];
  for (int k = 0; k < 4; ++k) p[k] = cascade_sum_f64(x + k * st, s, 4 * st);
  for (long long i = 4 * s; i < len; ++i) p[0] = p[0] + x[i * st];
  return ((p[0] + p[1]) + p[2]) + p[3];
}

static double inner_sum_f64(const double* x, long long m) {  /* 4 lanes */
  const long long vs = m / 4;
  double fin = 0.0;
  for (long long k = vs * 4; k < m; ++k) fin = fin + x[k];
  for (int l = 0; l < 4; ++l) fin = fin + ilp_sum_f64(x + l, vs, 4);
  return fin;
}

size_t oracle_chunk_mean_ilp_begin_f64(int m, size_t n, int threads) { return ilp_begin_gen(m, n, threads, 8, 4); }

int oracle_chunk_mean_f64(const double* const* in, int m, double* out, size_t n, int threads) {
  if (m < 1 || !in || !out) return -1;
  const size_t cb = 4096;
  double* col = (double*)malloc(sizeof(double) * (size_t)m * cb);
  if (!col) return -2;
  const size_t ib = oracle_chunk_mean_ilp_begin_f64(m, n, threads);
  for (size_t j0 = 0; j0 < n; j0 += cb) {
    const size_t c = n - j0 < cb ? n - j0 : cb;
    for (size_t j = 0; j < c; ++j)
      for (int i = 0; i < m; ++i) col[j * (size_t)m + i] = in[i][j0 + j];
    for (size_t j = 0; j < c; ++j) {
      const double* x = col + j * (size_t)m;
      const size_t g = j0 + j;
      double s;
      if (n == 1) s = m >= 4 ? inner_sum_f64(x, m) : ilp_sum_f64(x, m, 1);
      else if (g < ib) s = cascade_sum_f64(x, m, 1);
      else s = ilp_sum_f64(x, m, 1);
      out[g] = s / (double)m;
    }
  }
  free(col);
  return 0;
}

size_t oracle_chunk_mean_ilp_begin(int m, size_t n, int threads) {
  if (n == 0) return 0;
  if (n == 1) return 0;
  size_t b = 0, e = n;
  if (!((unsigned long long)m * n < 32768ULL || threads <= 1)) {
    const size_t tp = (size_t)threads < n ? (size_t)threads : n;
    const size_t cs = (n + tp - 1) / tp;
    for (size_t t = 0; t < tp; ++t) {
      size_t tb = t * cs;
      if (tb >= n) break;
      size_t te = tb + cs < n ? tb + cs : n;
      tb -= tb % 32;
      if (te != n) te -= te % 32;
      if (tb < te) { b = tb; e = te; }
    }
  }
  const size_t s1 = e - b;
  const size_t main = s1 >= 8 ? s1 / 32 * 32 : s1 / 4 * 4;
  return b + main;
}

int oracle_chunk_mean_f32(const float* const* in, int m, float* out, size_t n, int threads) {
  if (m < 1 || !in || !out) return -1;
  const size_t cb = 4096;
  float* col = (float*)malloc(sizeof(float) * (size_t)m * cb);
  if (!col) return -2;
  const size_t ib = oracle_chunk_mean_ilp_begin(m, n, threads);
  for (size_t j0 = 0; j0 < n; j0 += cb) {
    const size_t c = n - j0 < cb ? n - j0 : cb;
    for (size_t j = 0; j < c; ++j)
      for (int i = 0; i < m; ++i) col[j * (size_t)m + i] = in[i][j0 + j];
    for (size_t j = 0; j < c; ++j) {
      const float* x = col + j * (size_t)m;
      const size_t g = j0 + j;
      float s;
      if (n == 1) s = m >= 8 ? inner_sum(x, m) : ilp_sum(x, m, 1);
      else if (g < ib) s = cascade_sum(x, m, 1);
      else s = ilp_sum(x, m, 1);
      out[g] = s / (float)m;
    }
  }
  free(col);
  return 0;
}

static int chunk_mean_h16(const uint16_t* const* in, int m, uint16_t* out, size_t n, int threads, h2f_fn h2f,
                          f2h_fn f2h) {
  if (m < 1 || !in || !out) return -1;
  float* tmp = (float*)malloc(sizeof(float) * (n ? n : 1));
  float** rows = (float**)malloc(sizeof(float*) * (size_t)m);
  if (!tmp || !rows) { free(tmp); free(rows); return -2; }
  int rc = 0;
  /* widen each row to fp32 (the sum_out(Float) input cast), then the fp32 order */
  for (int i = 0; i < m && rc == 0; ++i) {
    rows[i] = (float*)malloc(sizeof(float) * (n ? n : 1));
    if (!rows[i]) { rc = -2; for (int k = 0; k < i; ++k) free(rows[k]); break; }
    for (size_t j = 0; j < n; ++j) rows[i][j] = h2f(in[i][j]);
  }
  if (rc == 0) {
    rc = oracle_chunk_mean_f32((const float* const*)rows, m, tmp, n, threads);
    for (size_t j = 0; j < n && rc == 0; ++j) out[j] = f2h(tmp[j]);
    for (int i = 0; i < m; ++i) free(rows[i]);
  }
  free(tmp);
  free(rows);
  return rc;
}

int oracle_chunk_mean_bf16(const uint16_t* const* in, int m, uint16_t* out, size_t n, int threads) {
  return chunk_mean_h16(in, m, out, n, threads, oracle_bf16_to_f32, oracle_f32_to_bf16);
}

int oracle_chunk_mean_f16(const uint16_t* const* in, int m, uint16_t* out, size_t n, int threads) {
  return chunk_mean_h16(in, m, out, n, threads, oracle_f16_to_f32, oracle_f32_to_f16);
}
