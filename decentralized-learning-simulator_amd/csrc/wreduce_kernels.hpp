// wreduce_kernels.hpp — gfx950 streaming kernels for the N-way weighted
// reduce of peer model parameters (the arithmetic of FedAvg.aggregate,
// reference dasklearn/gradient_aggregation/fedavg.py:12-26).
//
// Shape of the work: N input streams of P elements, one output stream of P
// elements, 1 multiply + 1 add per input element (~0.25 flop/byte in fp32).
// That is HBM-bound by a factor of ~100 over the vector ALU, so the design is
// a pure streaming kernel: 16 B per lane per load (global_load_dwordx4),
// every input of a group issued before the first add so each lane keeps
// G x VPT x 16 B in flight, accumulators in registers, one 16 B store per
// lane per vector. No LDS: the reference's summation order is strictly
// sequential in the input index, so splitting N across lanes (and combining
// partials through LDS) would change the rounding; within one element the
// N terms are folded in order by a single lane.
//
// Rounding contract (DLSIM_EXACT), per element j:
//   acc = x0[j] * 0                                (fedavg.py:21-22, p.mul_(0))
//   for i in 0..n-1: acc = acc + fl(w_i * x_i[j])  (fedavg.py:23-25, c1.add_(w*p1))
// fp32: each * and + rounded to fp32 (no contraction — see the pragma below).
// bf16: operands widened to fp32, each product and each sum rounded to bf16
// (round-to-nearest-even), which is PyTorch's CPU opmath behaviour for a
// bf16 tensor times a Python-float scalar and for bf16 add_.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

// Multiply and add must stay separate roundings: hipcc defaults to
// -ffp-contract=fast-honor-pragmas, which would fuse acc + w*x into v_fma_f32
// and change ~55% of the results (hard part (a)).
#pragma clang fp contract(off)

namespace dlsim {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// ---- bf16 helpers -----------------------------------------------------------
// Round fp32 -> bf16 (returned widened back to fp32), nearest-even. A NaN
// becomes the canonical quiet NaN 0x7FC0 (c10::BFloat16's scalar rule; the
// reference's vectorised CPU path writes 0xFFFF instead — NaN payloads are
// outside the parity contract, NaN-ness is inside it).
__device__ __forceinline__ float bf16_round(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return __uint_as_float(0x7fc00000u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return __uint_as_float(u & 0xffff0000u);
}

// Round-to-nearest-even fp32 -> bf16 of a pair, returned widened to fp32,
// with one v_cvt_pk_bf16_f32 (hardware RNE; NaN stays NaN).
__device__ __forceinline__ void bf16_round2(float& a0, float& a1) {
  const f32x2 v = {a0, a1};
  const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
  a0 = __uint_as_float(u << 16);
  a1 = __uint_as_float(u & 0xffff0000u);
}

// ---- fp16 helpers -------------------------------------------------------------
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// An fp32 value pinned in a VGPR. Without it the backend selects
// v_fma_mix{lo}_f16 for fptrunc(w * x) and fptrunc(a + b): one rounding of the
// exact result straight to fp16 (and an fma with a +0 addend, which turns a
// -0 product into +0) instead of the reference's fp32 rounding followed by
// the fp16 one. Found by scripts/fuzz_parity.py.
__device__ __forceinline__ float pin_f32(float v) {
  asm volatile("" : "+v"(v));
  return v;
}

// fp32 -> fp16 -> fp32, nearest-even (hardware conversion; NaN stays NaN,
// overflow to inf, fp16 subnormals kept).
__device__ __forceinline__ float f16_round(float f) { return static_cast<float>(static_cast<_Float16>(f)); }

__device__ __forceinline__ void f16_round2(float& a0, float& a1) {
  const f32x2 v = {a0, a1};
  const f32x2 r = __builtin_convertvector(__builtin_convertvector(v, f16x2), f32x2);
  a0 = r[0];
  a1 = r[1];
}

// Element formats: what a 16-bit element means (kBytes == 2 policies).
constexpr int kFmtF32 = 0, kFmtBF16 = 1, kFmtF16 = 2;

// ---- element policies -------------------------------------------------------
// E  = elements per 16-byte vector
// init(x0): value of acc after p.mul_(0)
// step(acc, w, x): one `c1.add_(w * p1)` on one element (scalar/tail path)
// step2: the same on two adjacent elements (vector path; lets the compiler
//        use v_pk_mul_f32 / v_pk_add_f32 and the packed bf16 convert)
struct F32Exact {
  static constexpr int E = 4;
  static constexpr int kBytes = 4;
  static constexpr int kFmt = kFmtF32;
  __device__ static float init(float x) { return x * 0.0f; }
  __device__ static float step(float acc, float w, float x) {
    const float p = w * x;  // rounded: contraction is off
    return acc + p;
  }
  __device__ static void step2(float& a0, float& a1, float w, float x0, float x1) {
    a0 = step(a0, w, x0);
    a1 = step(a1, w, x1);
  }
  __device__ static float finish(float a, float) { return a; }
};

struct F32Fast {
  static constexpr int E = 4;
  static constexpr int kBytes = 4;
  static constexpr int kFmt = kFmtF32;
  __device__ static float init(float x) { return x * 0.0f; }
  __device__ static float step(float acc, float w, float x) { return __builtin_fmaf(w, x, acc); }
  __device__ static void step2(float& a0, float& a1, float w, float x0, float x1) {
    a0 = step(a0, w, x0);
    a1 = step(a1, w, x1);
  }
  __device__ static float finish(float a, float) { return a; }
};

// bf16 exact: product and sum each rounded to bf16. x * 0 is +-0 or NaN,
// already bf16-exact, so init needs no rounding.
struct BF16Exact {
  static constexpr int E = 8;
  static constexpr int kBytes = 2;
  static constexpr int kFmt = kFmtBF16;
  __device__ static float init(float x) { return x * 0.0f; }
  __device__ static float step(float acc, float w, float x) {
    const float p = bf16_round(w * x);
    return bf16_round(acc + p);
  }
  __device__ static void step2(float& a0, float& a1, float w, float x0, float x1) {
    float p0 = w * x0, p1 = w * x1;
    bf16_round2(p0, p1);
    a0 = a0 + p0;
    a1 = a1 + p1;
    bf16_round2(a0, a1);
  }
  __device__ static float finish(float a, float) { return a; }
};

struct BF16Fast {
  static constexpr int E = 8;
  static constexpr int kBytes = 2;
  static constexpr int kFmt = kFmtBF16;
  __device__ static float init(float x) { return x * 0.0f; }
  __device__ static float step(float acc, float w, float x) { return __builtin_fmaf(w, x, acc); }
  __device__ static void step2(float& a0, float& a1, float w, float x0, float x1) {
    a0 = step(a0, w, x0);
    a1 = step(a1, w, x1);
  }
  __device__ static float finish(float a, float) { return bf16_round(a); }
};

// fp16 exact: as bf16 (PyTorch's CPU opmath for Half is fp32 too): the
// product and the sum each rounded to fp16, nearest-even.
struct F16Exact {
  static constexpr int E = 8;
  static constexpr int kBytes = 2;
  static constexpr int kFmt = kFmtF16;
  __device__ static float init(float x) { return x * 0.0f; }
  __device__ static float step(float acc, float w, float x) {
    const float p = f16_round(pin_f32(w * x));
    return f16_round(pin_f32(acc + p));
  }
  __device__ static void step2(float& a0, float& a1, float w, float x0, float x1) {
    float p0 = pin_f32(w * x0), p1 = pin_f32(w * x1);
    f16_round2(p0, p1);
    a0 = pin_f32(a0 + p0);
    a1 = pin_f32(a1 + p1);
    f16_round2(a0, a1);
  }
  __device__ static float finish(float a, float) { return a; }
};

struct F16Fast {
  static constexpr int E = 8;
  static constexpr int kBytes = 2;
  static constexpr int kFmt = kFmtF16;
  __device__ static float init(float x) { return x * 0.0f; }
  __device__ static float step(float acc, float w, float x) { return __builtin_fmaf(w, x, acc); }
  __device__ static void step2(float& a0, float& a1, float w, float x0, float x1) {
    a0 = step(a0, w, x0);
    a1 = step(a1, w, x1);
  }
  __device__ static float finish(float a, float) { return f16_round(a); }
};

// fp64 (a double model, dlsim_wreduce_f64): `w * p1` keeps the Python float
// exact as a double scalar and every product and sum is rounded to double
// (PyTorch's CPU opmath for a double tensor), so acc, weights and elements are
// doubles. T / W name the accumulator and weight types of a policy (float for
// every other policy, see acc_t / wt_t below).
struct F64Exact {
  using T = double;
  using W = double;
  static constexpr int E = 2;
  static constexpr int kBytes = 8;
  static constexpr int kFmt = kFmtF32;
  __device__ static double init(double x) { return x * 0.0; }
  __device__ static double step(double acc, double w, double x) {
    const double p = w * x;  // rounded: contraction is off
    return acc + p;
  }
  __device__ static void step2(double& a0, double& a1, double w, double x0, double x1) {
    a0 = step(a0, w, x0);
    a1 = step(a1, w, x1);
  }
  __device__ static double finish(double a, float) { return a; }
};

struct F64Fast {
  using T = double;
  using W = double;
  static constexpr int E = 2;
  static constexpr int kBytes = 8;
  static constexpr int kFmt = kFmtF32;
  __device__ static double init(double x) { return x * 0.0; }
  __device__ static double step(double acc, double w, double x) { return __builtin_fma(w, x, acc); }
  __device__ static void step2(double& a0, double& a1, double w, double x0, double x1) {
    a0 = step(a0, w, x0);
    a1 = step(a1, w, x1);
  }
  __device__ static double finish(double a, float) { return a; }
};

// Accumulator and weight types of a policy: float unless it names T / W.
template <class Op, class = void>
struct OpTypes {
  using T = float;
  using W = float;
};
template <class Op>
struct OpTypes<Op, std::void_t<typename Op::T>> {
  using T = typename Op::T;
  using W = typename Op::W;
};
template <class Op> using acc_t = typename OpTypes<Op>::T;
template <class Op> using wt_t = typename OpTypes<Op>::W;

// Mean of the inputs in input order (dlsim_mean): acc starts at +0 (the
// reduction's identity), adds every input in order, then one division by n
// (weights unused). bf16: the sum is accumulated in fp32, divided in fp32 and
// rounded once (PyTorch's CPU mean of a bf16 tensor sums in fp32, divides,
// and casts back). PyTorch's own CPU order for torch.mean(torch.stack(...),
// 0) — what ChunkManager.reconstruct_model (chunk_manager.py:38-40) needs —
// is chunk_mean_kernels.hpp; these policies also carry its element format.
struct F32Mean {
  static constexpr int E = 4;
  static constexpr int kBytes = 4;
  static constexpr int kFmt = kFmtF32;
  __device__ static float init(float) { return 0.0f; }
  __device__ static float step(float acc, float, float x) { return acc + x; }
  __device__ static void step2(float& a0, float& a1, float, float x0, float x1) {
    a0 = a0 + x0;
    a1 = a1 + x1;
  }
  __device__ static float finish(float a, float div) { return a / div; }
};

struct BF16Mean {
  static constexpr int E = 8;
  static constexpr int kBytes = 2;
  static constexpr int kFmt = kFmtBF16;
  __device__ static float init(float) { return 0.0f; }
  __device__ static float step(float acc, float, float x) { return acc + x; }
  __device__ static void step2(float& a0, float& a1, float, float x0, float x1) {
    a0 = a0 + x0;
    a1 = a1 + x1;
  }
  __device__ static float finish(float a, float div) { return bf16_round(a / div); }
};

struct F16Mean {
  static constexpr int E = 8;
  static constexpr int kBytes = 2;
  static constexpr int kFmt = kFmtF16;
  __device__ static float init(float) { return 0.0f; }
  __device__ static float step(float acc, float, float x) { return acc + x; }
  __device__ static void step2(float& a0, float& a1, float, float x0, float x1) {
    a0 = a0 + x0;
    a1 = a1 + x1;
  }
  __device__ static float finish(float a, float div) { return f16_round(pin_f32(a / div)); }
};

// fp64 chunk mean (ChunkManager on a double model, chunk_manager.py:40): the
// sum in double (chunk_mean_kernels.hpp's orders), one double division by m.
struct F64Mean {
  using T = double;
  using W = double;
  static constexpr int E = 2;
  static constexpr int kBytes = 8;
  static constexpr int kFmt = kFmtF32;
  __device__ static double init(double) { return 0.0; }
  __device__ static double step(double acc, double, double x) { return acc + x; }
  __device__ static void step2(double& a0, double& a1, double, double x0, double x1) {
    a0 = a0 + x0;
    a1 = a1 + x1;
  }
  __device__ static double finish(double a, float div) { return a / static_cast<double>(div); }
};

// ---- 16-byte vector <-> E floats --------------------------------------------
template <class Op>
__device__ __forceinline__ void unpack(const u32x4& r, acc_t<Op> (&x)[Op::E]) {
  if constexpr (Op::kBytes == 8) {
#pragma unroll
    for (int e = 0; e < 2; ++e)
      x[e] = __builtin_bit_cast(double, static_cast<uint64_t>(r[2 * e]) | (static_cast<uint64_t>(r[2 * e + 1]) << 32));
  } else if constexpr (Op::kBytes == 4) {
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = __uint_as_float(r[e]);
  } else if constexpr (Op::kFmt == kFmtF16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t u = r[e];
      x[2 * e] = static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(u & 0xffffu)));
      x[2 * e + 1] = static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(u >> 16)));
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[2 * e] = __uint_as_float(r[e] << 16);
      x[2 * e + 1] = __uint_as_float(r[e] & 0xffff0000u);
    }
  }
}

template <class Op>
__device__ __forceinline__ u32x4 pack(const acc_t<Op> (&a)[Op::E], float div) {
  u32x4 r;
  if constexpr (Op::kBytes == 8) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const uint64_t u = __builtin_bit_cast(uint64_t, Op::finish(a[e], div));
      r[2 * e] = static_cast<uint32_t>(u);
      r[2 * e + 1] = static_cast<uint32_t>(u >> 32);
    }
  } else if constexpr (Op::kBytes == 4) {
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = __float_as_uint(Op::finish(a[e], div));
  } else if constexpr (Op::kFmt == kFmtF16) {
    // finish() already rounded to fp16, so the conversion is exact
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t lo = __builtin_bit_cast(uint16_t, static_cast<_Float16>(Op::finish(a[2 * e], div)));
      const uint32_t hi = __builtin_bit_cast(uint16_t, static_cast<_Float16>(Op::finish(a[2 * e + 1], div)));
      r[e] = lo | (hi << 16);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t lo = __float_as_uint(Op::finish(a[2 * e], div)) >> 16;
      const uint32_t hi = __float_as_uint(Op::finish(a[2 * e + 1], div)) & 0xffff0000u;
      r[e] = lo | hi;
    }
  }
  return r;
}

// ---- scalar element load/store (tail and misaligned paths) ------------------
template <class Op>
__device__ __forceinline__ acc_t<Op> load_elem(const void* p, size_t j) {
  if constexpr (Op::kBytes == 8) {
    return static_cast<const double*>(p)[j];
  } else if constexpr (Op::kBytes == 4) {
    return static_cast<const float*>(p)[j];
  } else if constexpr (Op::kFmt == kFmtF16) {
    return static_cast<float>(static_cast<const _Float16*>(p)[j]);
  } else {
    return __uint_as_float(static_cast<uint32_t>(static_cast<const uint16_t*>(p)[j]) << 16);
  }
}

template <class Op>
__device__ __forceinline__ void store_elem(void* p, size_t j, acc_t<Op> a, float div) {
  if constexpr (Op::kBytes == 8) {
    static_cast<double*>(p)[j] = Op::finish(a, div);
  } else if constexpr (Op::kBytes == 4) {
    static_cast<float*>(p)[j] = Op::finish(a, div);
  } else if constexpr (Op::kFmt == kFmtF16) {
    static_cast<_Float16*>(p)[j] = static_cast<_Float16>(Op::finish(a, div));
  } else {
    static_cast<uint16_t*>(p)[j] = static_cast<uint16_t>(__float_as_uint(Op::finish(a, div)) >> 16);
  }
}

// Load policies: 0 = plain global_load, 1 = global_load ... nt; values
// >= kLdBuffer are buffer_load_dwordx4 with cache-policy bits (LDP - kLdBuffer:
// sc0 = 1, nt = 2, sc1 = 16). Buffer loads use 32-bit byte offsets: one launch
// reads < 2 GiB per input (the host splits longer ranges).
constexpr int kLdBuffer = 100;

template <int LDP>
__device__ __forceinline__ u32x4 ld16(const void* base, size_t v) {
  if constexpr (LDP >= kLdBuffer) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(v * 16), 0,
                                                                           LDP - kLdBuffer));
  } else {
    const u32x4* p = static_cast<const u32x4*>(base) + v;
    if constexpr (LDP == 1) return __builtin_nontemporal_load(p);
    else return *p;
  }
}

template <bool NT>
__device__ __forceinline__ void st16(void* base, size_t v, const u32x4& r) {
  u32x4* p = static_cast<u32x4*>(base) + v;
  if constexpr (NT) __builtin_nontemporal_store(r, p);
  else *p = r;
}

// ---- output store policies ----------------------------------------------------
// kStPlain / kStNT: global_store_dwordx4 (nt = non-temporal). Values >= 0 are
// buffer_store_dwordx4 cache-policy bits (gfx950: sc0 = 1, nt = 2, sc1 = 16),
// e.g. 16 = sc1 write-through: nothing of the output is left dirty in L2 at
// the kernel boundary.
constexpr int kStPlain = -1;
constexpr int kStNT = -2;

struct OutRef {
  void* ptr;
  __amdgpu_buffer_rsrc_t rsrc;
};

template <int STP>
__device__ __forceinline__ void store_vec(const OutRef& o, size_t v, const u32x4& r) {
  if constexpr (STP == kStPlain) {
    st16<false>(o.ptr, v, r);
  } else if constexpr (STP == kStNT) {
    st16<true>(o.ptr, v, r);
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(r, o.rsrc, static_cast<int>(v * 16), 0, STP);
  }
}

template <int STP>
__device__ __forceinline__ OutRef make_out(void* out, size_t nvec) {
  OutRef o;
  o.ptr = out;
  if constexpr (STP >= 0) {
    // wave-uniform descriptor from kernel arguments only (no waterfall loops)
    o.rsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, static_cast<int>(nvec * 16), 0x00020000);
  }
  return o;
}

// ---- kernel arguments -------------------------------------------------------
// Input pointers and fp32 weights travel in the kernarg segment (read with
// scalar loads, wave-uniform), NB slots; n <= NB inputs used.
template <int NB, class W = float>
struct Slots {
  const void* p[NB];
  W w[NB];
  float div;  // final divisor of the mean policies (1 for the weighted reduce)
  __device__ const void* ptr(int i) const { return p[i]; }
  __device__ W wt(int i) const { return w[i]; }
  __device__ float divisor() const { return div; }
};

// Fan-in above the kernarg slots (n > DLSIM_MAX_FUSED_INPUTS): the pointers
// and weights sit in a small device array the host uploads on the launch
// stream (read with scalar loads like the kernargs), so every n is one pass
// over the inputs: each output element is written once, after all n of its
// terms are folded.
template <class W = float>
struct DevSlots {
  const void* const* p;
  const W* w;
  float div;
  __device__ const void* ptr(int i) const { return p[i]; }
  __device__ W wt(int i) const { return w[i]; }
  __device__ float divisor() const { return div; }
};

// Scalar fold of one element over all n inputs (tail / misaligned path).
template <class Op, class S>
__device__ __forceinline__ void fold_scalar(const S& s, int n, void* out, size_t j) {
  // Every load of a chunk of 8 inputs issues before its first use: one HBM
  // round trip per chunk, not one per input. The first input doubles as the
  // x0*0 seed (n >= 1).
  acc_t<Op> a = 0;
  for (int i = 0; i < n; i += 8) {
    acc_t<Op> x[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) x[g] = (i + g < n) ? load_elem<Op>(s.ptr(i + g), j) : 0.0f;
    if (i == 0) a = Op::init(x[0]);
#pragma unroll
    for (int g = 0; g < 8; ++g)
      if (i + g < n) a = Op::step(a, s.wt(i + g), x[g]);
  }
  store_elem<Op>(out, j, a, s.divisor());
}

// Scalar kernel: any alignment, one element per thread.
template <class Op, class S>
__global__ __launch_bounds__(kBlock) void k_wreduce_scalar(const S s, int n, void* __restrict__ out,
                                                           size_t nelem) {
  const size_t j = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (j < nelem) fold_scalar<Op, S>(s, n, out, j);
}

// ---- tiled kernel ------------------------------------------------------------
// A tile is kBlock*VPT 16-byte vectors; lane t of a block owns vectors
// t + k*kBlock of the tile (coalesced 1 KiB per wave per k). Full tiles run
// without bounds checks (no exec-mask branches around the loads); the last
// partial tile and the < E scalar tail go to the grid's last block, which
// holds the fewest full tiles under the grid-stride deal below.
//
// NF > 0: the fan-in n == NF is a compile-time constant: every input's loads
// are issued back to back with no group branches. NF == 0: runtime n in
// groups of G (first group peeled).
template <class Op, int VPT, int NT, bool CHECK, int VS = kBlock>
__device__ __forceinline__ void load_tile(const void* src, size_t v0, size_t nvec,
                                          u32x4 (&r)[VPT]) {
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const size_t idx = v0 + static_cast<size_t>(v) * VS;
    if constexpr (CHECK) {
      r[v] = u32x4{0u, 0u, 0u, 0u};
      if (idx < nvec) r[v] = ld16<NT>(src, idx);
    } else {
      r[v] = ld16<NT>(src, idx);
    }
  }
}

template <class Op, int VPT>
__device__ __forceinline__ void fold_tile(acc_t<Op> (&a)[VPT][Op::E], wt_t<Op> w, const u32x4 (&r)[VPT]) {
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    acc_t<Op> x[Op::E];
    unpack<Op>(r[v], x);
#pragma unroll
    for (int e = 0; e < Op::E; e += 2) Op::step2(a[v][e], a[v][e + 1], w, x[e], x[e + 1]);
  }
}

template <class Op, int VPT>
__device__ __forceinline__ void init_tile(acc_t<Op> (&a)[VPT][Op::E], const u32x4 (&r)[VPT], bool from_acc) {
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    acc_t<Op> x[Op::E];
    unpack<Op>(r[v], x);
#pragma unroll
    for (int e = 0; e < Op::E; ++e) a[v][e] = from_acc ? x[e] : Op::init(x[e]);
  }
}

template <class Op, class S, int NF, int G, int VPT, int NT, bool CHECK, int STP, int VS = kBlock>
__device__ __forceinline__ void reduce_tile(const S& s, int n, const OutRef& out, size_t v0, size_t nvec) {
  acc_t<Op> a[VPT][Op::E];
  if constexpr (NF > 0) {
    u32x4 r[NF][VPT];
#pragma unroll
    for (int i = 0; i < NF; ++i) load_tile<Op, VPT, NT, CHECK, VS>(s.ptr(i), v0, nvec, r[i]);
    init_tile<Op, VPT>(a, r[0], false);
#pragma unroll
    for (int i = 0; i < NF; ++i) fold_tile<Op, VPT>(a, s.wt(i), r[i]);
  } else {
    // first group: up to G inputs, input 0 seeding acc = x0 * 0
    {
      u32x4 r[G][VPT];
      const int cnt = n < G ? n : G;
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (g < cnt) load_tile<Op, VPT, NT, CHECK, VS>(s.ptr(g), v0, nvec, r[g]);
      init_tile<Op, VPT>(a, r[0], false);
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (g < cnt) fold_tile<Op, VPT>(a, s.wt(g), r[g]);
    }
    for (int i0 = G; i0 < n; i0 += G) {
      u32x4 r[G][VPT];
      const int cnt = (n - i0) < G ? (n - i0) : G;
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (g < cnt) load_tile<Op, VPT, NT, CHECK, VS>(s.ptr(i0 + g), v0, nvec, r[g]);
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (g < cnt) fold_tile<Op, VPT>(a, s.wt(i0 + g), r[g]);
    }
  }
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const size_t idx = v0 + static_cast<size_t>(v) * VS;
    if (!CHECK || idx < nvec) store_vec<STP>(out, idx, pack<Op>(a[v], s.divisor()));
  }
}

// STP: output store policy (above). Buffer-store policies need the output's
// vector part to be < 2 GiB (32-bit byte offsets); the host checks.
//
// Block 0 — dispatched first — folds the ragged end (the last partial tile,
// then the < E scalar tail), so that latency hides under the rest of the
// grid instead of trailing it; blocks 1.. take the full tiles, one per block
// when the grid is full + 1 blocks, otherwise grid-strided. A one-block grid
// does everything. (Splitting the two ragged parts over blocks 0 and 1 was
// measured and did not pay: profiles/r01_tune_ragged.log.)
// WAVEMAP: lane l of wave w reads vectors w*64*VPT + l + k*64 of a tile (each
// wave sweeps VPT contiguous KiB per stream) instead of l' + k*kBlock.
template <class Op, class S, int NF, int G, int VPT, int NT, int STP, bool WAVEMAP>
__device__ __forceinline__ void tiles_body(const S& s, int n, void* __restrict__ out, size_t nvec, size_t nelem) {
  constexpr size_t kTile = static_cast<size_t>(kBlock) * VPT;
  const size_t full = nvec / kTile;
  const OutRef o = make_out<STP>(out, nvec);
  const size_t nb = gridDim.x;
  if (blockIdx.x == 0) {
    if (full * kTile < nvec)
      reduce_tile<Op, S, NF, G, VPT, NT, true, STP>(s, n, o, full * kTile + threadIdx.x, nvec);
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < nelem) fold_scalar<Op, S>(s, n, out, j);
    if (nb > 1) return;
  }
  const size_t workers = nb > 1 ? nb - 1 : 1;
  const size_t first = nb > 1 ? blockIdx.x - 1 : 0;
  if constexpr (WAVEMAP) {
    const size_t lane_off = (threadIdx.x >> 6) * 64 * VPT + (threadIdx.x & 63);
    for (size_t t = first; t < full; t += workers)
      reduce_tile<Op, S, NF, G, VPT, NT, false, STP, 64>(s, n, o, t * kTile + lane_off, nvec);
  } else {
    for (size_t t = first; t < full; t += workers)
      reduce_tile<Op, S, NF, G, VPT, NT, false, STP>(s, n, o, t * kTile + threadIdx.x, nvec);
  }
}

template <class Op, class S, int NF, int G, int VPT, int NT, int STP = (NT ? kStNT : kStPlain),
          bool WAVEMAP = false>
__global__ __launch_bounds__(kBlock) void k_wreduce_tiles(const S s, int n, void* __restrict__ out, size_t nvec,
                                                          size_t nelem) {
  tiles_body<Op, S, NF, G, VPT, NT, STP, WAVEMAP>(s, n, out, nvec, nelem);
}

// ---- preloaded arguments (round 6) ----------------------------------------------
// A block's first input loads wait for the kernel arguments that address them.
// Arguments that lead the list are preloaded into SGPRs at wave launch
// (-mllvm -amdgpu-kernarg-preload-count; 14 dwords fit beside the kernarg
// segment pointer): the fixed fan-in deferred kernel takes nvec, the output
// and the first kPre input pointers there, so those loads issue at once and
// only the rest wait for the argument loads (the output must be among them:
// the buffer resource built from it is set up before the first load, and a
// wait for one scalar load waits for all of them). Every deferred block of a
// launch starts at once, so that wait is on the kernel's critical path
// (scripts/probes/kernarg_preload_probe.hip, profiles/r06_kpp/: an 8-input
// reduce 10.04-10.08 -> 9.75-9.79 us; the product's gains and the tiled
// kernel's loss: dispatch.hpp launch_defer_kernel).
constexpr int kPre = 5;
template <class S>
struct PreSlots {
  const void* q[kPre];
  const S& s;
  __device__ const void* ptr(int i) const { return i < kPre ? q[i] : s.ptr(i); }
  __device__ auto wt(int i) const { return s.wt(i); }
  __device__ float divisor() const { return s.divisor(); }
};


// ---- deferred-store kernel (round 5) -----------------------------------------
// HBM pays a bus turnaround each time the traffic switches between reads and
// writes; the tiled kernel's blocks interleave their 16 KiB stores with the
// other blocks' loads all along the launch. Here the output is cut into rows
// of kDeferBlock vectors (lane t of a block owns vector t of a row) and block
// b folds rows [b*R, (b+1)*R): the R results per lane stay in registers until
// all R rows are folded, then go out together, so each CU writes R * 8 KiB
// at a time instead of 16 KiB. The host picks R so the grid's last round of
// blocks keeps most CUs busy (dispatch.hpp defer_rows; DESIGN.md §5e,
// profiles/r05s/ .. r05y/).
//
// R is a runtime argument (uniform, 1 <= R <= RMAX): the loads of U rows
// issue back to back, then fold (a row past R re-reads row r0, which the
// same wave's first load already brings in: no extra HBM traffic); the
// compiler must not hoist later groups' loads above the fold (NF * RMAX live
// vectors would spill), hence the barrier per group. Uniform `if`s instead
// of `break`s keep the loops unrolled and res[] in VGPRs.
constexpr int kDeferBlock = 512;
// U rows' vectors of one group of inputs [i0, i0 + cnt) (cnt <= G; NF > 0: all
// NF inputs, cnt unused).
template <class Op, class S, int NF, int G, int U>
__device__ __forceinline__ void defer_fold_group(const S& s, int i0, int cnt, size_t base, int r0, int R, bool first,
                                                 acc_t<Op> (&a)[U][1][Op::E]) {
  constexpr int K = NF > 0 ? NF : G;
  u32x4 x[K][U];
#pragma unroll
  for (int g = 0; g < K; ++g)
    if (NF > 0 || g < cnt)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = r0 + u < R ? r0 + u : r0;
        x[g][u] = ld16<1>(s.ptr(i0 + g), base + static_cast<size_t>(row) * kDeferBlock);
      }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (first) {
      const u32x4 x0[1] = {x[0][u]};
      init_tile<Op, 1>(a[u], x0, false);
    }
#pragma unroll
    for (int g = 0; g < K; ++g)
      if (NF > 0 || g < cnt) {
        const u32x4 xg[1] = {x[g][u]};
        fold_tile<Op, 1>(a[u], s.wt(i0 + g), xg);
      }
  }
}
// Compile-time R (RC): every row group and store unguarded. NF == 0: the
// grouped form (runtime fan-in in groups of G, input order).
template <class Op, class S, int NF, int G, int RC, int U, int STP>
__device__ __forceinline__ void defer_rows_c(const S& s, int n, const OutRef& o, size_t base) {
  static_assert(RC % U == 0, "whole row groups");
  u32x4 res[RC];
#pragma unroll
  for (int r0 = 0; r0 < RC; r0 += U) {
    if constexpr (NF == 0) {
      acc_t<Op> a[U][1][Op::E];
      defer_fold_group<Op, S, 0, G, U>(s, 0, n < G ? n : G, base, r0, RC, true, a);
      for (int i0 = G; i0 < n; i0 += G)
        defer_fold_group<Op, S, 0, G, U>(s, i0, (n - i0) < G ? (n - i0) : G, base, r0, RC, false, a);
#pragma unroll
      for (int u = 0; u < U; ++u) res[r0 + u] = pack<Op>(a[u][0], s.divisor());
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      continue;
    }
    constexpr int K = NF > 0 ? NF : 1;
    u32x4 x[K][U];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
      for (int u = 0; u < U; ++u) x[i][u] = ld16<1>(s.ptr(i), base + static_cast<size_t>(r0 + u) * kDeferBlock);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc_t<Op> a[1][Op::E];
      const u32x4 x0[1] = {x[0][u]};
      init_tile<Op, 1>(a, x0, false);
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const u32x4 xi[1] = {x[i][u]};
        fold_tile<Op, 1>(a, s.wt(i), xi);
      }
      res[r0 + u] = pack<Op>(a[0], s.divisor());
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int r = 0; r < RC; ++r) store_vec<STP>(o, base + static_cast<size_t>(r) * kDeferBlock, res[r]);
}
template <class Op, class S, int NF, int G, int RMAX, int U, int STP>
__device__ __forceinline__ void defer_rows(const S& s, int n, const OutRef& o, size_t base, int R, size_t nvec) {
  u32x4 res[RMAX];
#pragma unroll
  for (int r0 = 0; r0 < RMAX; r0 += U) {
    if (r0 < R) {
      if constexpr (NF > 0) {
        // (this exact form: folding through defer_fold_group, as the grouped
        // form does, schedules differently and lost the north star's 0.5 us)
        u32x4 x[NF][U];
#pragma unroll
        for (int i = 0; i < NF; ++i)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int row = r0 + u < R ? r0 + u : r0;
            x[i][u] = ld16<1>(s.ptr(i), base + static_cast<size_t>(row) * kDeferBlock);
          }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          acc_t<Op> a[1][Op::E];
          const u32x4 x0[1] = {x[0][u]};
          init_tile<Op, 1>(a, x0, false);
#pragma unroll
          for (int i = 0; i < NF; ++i) {
            const u32x4 xi[1] = {x[i][u]};
            fold_tile<Op, 1>(a, s.wt(i), xi);
          }
          res[r0 + u] = pack<Op>(a[0], s.divisor());
        }
      } else {  // runtime fan-in in groups of G, input order; the first seeds x0 * 0
        acc_t<Op> a[U][1][Op::E];
        defer_fold_group<Op, S, 0, G, U>(s, 0, n < G ? n : G, base, r0, R, true, a);
        for (int i0 = G; i0 < n; i0 += G)
          defer_fold_group<Op, S, 0, G, U>(s, i0, (n - i0) < G ? (n - i0) : G, base, r0, R, false, a);
#pragma unroll
        for (int u = 0; u < U; ++u) res[r0 + u] = pack<Op>(a[u][0], s.divisor());
      }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  // The stores run straight-line: a row past R goes to vector nvec, the first
  // past the output's buffer range, which the hardware drops (a guarded
  // store per row left a chain of branches around out-of-line stores).
  static_assert(STP >= 0, "buffer stores: out-of-range rows are dropped");
#pragma unroll
  for (int r = 0; r < RMAX; ++r)
    store_vec<STP>(o, r < R ? base + static_cast<size_t>(r) * kDeferBlock : nvec, res[r]);
}
// Full blocks defer; the grid's last block, when partial, folds its rows one
// at a time with bounds checks; block 0 also folds the < E scalar tail.
// NF > 0: fixed fan-in n == NF; NF == 0: runtime n in groups of G.
template <class Op, class S, int NF, int G, int RMAX, int U, int STP, int RC>
__device__ __forceinline__ void defer_body(const S& s, int n, int Rrt, void* __restrict__ out, size_t nvec,
                                           size_t nelem) {
  const int R = RC > 0 ? RC : Rrt;
  const size_t span = static_cast<size_t>(kDeferBlock) * static_cast<size_t>(R);
  const size_t base = static_cast<size_t>(blockIdx.x) * span + threadIdx.x;
  const OutRef o = make_out<STP>(out, nvec);
  if (static_cast<size_t>(blockIdx.x + 1) * span <= nvec) {
    if constexpr (RC > 0 && NF > 0) {
      defer_rows_c<Op, S, NF, G, RC, U, STP>(s, n, o, base);
    } else if constexpr (RC > 0) {
      const S* ks = (const S*)__builtin_amdgcn_kernarg_segment_ptr();  // (below)
      defer_rows_c<Op, S, 0, G, RC, U, STP>(*ks, n, o, base);
    } else if constexpr (NF > 0) {
      defer_rows<Op, S, NF, G, RMAX, U, STP>(s, n, o, base, R, nvec);
    } else {
      // The grouped form indexes the slots at run time from 16 unrolled row
      // groups; read through `s` the compiler keeps a private copy of the
      // whole argument (1.5 KiB of scratch per lane for Slots<128>). `s` is
      // the first kernel argument: read it in place in the kernarg segment.
      const S* ks = (const S*)__builtin_amdgcn_kernarg_segment_ptr();
      defer_rows<Op, S, NF, G, RMAX, U, STP>(*ks, n, o, base, R, nvec);
    }
  } else {
    for (int r = 0; r < R; ++r)
      reduce_tile<Op, S, NF, G, 1, 1, true, STP, kDeferBlock>(s, NF > 0 ? NF : n, o,
                                                              base + static_cast<size_t>(r) * kDeferBlock, nvec);
  }
  if (blockIdx.x == 0) {
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < nelem) fold_scalar<Op, S>(s, NF > 0 ? NF : n, out, j);
  }
}

template <class Op, class S, int NF, int G, int RMAX, int U, int STP, int RC = 0>
__global__ __launch_bounds__(kDeferBlock) void k_wreduce_defer(const S s, int n, int Rrt, void* __restrict__ out,
                                                               size_t nvec, size_t nelem) {
  defer_body<Op, S, NF, G, RMAX, U, STP, RC>(s, n, Rrt, out, nvec, nelem);
}

// The fixed fan-in deferred kernel with nvec and the first kPre pointers
// preloaded (PreSlots above). The grouped form (NF == 0) reads its slots in
// place in the kernarg segment, at offset 0: it keeps k_wreduce_defer.
template <class Op, class S, int NF, int G, int RMAX, int U, int STP, int RC = 0>
__global__ __launch_bounds__(kDeferBlock) void k_wreduce_defer_pre(size_t nvec, void* __restrict__ out,
                                                                   const void* q0, const void* q1, const void* q2,
                                                                   const void* q3, const void* q4, const S s, int n,
                                                                   int Rrt, size_t nelem) {
  static_assert(NF > 0, "fixed fan-in");
  const PreSlots<S> ps{{q0, q1, q2, q3, q4}, s};
  defer_body<Op, PreSlots<S>, NF, G, RMAX, U, STP, RC>(ps, n, Rrt, out, nvec, nelem);
}

// ---- batched launch: many independent aggregates in one grid -----------------
// The aggregate tasks of one simulated round (every peer's neighbour mix) are
// independent; small models (GNLeNet: 3 MB per task) are launch-bound when
// each is its own kernel. One grid covers every task: blocks 0 .. ntasks-1
// fold the tasks' ragged ends (the partial tile, then the scalar tail: two
// dependent phases), so they are all dispatched first and finish under the
// full tiles instead of the last task's trailing the grid; block ntasks + f is
// full tile f of the concatenated tasks (task t's full tiles start at
// block_start[t]). Descriptors travel as kernel arguments (read with scalar
// loads); the host splits larger batches.
constexpr int kBatchMaxTasks = 32;
constexpr int kBatchMaxPtrs = 192;

struct BatchSlots {
  const void* p[kBatchMaxPtrs];
  float w[kBatchMaxPtrs];
  void* out[kBatchMaxTasks];
  size_t nvec[kBatchMaxTasks];
  size_t nelem[kBatchMaxTasks];
  float div[kBatchMaxTasks];  // final divisor per task (mean policies; 1 for the reduce)
  uint32_t block_start[kBatchMaxTasks + 1];  // first full tile of each task
  uint32_t ptr_off[kBatchMaxTasks];  // 32-bit: read with scalar loads at a run-time index (16-bit
  uint32_t fan_in[kBatchMaxTasks];   // fields compiled to vector loads; round 6)
  int ntasks;
};
static_assert(sizeof(BatchSlots) <= 4096, "kernel arguments");

// The task of full-tile entry f: the last t with block_start[t] <= f, as a
// count over a compile-time range (wide scalar loads, scalar compares) instead
// of a scan waiting on one dependent load per task passed (round 6).
__device__ __forceinline__ int batch_find_task(const BatchSlots& s, uint32_t f) {
  int t = 0;
#pragma unroll
  for (int j = 1; j < kBatchMaxTasks; ++j) t += (j < s.ntasks && f >= s.block_start[j]) ? 1 : 0;
  return t;
}

// One task's view of the batch (same accessor interface as Slots).
struct TaskArgs {
  const BatchSlots& b;
  int off;
  float d;
  __device__ const void* ptr(int i) const { return b.p[off + i]; }
  __device__ float wt(int i) const { return b.w[off + i]; }
  __device__ float divisor() const { return d; }
};

template <class Op, int NF, int G, int VPT, int NT, int STP, bool WAVEMAP = false>
__global__ __launch_bounds__(kBlock) void k_wreduce_batch(const BatchSlots s) {
  const uint32_t bid = blockIdx.x;
  int t = 0;
  uint32_t local = 0;
  if (bid < static_cast<uint32_t>(s.ntasks)) {
    t = static_cast<int>(bid);
  } else {
    const uint32_t f = bid - static_cast<uint32_t>(s.ntasks);
    t = batch_find_task(s, f);
    local = f - s.block_start[t] + 1;
  }
  const TaskArgs a{s, static_cast<int>(s.ptr_off[t]), s.div[t]};
  const int n = NF > 0 ? NF : static_cast<int>(s.fan_in[t]);
  const size_t nvec = s.nvec[t];
  constexpr size_t kTile = static_cast<size_t>(kBlock) * VPT;
  const size_t full = nvec / kTile;
  const OutRef o = make_out<STP>(s.out[t], nvec);
  if (local == 0) {
    if (full * kTile < nvec)
      reduce_tile<Op, TaskArgs, NF, G, VPT, NT, true, STP>(a, n, o, full * kTile + threadIdx.x, nvec);
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < s.nelem[t]) fold_scalar<Op, TaskArgs>(a, n, s.out[t], j);
    return;
  }
  if constexpr (WAVEMAP) {
    const size_t lane_off = (threadIdx.x >> 6) * 64 * VPT + (threadIdx.x & 63);
    reduce_tile<Op, TaskArgs, NF, G, VPT, NT, false, STP, 64>(a, n, o, (local - 1) * kTile + lane_off, nvec);
  } else {
    reduce_tile<Op, TaskArgs, NF, G, VPT, NT, false, STP>(a, n, o, (local - 1) * kTile + threadIdx.x, nvec);
  }
}

// ---- batched launch from a device descriptor table ----------------------------
// Same work as k_wreduce_batch for any number of tasks: the descriptors live
// in a device buffer the caller uploads (dlsim_batch_table_*), each block
// finds its task with one read of a block -> task map (scalar loads, the
// index is wave-uniform). The same block order: the ntasks ragged-end blocks
// first, then every task's full tiles (a task's block_start is one before its
// first full-tile block, so local = blockIdx.x - block_start >= 1 there).
struct BatchTableHeader {
  uint32_t ntasks;
  uint32_t nblocks;
  uint32_t uniform_fan_in;  // fan-in shared by every task, or 0
  uint32_t vpt;             // vectors per lane the block map was laid out for (1 or 4)
  uint64_t tasks_off;       // byte offsets from the table base
  uint64_t map_off;
  uint64_t ptrs_off;
  uint64_t w_off;
};

struct BatchTaskDesc {
  void* out;
  uint64_t nvec;
  uint64_t nelem;
  uint32_t block_start;
  uint32_t ptr_off;
  uint32_t fan_in;
  uint32_t reserved;
};

struct TableArgs {
  const void* const* p;
  const float* w;
  __device__ const void* ptr(int i) const { return p[i]; }
  __device__ float wt(int i) const { return w[i]; }
  __device__ float divisor() const { return 1.0f; }
};

template <class Op, int NF, int G, int VPT, int NT, int STP, bool WAVEMAP = false>
__global__ __launch_bounds__(kBlock) void k_wreduce_batch_table(const unsigned char* __restrict__ table) {
  const BatchTableHeader* h = reinterpret_cast<const BatchTableHeader*>(table);
  const uint32_t* map = reinterpret_cast<const uint32_t*>(table + h->map_off);
  const uint32_t t = map[blockIdx.x];
  const BatchTaskDesc d = reinterpret_cast<const BatchTaskDesc*>(table + h->tasks_off)[t];
  const TableArgs a{reinterpret_cast<const void* const*>(table + h->ptrs_off) + d.ptr_off,
                    reinterpret_cast<const float*>(table + h->w_off) + d.ptr_off};
  const int n = NF > 0 ? NF : static_cast<int>(d.fan_in);
  const size_t nvec = d.nvec;
  constexpr size_t kTile = static_cast<size_t>(kBlock) * VPT;
  const size_t full = nvec / kTile;
  const OutRef o = make_out<STP>(d.out, nvec);
  const uint32_t local = blockIdx.x < h->ntasks ? 0u : blockIdx.x - d.block_start;
  if (local == 0) {
    if (full * kTile < nvec)
      reduce_tile<Op, TableArgs, NF, G, VPT, NT, true, STP>(a, n, o, full * kTile + threadIdx.x, nvec);
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < d.nelem) fold_scalar<Op, TableArgs>(a, n, d.out, j);
    return;
  }
  if constexpr (WAVEMAP) {
    const size_t lane_off = (threadIdx.x >> 6) * 64 * VPT + (threadIdx.x & 63);
    reduce_tile<Op, TableArgs, NF, G, VPT, NT, false, STP, 64>(a, n, o, (local - 1) * kTile + lane_off, nvec);
  } else {
    reduce_tile<Op, TableArgs, NF, G, VPT, NT, false, STP>(a, n, o, (local - 1) * kTile + threadIdx.x, nvec);
  }
}

// Memory-only probe (dlsim_probe_pattern): the element policy of the reduce
// with the weighted fold replaced by a bitwise XOR of the inputs' bits, run
// through the same dispatch (kernel, launch shape, load and store policies).
// Its time is what the memory system allows for exactly the reduce's
// read/write mix; the reduce is timed against it. n = 1 is a
// bit-exact copy.
template <int BYTES>
struct XorProbe {
  static constexpr int E = 16 / BYTES;
  static constexpr int kBytes = BYTES;
  static constexpr int kFmt = BYTES == 4 ? kFmtF32 : kFmtBF16;
  __device__ static float init(float) { return 0.0f; }
  __device__ static float step(float acc, float, float x) {
    float r = __uint_as_float(__float_as_uint(acc) ^ __float_as_uint(x));
    // XOR is associative: without this pin the compiler may re-associate the
    // chain and schedule the loads unlike the reduce's strictly ordered fold
    // (seen as a probe slower than the reduce for the grouped VPT 1 shape)
    asm volatile("" : "+v"(r));
    return r;
  }
  __device__ static void step2(float& a0, float& a1, float w, float x0, float x1) {
    a0 = step(a0, w, x0);
    a1 = step(a1, w, x1);
  }
  __device__ static float finish(float a, float) { return a; }
};

// ---- parameters of different dtypes at one position (round 5) -----------------
// fedavg.py:20-25 when a model's parameter t has another dtype than
// models[0]'s: c1 (models[0]'s dtype cd) starts as
// models[0][t] * 0, then per input i `c1.add_(w_i * p1)` with torch's type
// promotion: the product in p1's dtype pd (float(w) * x rounded to fp32 and then
// to pd for fp32 / bf16 / fp16; the exact double w times x for fp64), the add
// in result_type(cd, pd) (fp32 for any pair of fp32 / bf16 / fp16, fp64 with a
// double on either side), cast back into cd the way c10 casts (a double to
// bf16 / fp16 goes through float). Pinned by tests/golden/mixed_*.npz, made by
// running the reference. One element per lane, values carried as exact
// doubles; a rare path (simulations aggregate one architecture), so no
// vector loads. dtype codes are include/dlsim.h's DLSIM_F32/BF16/F16/F64.
constexpr int kMixedMaxInputs = 32;
struct MixedSlots {
  const void* p[kMixedMaxInputs];
  double w[kMixedMaxInputs];
  int dt[kMixedMaxInputs];
  int n;       // inputs of this pass
  int out_dt;  // cd
  int seed;    // 1: start from input 0 * 0; 0: continue from the output (a later pass)
};

__device__ __forceinline__ double pin_f64(double v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ double mixed_load(const void* p, int dt, size_t j) {
  switch (dt) {
    case 0: return static_cast<double>(static_cast<const float*>(p)[j]);
    case 1: return static_cast<double>(__uint_as_float(static_cast<uint32_t>(static_cast<const uint16_t*>(p)[j]) << 16));
    case 2: return static_cast<double>(static_cast<float>(static_cast<const _Float16*>(p)[j]));
    default: return static_cast<const double*>(p)[j];
  }
}

// a float result cast to dt (f32 / bf16 / f16), as an exact double
__device__ __forceinline__ double mixed_round_f32(float x, int dt) {
  x = pin_f32(x);
  if (dt == 1) return static_cast<double>(bf16_round(x));
  if (dt == 2) return static_cast<double>(pin_f32(f16_round(x)));
  return static_cast<double>(x);
}

// a double result cast to dt: c10 converts a double to float first, and a
// bf16 / fp16 from that float
__device__ __forceinline__ double mixed_round_f64(double x, int dt) {
  if (dt == 3) return x;
  return mixed_round_f32(static_cast<float>(x), dt);
}

__device__ __forceinline__ void mixed_store(void* p, int dt, size_t j, double v) {
  switch (dt) {  // v is exactly representable in dt (bf16: a canonical NaN if NaN)
    case 0: static_cast<float*>(p)[j] = static_cast<float>(v); break;
    case 1: static_cast<uint16_t*>(p)[j] = static_cast<uint16_t>(__float_as_uint(static_cast<float>(v)) >> 16); break;
    case 2: static_cast<_Float16*>(p)[j] = static_cast<_Float16>(static_cast<float>(v)); break;
    default: static_cast<double*>(p)[j] = v;
  }
}

// (a template so that the header, included by every unit, defines it once:
// instantiated with MixedSlots by dlsim_abi.hip)
template <class S>
__global__ __launch_bounds__(kBlock) void k_wreduce_mixed(const S s, void* __restrict__ out, size_t nelem) {
  const int cd = s.out_dt;
  for (size_t j = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; j < nelem;
       j += static_cast<size_t>(gridDim.x) * kBlock) {
    double acc;
    if (s.seed) {
      const double x0 = mixed_load(s.p[0], cd, j);
      acc = cd == 3 ? pin_f64(x0 * 0.0) : mixed_round_f32(static_cast<float>(x0) * 0.0f, cd);
    } else {
      acc = mixed_load(out, cd, j);
    }
    for (int i = 0; i < s.n; ++i) {
      const int pd = s.dt[i];
      const double x = mixed_load(s.p[i], pd, j);
      const double prod = pd == 3 ? pin_f64(s.w[i] * x)
                                  : mixed_round_f32(static_cast<float>(s.w[i]) * static_cast<float>(x), pd);
      if (cd == 3 || pd == 3)
        acc = mixed_round_f64(pin_f64(acc + prod), cd);
      else
        acc = mixed_round_f32(static_cast<float>(acc) + static_cast<float>(prod), cd);
    }
    mixed_store(out, cd, j, acc);
  }
}

}  // namespace dlsim
