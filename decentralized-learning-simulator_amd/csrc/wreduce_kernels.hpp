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

// Multiply and add must stay separate roundings: hipcc defaults to
// -ffp-contract=fast-honor-pragmas, which would fuse acc + w*x into v_fma_f32
// and change ~55% of the results (hard part (a)).
#pragma clang fp contract(off)

namespace dlsim {

constexpr int kBlock = 256;  // 4 waves of 64 lanes

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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

// ---- element policies -------------------------------------------------------
// E  = elements per 16-byte vector
// init(x0): value of acc after p.mul_(0)
// step(acc, w, x): one `c1.add_(w * p1)`
struct F32Exact {
  static constexpr int E = 4;
  static constexpr int kBytes = 4;
  __device__ static float init(float x) { return x * 0.0f; }
  __device__ static float step(float acc, float w, float x) {
    const float p = w * x;  // rounded: contraction is off
    return acc + p;
  }
  __device__ static float finish(float a) { return a; }
};

struct F32Fast {
  static constexpr int E = 4;
  static constexpr int kBytes = 4;
  __device__ static float init(float x) { return x * 0.0f; }
  __device__ static float step(float acc, float w, float x) { return __builtin_fmaf(w, x, acc); }
  __device__ static float finish(float a) { return a; }
};

struct BF16Exact {
  static constexpr int E = 8;
  static constexpr int kBytes = 2;
  __device__ static float init(float x) { return bf16_round(x * 0.0f); }
  __device__ static float step(float acc, float w, float x) {
    const float p = bf16_round(w * x);
    return bf16_round(acc + p);
  }
  __device__ static float finish(float a) { return a; }
};

struct BF16Fast {
  static constexpr int E = 8;
  static constexpr int kBytes = 2;
  __device__ static float init(float x) { return x * 0.0f; }
  __device__ static float step(float acc, float w, float x) { return __builtin_fmaf(w, x, acc); }
  __device__ static float finish(float a) { return bf16_round(a); }
};

// ---- 16-byte vector <-> E floats --------------------------------------------
template <class Op>
__device__ __forceinline__ void unpack(const u32x4& r, float (&x)[Op::E]) {
  if constexpr (Op::kBytes == 4) {
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = __uint_as_float(r[e]);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[2 * e] = __uint_as_float(r[e] << 16);
      x[2 * e + 1] = __uint_as_float(r[e] & 0xffff0000u);
    }
  }
}

template <class Op>
__device__ __forceinline__ u32x4 pack(const float (&a)[Op::E]) {
  u32x4 r;
  if constexpr (Op::kBytes == 4) {
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = __float_as_uint(Op::finish(a[e]));
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t lo = __float_as_uint(Op::finish(a[2 * e])) >> 16;
      const uint32_t hi = __float_as_uint(Op::finish(a[2 * e + 1])) & 0xffff0000u;
      r[e] = lo | hi;
    }
  }
  return r;
}

// ---- scalar element load/store (tail and misaligned paths) ------------------
template <class Op>
__device__ __forceinline__ float load_elem(const void* p, size_t j) {
  if constexpr (Op::kBytes == 4) {
    return static_cast<const float*>(p)[j];
  } else {
    return __uint_as_float(static_cast<uint32_t>(static_cast<const uint16_t*>(p)[j]) << 16);
  }
}

template <class Op>
__device__ __forceinline__ void store_elem(void* p, size_t j, float a) {
  if constexpr (Op::kBytes == 4) {
    static_cast<float*>(p)[j] = Op::finish(a);
  } else {
    static_cast<uint16_t*>(p)[j] = static_cast<uint16_t>(__float_as_uint(Op::finish(a)) >> 16);
  }
}

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const void* base, size_t v) {
  const u32x4* p = static_cast<const u32x4*>(base) + v;
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <bool NT>
__device__ __forceinline__ void st16(void* base, size_t v, const u32x4& r) {
  u32x4* p = static_cast<u32x4*>(base) + v;
  if constexpr (NT) __builtin_nontemporal_store(r, p);
  else *p = r;
}

// ---- kernel arguments -------------------------------------------------------
// Input pointers and fp32 weights travel in the kernarg segment (read with
// scalar loads, wave-uniform), NB slots; n <= NB inputs used.
template <int NB>
struct Slots {
  const void* p[NB];
  float w[NB];
};

// One group of up to G inputs: issue every load first, then fold in order.
// FIRST: the group starts the sum (acc from x0*0, or from acc_in).
template <class Op, int NB, int G, int VPT, bool NT, bool FIRST>
__device__ __forceinline__ void fold_group(const Slots<NB>& s, int i0, int cnt,
                                           const void* acc_in, const size_t (&vi)[VPT],
                                           const bool (&live)[VPT],
                                           float (&a)[VPT][Op::E]) {
  // Lanes past the end keep zeros (never stored); no value is left undefined.
  u32x4 r[G][VPT];
  u32x4 racc[VPT];
#pragma unroll
  for (int v = 0; v < VPT; ++v) racc[v] = u32x4{0u, 0u, 0u, 0u};
  if constexpr (FIRST) {
    if (acc_in) {
#pragma unroll
      for (int v = 0; v < VPT; ++v)
        if (live[v]) racc[v] = ld16<NT>(acc_in, vi[v]);
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int v = 0; v < VPT; ++v) r[g][v] = u32x4{0u, 0u, 0u, 0u};
    if (g < cnt) {
      const void* src = s.p[i0 + g];
#pragma unroll
      for (int v = 0; v < VPT; ++v)
        if (live[v]) r[g][v] = ld16<NT>(src, vi[v]);
    }
  }
  if constexpr (FIRST) {
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      float x[Op::E];
      if (acc_in) {
        unpack<Op>(racc[v], x);
#pragma unroll
        for (int e = 0; e < Op::E; ++e) a[v][e] = x[e];
      } else {
        unpack<Op>(r[0][v], x);
#pragma unroll
        for (int e = 0; e < Op::E; ++e) a[v][e] = Op::init(x[e]);
      }
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    if (g < cnt) {
      const float w = s.w[i0 + g];
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        float x[Op::E];
        unpack<Op>(r[g][v], x);
#pragma unroll
        for (int e = 0; e < Op::E; ++e) a[v][e] = Op::step(a[v][e], w, x[e]);
      }
    }
  }
}

// Scalar fold of one element over all n inputs (tail / misaligned path).
template <class Op, int NB>
__device__ __forceinline__ void fold_scalar(const Slots<NB>& s, int n, const void* acc_in,
                                            void* out, size_t j) {
  float a = acc_in ? load_elem<Op>(acc_in, j) : Op::init(load_elem<Op>(s.p[0], j));
  int i = 0;
  // Loads of a chunk of 8 inputs are independent of the running sum; the
  // unrolled chunk lets them issue together.
  for (; i + 8 <= n; i += 8) {
    float x[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) x[g] = load_elem<Op>(s.p[i + g], j);
#pragma unroll
    for (int g = 0; g < 8; ++g) a = Op::step(a, s.w[i + g], x[g]);
  }
  for (; i < n; ++i) a = Op::step(a, s.w[i], load_elem<Op>(s.p[i], j));
  store_elem<Op>(out, j, a);
}

// Vector kernel: thread t of block b owns 16-byte vectors
//   b*kBlock*VPT + t + k*kBlock,  k < VPT   (coalesced per k)
// over [0, nvec). Elements [nvec*E, nelem) — fewer than E — are folded by
// block 0 afterwards (block 0 is dispatched first, so that latency hides
// under the rest of the grid).
template <class Op, int NB, int G, int VPT, bool NT>
__global__ __launch_bounds__(kBlock) void k_wreduce_vec(const Slots<NB> s, int n,
                                                        const void* __restrict__ acc_in,
                                                        void* __restrict__ out, size_t nvec,
                                                        size_t nelem) {
  const size_t base = static_cast<size_t>(blockIdx.x) * (kBlock * VPT) + threadIdx.x;
  size_t vi[VPT];
  bool live[VPT];
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    vi[v] = base + static_cast<size_t>(v) * kBlock;
    live[v] = vi[v] < nvec;
  }
  float a[VPT][Op::E];
  int cnt0 = n < G ? n : G;
  fold_group<Op, NB, G, VPT, NT, true>(s, 0, cnt0, acc_in, vi, live, a);
  for (int i0 = G; i0 < n; i0 += G) {
    const int cnt = (n - i0) < G ? (n - i0) : G;
    fold_group<Op, NB, G, VPT, NT, false>(s, i0, cnt, acc_in, vi, live, a);
  }
#pragma unroll
  for (int v = 0; v < VPT; ++v)
    if (live[v]) st16<NT>(out, vi[v], pack<Op>(a[v]));

  if (blockIdx.x == 0) {
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < nelem) fold_scalar<Op, NB>(s, n, acc_in, out, j);
  }
}

// Scalar kernel: any alignment, one element per thread.
template <class Op, int NB>
__global__ __launch_bounds__(kBlock) void k_wreduce_scalar(const Slots<NB> s, int n,
                                                           const void* __restrict__ acc_in,
                                                           void* __restrict__ out,
                                                           size_t nelem) {
  const size_t j = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (j < nelem) fold_scalar<Op, NB>(s, n, acc_in, out, j);
}

// Copy probe: the achievable streaming ceiling on this device.
template <int VPT>
__global__ __launch_bounds__(kBlock) void k_copy16(const u32x4* __restrict__ src,
                                                   u32x4* __restrict__ dst, size_t nvec) {
  const size_t base = static_cast<size_t>(blockIdx.x) * (kBlock * VPT) + threadIdx.x;
  u32x4 r[VPT];
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const size_t i = base + static_cast<size_t>(v) * kBlock;
    if (i < nvec) r[v] = src[i];
  }
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const size_t i = base + static_cast<size_t>(v) * kBlock;
    if (i < nvec) dst[i] = r[v];
  }
}

}  // namespace dlsim
