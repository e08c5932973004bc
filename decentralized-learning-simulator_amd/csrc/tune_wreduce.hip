// tune_wreduce.hip — standalone tuning harness for the reduce kernels.
// Times launch-shape variants of k_wreduce_tiles on rotating input sets (so
// the 256 MiB Infinity Cache cannot serve re-reads) with hipEvents around
// each launch, checks every variant bit-for-bit against the shipped shape,
// and prints one line per variant. Not part of the product library.
//
//   tune_wreduce [n] [P] [dtype f32|bf16] [mode exact|fast] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <map>
#include <vector>

#include "wreduce_kernels.hpp"
#include "chunk_mean_kernels.hpp"

namespace dlsim {
// Experimental bf16-exact element policies (compared against the shipped
// BF16Exact, which rounds with v_cvt_pk_bf16_f32).
struct BF16ExactOld {  // integer RNE with an explicit NaN branch (round-1 shape)
  static constexpr int E = 8;
  static constexpr int kBytes = 2;
  static constexpr int kFmt = kFmtBF16;
  __device__ static float init(float x) { return bf16_round(x * 0.0f); }
  __device__ static float step(float acc, float w, float x) {
    return bf16_round(acc + bf16_round(w * x));
  }
  __device__ static void step2(float& a0, float& a1, float w, float x0, float x1) {
    a0 = step(a0, w, x0);
    a1 = step(a1, w, x1);
  }
  __device__ static float finish(float a, float) { return a; }
};
__device__ __forceinline__ float bf16_round_nonan(float f) {  // valid when NaNs have zero low halves
  uint32_t u = __float_as_uint(f);
  return __uint_as_float((u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u);
}
struct BF16ExactInt {
  static constexpr int E = 8;
  static constexpr int kBytes = 2;
  static constexpr int kFmt = kFmtBF16;
  __device__ static float init(float x) { return x * 0.0f; }
  __device__ static float step(float acc, float w, float x) {
    return bf16_round_nonan(acc + bf16_round_nonan(w * x));
  }
  __device__ static void step2(float& a0, float& a1, float w, float x0, float x1) {
    a0 = step(a0, w, x0);
    a1 = step(a1, w, x1);
  }
  __device__ static float finish(float a, float) { return a; }
};
// ---- LDS-DMA variant (experiment, not shipped: no gain over register
// streaming on MI355X) -------------------------------------------
// Each wave streams its inputs global -> LDS with global_load_lds_dwordx4
// (no VGPR destination; aux = 2 is the non-temporal policy), waits on its own
// vmcnt, then reads its lane's 16 B back with ds_read_b128. Waves never share
// LDS, so no barrier is needed. NF inputs, VPT vectors per lane, full tiles
// only (the caller handles ragged ends with k_wreduce_tiles).
template <class Op, int NF, int VPT, int AUX>
__global__ __launch_bounds__(kBlock) void k_wreduce_lds(const Slots<128> s, void* __restrict__ out,
                                                        size_t full_tiles) {
  constexpr int kWaves = kBlock / 64;
  __shared__ u32x4 lds[kWaves][NF * VPT][64];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  constexpr size_t kTile = static_cast<size_t>(kBlock) * VPT;
  for (size_t t = blockIdx.x; t < full_tiles; t += gridDim.x) {
    // wave w covers vectors [t*kTile + w*64*VPT, +64*VPT): VPT contiguous KiB
    const size_t v0 = t * kTile + static_cast<size_t>(wave) * 64 * VPT + lane;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
#pragma unroll
      for (int v = 0; v < VPT; ++v) {
        const u32x4* g = static_cast<const u32x4*>(s.p[i]) + v0 + v * 64;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                         (__attribute__((address_space(3))) void*)&lds[wave][i * VPT + v][0],
                                         16, 0, AUX);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float a[VPT][Op::E];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      u32x4 r[VPT];
#pragma unroll
      for (int v = 0; v < VPT; ++v) r[v] = lds[wave][i * VPT + v][lane];
      if (i == 0) init_tile<Op, VPT>(a, r, false);
      fold_tile<Op, VPT>(a, s.w[i], r);
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v) st16<true>(out, v0 + v * 64, pack<Op>(a[v], s.div));
    // the next tile's DMA must not overwrite LDS this wave is still reading
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// ---- round 3: the ceiling of the 8:1 read/write mix ---------------------------
// Read-only probe: the shipped large fp32 shape (wave map, VPT 4, global nt
// loads) with the fold replaced by the pinned XOR and the store kept only
// behind a data-dependent branch that never fires for the harness's finite
// inputs (the XOR of finite fp32 words is never the sentinel), so every load
// stays and nothing is written.
template <int NF, int VPT>
__global__ __launch_bounds__(kBlock) void k_probe_rdonly(const Slots<128> s, void* __restrict__ out, size_t nvec) {
  constexpr size_t kTile = static_cast<size_t>(kBlock) * VPT;
  const size_t t = blockIdx.x;
  if (t >= nvec / kTile) return;
  const size_t v0 = t * kTile + (threadIdx.x >> 6) * 64 * VPT + (threadIdx.x & 63);
  u32x4 r[NF][VPT];
#pragma unroll
  for (int i = 0; i < NF; ++i) load_tile<F32Exact, VPT, 1, false, 64>(s.p[i], v0, nvec, r[i]);
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
      x ^= r[i][v][0] ^ r[i][v][1] ^ r[i][v][2] ^ r[i][v][3];
      asm volatile("" : "+v"(x));
    }
  if (x == 0x7fbadbadu) static_cast<uint32_t*>(out)[v0] = x;
}

// Write-only probe: the same tiles and sc1 buffer stores of the output, no
// loads (the value is the vector index, so the stores cannot be merged away).
template <int VPT, int STP = 16>
__global__ __launch_bounds__(kBlock) void k_probe_wronly(void* __restrict__ out, size_t nvec) {
  constexpr size_t kTile = static_cast<size_t>(kBlock) * VPT;
  const size_t t = blockIdx.x;
  if (t >= nvec / kTile) return;
  const OutRef o = make_out<STP>(out, nvec);
  const size_t v0 = t * kTile + (threadIdx.x >> 6) * 64 * VPT + (threadIdx.x & 63);
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const uint32_t k = static_cast<uint32_t>(v0 + v * 64);
    store_vec<STP>(o, v0 + v * 64, u32x4{k, k + 1, k + 2, k + 3});
  }
}

// Pipelined LDS-DMA ring: a persistent grid; each wave
// owns a ring of ST slots of NF KiB in LDS (one 1 KiB global_load_lds_dwordx4
// per input per wave tile of 64 vectors) and keeps ST-1 wave tiles of DMA in
// flight while it folds the oldest slot from LDS. Wave tiles are dealt
// round-robin over all waves of the grid (neighbouring KiB on different CUs,
// as the shipped map). AUX is the load cache policy (2 = nt). The wait before
// reading slot k is vmcnt((ST-1)*NF): everything issued after tile k's DMA
// is at least (ST-1)*NF loads (plus stores), so it is safe whether stores
// retire in order with the loads or not. Full wave tiles only; the harness
// sizes keep the ragged rest out of the comparison (the `same` column).
template <class Op, int NF, int ST, int AUX, int WPB, int STP = 16>
__global__ __launch_bounds__(64 * WPB) void k_wreduce_ldsring(const Slots<128> s, void* __restrict__ out,
                                                              size_t nvec) {
  __shared__ u32x4 ring[WPB][ST][NF][64];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const size_t nwt = nvec / 64;  // full wave tiles
  const size_t gw = static_cast<size_t>(blockIdx.x) * WPB + wave;
  const size_t stride = static_cast<size_t>(gridDim.x) * WPB;
  const OutRef o = make_out<STP>(out, nvec);
  auto issue = [&](size_t wt, int slot) {
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const u32x4* g = static_cast<const u32x4*>(s.p[i]) + wt * 64 + lane;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                       (__attribute__((address_space(3))) void*)&ring[wave][slot][i][0], 16, 0, AUX);
    }
  };
  // prologue: ST-1 tiles in flight
#pragma unroll
  for (int k = 0; k < ST - 1; ++k) {
    const size_t wt = gw + k * stride;
    if (wt < nwt) issue(wt, k);
  }
  int slot = 0;
  for (size_t wt = gw; wt < nwt; wt += stride) {
    const size_t ahead = wt + (ST - 1) * stride;
    if (ahead < nwt) {
      issue(ahead, (slot + ST - 1) % ST);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((ST - 1) * NF) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    acc_t<Op> a[1][Op::E];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      u32x4 r[1];
      r[0] = ring[wave][slot][i][lane];
      if (i == 0) init_tile<Op, 1>(a, r, false);
      fold_tile<Op, 1>(a, s.w[i], r);
    }
    // the slot is refilled by the next iteration's DMA: its reads must be done
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    store_vec<STP>(o, wt * 64 + lane, pack<Op>(a[0], s.div));
    slot = (slot + 1) % ST;
  }
}

// Block-size experiment: wave-contiguous map (stride 64 per vector) with
// BLOCK threads per workgroup; tile = BLOCK * VPT vectors; block 0 takes the
// ragged end (none for tile-multiple P) like the shipped kernel.
template <class Op, int NF, int VPT, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_tiles_block(const Slots<128> s, int n, void* __restrict__ out,
                                                       size_t nvec) {
  constexpr size_t kT = static_cast<size_t>(BLOCK) * VPT;
  const size_t full = nvec / kT;
  const OutRef o = make_out<16>(out, nvec);
  if (blockIdx.x == 0) return;  // tile-multiple sizes only in this experiment
  const size_t t = blockIdx.x - 1;
  if (t >= full) return;
  const size_t lane_off = (threadIdx.x >> 6) * 64 * VPT + (threadIdx.x & 63);
  reduce_tile<Op, Slots<128>, NF, 8, VPT, 1, false, 16, 64>(s, n, o, t * kT + lane_off, nvec);
}

// XCD-aware tile map experiment: workgroups are dispatched round-robin over
// the 8 XCDs, so block k+1 runs on XCD (k+1) % 8; this map gives each XCD one
// contiguous 1/8 of the tiles (its own L2 / TLB footprint) instead of every
// 8th tile. Tile-multiple sizes only; grid = 8 * per + 1.
template <class Op, int NF, int VPT>
__global__ __launch_bounds__(kBlock) void k_tiles_xcd(const Slots<128> s, int n, void* __restrict__ out,
                                                      size_t nvec, size_t per) {
  constexpr size_t kT = static_cast<size_t>(kBlock) * VPT;
  const OutRef o = make_out<16>(out, nvec);
  if (blockIdx.x == 0) return;
  const size_t k = blockIdx.x - 1;
  const size_t t = (k & 7) * per + (k >> 3);
  if (t >= nvec / kT) return;
  const size_t lane_off = (threadIdx.x >> 6) * 64 * VPT + (threadIdx.x & 63);
  reduce_tile<Op, Slots<128>, NF, 8, VPT, 1, false, 16, 64>(s, n, o, t * kT + lane_off, nvec);
}
// Translation-reach experiment (round 4, DLSIM_TUNE_TLB): the blocks that
// share an XCD (blockIdx % 8) take runs of C consecutive tiles, the XCDs
// advancing side by side through super-chunks of 8*C tiles, so one XCD's
// translations cover ~1/8 of the pages in flight (C = 128 tiles of 16 KiB =
// one 2 MiB page per stream). Full tiles only; block 0 idles.
template <class Op, int NF, int VPT, int C>
__global__ __launch_bounds__(kBlock) void k_tiles_xcdc(const Slots<128> s, int n, void* __restrict__ out,
                                                       size_t nvec) {
  constexpr size_t kT = static_cast<size_t>(kBlock) * VPT;
  const OutRef o = make_out<16>(out, nvec);
  if (blockIdx.x == 0) return;
  const size_t k = blockIdx.x - 1;
  const size_t j = k >> 3;
  const size_t t = (j / C) * 8 * C + (k & 7) * C + (j % C);
  if (t >= nvec / kT) return;
  const size_t lane_off = (threadIdx.x >> 6) * 64 * VPT + (threadIdx.x & 63);
  reduce_tile<Op, Slots<128>, NF, 8, VPT, 1, false, 16, 64>(s, n, o, t * kT + lane_off, nvec);
}
}  // namespace dlsim

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

using namespace dlsim;

__global__ void k_fill(uint32_t* p, size_t nwords, uint32_t seed, int bf16) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < nwords; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
    // finite values of moderate magnitude: exponent 120..127, random mantissa/sign
    uint32_t f = (h & 0x807fffffu) | ((120u + (h >> 28) % 8u) << 23);
    if (bf16) {
      const uint32_t lo = (h & 0x807fu) | ((120u + ((h >> 8) & 7u)) << 7);
      const uint32_t hi = ((h >> 16) & 0x807fu) | ((120u + ((h >> 24) & 7u)) << 7);
      f = lo | (hi << 16);
    }
    p[i] = f;
  }
}

struct Variant {
  std::string name;
  void (*launch)(const Slots<128>&, int, void*, size_t, size_t, hipStream_t, int);
  int gm;  // grid: 0 = one tile per block, k = k*256 blocks (grid-stride)
  double moved = 1.0;  // bytes the variant moves, as a fraction of the reduce's (probes)
};

template <class Op, int NF, int G, int VPT, bool NT>
void launch_t(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int gm) {
  const size_t tile = (size_t)kBlock * VPT;
  const size_t full = nvec / tile;
  size_t grid = full + 1;
  if (gm > 0) grid = std::min<size_t>(grid, (size_t)gm * 256);
  hipLaunchKernelGGL((k_wreduce_tiles<Op, Slots<128>, NF, G, VPT, NT>), dim3((unsigned)grid), dim3(kBlock), 0,
                     st, s, n, out, nvec, nelem);
}

template <class Op, int NF, int G, int VPT, int NT, int NTS, bool WM = false>
void launch_ts(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int gm) {
  const size_t tile = (size_t)kBlock * VPT;
  const size_t full = nvec / tile;
  size_t grid = full + 1;
  // gm > 0: grid-stride with gm*256 blocks; gm < 0: one tile per block, at most
  // -gm blocks per CU (occupancy capped by dynamic LDS: 160 KiB / -gm each)
  size_t lds = 0;
  if (gm > 0) grid = std::min<size_t>(grid, (size_t)gm * 256);
  if (gm < 0) lds = (160 * 1024) / (size_t)(-gm) - 512;
  hipLaunchKernelGGL((k_wreduce_tiles<Op, Slots<128>, NF, G, VPT, NT, NTS, WM>), dim3((unsigned)grid), dim3(kBlock), lds,
                     st, s, n, out, nvec, nelem);
}

// The same kernel with the library's argument carriers (round 3, session 3:
// is the harness/bench gap the kernel-argument size?): Slots<16> as
// dlsim_wreduce passes n <= 16, and DevSlots (pointers and weights read from a
// device buffer, uploaded once per slot set).
template <class Op, int NF, int G, int VPT, int NT, int NTS, bool WM = false>
void launch_ts16(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int) {
  Slots<16> s16;
  memset(&s16, 0, sizeof(s16));
  for (int i = 0; i < n && i < 16; ++i) {
    s16.p[i] = s.p[i];
    s16.w[i] = s.w[i];
  }
  const size_t grid = nvec / ((size_t)kBlock * VPT) + 1;
  hipLaunchKernelGGL((k_wreduce_tiles<Op, Slots<16>, NF, G, VPT, NT, NTS, WM>), dim3((unsigned)grid), dim3(kBlock), 0,
                     st, s16, n, out, nvec, nelem);
}
template <class Op, int NF, int G, int VPT, int NT, int NTS, bool WM = false>
void launch_tsdev(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int) {
  static std::map<const void*, void*> dev;  // slot set -> its device copy (pointers, then weights)
  void*& d = dev[&s];
  if (!d) {
    std::vector<char> h(128 * sizeof(void*) + 128 * sizeof(float));
    memcpy(h.data(), s.p, 128 * sizeof(void*));
    memcpy(h.data() + 128 * sizeof(void*), s.w, 128 * sizeof(float));
    CK(hipMalloc(&d, h.size()));
    CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  }
  DevSlots<float> ds{static_cast<const void* const*>(d),
                     reinterpret_cast<const float*>(static_cast<char*>(d) + 128 * sizeof(void*)), 1.0f};
  const size_t grid = nvec / ((size_t)kBlock * VPT) + 1;
  hipLaunchKernelGGL((k_wreduce_tiles<Op, DevSlots<float>, NF, G, VPT, NT, NTS, WM>), dim3((unsigned)grid),
                     dim3(kBlock), 0, st, ds, n, out, nvec, nelem);
}

// LDS-DMA body over full tiles; ragged end by the tiled kernel's last block
// (only exact for inputs whose nvec is a multiple of the tile: the harness
// flags any mismatch through `same`).
template <class Op, int NF, int VPT, int AUX>
void launch_l(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int gm) {
  const size_t tile = (size_t)kBlock * VPT;
  const size_t full = nvec / tile;
  size_t grid = std::max<size_t>(1, full);
  if (gm > 0) grid = std::min<size_t>(grid, (size_t)gm * 256);
  hipLaunchKernelGGL((k_wreduce_lds<Op, NF, VPT, AUX>), dim3((unsigned)grid), dim3(kBlock), 0, st, s, out, full);
}

// Representative shapes (the full round-1 sweep is in profiles/r01_tune_*):
// the shipped fp32 shape (wave map + sc1), the block map, nt stores, buffer
// nt loads and the LDS-DMA experiment.
template <class Op, int NF, int VPT, int BLOCK>
void launch_b(const Slots<128>& s, int n, void* out, size_t nvec, size_t, hipStream_t st, int) {
  const size_t full = nvec / ((size_t)BLOCK * VPT);
  hipLaunchKernelGGL((k_tiles_block<Op, NF, VPT, BLOCK>), dim3((unsigned)(full + 1)), dim3(BLOCK), 0, st, s, n,
                     out, nvec);
}

template <class Op, int NF, int VPT>
void launch_x(const Slots<128>& s, int n, void* out, size_t nvec, size_t, hipStream_t st, int) {
  const size_t full = nvec / ((size_t)kBlock * VPT);
  const size_t per = (full + 7) / 8;
  hipLaunchKernelGGL((k_tiles_xcd<Op, NF, VPT>), dim3((unsigned)(8 * per + 1)), dim3(kBlock), 0, st, s, n, out,
                     nvec, per);
}

template <class Op, int NF, int VPT, int C>
void launch_xc(const Slots<128>& s, int n, void* out, size_t nvec, size_t, hipStream_t st, int) {
  const size_t full = nvec / ((size_t)kBlock * VPT);
  const size_t super = 8 * (size_t)C;
  const size_t grid = (full + super - 1) / super * super + 1;
  hipLaunchKernelGGL((k_tiles_xcdc<Op, NF, VPT, C>), dim3((unsigned)grid), dim3(kBlock), 0, st, s, n, out, nvec);
}

// Memory-ceiling probe: the shipped fp32 access pattern (wave map, nt
// loads, sc1 stores, same tiles) with the arithmetic replaced by a bitwise
// XOR of the inputs. Its time is what the HBM allows for exactly this
// read/write mix; the exact reduce is compared against it.
using XorProbeF32 = XorProbe<4>;  // wreduce_kernels.hpp

template <class Op, int NF>
void launch_probe(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int) {
  if constexpr (Op::kBytes == 4) {
    const size_t full = nvec / ((size_t)kBlock * 4);
    hipLaunchKernelGGL((k_wreduce_tiles<XorProbeF32, Slots<128>, NF, 8, 4, 1, 16, true>), dim3((unsigned)(full + 1)),
                       dim3(kBlock), 0, st, s, n, out, nvec, nelem);
  }
}

// Contiguous persistent: gm*256 blocks, block b sweeps tiles
// [b*T/B, (b+1)*T/B) in order (wave map), so each wave streams long
// contiguous runs of every input instead of one 4 KiB piece per block.
template <class Op, int NF>
__global__ __launch_bounds__(kBlock) void k_tiles_contig(const Slots<128> s, int n, void* __restrict__ out,
                                                         size_t nvec, size_t nelem) {
  constexpr size_t kTile = (size_t)kBlock * 4;
  const size_t full = nvec / kTile;
  const OutRef o = make_out<16>(out, nvec);
  const size_t B = gridDim.x;
  if (blockIdx.x == 0) {
    if (full * kTile < nvec)
      reduce_tile<Op, Slots<128>, NF, 8, 4, 1, true, 16>(s, n, o, full * kTile + threadIdx.x, nvec);
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < nelem) fold_scalar<Op, Slots<128>>(s, n, out, j);
  }
  const size_t t0 = full * blockIdx.x / B, t1 = full * (blockIdx.x + 1) / B;
  const size_t lo = (threadIdx.x >> 6) * 64 * 4 + (threadIdx.x & 63);
  for (size_t t = t0; t < t1; ++t)
    reduce_tile<Op, Slots<128>, NF, 8, 4, 1, false, 16, 64>(s, n, o, t * kTile + lo, nvec);
}

template <class Op, int NF>
void launch_contig(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int gm) {
  hipLaunchKernelGGL((k_tiles_contig<Op, NF>), dim3((unsigned)(gm * 256)), dim3(kBlock), 0, st, s, n, out, nvec,
                     nelem);
}

// Two tile sizes in one grid: the first ~gm percent of the vectors in big
// tiles (VB vectors per lane), the rest in small tiles (VSM) dispatched last,
// so the blocks still running at the end of the launch are short (a finer
// tail). Wave map + sc1 stores as the shipped fp32 shape; block 0 takes the
// ragged end.
template <class Op, int NF, int VB, int VSM>
__global__ __launch_bounds__(kBlock) void k_tiles_split(const Slots<128> s, int n, void* __restrict__ out,
                                                        size_t nvec, size_t nelem, size_t big_tiles) {
  constexpr size_t kBig = (size_t)kBlock * VB, kSm = (size_t)kBlock * VSM;
  const OutRef o = make_out<16>(out, nvec);
  const size_t base = big_tiles * kBig;
  const size_t small_full = (nvec - base) / kSm;
  if (blockIdx.x == 0) {
    if (base + small_full * kSm < nvec)
      reduce_tile<Op, Slots<128>, NF, 8, VSM, 1, true, 16>(s, n, o, base + small_full * kSm + threadIdx.x,
                                                         nvec);
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < nelem) fold_scalar<Op, Slots<128>>(s, n, out, j);
    return;
  }
  const size_t b = blockIdx.x - 1;
  if (b < big_tiles) {
    const size_t lo = (threadIdx.x >> 6) * 64 * VB + (threadIdx.x & 63);
    reduce_tile<Op, Slots<128>, NF, 8, VB, 1, false, 16, 64>(s, n, o, b * kBig + lo, nvec);
  } else {
    const size_t lo = (threadIdx.x >> 6) * 64 * VSM + (threadIdx.x & 63);
    reduce_tile<Op, Slots<128>, NF, 8, VSM, 1, false, 16, 64>(s, n, o, base + (b - big_tiles) * kSm + lo,
                                                            nvec);
  }
}

template <class Op, int NF, int VB, int VSM>
void launch_split(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int pct) {
  const size_t kBig = (size_t)kBlock * VB, kSm = (size_t)kBlock * VSM;
  const size_t big = (size_t)((double)nvec * pct / 100.0) / kBig;
  const size_t small_full = (nvec - big * kBig) / kSm;
  hipLaunchKernelGGL((k_tiles_split<Op, NF, VB, VSM>), dim3((unsigned)(1 + big + small_full)), dim3(kBlock), 0,
                     st, s, n, out, nvec, nelem, big);
}

template <int NF, int VPT>
void launch_rdonly(const Slots<128>& s, int, void* out, size_t nvec, size_t, hipStream_t st, int) {
  hipLaunchKernelGGL((k_probe_rdonly<NF, VPT>), dim3((unsigned)(nvec / ((size_t)kBlock * VPT))), dim3(kBlock), 0, st,
                     s, out, nvec);
}
template <int VPT, int STP = 16>
void launch_wronly(const Slots<128>&, int, void* out, size_t nvec, size_t, hipStream_t st, int) {
  hipLaunchKernelGGL((k_probe_wronly<VPT, STP>), dim3((unsigned)(nvec / ((size_t)kBlock * VPT))), dim3(kBlock), 0, st,
                     out, nvec);
}
// gm = blocks per CU of the persistent ring grid (256 CUs)
template <class Op, int NF, int ST, int AUX, int WPB, int STP = 16>
void launch_ring(const Slots<128>& s, int, void* out, size_t nvec, size_t, hipStream_t st, int gm) {
  hipLaunchKernelGGL((k_wreduce_ldsring<Op, NF, ST, AUX, WPB, STP>), dim3((unsigned)(gm * 256)), dim3(64 * WPB), 0, st,
                     s, out, nvec);
}

// Round 5: small slices. A one-tile-per-block grid at
// 1.4 M elements has every block resident at once: all loads issue at the
// start and all stores at the end, read and write phases apart. The
// pipelined grid keeps gm*256 blocks; block b takes tiles b-1, b-1+W, ...
// (W = blocks - 1; block 0 the ragged end) and issues the loads of its next
// tile before it folds and stores the current one (two register buffers),
// so stores overlap loads inside every block. Same fold order: bit-exact.
template <class Op, int NF, int VPT, int VS>
__device__ __forceinline__ void pipe_load(const Slots<128>& s, size_t v0, size_t nvec, u32x4 (&r)[NF][VPT]) {
#pragma unroll
  for (int i = 0; i < NF; ++i) load_tile<Op, VPT, 1, false, VS>(s.ptr(i), v0, nvec, r[i]);
}
template <class Op, int NF, int VPT, int VS, int STP = 16>
__device__ __forceinline__ void pipe_fold_store(const Slots<128>& s, const OutRef& o, size_t v0,
                                                const u32x4 (&r)[NF][VPT]) {
  acc_t<Op> a[VPT][Op::E];
  init_tile<Op, VPT>(a, r[0], false);
#pragma unroll
  for (int i = 0; i < NF; ++i) fold_tile<Op, VPT>(a, s.wt(i), r[i]);
#pragma unroll
  for (int v = 0; v < VPT; ++v) store_vec<STP>(o, v0 + static_cast<size_t>(v) * VS, pack<Op>(a[v], s.divisor()));
}
template <class Op, int NF, int VPT, bool WM, int STP = 16>
__global__ __launch_bounds__(kBlock) void k_tiles_pipe(const Slots<128> s, int n, void* __restrict__ out,
                                                       size_t nvec, size_t nelem) {
  constexpr size_t kTile = (size_t)kBlock * VPT;
  constexpr int VS = WM ? 64 : kBlock;
  const size_t full = nvec / kTile;
  const OutRef o = make_out<STP>(out, nvec);
  if (blockIdx.x == 0) {
    if (full * kTile < nvec)
      reduce_tile<Op, Slots<128>, NF, 8, VPT, 1, true, STP>(s, n, o, full * kTile + threadIdx.x, nvec);
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < nelem) fold_scalar<Op, Slots<128>>(s, n, out, j);
    return;
  }
  const size_t W = gridDim.x - 1;
  const size_t lo = WM ? (threadIdx.x >> 6) * 64 * VPT + (threadIdx.x & 63) : threadIdx.x;
  size_t t = blockIdx.x - 1;
  if (t >= full) return;
  u32x4 ra[NF][VPT], rb[NF][VPT];
  pipe_load<Op, NF, VPT, VS>(s, t * kTile + lo, nvec, ra);
  while (true) {
    size_t t2 = t + W;
    if (t2 < full) pipe_load<Op, NF, VPT, VS>(s, t2 * kTile + lo, nvec, rb);
    pipe_fold_store<Op, NF, VPT, VS, STP>(s, o, t * kTile + lo, ra);
    if (t2 >= full) break;
    t = t2;
    t2 = t + W;
    if (t2 < full) pipe_load<Op, NF, VPT, VS>(s, t2 * kTile + lo, nvec, ra);
    pipe_fold_store<Op, NF, VPT, VS, STP>(s, o, t * kTile + lo, rb);
    if (t2 >= full) break;
    t = t2;
  }
}
// gm > 0: 1 + gm*256 blocks; gm < 0: 1 + ceil(full / -gm) blocks (-gm tiles per block)
template <class Op, int NF, int VPT, bool WM, int STP = 16>
void launch_pipe(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int gm) {
  const size_t full = nvec / ((size_t)kBlock * VPT);
  size_t workers = gm > 0 ? (size_t)gm * 256 : (full + (size_t)(-gm) - 1) / (size_t)(-gm);
  workers = std::max<size_t>(1, std::min(workers, full));
  hipLaunchKernelGGL((k_tiles_pipe<Op, NF, VPT, WM, STP>), dim3((unsigned)(workers + 1)), dim3(kBlock), 0, st, s, n, out,
                     nvec, nelem);
}
// Balanced one-shot grid (round 5): B = 256*k blocks, block b owns the
// vectors [b*nvec/B, (b+1)*nvec/B) (boundaries rounded down to 8 vectors,
// 128 B), every lane loads its up to VPT vectors of every input at once
// (masked), folds and stores: each CU gets the same bytes, where a grid of
// whole tiles leaves some CUs one tile more than others (at 1.4 M fp32 the
// VPT 2 grid has 2.67 tiles per CU, the VPT 4 grid 1.33). Block 0 also folds
// the scalar tail. LDS > 0: dynamic LDS that caps the blocks per CU.
template <class Op, int NF, int VPT>
__global__ __launch_bounds__(kBlock) void k_bal(const Slots<128> s, int n, void* __restrict__ out, size_t nvec,
                                                size_t nelem) {
  const size_t B = gridDim.x, b = blockIdx.x;
  const size_t r0 = (b * nvec / B) & ~(size_t)7;
  const size_t r1 = b + 1 == B ? nvec : ((b + 1) * nvec / B) & ~(size_t)7;
  const OutRef o = make_out<16>(out, nvec);
  reduce_tile<Op, Slots<128>, NF, 8, VPT, 1, true, 16>(s, n, o, r0 + threadIdx.x, r1);
  if (b == 0) {
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < nelem) fold_scalar<Op, Slots<128>>(s, n, out, j);
  }
}
template <class Op, int NF, int V>
void bal_go(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, size_t B, size_t lds) {
  hipLaunchKernelGGL((k_bal<Op, NF, V>), dim3((unsigned)B), dim3(kBlock), lds, st, s, n, out, nvec, nelem);
}
template <class Op, int NF, int LDSK>
void launch_bal(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int gm) {
  const size_t B = (size_t)gm * 256;
  const size_t per = (nvec + B - 1) / B + 8;  // + the 128-B rounding of the boundaries
  const size_t vpt = (per + kBlock - 1) / kBlock;
  const size_t lds = LDSK ? (160 * 1024) / LDSK - 512 : 0;
  switch (vpt) {
    case 1: bal_go<Op, NF, 1>(s, n, out, nvec, nelem, st, B, lds); break;
    case 2: bal_go<Op, NF, 2>(s, n, out, nvec, nelem, st, B, lds); break;
    case 3: bal_go<Op, NF, 3>(s, n, out, nvec, nelem, st, B, lds); break;
    case 4: bal_go<Op, NF, 4>(s, n, out, nvec, nelem, st, B, lds); break;
    case 5: bal_go<Op, NF, 5>(s, n, out, nvec, nelem, st, B, lds); break;
    case 6: bal_go<Op, NF, 6>(s, n, out, nvec, nelem, st, B, lds); break;
    case 7: bal_go<Op, NF, 7>(s, n, out, nvec, nelem, st, B, lds); break;
    case 8: bal_go<Op, NF, 8>(s, n, out, nvec, nelem, st, B, lds); break;
    default: fprintf(stderr, "k_bal: %zu vectors per lane\n", vpt); exit(1);
  }
}

// Round 5: deferred stores. With the outputs beyond the Infinity Cache the
// reduce runs at a copy's rate (6.3 TB/s) while its eight read streams alone
// reach 0.84 of peak: the read/write turnaround costs ~8 %. Here every block
// folds R tiles (256 vectors each) and keeps the R packed results in
// registers, then stores them all at the end: with one residency wave of
// blocks (R chosen so the grid fits the chip) the whole chip reads first and
// writes last, so HBM turns around far less often. U tiles' loads are issued
// together. Same fold order as reduce_tile: bit-exact.
// Grid-wide rendezvous between the read phase and the stores (round 5
// experiment): every block adds 1 to a counter that only grows (the launch's
// target is epoch * grid) and waits, bounded by a ~1 ms timeout after which it
// stores anyway -- no result depends on it; it only lines the phases up.
__device__ __forceinline__ void grid_rendezvous(unsigned* counter, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(counter, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (wall_clock64() - t0 > 100000) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}
template <class Op, int NF, int R, int U, int STP, int BS, bool BAR = false>
__device__ __forceinline__ void defer_body(const Slots<128>& s, const OutRef& o, size_t base,
                                           unsigned* counter = nullptr, unsigned target = 0) {
  u32x4 res[R];
#pragma unroll
  for (int r0 = 0; r0 < R; r0 += U) {
    u32x4 x[NF][U];
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int u = 0; u < U; ++u) x[i][u] = ld16<1>(s.p[i], base + static_cast<size_t>(r0 + u) * BS);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      acc_t<Op> a[1][Op::E];
      u32x4 r0v[1] = {x[0][u]};
      init_tile<Op, 1>(a, r0v, false);
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        u32x4 ri[1] = {x[i][u]};
        fold_tile<Op, 1>(a, s.w[i], ri);
      }
      res[r0 + u] = pack<Op>(a[0], s.div);
    }
    // keep the next group's loads behind this fold: hoisting every group's
    // loads to the top would need NF * R vector registers and spill
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (BAR) grid_rendezvous(counter, target);
#pragma unroll
  for (int r = 0; r < R; ++r) store_vec<STP>(o, base + static_cast<size_t>(r) * BS, res[r]);
}
// BS threads per block; LDS > 0: that much dynamic LDS per block pins one
// block per CU (the grid is sized to about one block per CU).
template <class Op, int NF, int R, int U, int STP, int MINB = 2, int BS = kBlock>
__global__ __launch_bounds__(BS, MINB) void k_defer(const Slots<128> s, int n, void* __restrict__ out, size_t nvec,
                                                    size_t nelem) {
  const size_t base = static_cast<size_t>(blockIdx.x) * BS * R + threadIdx.x;
  const OutRef o = make_out<STP>(out, nvec);
  if (static_cast<size_t>(blockIdx.x + 1) * BS * R <= nvec) {
    defer_body<Op, NF, R, U, STP, BS>(s, o, base);
  } else {  // the last, partial block: tile by tile with bounds checks
    for (int r = 0; r < R; ++r)
      reduce_tile<Op, Slots<128>, NF, 8, 1, 1, true, STP, BS>(s, n, o, base + static_cast<size_t>(r) * BS, nvec);
  }
  if (blockIdx.x == 0 && threadIdx.x < kBlock) {
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < nelem) fold_scalar<Op, Slots<128>>(s, n, out, j);
  }
}
// k_defer with the rendezvous: every block of the grid must be resident at
// once (grid <= CUs, one block per CU by the LDS pin); the partial last block
// joins the rendezvous too.
template <class Op, int NF, int R, int U, int STP, int BS>
__global__ __launch_bounds__(BS, 1) void k_defer_bar(const Slots<128> s, int n, void* __restrict__ out, size_t nvec,
                                                     size_t nelem, unsigned* counter, unsigned target) {
  const size_t base = static_cast<size_t>(blockIdx.x) * BS * R + threadIdx.x;
  const OutRef o = make_out<STP>(out, nvec);
  if (static_cast<size_t>(blockIdx.x + 1) * BS * R <= nvec) {
    defer_body<Op, NF, R, U, STP, BS, true>(s, o, base, counter, target);
  } else {
    grid_rendezvous(counter, target);
    for (int r = 0; r < R; ++r)
      reduce_tile<Op, Slots<128>, NF, 8, 1, 1, true, STP, BS>(s, n, o, base + static_cast<size_t>(r) * BS, nvec);
  }
  if (blockIdx.x == 0 && threadIdx.x < kBlock) {
    const size_t j = nvec * Op::E + threadIdx.x;
    if (j < nelem) fold_scalar<Op, Slots<128>>(s, n, out, j);
  }
}
template <class Op, int NF, int R, int U, int STP, int BS, int LDSKB>
void launch_defer_bar(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int) {
  static unsigned* counter = nullptr;
  static unsigned epoch = 0;
  if (!counter) {
    CK(hipMalloc(&counter, 256));
    CK(hipMemset(counter, 0, 256));
  }
  const size_t per = static_cast<size_t>(BS) * R;
  const unsigned grid = static_cast<unsigned>((nvec + per - 1) / per);
  ++epoch;
  hipLaunchKernelGGL((k_defer_bar<Op, NF, R, U, STP, BS>), dim3(grid), dim3(BS), (size_t)LDSKB * 1024, st, s, n, out,
                     nvec, nelem, counter, epoch * grid);
}

template <class Op, int NF, int R, int U, int STP, int MINB = 2, int BS = kBlock, int LDSKB = 0>
void launch_defer(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int) {
  const size_t per = static_cast<size_t>(BS) * R;
  hipLaunchKernelGGL((k_defer<Op, NF, R, U, STP, MINB, BS>), dim3((unsigned)((nvec + per - 1) / per)), dim3(BS),
                     (size_t)LDSKB * 1024, st, s, n, out, nvec, nelem);
}

// The library's deferred kernel (wreduce_kernels.hpp k_wreduce_defer, runtime
// R) on the harness's buffers: R rows per block, LDSKB of dynamic LDS.
template <class Op, int NF, int R, int LDSKB>
void launch_libdefer(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int) {
  const size_t per = static_cast<size_t>(kDeferBlock) * R;
  hipLaunchKernelGGL((dlsim::k_wreduce_defer<Op, Slots<128>, NF, 8, 32, 2, 2>), dim3((unsigned)((nvec + per - 1) / per)),
                     dim3(kDeferBlock), (size_t)LDSKB * 1024, st, s, n, R, out, nvec, nelem);
}

template <class Op, int NF, int R>
void launch_libdefer_c(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int) {
  const size_t per = static_cast<size_t>(kDeferBlock) * R;
  hipLaunchKernelGGL((dlsim::k_wreduce_defer<Op, Slots<128>, NF, 8, 32, 2, 2, R>),
                     dim3((unsigned)((nvec + per - 1) / per)), dim3(kDeferBlock), 0, st, s, n, R, out, nvec, nelem);
}

// k_defer with R chosen from the size: the smallest R of the list with
// ceil(nvec / (BS * R)) <= 256 blocks (one per CU), or the largest R (then
// more than one block per CU).
template <class Op, int NF, int U, int BS, int LDSKB>
void launch_defer_auto(const Slots<128>& s, int n, void* out, size_t nvec, size_t nelem, hipStream_t st, int gm) {
  const size_t cus = gm > 0 ? (size_t)gm : 256;
  const size_t need = (nvec + cus * BS - 1) / (cus * BS);
#define DEFER_R(RR) \
  if (need <= RR) return launch_defer<Op, NF, RR, (RR % U == 0 ? U : 1), 2, 1, BS, LDSKB>(s, n, out, nvec, nelem, st, 0);
  DEFER_R(1) DEFER_R(2) DEFER_R(4) DEFER_R(6) DEFER_R(8) DEFER_R(12) DEFER_R(16) DEFER_R(22) DEFER_R(28)
#undef DEFER_R
  launch_defer<Op, NF, 32, U, 2, 1, BS, LDSKB>(s, n, out, nvec, nelem, st, 0);
}

// Round 5: the shipped shapes with sc1 (write-through) stores against
// non-temporal buffer stores (nt = 2), for fixed fan-in 2 / 8 and the grouped
// kernel, fp32 and bf16 (DLSIM_TUNE_NTSWEEP; run with DLSIM_TUNE_OUT_SETS so
// the outputs do not stay in the Infinity Cache).
template <class Op>
void add_ntsweep(std::vector<Variant>& vs, int n) {
  if constexpr (Op::kBytes >= 4) {
    if (n == 8) {
      vs.push_back({"NF8_V2_sc1_blk", launch_ts<Op, 8, 8, 2, 1, 16, false>, 0});
      vs.push_back({"NF8_V2_bnt_blk", launch_ts<Op, 8, 8, 2, 1, 2, false>, 0});
      vs.push_back({"NF8_V4_sc1_blk", launch_ts<Op, 8, 8, 4, 1, 16, false>, 0});
      vs.push_back({"NF8_V4_bnt_blk", launch_ts<Op, 8, 8, 4, 1, 2, false>, 0});
      vs.push_back({"NF8_V4_sc1_wave", launch_ts<Op, 8, 8, 4, 1, 16, true>, 0});
      vs.push_back({"NF8_V4_bnt_wave", launch_ts<Op, 8, 8, 4, 1, 2, true>, 0});
      vs.push_back({"NF8_V4_nt_wave", launch_ts<Op, 8, 8, 4, 1, kStNT, true>, 0});
    } else if (n == 2) {
      vs.push_back({"NF2_V2_sc1_blk", launch_ts<Op, 2, 8, 2, 1, 16, false>, 0});
      vs.push_back({"NF2_V2_bnt_blk", launch_ts<Op, 2, 8, 2, 1, 2, false>, 0});
      vs.push_back({"NF2_V4_sc1_wave", launch_ts<Op, 2, 8, 4, 1, 16, true>, 0});
      vs.push_back({"NF2_V4_bnt_wave", launch_ts<Op, 2, 8, 4, 1, 2, true>, 0});
    } else {
      vs.push_back({"T_G8_V1_sc1_wave", launch_ts<Op, 0, 8, 1, 1, 16, true>, 0});
      vs.push_back({"T_G8_V1_bnt_wave", launch_ts<Op, 0, 8, 1, 1, 2, true>, 0});
      vs.push_back({"T_G8_V4_sc1_blk", launch_ts<Op, 0, 8, 4, 1, 16, false>, 0});
      vs.push_back({"T_G8_V4_bnt_blk", launch_ts<Op, 0, 8, 4, 1, 2, false>, 0});
    }
  } else {
    if (n == 2) {
      vs.push_back({"NF2_V1_sc1_wave", launch_ts<Op, 2, 4, 1, 1, 16, true>, 0});
      vs.push_back({"NF2_V1_bnt_wave", launch_ts<Op, 2, 4, 1, 1, 2, true>, 0});
      vs.push_back({"NF2_V4_nt_blk", launch_ts<Op, 2, 4, 4, 1, kStNT, false>, 0});
      vs.push_back({"NF2_V4_bnt_blk", launch_ts<Op, 2, 4, 4, 1, 2, false>, 0});
      vs.push_back({"NF2_V4_sc1_blk", launch_ts<Op, 2, 4, 4, 1, 16, false>, 0});
    } else {
      vs.push_back({"T_G4_V1_sc1_wave", launch_ts<Op, 0, 4, 1, 1, 16, true>, 0});
      vs.push_back({"T_G4_V1_bnt_wave", launch_ts<Op, 0, 4, 1, 1, 2, true>, 0});
      vs.push_back({"T_G4_V4_nt_blk", launch_ts<Op, 0, 4, 4, 1, kStNT, false>, 0});
    }
  }
}

template <class Op, int NF>
void add_small(std::vector<Variant>& vs, int n) {
  if constexpr (!std::is_same<Op, F32Exact>::value) return;
  else {
  if (n != NF) return;
  const std::string p = "NF" + std::to_string(NF);
  vs.push_back({p + "_V2_sc1_blk", launch_ts<Op, NF, 8, 2, 1, 16, false>, 0});  // shipped below 2 M fp32
  vs.push_back({p + "_V1_sc1_blk", launch_ts<Op, NF, 8, 1, 1, 16, false>, 0});
  vs.push_back({p + "_V4_sc1_blk", launch_ts<Op, NF, 8, 4, 1, 16, false>, 0});
  vs.push_back({p + "_xorprobe_V4w", launch_probe<Op, NF>, 0});
  vs.push_back({p + "_bal_k1", launch_bal<Op, NF, 0>, 1});
  vs.push_back({p + "_bal_k2", launch_bal<Op, NF, 0>, 2});
  vs.push_back({p + "_bal_k3", launch_bal<Op, NF, 0>, 3});
  vs.push_back({p + "_bal_k4", launch_bal<Op, NF, 0>, 4});
  vs.push_back({p + "_bal_k1_lds1", launch_bal<Op, NF, 1>, 1});
  vs.push_back({p + "_bal_k2_lds2", launch_bal<Op, NF, 2>, 2});
  vs.push_back({p + "_bal_k3_lds3", launch_bal<Op, NF, 3>, 3});
  if (getenv("DLSIM_TUNE_SMALL_BAL")) return;
  vs.push_back({p + "_pipe_V1_blk_g1", launch_pipe<Op, NF, 1, false>, 1});
  vs.push_back({p + "_pipe_V1_blk_g2", launch_pipe<Op, NF, 1, false>, 2});
  vs.push_back({p + "_pipe_V1_blk_g3", launch_pipe<Op, NF, 1, false>, 3});
  vs.push_back({p + "_pipe_V1_blk_t2", launch_pipe<Op, NF, 1, false>, -2});
  vs.push_back({p + "_pipe_V1_blk_t3", launch_pipe<Op, NF, 1, false>, -3});
  vs.push_back({p + "_pipe_V1_wave_g2", launch_pipe<Op, NF, 1, true>, 2});
  vs.push_back({p + "_pipe_V2_blk_g1", launch_pipe<Op, NF, 2, false>, 1});
  vs.push_back({p + "_pipe_V2_blk_t2", launch_pipe<Op, NF, 2, false>, -2});
  vs.push_back({p + "_pipe_V2_wave_g1", launch_pipe<Op, NF, 2, true>, 1});
  vs.push_back({p + "_pipe_V2_wave_t2", launch_pipe<Op, NF, 2, true>, -2});
  }
}

// Round 5: deferred stores (k_defer), outputs beyond the MALL.
template <class Op, int NF>
void add_defer(std::vector<Variant>& vs, int n) {
  if constexpr (!std::is_same<Op, F32Exact>::value) return;
  else {
  if (n != NF) return;
  const std::string p = "NF" + std::to_string(NF);
  vs.push_back({p + "_V4_sc1_wave", launch_ts<Op, NF, 8, 4, 1, 16, true>, 0});
    {
      vs.push_back({p + "_V4_bnt_wave", launch_ts<Op, NF, 8, 4, 1, 2, true>, 0});
      vs.push_back({p + "_V4_bnt_blk", launch_ts<Op, NF, 8, 4, 1, 2, false>, 0});
      vs.push_back({p + "_V2_bnt_blk", launch_ts<Op, NF, 8, 2, 1, 2, false>, 0});
    }
    vs.push_back({p + "_dauto_B512_U2_lds", launch_defer_auto<Op, NF, 2, 512, 96>, 0});
    if constexpr (NF == 8) {
      // the grid rendezvous before the stores: 167-172 us (profiles/r05_defer/r05ak/)
      if (getenv("DLSIM_TUNE_RENDEZVOUS"))
        vs.push_back({p + "_dbar_R22_B512_U2_lds", launch_defer_bar<Op, NF, 22, 2, 2, 512, 96>, 0});
      vs.push_back({p + "_d_R22_B512_U2_lds", launch_defer<Op, NF, 22, 2, 2, 1, 512, 96>, 0});
      vs.push_back({p + "_lib_R22", launch_libdefer<Op, NF, 22, 0>, 0});
      vs.push_back({p + "_lib_R22_lds", launch_libdefer<Op, NF, 22, 96>, 0});
      vs.push_back({p + "_libc_R22", launch_libdefer_c<Op, NF, 22>, 0});
      vs.push_back({p + "_d_R24_B512_U2_lds", launch_defer<Op, NF, 24, 2, 2, 1, 512, 96>, 0});
      vs.push_back({p + "_d_R24_B512_U4_lds", launch_defer<Op, NF, 24, 4, 2, 1, 512, 96>, 0});
      vs.push_back({p + "_d_R24_B512_U3_lds", launch_defer<Op, NF, 24, 3, 2, 1, 512, 96>, 0});
      vs.push_back({p + "_d_R12_B1024_U2_lds", launch_defer<Op, NF, 12, 2, 2, 1, 1024, 96>, 0});
    }
    vs.push_back({p + "_dauto_B512_U2", launch_defer_auto<Op, NF, 2, 512, 0>, 0});
    vs.push_back({p + "_dauto_B512_U1_lds", launch_defer_auto<Op, NF, 1, 512, 96>, 0});
    vs.push_back({p + "_dauto_B256_U2_lds", launch_defer_auto<Op, NF, 2, 256, 96>, 0});
    vs.push_back({p + "_dauto_B1024_U2_lds", launch_defer_auto<Op, NF, 2, 1024, 96>, 0});
    vs.push_back({p + "_dauto_B512_U2_lds_c2", launch_defer_auto<Op, NF, 2, 512, 60>, 512});
  }
}

// Round 3: the shipped large shape, the memory-only
// probe, read-only and write-only probes of the same tiles, and pipelined
// LDS-DMA rings (nt and default policy) at 1-2 blocks per CU.
template <class Op, int NF>
void add_r03(std::vector<Variant>& vs, int n) {
  if constexpr (!std::is_same<Op, F32Exact>::value) return;
  else {
  if (n != NF) return;
  const std::string p = "NF" + std::to_string(NF);
  const double rd = (double)NF / (NF + 1), wr = 1.0 / (NF + 1);
  vs.push_back({p + "_V4_sc1_wave", launch_ts<Op, NF, 8, 4, 1, 16, true>, 0});
  if (getenv("DLSIM_TUNE_ARGS")) {  // kernel-argument carriers only
    vs.push_back({p + "_V4_sc1_wave_S16", launch_ts16<Op, NF, 8, 4, 1, 16, true>, 0});
    vs.push_back({p + "_V4_sc1_wave_dev", launch_tsdev<Op, NF, 8, 4, 1, 16, true>, 0});
    vs.push_back({p + "_V4_sc1_wave_b", launch_ts<Op, NF, 8, 4, 1, 16, true>, 0});
    return;
  }
  if (getenv("DLSIM_TUNE_DEFER")) return add_defer<Op, NF>(vs, n);
  if (getenv("DLSIM_TUNE_HONEST")) {  // round 5: shapes with nt buffer stores, outputs beyond the MALL
    vs.push_back({p + "_V4_bnt_wave", launch_ts<Op, NF, 8, 4, 1, 2, true>, 0});
    vs.push_back({p + "_V8_bnt_wave", launch_ts<Op, NF, 8, 8, 1, 2, true>, 0});
    vs.push_back({p + "_V2_bnt_wave", launch_ts<Op, NF, 8, 2, 1, 2, true>, 0});
    vs.push_back({p + "_V1_bnt_wave", launch_ts<Op, NF, 8, 1, 1, 2, true>, 0});
    vs.push_back({p + "_V4_bnt_g2", launch_ts<Op, NF, 8, 4, 1, 2, true>, 2});
    vs.push_back({p + "_V4_bnt_g4", launch_ts<Op, NF, 8, 4, 1, 2, true>, 4});
    vs.push_back({p + "_pipe_V2w_bnt_g1", launch_pipe<Op, NF, 2, true, 2>, 1});
    vs.push_back({p + "_pipe_V4w_bnt_g1", launch_pipe<Op, NF, 4, true, 2>, 1});
    vs.push_back({p + "_pipe_V2w_bnt_g2", launch_pipe<Op, NF, 2, true, 2>, 2});
    vs.push_back({p + "_ring_S3_nt_W4_g1_bnt", launch_ring<Op, NF, 3, 2, 4, 2>, 1});
    vs.push_back({p + "_ring_S4_nt_W4_g1_bnt", launch_ring<Op, NF, 4, 2, 4, 2>, 1});
    vs.push_back({p + "_rdonly_V4w", launch_rdonly<NF, 4>, 0, (double)NF / (NF + 1)});
    vs.push_back({p + "_wronly_V4w_bnt", launch_wronly<4, 2>, 0, 1.0 / (NF + 1)});
    vs.push_back({p + "_wronly_V4w_sc1", launch_wronly<4, 16>, 0, 1.0 / (NF + 1)});
    return;
  }
  if (getenv("DLSIM_TUNE_STPOL")) {  // every buffer-store cache policy (round 5: outputs beyond the MALL)
    vs.push_back({p + "_V4_sc1_wave", launch_ts<Op, NF, 8, 4, 1, 16, true>, 0});
    vs.push_back({p + "_V4_nt_wave", launch_ts<Op, NF, 8, 4, 1, kStNT, true>, 0});
    vs.push_back({p + "_V4_b0_wave", launch_ts<Op, NF, 8, 4, 1, 0, true>, 0});
    vs.push_back({p + "_V4_bsc0_wave", launch_ts<Op, NF, 8, 4, 1, 1, true>, 0});
    vs.push_back({p + "_V4_bnt_wave", launch_ts<Op, NF, 8, 4, 1, 2, true>, 0});
    vs.push_back({p + "_V4_bsc0nt_wave", launch_ts<Op, NF, 8, 4, 1, 3, true>, 0});
    vs.push_back({p + "_V4_bsc01_wave", launch_ts<Op, NF, 8, 4, 1, 17, true>, 0});
    vs.push_back({p + "_V4_bsc1nt_wave", launch_ts<Op, NF, 8, 4, 1, 18, true>, 0});
    vs.push_back({p + "_V4_bsc01nt_wave", launch_ts<Op, NF, 8, 4, 1, 19, true>, 0});
    vs.push_back({p + "_V4_sc1_ldb_nt", launch_ts<Op, NF, 8, 4, kLdBuffer + 2, 16, true>, 0});
    vs.push_back({p + "_V4_nt_ldb_nt", launch_ts<Op, NF, 8, 4, kLdBuffer + 2, kStNT, true>, 0});
    return;
  }
  if (getenv("DLSIM_TUNE_STORES")) {  // store policies and shapes on contiguous blocks (round 4)
    vs.push_back({p + "_V4_nt_wave", launch_ts<Op, NF, 8, 4, 1, kStNT, true>, 0});
    vs.push_back({p + "_V4_plain_wave", launch_ts<Op, NF, 8, 4, 1, kStPlain, true>, 0});
    vs.push_back({p + "_V4_sc1_blk", launch_ts<Op, NF, 8, 4, 1, 16, false>, 0});
    vs.push_back({p + "_V2_sc1_wave", launch_ts<Op, NF, 8, 2, 1, 16, true>, 0});
    vs.push_back({p + "_V8_sc1_wave", launch_ts<Op, NF, 8, 8, 1, 16, true>, 0});
    vs.push_back({p + "_xorprobe", launch_probe<Op, NF>, 0});
    return;
  }
  if (getenv("DLSIM_TUNE_TLB")) {  // tile orders against translation reach
    vs.push_back({p + "_xorprobe", launch_probe<Op, NF>, 0});
    vs.push_back({p + "_xcd_split", launch_x<Op, NF, 4>, 0});
    vs.push_back({p + "_xcdc_16", launch_xc<Op, NF, 4, 16>, 0});
    vs.push_back({p + "_xcdc_64", launch_xc<Op, NF, 4, 64>, 0});
    vs.push_back({p + "_xcdc_128", launch_xc<Op, NF, 4, 128>, 0});
    vs.push_back({p + "_xcdc_512", launch_xc<Op, NF, 4, 512>, 0});
    return;
  }
  vs.push_back({p + "_xorprobe", launch_probe<Op, NF>, 0});
  vs.push_back({p + "_rdonly_V4w", launch_rdonly<NF, 4>, 0, rd});
  vs.push_back({p + "_rdonly_V2w", launch_rdonly<NF, 2>, 0, rd});
  vs.push_back({p + "_wronly_V4w", launch_wronly<4>, 0, wr});
  vs.push_back({p + "_wronly_V1w", launch_wronly<1>, 0, wr});
  vs.push_back({p + "_ring_S3_nt_W4_g1", launch_ring<Op, NF, 3, 2, 4>, 1});
  vs.push_back({p + "_ring_S4_nt_W4_g1", launch_ring<Op, NF, 4, 2, 4>, 1});
  vs.push_back({p + "_ring_S2_nt_W4_g2", launch_ring<Op, NF, 2, 2, 4>, 2});
  vs.push_back({p + "_ring_S2_nt_W8_g1", launch_ring<Op, NF, 2, 2, 8>, 1});
  vs.push_back({p + "_ring_S4_def_W4_g1", launch_ring<Op, NF, 4, 0, 4>, 1});
  vs.push_back({p + "_ring_S3_def_W4_g1", launch_ring<Op, NF, 3, 0, 4>, 1});
  }
}

// Round 3 layout sweep (DLSIM_TUNE_LAYOUT): the shipped launch shapes of
// every size class for fan-in n (fixed kernels for n = 2 and 8, the grouped
// kernel for any n), to time one layout of the inputs and outputs.
template <class Op, int NF>
void add_fixed_shapes(std::vector<Variant>& vs, int n) {
  if (n != NF) return;
  const std::string p = "NF" + std::to_string(NF);
  if constexpr (Op::kBytes >= 4) {
    vs.push_back({p + "_V2_sc1_blk", launch_ts<Op, NF, 8, 2, 1, 16, false>, 0});
    vs.push_back({p + "_V4_sc1_blk", launch_ts<Op, NF, 8, 4, 1, 16, false>, 0});
    vs.push_back({p + "_V4_sc1_wave", launch_ts<Op, NF, 8, 4, 1, 16, true>, 0});
  } else {
    vs.push_back({p + "_V1_sc1_wave", launch_ts<Op, NF, 4, 1, 1, 16, true>, 0});
    vs.push_back({p + "_V4_nt_blk", launch_ts<Op, NF, 4, 4, 1, kStNT, false>, 0});
  }
}
template <class Op>
void add_layout(std::vector<Variant>& vs, int n) {
  add_fixed_shapes<Op, 2>(vs, n);
  add_fixed_shapes<Op, 8>(vs, n);
  if constexpr (Op::kBytes >= 4) {
    vs.push_back({"T_G8_V1_sc1_wave", launch_ts<Op, 0, 8, 1, 1, 16, true>, 0});
    vs.push_back({"T_G8_V4_sc1_blk", launch_ts<Op, 0, 8, 4, 1, 16, false>, 0});
  } else {
    vs.push_back({"T_G4_V1_sc1_wave", launch_ts<Op, 0, 4, 1, 1, 16, true>, 0});
    vs.push_back({"T_G4_V4_nt_blk", launch_ts<Op, 0, 4, 4, 1, kStNT, false>, 0});
  }
}

template <class Op, int NF>
void add_nf(std::vector<Variant>& vs, int n) {
  if (n != NF) return;
  const std::string p = "NF" + std::to_string(NF);
  vs.push_back({p + "_V4", launch_t<Op, NF, 8, 4, true>, 0});
  vs.push_back({p + "_V4_sc1", launch_ts<Op, NF, 8, 4, 1, 16>, 0});
  vs.push_back({p + "_V4_sc1_wave", launch_ts<Op, NF, 8, 4, 1, 16, true>, 0});
  vs.push_back({p + "_V4_sc1_bnt", launch_ts<Op, NF, 8, 4, kLdBuffer + 2, 16>, 0});
  vs.push_back({p + "_V2_sc1", launch_ts<Op, NF, 8, 2, 1, 16>, 0});
  vs.push_back({p + "_lds_V2_nt", launch_l<Op, NF, 2, 2>, 0});
  vs.push_back({p + "_B128_V4", launch_b<Op, NF, 4, 128>, 0});
  vs.push_back({p + "_B256_V4", launch_b<Op, NF, 4, 256>, 0});
  vs.push_back({p + "_B512_V4", launch_b<Op, NF, 4, 512>, 0});
  vs.push_back({p + "_B1024_V4", launch_b<Op, NF, 4, 1024>, 0});
  vs.push_back({p + "_B512_V2", launch_b<Op, NF, 2, 512>, 0});
  vs.push_back({p + "_B64_V4", launch_b<Op, NF, 4, 64>, 0});
  vs.push_back({p + "_V2_sc1_wave", launch_ts<Op, NF, 8, 2, 1, 16, true>, 0});
  vs.push_back({p + "_V1_sc1_wave", launch_ts<Op, NF, 8, 1, 1, 16, true>, 0});
  vs.push_back({p + "_xcd_V4", launch_x<Op, NF, 4>, 0});
  vs.push_back({p + "_xcd_V2", launch_x<Op, NF, 2>, 0});
  vs.push_back({p + "_xorprobe", launch_probe<Op, NF>, 0});
  vs.push_back({p + "_contig2", launch_contig<Op, NF>, 2});
  vs.push_back({p + "_contig3", launch_contig<Op, NF>, 3});
  vs.push_back({p + "_contig6", launch_contig<Op, NF>, 6});
  vs.push_back({p + "_split80_V1", launch_split<Op, NF, 4, 1>, 80});
  vs.push_back({p + "_split90_V1", launch_split<Op, NF, 4, 1>, 90});
  vs.push_back({p + "_split95_V1", launch_split<Op, NF, 4, 1>, 95});
  vs.push_back({p + "_split90_V2", launch_split<Op, NF, 4, 2>, 90});
  vs.push_back({p + "_split97_V1", launch_split<Op, NF, 4, 1>, 97});
  // small-launch shapes (strong-scaling slices): block map at VPT 1/2,
  // grid-stride grids of k*256 blocks, nt stores
  vs.push_back({p + "_V2_sc1_blk", launch_ts<Op, NF, 8, 2, 1, 16, false>, 0});
  vs.push_back({p + "_V1_sc1_g1", launch_ts<Op, NF, 8, 1, 1, 16, true>, 1});
  vs.push_back({p + "_V1_sc1_g2", launch_ts<Op, NF, 8, 1, 1, 16, true>, 2});
  vs.push_back({p + "_V1_sc1_g4", launch_ts<Op, NF, 8, 1, 1, 16, true>, 4});
  vs.push_back({p + "_V2_sc1_g1", launch_ts<Op, NF, 8, 2, 1, 16, true>, 1});
  vs.push_back({p + "_V2_sc1_g2", launch_ts<Op, NF, 8, 2, 1, 16, true>, 2});
  vs.push_back({p + "_V4_sc1_g1", launch_ts<Op, NF, 8, 4, 1, 16, true>, 1});
  vs.push_back({p + "_V1_nt", launch_ts<Op, NF, 8, 1, 1, kStNT, true>, 0});
  vs.push_back({p + "_V2_nt_wave", launch_ts<Op, NF, 8, 2, 1, kStNT, true>, 0});
  vs.push_back({p + "_V4_nt_wave", launch_ts<Op, NF, 8, 4, 1, kStNT, true>, 0});
  vs.push_back({p + "_V1_plain", launch_ts<Op, NF, 8, 1, 1, kStPlain, true>, 0});
  vs.push_back({p + "_V1_sc1_ldplain", launch_ts<Op, NF, 8, 1, 0, 16, true>, 0});
  // load cache-policy bits on the shipped large shape (round 2, session 2):
  // buffer loads with sc0 = 1, nt = 2, sc1 = 16 combinations
  vs.push_back({p + "_V4w_ldb_nt", launch_ts<Op, NF, 8, 4, kLdBuffer + 2, 16, true>, 0});
  vs.push_back({p + "_V4w_ldb_sc0nt", launch_ts<Op, NF, 8, 4, kLdBuffer + 3, 16, true>, 0});
  vs.push_back({p + "_V4w_ldb_sc1nt", launch_ts<Op, NF, 8, 4, kLdBuffer + 18, 16, true>, 0});
  vs.push_back({p + "_V4w_ldb_sc01nt", launch_ts<Op, NF, 8, 4, kLdBuffer + 19, 16, true>, 0});
  vs.push_back({p + "_V4w_ldb_sc1", launch_ts<Op, NF, 8, 4, kLdBuffer + 16, 16, true>, 0});
  vs.push_back({p + "_V4w_ldb_sc01", launch_ts<Op, NF, 8, 4, kLdBuffer + 17, 16, true>, 0});
  vs.push_back({p + "_V4w_ldb_plain", launch_ts<Op, NF, 8, 4, kLdBuffer + 0, 16, true>, 0});
}

template <class Op>
std::vector<Variant> variants(int n) {
  std::vector<Variant> vs = {
      {"T_G8_V2", launch_t<Op, 0, 8, 2, true>, 0},
      {"T_G8_V4", launch_t<Op, 0, 8, 4, true>, 0},
      {"T_G8_V4_sc1", launch_ts<Op, 0, 8, 4, 1, 16>, 0},
      {"T_G8_V4_sc1_wave", launch_ts<Op, 0, 8, 4, 1, 16, true>, 0},
      // grouped (runtime fan-in) shapes beyond the shipped VPT 4 (round 2)
      {"T_G8_V2_sc1_blk", launch_ts<Op, 0, 8, 2, 1, 16, false>, 0},
      {"T_G8_V2_sc1_wave", launch_ts<Op, 0, 8, 2, 1, 16, true>, 0},
      {"T_G8_V1_sc1_wave", launch_ts<Op, 0, 8, 1, 1, 16, true>, 0},
      {"T_G4_V4_sc1_wave", launch_ts<Op, 0, 4, 4, 1, 16, true>, 0},
      {"T_G4_V2_sc1_wave", launch_ts<Op, 0, 4, 2, 1, 16, true>, 0},
      {"T_G16_V2_sc1_wave", launch_ts<Op, 0, 16, 2, 1, 16, true>, 0},
      {"T_G16_V1_sc1_wave", launch_ts<Op, 0, 16, 1, 1, 16, true>, 0},
      {"T_G8_V4_nt_wave", launch_ts<Op, 0, 8, 4, 1, kStNT, true>, 0},
      // 2-byte elements group 4 inputs; the shipped grouped shape is G4 V4 nt block
      {"T_G4_V4_nt_blk", launch_ts<Op, 0, 4, 4, 1, kStNT, false>, 0},
      {"T_G4_V2_nt_blk", launch_ts<Op, 0, 4, 2, 1, kStNT, false>, 0},
      {"T_G4_V1_sc1_wave", launch_ts<Op, 0, 4, 1, 1, 16, true>, 0},
      {"T_G4_V1_nt_wave", launch_ts<Op, 0, 4, 1, 1, kStNT, true>, 0},
      {"T_G4_V2_sc1_blk", launch_ts<Op, 0, 4, 2, 1, 16, false>, 0},
      {"T_xorprobe", launch_probe<Op, 0>, 0},
  };
  add_nf<Op, 2>(vs, n);
  add_nf<Op, 8>(vs, n);
  add_nf<Op, 17>(vs, n);
  return vs;
}

template <class Op>
int run(int n, size_t P, int reps, double peak_gbs) {
  const size_t bytes = P * Op::kBytes;
  // enough rotating input sets that their footprint is >= 1 GiB (4x the
  // 256 MiB Infinity Cache): small slices must not be served from it
  const double set_bytes = (double)(n + 1) * bytes;
  int sets = std::max(3, std::min(64, (int)((1ull << 30) / set_bytes) + 1));
  if (const char* ns = getenv("DLSIM_TUNE_SETS")) sets = std::max(1, atoi(ns));  // rotation length A/B
  printf("sets=%d footprint=%.0fMB\n", sets, sets * set_bytes / 1e6);
  const size_t nvec = P / Op::E;
  std::vector<void*> in((size_t)sets * n);
  // DLSIM_TUNE_OUT_SETS=k: the outputs rotate over k buffers instead of one
  // per input set (round 5: does the 256 MiB Infinity Cache hold a short
  // rotation of outputs, so their writes never reach HBM?)
  const int osets = getenv("DLSIM_TUNE_OUT_SETS") ? std::max(1, atoi(getenv("DLSIM_TUNE_OUT_SETS"))) : sets;
  printf("out_sets=%d\n", osets);
  std::vector<void*> out(osets);
  // Input layout experiment: DLSIM_TUNE_STAGGER unset = one hipMalloc per
  // input; set to S (bytes, multiple of 256) = all inputs rows of one arena,
  // row stride = bytes rounded up to 256 B, plus S more per row (S = 0 is the
  // bench's (n, p_pad) layout).
  const char* stg = getenv("DLSIM_TUNE_STAGGER");
  void* arena = nullptr;
  // DLSIM_TUNE_ALIGN=A (power of two >= 256): rows start A-aligned (the row
  // is rounded up to A before the stagger is added)
  const char* alg = getenv("DLSIM_TUNE_ALIGN");
  const size_t align = alg ? std::max<size_t>(256, strtoull(alg, nullptr, 10)) : 256;
  if (stg || alg) {
    const size_t stagger = stg ? strtoull(stg, nullptr, 10) & ~(size_t)255 : 0;
    const size_t stride = ((bytes + align - 1) / align) * align + stagger;
    if (getenv("DLSIM_TUNE_CONTIG"))  // physically contiguous
      CK(hipExtMallocWithFlags(&arena, stride * in.size() + align, hipDeviceMallocContiguous));
    else
      CK(hipMalloc(&arena, stride * in.size() + align));
    char* base = (char*)((((uintptr_t)arena) + align - 1) / align * align);
    for (size_t k = 0; k < in.size(); ++k) in[k] = base + k * stride;
    printf("layout=arena stride=%zu stagger=%zu align=%zu\n", stride, stagger, align);
  } else {
    for (auto& p : in) CK(hipMalloc(&p, bytes + 256));
    printf("layout=separate\n");
  }
  // DLSIM_TUNE_OUT_OFFSET=B: each output starts B bytes past its (2 MiB
  // aligned) allocation
  const size_t out_off = getenv("DLSIM_TUNE_OUT_OFFSET") ? strtoull(getenv("DLSIM_TUNE_OUT_OFFSET"), nullptr, 10) & ~(size_t)15 : 0;
  std::vector<void*> out_alloc(osets);
  for (int k = 0; k < osets; ++k) {
    if (getenv("DLSIM_TUNE_CONTIG"))
      CK(hipExtMallocWithFlags(&out_alloc[k], bytes + 256 + out_off, hipDeviceMallocContiguous));
    else
      CK(hipMalloc(&out_alloc[k], bytes + 256 + out_off));
    out[k] = (char*)out_alloc[k] + out_off;
  }
  printf("addr_mod_2MiB in0=%zu in1=%zu out0=%zu\n", (size_t)((uintptr_t)in[0] % (2u << 20)),
         (size_t)((uintptr_t)in[n > 1 ? 1 : 0] % (2u << 20)), (size_t)((uintptr_t)out[0] % (2u << 20)));
  for (size_t k = 0; k < in.size(); ++k)
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, (uint32_t*)in[k], bytes / 4,
                       (uint32_t)(k * 7919 + 1), Op::kBytes == 2);
  CK(hipDeviceSynchronize());
  std::vector<Slots<128>> slots(sets);
  for (int s = 0; s < sets; ++s) {
    memset(&slots[s], 0, sizeof(Slots<128>));
    for (int i = 0; i < n; ++i) {
      slots[s].p[i] = in[(size_t)s * n + i];
      slots[s].w[i] = 1.0f / n + 0.001f * i;
    }
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::vector<hipEvent_t> ev(2 * reps);
  for (auto& e : ev) CK(hipEventCreate(&e));
  const double alg_bytes = (double)(n + 1) * bytes;

  const bool r03 = getenv("DLSIM_TUNE_R03") != nullptr || getenv("DLSIM_TUNE_LAYOUT") != nullptr ||
                   getenv("DLSIM_TUNE_SMALL") != nullptr || getenv("DLSIM_TUNE_NTSWEEP") != nullptr;
  std::vector<Variant> vs;
  if (getenv("DLSIM_TUNE_NTSWEEP")) {
    add_ntsweep<Op>(vs, n);
  } else if (getenv("DLSIM_TUNE_SMALL")) {
    add_small<Op, 2>(vs, n);
    add_small<Op, 4>(vs, n);
    add_small<Op, 8>(vs, n);
    if (vs.empty()) {
      fprintf(stderr, "DLSIM_TUNE_SMALL needs f32 exact, n = 2, 4 or 8\n");
      return 1;
    }
  } else if (getenv("DLSIM_TUNE_LAYOUT")) {
    add_layout<Op>(vs, n);
  } else if (r03) {
    add_r03<Op, 8>(vs, n);
    if (getenv("DLSIM_TUNE_DEFER")) {
      add_defer<Op, 2>(vs, n);
      add_defer<Op, 4>(vs, n);
    }
    if (vs.empty()) {
      fprintf(stderr, "DLSIM_TUNE_R03 needs f32 exact, n = 8\n");
      return 1;
    }
  } else {
#ifdef DLSIM_TUNE_F32_ONLY  // the fast build carries the round-3 list only
    fprintf(stderr, "the tune_f32 build needs DLSIM_TUNE_R03=1\n");
    return 1;
#else
    vs = variants<Op>(n);
#endif
  }
  const int refv = r03 ? 0 : 1;
  if (const char* only = getenv("DLSIM_TUNE_ONLY")) {  // comma-separated exact names
    const std::string keep = std::string(",") + only + ",";
    std::vector<Variant> sel;
    for (auto& v : vs)
      if (keep.find("," + v.name + ",") != std::string::npos) sel.push_back(v);
    if (sel.size() < 2) {
      fprintf(stderr, "DLSIM_TUNE_ONLY must keep at least 2 variants\n");
      return 1;
    }
    vs = sel;
  }
  // reference output of the first (shipped-like) variant on set 0
  std::vector<char> ref(bytes), got(bytes);
  vs[refv].launch(slots[0], n, out[0], nvec, P, st, vs[refv].gm);
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(ref.data(), out[0], bytes, hipMemcpyDeviceToHost));
  {  // FNV-1a of the reference output: compare across element policies
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < bytes; ++i) h = (h ^ (unsigned char)ref[i]) * 1099511628211ull;
    printf("output_fnv1a=%016llx\n", (unsigned long long)h);
  }

  // interleaved rounds (one process, same device) — rule 24 of the guide
  const int rounds = 3;
  std::vector<std::vector<double>> med(vs.size()), bat(vs.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t v = 0; v < vs.size(); ++v) {
      for (int w = 0; w < 10; ++w) vs[v].launch(slots[w % sets], n, out[w % osets], nvec, P, st, vs[v].gm);
      for (int k = 0; k < reps; ++k) {
        CK(hipEventRecord(ev[2 * k], st));
        vs[v].launch(slots[k % sets], n, out[k % osets], nvec, P, st, vs[v].gm);
        CK(hipEventRecord(ev[2 * k + 1], st));
      }
      CK(hipStreamSynchronize(st));
      std::vector<double> t(reps);
      for (int k = 0; k < reps; ++k) {
        float ms;
        CK(hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]));
        t[k] = ms * 1e3;
      }
      std::sort(t.begin(), t.end());
      med[v].push_back(t[reps / 2]);
      // batch: one event pair around `reps` back-to-back launches
      CK(hipEventRecord(ev[0], st));
      for (int k = 0; k < reps; ++k) vs[v].launch(slots[k % sets], n, out[k % osets], nvec, P, st, vs[v].gm);
      CK(hipEventRecord(ev[1], st));
      CK(hipEventSynchronize(ev[1]));
      float bms;
      CK(hipEventElapsedTime(&bms, ev[0], ev[1]));
      bat[v].push_back(bms * 1e3 / reps);
    }
  }
  for (size_t v = 0; v < vs.size(); ++v) {
    vs[v].launch(slots[0], n, out[0], nvec, P, st, vs[v].gm);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(got.data(), out[0], bytes, hipMemcpyDeviceToHost));
    // compare only the vector part (tail elements are folded by every variant identically)
    const bool same = memcmp(ref.data(), got.data(), bytes) == 0;
    std::sort(med[v].begin(), med[v].end());
    std::sort(bat[v].begin(), bat[v].end());
    const double us = med[v][rounds / 2];
    const double bus = bat[v][rounds / 2];
    const double gbs = alg_bytes / (us * 1e-6) / 1e9;
    const double bgbs = alg_bytes / (bus * 1e-6) / 1e9;
    printf("variant=%-16s n=%d P=%zu bytes=%.1fMB median_us=%.2f GBps=%.0f frac=%.3f batch_us=%.2f batch_GBps=%.0f bfrac=%.3f same=%d moved=%.4f moved_bfrac=%.3f\n",
           vs[v].name.c_str(), n, P, alg_bytes / 1e6, us, gbs, gbs / peak_gbs, bus, bgbs, bgbs / peak_gbs, (int)same,
           vs[v].moved, bgbs * vs[v].moved / peak_gbs);
  }
  // copy ceiling on the same per-launch footprint, rotating >= 1 GiB of
  // buffers like the inputs (a fixed pair would be served from the MALL)
  {
    const size_t cbytes = (size_t)(alg_bytes / 2) & ~(size_t)15;
    const int csets = std::max(2, std::min(64, (int)((1ull << 30) / (2.0 * cbytes)) + 1));
    std::vector<void*> ca(csets), cb(csets);
    for (int k = 0; k < csets; ++k) {
      CK(hipMalloc(&ca[k], cbytes));
      CK(hipMalloc(&cb[k], cbytes));
      CK(hipMemset(ca[k], 1, cbytes));
    }
    const size_t nv = cbytes / 16;
    auto launch_copy = [&](int k) {
      Slots<128> cs;
      memset(&cs, 0, sizeof(cs));
      cs.p[0] = ca[k % csets];
      cs.w[0] = 1.0f;
      cs.div = 1.0f;
      launch_ts<XorProbeF32, 1, 8, 4, 1, 16, true>(cs, 1, cb[k % csets], nv, nv * 4, st, 0);
    };
    for (int k = 0; k < 10; ++k) launch_copy(k);
    CK(hipEventRecord(ev[0], st));
    for (int k = 0; k < reps; ++k) launch_copy(k);
    CK(hipEventRecord(ev[1], st));
    CK(hipEventSynchronize(ev[1]));
    float ms;
    CK(hipEventElapsedTime(&ms, ev[0], ev[1]));
    const double us = ms * 1e3 / reps;
    printf("copy16 sets=%d bytes_moved=%.1fMB batch_us=%.2f GBps=%.0f frac=%.3f\n", csets, 2.0 * cbytes / 1e6, us,
           2.0 * cbytes / (us * 1e-6) / 1e9, 2.0 * cbytes / (us * 1e-6) / 1e9 / peak_gbs);
    for (int k = 0; k < csets; ++k) {
      CK(hipFree(ca[k]));
      CK(hipFree(cb[k]));
    }
  }
  if (arena) CK(hipFree(arena));
  else
    for (auto& p : in) CK(hipFree(p));
  for (auto& p : out_alloc) CK(hipFree(p));
  return 0;
}

// ---- round 3: the chunk mean's shapes and its memory-only ceiling ----------------
//  DLSIM_TUNE_CHUNK=1: `tasks` chunk indices of n
// elements each, m contributors, one k_chunk_mean_batch launch per step, as
// ChunkManager.reconstruct_model runs them: contributor p's flat model is one
// arena row (the product's row rule), chunk c its slice [c n, (c+1) n), the
// means back to back. Variants: cascade tile shapes, and the XOR pattern probe
// of the shipped shape (same dispatch, arithmetic removed).
static size_t cm_ilp_begin(int m, size_t n, int threads) {  // dispatch.hpp chunk_mean_ilp_begin, fp32
  if (n <= 1) return 0;
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
  return b + (s1 >= 8 ? s1 / 32 * 32 : s1 / 4 * 4);
}

struct CmVariant {
  std::string name;
  void (*launch)(const ChunkMeanSlots&, unsigned, hipStream_t);
  int vpt;
  bool probe;
};
template <class Op, class SH>
void cm_launch(const ChunkMeanSlots& s, unsigned blocks, hipStream_t st) {
  hipLaunchKernelGGL((k_chunk_mean_batch<Op, SH>), dim3(blocks), dim3(kBlock), 0, st, s);
}

static size_t row_rule_bytes(size_t bytes) {  // arena.row_stride for 4-byte rows
  const size_t mib2 = size_t{2} << 20;
  if (bytes >= (size_t{16} << 20)) {
    size_t k = (bytes + mib2 - 1) / mib2;
    if (k % 4 == 0) ++k;
    return k * mib2;
  }
  size_t r = (bytes + 255) / 256 * 256;
  if (r % 65536 == 0) r += 4096;
  return r;
}

int run_chunk(int m, size_t n, int tasks, int reps) {
  const double peak = 8000.0;
  std::vector<CmVariant> vs = {
      {"cm_V4_wave_RF8", cm_launch<F32Mean, CmShape<4, true, 8>>, 4, false},
      {"cm_V4_blk_RF8", cm_launch<F32Mean, CmShape<4, false, 8>>, 4, false},
      {"cm_V2_wave_RF8", cm_launch<F32Mean, CmShape<2, true, 8>>, 2, false},
      {"cm_V1_wave_RF8", cm_launch<F32Mean, CmShape<1, true, 8>>, 1, false},
      {"cm_V4_wave_RF4", cm_launch<F32Mean, CmShape<4, true, 4>>, 4, false},
      {"cm_V4_wave_RF16", cm_launch<F32Mean, CmShape<4, true, 16>>, 4, false},
      {"cm_V2_wave_RF16", cm_launch<F32Mean, CmShape<2, true, 16>>, 2, false},
      {"cm_V1_wave_RF16", cm_launch<F32Mean, CmShape<1, true, 16>>, 1, false},
      {"cm_xorprobe_V4_wave_RF8", cm_launch<XorProbe<4>, CmShape<4, true, 8>>, 4, true},
  };
  if (m > kCmMaxPtrs / tasks || tasks > kCmMaxTasks) {
    fprintf(stderr, "m * tasks must fit one kernel-argument batch\n");
    return 1;
  }
  const size_t model_bytes = (size_t)tasks * n * 4;
  const size_t stride = row_rule_bytes(model_bytes);
  const double alg = (double)tasks * n * (m + 1) * 4;
  const int sets = std::max(3, std::min(64, (int)((1ull << 30) / ((double)m * stride + model_bytes)) + 1));
  void* arena = nullptr;
  const size_t al = size_t{2} << 20;
  CK(hipMalloc(&arena, stride * (size_t)m * sets + al));
  char* base = (char*)((((uintptr_t)arena) + al - 1) / al * al);
  std::vector<void*> outs(sets);
  for (auto& o : outs) CK(hipMalloc(&o, model_bytes + 256));
  for (size_t k = 0; k < (size_t)m * sets; ++k)
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, (uint32_t*)(base + k * stride), model_bytes / 4,
                       (uint32_t)(k * 7919 + 1), 0);
  CK(hipDeviceSynchronize());
  printf("chunk m=%d n=%zu tasks=%d sets=%d stride=%zu bytes=%.1fMB\n", m, n, tasks, sets, stride, alg / 1e6);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  auto slots = [&](int set, int vpt) {
    ChunkMeanSlots s;
    memset(&s, 0, sizeof(s));
    const size_t tile = (size_t)kBlock * vpt;
    size_t blocks = 0;
    int np = 0;
    for (int t = 0; t < tasks; ++t) {
      s.ptr_off[t] = (uint16_t)np;
      for (int i = 0; i < m; ++i) s.p[np++] = base + ((size_t)set * m + i) * stride + (size_t)t * n * 4;
      s.out[t] = (char*)outs[set] + (size_t)t * n * 4;
      s.nelem[t] = n;
      s.m[t] = (uint16_t)m;
      const size_t ib = cm_ilp_begin(m, n, 4);
      s.ilp_begin[t] = ib;
      s.flags[t] = (n * 4) % 16 == 0 ? kCmVec : 0;
      s.block_start[t] = (uint32_t)(blocks - t);  // full tiles before task t (ragged ends first)
      blocks += ib / 4 / tile + 1;
    }
    s.block_start[tasks] = (uint32_t)(blocks - tasks);
    s.ntasks = tasks;
    return std::make_pair(s, (unsigned)blocks);
  };
  std::vector<char> ref(model_bytes), got(model_bytes);
  {
    auto sb = slots(0, vs[0].vpt);
    vs[0].launch(sb.first, sb.second, st);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(ref.data(), outs[0], model_bytes, hipMemcpyDeviceToHost));
  }
  std::vector<hipEvent_t> ev(2);
  for (auto& e : ev) CK(hipEventCreate(&e));
  const int rounds = 3;
  std::vector<std::vector<double>> bat(vs.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      std::vector<std::pair<ChunkMeanSlots, unsigned>> sb;
      for (int k = 0; k < sets; ++k) sb.push_back(slots(k, vs[v].vpt));
      for (int w = 0; w < 10; ++w) vs[v].launch(sb[w % sets].first, sb[w % sets].second, st);
      CK(hipEventRecord(ev[0], st));
      for (int k = 0; k < reps; ++k) vs[v].launch(sb[k % sets].first, sb[k % sets].second, st);
      CK(hipEventRecord(ev[1], st));
      CK(hipEventSynchronize(ev[1]));
      float ms;
      CK(hipEventElapsedTime(&ms, ev[0], ev[1]));
      bat[v].push_back(ms * 1e3 / reps);
    }
  for (size_t v = 0; v < vs.size(); ++v) {
    auto sb = slots(0, vs[v].vpt);
    vs[v].launch(sb.first, sb.second, st);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(got.data(), outs[0], model_bytes, hipMemcpyDeviceToHost));
    std::sort(bat[v].begin(), bat[v].end());
    const double us = bat[v][rounds / 2];
    printf("variant=%-24s m=%d n=%zu tasks=%d batch_us=%.2f GBps=%.0f frac=%.3f same=%d\n", vs[v].name.c_str(), m, n,
           tasks, us, alg / (us * 1e-6) / 1e9, alg / (us * 1e-6) / 1e9 / peak,
           (int)(memcmp(ref.data(), got.data(), model_bytes) == 0));
  }
  CK(hipFree(arena));
  for (auto& o : outs) CK(hipFree(o));
  return 0;
}

int main(int argc, char** argv) {
  if (getenv("DLSIM_TUNE_CHUNK")) {  // tune_* chunk m n tasks reps
    const int m = argc > 1 ? atoi(argv[1]) : 4;
    const size_t n = argc > 2 ? strtoull(argv[2], nullptr, 10) : 1118164;
    const int tasks = argc > 3 ? atoi(argv[3]) : 10;
    const int reps = argc > 4 ? atoi(argv[4]) : 100;
    if (m < 1 || tasks < 1 || reps < 1 || n < 1) return 1;
    return run_chunk(m, n, tasks, reps);
  }
  int n = argc > 1 ? atoi(argv[1]) : 8;
  size_t P = argc > 2 ? strtoull(argv[2], nullptr, 10) : 11181642ull;
  std::string dt = argc > 3 ? argv[3] : "f32";
  std::string mode = argc > 4 ? argv[4] : "exact";
  int reps = argc > 5 ? atoi(argv[5]) : 50;
  if (n < 1 || n > 128 || reps < 1 || reps > 10000) {
    fprintf(stderr, "bad args\n");
    return 1;
  }
  const double peak = 8000.0;  // GB/s, MI355X HBM3E spec
#ifdef DLSIM_TUNE_F32_ONLY  // the fp32 / bf16 exact policies alone (fast to build: csrc/build/tune_f32)
  if (mode != "exact") {
    fprintf(stderr, "this build times the exact policies only\n");
    return 1;
  }
  return dt == "f32" ? run<F32Exact>(n, P, reps, peak) : run<BF16Exact>(n, P, reps, peak);
#endif
  if (dt == "f32")
    return mode == "exact" ? run<F32Exact>(n, P, reps, peak) : run<F32Fast>(n, P, reps, peak);
  if (mode == "exactold") return run<BF16ExactOld>(n, P, reps, peak);
  if (mode == "exactint") return run<BF16ExactInt>(n, P, reps, peak);
  return mode == "exact" ? run<BF16Exact>(n, P, reps, peak) : run<BF16Fast>(n, P, reps, peak);
}
