// dispatch.hpp — host-side dispatch of the reduce kernels (launch shapes,
// fan-in slots, size classes, batches, descriptor tables, chunk-mean tasks),
// shared by the C ABI (dlsim_abi.hip) and the per-policy instantiation units
// (inst_*.hip). The ABI unit declares every per-policy entry `extern
// template`; each inst_*.hip instantiates the ones of its element policies,
// so the device code of the policies compiles in parallel translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "dlsim.h"
#include "wreduce_kernels.hpp"
#include "chunk_mean_kernels.hpp"
#include "ab_env.hpp"

// Every DLSIM_* switch named below is an A/B switch, read through
// dlsim::ab_getenv: only when DLSIM_AB=1 is set as well (ab_env.hpp).

namespace dlsim_host __attribute__((visibility("hidden"))) {

// error reporting of the ABI (dlsim_abi.hip): set the thread's message, return code
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int hip_fail(hipError_t e, const char* what);

// Launch shape (tuned on MI355X with csrc/tune_wreduce.hip):
// 4 vectors of 16 B per lane (a 16 KiB tile per stream per block), one tile
// per block, non-temporal loads and stores. Small fan-in runs a kernel
// specialised on n (all n*4 loads issued back to back, fewer VGPRs than the
// grouped loop); larger n folds groups of G inputs. The specialised kernels
// are used only while they fit in 256 VGPRs (two waves per SIMD): past that
// the measured rate drops by up to 20% (profiles/r01_sweep_fanin_*.jsonl).
constexpr int kVpt = 4;
// Vectors per lane of the batched kernels (kernel-argument and table batches),
// by the largest task of the launch: VPT 1 when every task is under 1 MB per
// stream (100 GNLeNet tasks per launch: 0.787 against 0.759 at VPT 4), else
// VPT 4 (8 tasks of 1 M fp32: 0.797 against 0.778) (profiles/r02_batch_vpt/).
constexpr size_t kBatchSmallBytes = size_t{1} << 20;
template <class Op>
int batch_vpt(const size_t* nelem, int t0, int t1) {
  size_t mx = 0;
  for (int t = t0; t < t1; ++t) mx = nelem[t] > mx ? nelem[t] : mx;
  return mx * Op::kBytes < kBatchSmallBytes ? 1 : 4;
}
constexpr bool kNT = true;
// Output stores: buffer_store_dwordx4 with the nt bit (round 5). Rounds 1-4
// shipped sc1 (write-through), measured with outputs that rotated over 3
// buffers: those stay in the 256 MiB Infinity Cache, so their rewrites never
// reached HBM. With outputs that do not stay there (the bench now rotates
// >= 1 GiB of them, as a simulation's distinct aggregate outputs do) the nt
// store is faster in every shipped shape: north star 64.2 against 67.1 us,
// 2.8 M x 8 17.3 against 18.1, n = 17 at 11.2 M 126.0 against 130.9, bf16
// n = 2 at 31 M 30.2 against 30.5 (profiles/r05j/).
// The buffer's 32-bit byte offsets cap one launch's output at 2 GiB; longer
// outputs are split into independent launches over element ranges.
constexpr int kStore = 2;  // buffer store, nt
// Per element type (profiles/r01_tune_*): fp32 takes the buffer stores and
// the wave-contiguous lane map (each wave sweeps 4 KiB per stream, +1.3% on
// the north star); bf16, whose output is a third of the traffic in the
// 2-way merge, global non-temporal stores (+2% there) and the block map.
// These are the policies of the grouped (runtime fan-in) kernel and of the
// batched kernels.
// fp64 elements take the fp32 shapes (a 16-byte vector is 4 VGPRs in both).
template <class Op> constexpr int store_policy() { return Op::kBytes >= 4 ? kStore : dlsim::kStNT; }
template <class Op> constexpr bool wave_map() { return Op::kBytes >= 4; }
constexpr size_t kMaxLaunchOutBytes = (size_t{1} << 31) - (size_t{1} << 20);
template <class Op> constexpr int max_fixed_fan_in() { return Op::kBytes >= 4 ? 14 : 9; }
template <class Op> constexpr int group_size() { return Op::kBytes >= 4 ? 8 : 4; }

// Launch shape of the fixed fan-in kernels, chosen by the per-stream size
// class (size sweeps with arena rows as in bench.py and >= 1 GiB of rotating
// inputs: profiles/r01_tune_shape_sweep.log, profiles/r02_tune_slices/; the
// store policy re-chosen in round 5 with >= 1 GiB of rotating outputs,
// profiles/r05j/; "kStore" = buffer store, nt):
//   fp32  < 2 M elements   : VPT 2, block map, kStore (+7% at the 8-rank slice
//                            of the north star, 1.4 M: 9.85 vs 10.57 us)
//   fp32  2 M .. 5 M       : VPT 4, block map, kStore (1-4% over the wave map)
//   fp32 >= 5 M            : VPT 4, wave map,  kStore (~1% at 6-11 M)
//   bf16  < 48 M elements  : VPT 1, wave map, kStore (+7-12% at 4-33 M for n = 2)
//   bf16 >= 48 M           : VPT 4, block map, global nt (+1.5-2.5% at 64-125 M)
struct Shape {
  int vpt;
  int store;
  bool wave;
};
template <class Op, int C> constexpr Shape fixed_shape() {
  if constexpr (Op::kBytes >= 4) {
    if constexpr (C == 0) return Shape{2, kStore, false};
    else if constexpr (C == 1) return Shape{4, kStore, false};
    else return Shape{4, kStore, true};
  } else {
    if constexpr (C < 2) return Shape{1, kStore, true};
    else return Shape{4, dlsim::kStNT, false};
  }
}
//
// Round 5 (profiles/r05c/, fp32 rows of 0.5-2 M elements, n = 2, 4, 8): below
// 8 MB a one-tile-per-block grid has every block resident at once, and the
// launch runs at the pace of the CUs that hold the most whole tiles — about
// 37 GB/s per CU, so a CU with ceil(x) tiles where the average is x sets the
// time once ceil(x)/x exceeds ~1.25. For fan-in >= 6 the VPT 4 grid is the
// faster one whenever its tiles spread evenly (x4 = tiles per CU,
// ceil(x4)/x4 <= 1.25): n = 8 at 1.05 M (cfg2) 7.56 against 7.87 us, 1.70 M
// 11.09 against 11.78, 1.84 M 11.58 against 12.03; where they do not (the
// 8-rank slice of the north star, 1.4 M: x4 = 1.33) VPT 2 stays (9.60 against
// 10.45 us). Fan-in 2-4 showed no such rule and keep VPT 2.
int device_cus();  // multiProcessorCount of the current device (cached per device; dlsim_abi.hip)
inline bool v4_tiles_even(size_t nvec) {
  const double x = static_cast<double>(nvec / (static_cast<size_t>(dlsim::kBlock) * 4)) /
                   static_cast<double>(device_cus());
  return x >= 0.75 && std::ceil(x) / x <= 1.25;
}
// DLSIM_SMALL_SHAPE_R04 (read once; A/B runs): round 4's rule, VPT 2 below 8 MB.
inline bool small_shape_r04() {
  static const bool on = dlsim::ab_getenv("DLSIM_SMALL_SHAPE_R04") != nullptr;
  return on;
}
template <class Op> int size_class(size_t nelem, int fixed_fan_in = 0) {
  const size_t bytes = nelem * Op::kBytes;  // per stream
  if constexpr (Op::kBytes >= 4) {
    if (bytes < 8000000)
      return Op::kBytes == 4 && fixed_fan_in >= 6 && !small_shape_r04() && v4_tiles_even(nelem / Op::E) ? 1 : 0;
    return bytes < 20000000 ? 1 : 2;
  } else {
    return bytes < 96000000 ? 0 : 2;
  }
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// The fixed fan-in deferred launches pass nvec, the output and the first kPre
// input pointers as the leading, preloaded kernel arguments
// (k_wreduce_defer_pre, wreduce_kernels.hpp PreSlots). Measured in fresh
// bench processes, one box, two passes each (profiles/r06_preload_ab/): the
// 4-rank slice 16.66-16.70 -> 16.45-16.54 us, the north star 61.41-61.50 ->
// 61.29-61.43; the tiled kernel preloaded lost at small sizes (the 8-rank
// slice 9.76-9.77 -> 9.93-9.99, cfg2 7.63-7.75 -> 7.76-7.81: its blocks launch
// in several rounds and each wave's launch carries the preload), so it takes
// its arguments as before.
template <class S> inline const void* pre_ptr(const S& s, int nf, int i) { return i < nf ? s.p[i] : nullptr; }
static_assert(dlsim::kPre == 5, "the launches below pass five leading pointers");

template <class Op, class S, int NF, int VPT, int STP, bool WAVE>
hipError_t launch_shape(const S& s, int n, void* out, size_t nelem, hipStream_t st) {
  const size_t nvec = nelem / Op::E;
  const size_t tile = static_cast<size_t>(dlsim::kBlock) * VPT;
  const size_t blocks = nvec / tile + 1;  // full tiles + one block for the ragged end
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  hipLaunchKernelGGL((dlsim::k_wreduce_tiles<Op, S, NF, group_size<Op>(), VPT, kNT, STP, WAVE>),
                     dim3(static_cast<unsigned>(blocks)), dim3(dlsim::kBlock), 0, st, s, n, out, nvec, nelem);
  return hipGetLastError();
}

// Launch shape of the grouped (runtime fan-in, n > max_fixed_fan_in) kernel
// by the same size classes (sweeps: profiles/r02_tune_grouped/, fp32 n = 17
// and 100 at 11.2 M and at the 8-rank slice, 1.4 M; bf16 n = 17 and 12):
//   4/8-byte  < 8 MB per stream : VPT 1, wave map,  kStore (0.837 against 0.791
//                                 at n = 100, 0.646 against 0.595 at n = 17)
//   4/8-byte  larger            : VPT 4, block map, kStore (0.801 against 0.791
//                                 at n = 100 -- the memory-only probe's 0.802)
//   2-byte    < 96 MB per stream: VPT 1, wave map,  kStore (bf16 n = 17: 0.724
//                                 against 0.691 at 11.2 M, 0.400 against 0.309
//                                 at 1.4 M)
//   2-byte    larger            : VPT 4, block map, nt (0.771 at n = 12, 62.5 M)
template <class Op, int C> constexpr Shape grouped_shape() {
  if constexpr (C == 0) return Shape{1, kStore, true};
  else if constexpr (Op::kBytes >= 4) return Shape{4, kStore, false};
  else return Shape{4, dlsim::kStNT, false};
}

template <class Op, class S, int NF, int C>
hipError_t launch_class(const S& s, int n, void* out, size_t nelem, hipStream_t st) {
  constexpr Shape k = NF > 0 ? fixed_shape<Op, C>() : grouped_shape<Op, C>();
  return launch_shape<Op, S, NF, k.vpt, k.store, k.wave>(s, n, out, nelem, st);
}

// Deferred stores (dlsim::k_wreduce_defer): fp32 policies,
// fan-in >= 3 (fixed, and the grouped form above 14), >= 10 MB per stream
// (use_defer). One block (512
// lanes, ~190-250 VGPRs: one block per CU) folds R rows of 512 vectors.
// defer_rows picks an even R (profiles/r05_defer/, bench A/B in fresh
// processes, outputs rotating beyond the Infinity Cache; odd R re-reads a
// row per group and measured slower):
// * one round of blocks with every CU busy, R = ceil(rows / CUs), up to 24
//   rows: north star (8 x 11.2 M, 2,795,410 vectors, 256 CUs) R = 22, 249
//   blocks, 63.0 us against 63.4 tiled; n = 4 / 6 / 10 at 11.2 M 35.5 / 48.9 /
//   76.4 against 37.0 / 51.0 / 78.0;
// * else two rounds, R = ceil(rows / 2 CUs): a single round of 32 rows loses
//   to two of 16 at 16 M (n = 8: 90.1 against 88.3 us; n = 10: 111.3 against
//   107.6; tiled 92.2 / 113.1);
// * else R in [RMAX/2, RMAX] from a cost model of rounds of blocks: full
//   rounds cost R each, a last round with a fraction x of the CUs busy costs
//   R * max(x, 0.38 + 0.45 x) (fewer CUs each stream more, up to ~2.2x their
//   fair share), every round adds 0.1. 8 x 44.7 M: R = 30, 251.6 against
//   261.7 us. A thin last round is what to avoid (north star R = 10: 546
//   blocks, 70.9 us; R = 20: 273 blocks, 82.8).
// DLSIM_DEFER=0 (read once): the tiled kernel (A/B runs); DLSIM_DEFER_R=r
// (read once): that R.
constexpr int kDeferU = 2, kDeferRMin = 4, kDeferOneRoundMax = 24;
// results per lane a block can hold: 32 (128 VGPRs) while the fan-in's loads
// fit beside them, 24 from fan-in 12 (no spills: tests/test_isa_audit.py)
template <class Op, int NF> constexpr int defer_rmax() { return NF >= 12 ? 24 : 32; }  // NF = 0 (grouped): 32
// Fan-in 11-14 defers only from 16 rows per CU (8.4 M fp32 elements on 256
// CUs): 12 and 14 x 11.2 M 89.9 / 103.4 us against 92.1 / 106.2 tiled, but
// 14 x 5 M 48.4 against 46.9 (profiles/r05_defer/r05y*, r05z*).
// DLSIM_DEFER_MAX_FAN_IN=k (read once; A/B runs): no deferred launch above
// fan-in k.
// Instantiated for fp32 fan-in >= 2 and the grouped form; used from fan-in
// defer_min_fan_in(), 3: n = 3 at 11.2 M 28.74 against 29.80 us tiled, n = 2
// loses (23.79 against 22.55 at 11.2 M, 67.06 against 58.56 at 31 M). 2-byte
// elements were tried (fixed fan-in 2-6) and did not pay: bf16 n = 2 at 125 M
// (cfg4) 126.8 against 114.9 us, at 31 M 32.66 against 30.04, n = 4 at 11.2 M
// even (profiles/r05_defer/r05ai_*). DLSIM_DEFER_MIN_FAN_IN=k (read once; A/B
// runs).
template <class Op, int NF> constexpr bool defer_eligible() { return Op::kBytes == 4 && (NF >= 2 || NF == 0); }
inline int defer_min_fan_in() {
  static const int k = [] {
    const char* e = dlsim::ab_getenv("DLSIM_DEFER_MIN_FAN_IN");
    return e ? std::atoi(e) : 3;
  }();
  return k;
}
constexpr int kDeferWideFanIn = 10;
constexpr size_t kDeferWideRowsPerCu = 16;
inline bool defer_on() {
  static const bool on = [] {
    const char* e = dlsim::ab_getenv("DLSIM_DEFER");
    return !(e && e[0] == '0');
  }();
  return on;
}
inline int defer_max_fan_in() {
  static const int k = [] {
    const char* e = dlsim::ab_getenv("DLSIM_DEFER_MAX_FAN_IN");
    return e ? std::atoi(e) : 1 << 30;
  }();
  return k;
}
inline int defer_r_override() {
  static const int r = [] {
    const char* e = dlsim::ab_getenv("DLSIM_DEFER_R");
    return e ? std::atoi(e) : 0;
  }();
  return r;
}
inline int defer_rows(size_t nvec, size_t cus, int rmax) {
  if (defer_r_override() > 0) return std::min(defer_r_override(), rmax);
  const size_t T = (nvec + dlsim::kDeferBlock - 1) / dlsim::kDeferBlock;
  const size_t one = ((T + cus - 1) / cus + 1) & ~size_t{1};  // one round, every CU busy; even
  if (one <= static_cast<size_t>(std::min(rmax, kDeferOneRoundMax))) return std::max(static_cast<int>(one), kDeferRMin);
  const size_t two = ((T + 2 * cus - 1) / (2 * cus) + 1) & ~size_t{1};  // two rounds
  if (two <= static_cast<size_t>(rmax)) return static_cast<int>(two);
  int best = rmax;
  double best_cost = 1e300;
  for (int R = rmax / 2; R <= rmax; R += 2) {
    const double w = static_cast<double>((T + R - 1) / R) / static_cast<double>(cus);  // rounds (> 1)
    const double full = std::floor(w), x = w - full;
    const double cost = R * (full + (x > 0 ? std::max(x, 0.38 + 0.45 * x) : 0.0)) + 0.1 * std::ceil(w);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = R;
    }
  }
  return best;
}

// Does a launch of n inputs of nelem elements defer? From 10 MB per stream
// (fan-in 11-14 from 16 rows per CU). Grouped (runtime) fan-in, n > 14, the
// same (cfg3, 17 x 11.2 M: 123.8 -> 120.8 us; cfg5,
// 100 x 11.2 M: 676.6 -> 659.0; 17 x 16 M 182.5 -> 171.9; 30 x 11.2 M 212.6
// -> 204.3; profiles/r05_defer/r05ad_*). DLSIM_DEFER_GROUPED=0 (read once;
// A/B runs): the tiled grouped kernel.
inline bool defer_grouped_on() {
  static const bool on = [] {
    const char* e = dlsim::ab_getenv("DLSIM_DEFER_GROUPED");
    return !(e && e[0] == '0');
  }();
  return on;
}
// From 10 MB per stream (profiles/r05_defer/r05bb_*, r05bc_*): the north
// star's 4-rank slice (8 x 2.8 M) 16.55-16.58 against 17.08-17.19 us tiled,
// 8 x 3.5 M 20.35 against 21.76, 17 x 2.8 M 33.88 against 34.30, 3 x 2.8 M
// 9.01 against 9.15; below it the one round of rows leaves CUs idle or too
// few rows to defer: 8 x 2.1 M +1.6 % but 4 x 2.1 M -5 %, the 8-rank slice
// (8 x 1.4 M) 10.28-10.30 against 9.71, cfg2 (8 x 1 M) 9.06 against 7.62.
// DLSIM_DEFER_MIN_MB=x (read once; A/B runs): from x MB instead.
constexpr double kDeferMinMB = 10.0;
inline double defer_min_mb() {
  static const double x = [] {
    const char* e = dlsim::ab_getenv("DLSIM_DEFER_MIN_MB");
    return e ? std::atof(e) : kDeferMinMB;
  }();
  return x;
}
template <class Op> bool use_defer(int n, size_t nelem) {
  if (Op::kBytes != 4 || n < std::max(2, defer_min_fan_in()) || n > defer_max_fan_in() || !defer_on()) return false;
  if (static_cast<double>(nelem * Op::kBytes) < defer_min_mb() * 1e6) return false;
  if (n > max_fixed_fan_in<Op>()) return defer_grouped_on();
  if (n <= kDeferWideFanIn) return true;
  const size_t rows = nelem / Op::E / dlsim::kDeferBlock;
  return rows >= kDeferWideRowsPerCu * static_cast<size_t>(device_cus());
}

// The kernel run<Op> launches for n aligned inputs (dlsim_kernel_name).
template <class Op> const char* kernel_name(int n, size_t nelem) {
  if (nelem == 0 || n < 1) return "";
  const size_t first = std::min(nelem, kMaxLaunchOutBytes / Op::kBytes);
  if (use_defer<Op>(n, first)) return n <= max_fixed_fan_in<Op>() ? "dlsim::k_wreduce_defer_pre" : "dlsim::k_wreduce_defer";
  return "dlsim::k_wreduce_tiles";
}

// The exact fp32 policy with a fixed fan-in launches the kernel compiled for
// its R (every even R up to RMAX): the row groups and stores run unguarded
// and straight-line. A runtime R guards each with a branch: the north star
// ran 63.35-63.38 us that way against 61.60-61.63 compiled for R = 22, in one
// process of the tuning harness (profiles/r05_defer/r05aw/). The other
// policies (FAST, mean, the probe) and the grouped form take the runtime R
// (the grouped form compiled per R measured the same: cfg3 120.76-120.90 us,
// cfg5 661.9-662.3, profiles/r05_defer/r05az_*).
// One deferred launch, compiled for R = RC (0: runtime R); fixed fan-in with
// the leading arguments preloaded.
template <class Op, class S, int NF, int RC>
hipError_t launch_defer_kernel(const S& s, int n, void* out, size_t nvec, size_t nelem, int R, unsigned blocks,
                               hipStream_t st) {
  if constexpr (NF > 0) {
    hipLaunchKernelGGL(
        (dlsim::k_wreduce_defer_pre<Op, S, NF, group_size<Op>(), defer_rmax<Op, NF>(), kDeferU, kStore, RC>),
        dim3(blocks), dim3(dlsim::kDeferBlock), 0, st, nvec, out, pre_ptr(s, NF, 0), pre_ptr(s, NF, 1),
        pre_ptr(s, NF, 2), pre_ptr(s, NF, 3), pre_ptr(s, NF, 4), s, n, R, nelem);
  } else {
    hipLaunchKernelGGL(
        (dlsim::k_wreduce_defer<Op, S, NF, group_size<Op>(), defer_rmax<Op, NF>(), kDeferU, kStore, RC>),
        dim3(blocks), dim3(dlsim::kDeferBlock), 0, st, s, n, R, out, nvec, nelem);
  }
  return hipGetLastError();
}

template <class Op, class S, int NF, int RC>
hipError_t launch_defer_rc(const S& s, int n, void* out, size_t nvec, size_t nelem, int R, unsigned blocks,
                           hipStream_t st) {
  if constexpr (RC > defer_rmax<Op, NF>()) {
    return launch_defer_kernel<Op, S, NF, 0>(s, n, out, nvec, nelem, R, blocks, st);
  } else {
    if (R == RC) return launch_defer_kernel<Op, S, NF, RC>(s, n, out, nvec, nelem, R, blocks, st);
    return launch_defer_rc<Op, S, NF, RC + kDeferU>(s, n, out, nvec, nelem, R, blocks, st);
  }
}

template <class Op, class S, int NF>
hipError_t launch_defer(const S& s, int n, void* out, size_t nelem, hipStream_t st) {
  const size_t nvec = nelem / Op::E;
  const int R = defer_rows(nvec, static_cast<size_t>(device_cus()), defer_rmax<Op, NF>());
  const size_t span = static_cast<size_t>(dlsim::kDeferBlock) * static_cast<size_t>(R);
  const size_t blocks = (nvec + span - 1) / span;
  if (blocks == 0 || blocks > 0x7fffffffu) return hipErrorInvalidValue;
  // compiled R from kDeferRMin (defer_rows never returns less) for the fan-ins
  // that defer by default (>= 3); R = 2 and fan-in 2 (reachable only through
  // the A/B switches) take the runtime R
  if constexpr (NF >= 3 && std::is_same<Op, dlsim::F32Exact>::value)
    return launch_defer_rc<Op, S, NF, kDeferRMin>(s, n, out, nvec, nelem, R, static_cast<unsigned>(blocks), st);
  return launch_defer_kernel<Op, S, NF, 0>(s, n, out, nvec, nelem, R, static_cast<unsigned>(blocks), st);
}

template <class Op, class S, int NF>
hipError_t launch_tiles(const S& s, int n, void* out, size_t nelem, hipStream_t st) {
  if constexpr (NF > 0) {
    const int c = size_class<Op>(nelem, NF);
    if constexpr (defer_eligible<Op, NF>())
      if (use_defer<Op>(NF, nelem)) return launch_defer<Op, S, NF>(s, n, out, nelem, st);
    switch (c) {
      case 0: return launch_class<Op, S, NF, 0>(s, n, out, nelem, st);
      case 1: return launch_class<Op, S, NF, 1>(s, n, out, nelem, st);
      default: return launch_class<Op, S, NF, 2>(s, n, out, nelem, st);
    }
  } else {
    if constexpr (defer_eligible<Op, 0>())
      if (use_defer<Op>(n, nelem)) return launch_defer<Op, S, 0>(s, n, out, nelem, st);
    return size_class<Op>(nelem) == 0 ? launch_class<Op, S, 0, 0>(s, n, out, nelem, st)
                                      : launch_class<Op, S, 0, 2>(s, n, out, nelem, st);
  }
}

template <class Op, int K>
hipError_t launch_fixed_k(const dlsim::Slots<16, dlsim::wt_t<Op>>& s, int n, void* out, size_t nelem,
                          hipStream_t st) {
  if constexpr (K > max_fixed_fan_in<Op>()) {
    return hipErrorInvalidValue;
  } else {
    if (n == K) return launch_tiles<Op, dlsim::Slots<16, dlsim::wt_t<Op>>, K>(s, n, out, nelem, st);
    return launch_fixed_k<Op, K + 1>(s, n, out, nelem, st);
  }
}

template <class Op, class S>
hipError_t launch_any(const S& s, int n, void* out, size_t nelem, bool vec, hipStream_t st) {
  if (vec) {
    if constexpr (std::is_same<S, dlsim::Slots<16, dlsim::wt_t<Op>>>::value) {
      if (n <= max_fixed_fan_in<Op>()) return launch_fixed_k<Op, 1>(s, n, out, nelem, st);
    }
    return launch_tiles<Op, S, 0>(s, n, out, nelem, st);
  }
  const size_t blocks = (nelem + dlsim::kBlock - 1) / dlsim::kBlock;
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  hipLaunchKernelGGL((dlsim::k_wreduce_scalar<Op, S>), dim3(static_cast<unsigned>(blocks)), dim3(dlsim::kBlock), 0,
                     st, s, n, out, nelem);
  return hipGetLastError();
}

template <int NB, class W>
void fill_slots(dlsim::Slots<NB, W>& s, const void* const* in, const W* w, int n, float div) {
  std::memset(&s, 0, sizeof(s));
  for (int i = 0; i < n; ++i) {
    s.p[i] = in[i];
    s.w[i] = w ? w[i] : 1.0f;
  }
  s.div = div;
}

// One launch over [0, nelem) of n inputs: every output element is written
// once, after all n of its terms are folded in input order. Up to
// DLSIM_MAX_FUSED_INPUTS inputs travel as kernel arguments; above that the
// pointer/weight table goes to a stream-ordered device buffer (the pageable
// host copy is staged by the runtime before hipMemcpyAsync returns).
// div: final divisor (the mean policies; 1 for the weighted reduce).
template <class Op>
int run_range(const void* const* in, int n, const dlsim::wt_t<Op>* w, void* out, size_t nelem, bool vec, float div,
              hipStream_t st) {
  using W = dlsim::wt_t<Op>;
  hipError_t e;
  if (n <= 16) {
    dlsim::Slots<16, W> s;
    fill_slots(s, in, w, n, div);
    e = launch_any<Op>(s, n, out, nelem, vec, st);
  } else if (n <= DLSIM_MAX_FUSED_INPUTS) {
    dlsim::Slots<DLSIM_MAX_FUSED_INPUTS, W> s;
    fill_slots(s, in, w, n, div);
    e = launch_any<Op>(s, n, out, nelem, vec, st);
  } else {
    const size_t pbytes = static_cast<size_t>(n) * sizeof(void*);
    std::vector<unsigned char> h(pbytes + static_cast<size_t>(n) * sizeof(W));
    std::memcpy(h.data(), in, pbytes);
    for (int i = 0; i < n; ++i) {
      const W wi = w ? w[i] : W(1);
      std::memcpy(h.data() + pbytes + static_cast<size_t>(i) * sizeof(W), &wi, sizeof(W));
    }
    void* d = nullptr;
    e = hipMallocAsync(&d, h.size(), st);
    if (e != hipSuccess) return hip_fail(e, "fan-in table alloc");
    e = hipMemcpyAsync(d, h.data(), h.size(), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
      const dlsim::DevSlots<W> s{static_cast<const void* const*>(d),
                                 reinterpret_cast<const W*>(static_cast<unsigned char*>(d) + pbytes), div};
      e = launch_any<Op>(s, n, out, nelem, vec, st);
    }
    const hipError_t e2 = hipFreeAsync(d, st);
    if (e == hipSuccess) e = e2;
  }
  if (e != hipSuccess) return hip_fail(e, "kernel launch");
  return DLSIM_OK;
}

// Elements are independent: an output longer than one launch's 2 GiB store
// window is reduced as consecutive ranges (pointers offset by the range start).
template <class Op>
int run(const void* const* in, int n, const dlsim::wt_t<Op>* w, void* out, size_t nelem, hipStream_t st,
        float div = 1.0f) {
  if (nelem == 0) return DLSIM_OK;
  bool vec = aligned16(out);
  for (int i = 0; i < n && vec; ++i) vec = aligned16(in[i]);
  const size_t chunk = kMaxLaunchOutBytes / Op::kBytes;  // multiple of every tile size
  if (!vec || nelem <= chunk) return run_range<Op>(in, n, w, out, nelem, vec, div, st);
  std::vector<const void*> sub(static_cast<size_t>(n));
  for (size_t b = 0; b < nelem; b += chunk) {
    const size_t len = std::min(chunk, nelem - b);
    for (int i = 0; i < n; ++i) sub[i] = static_cast<const char*>(in[i]) + b * Op::kBytes;
    int rc = run_range<Op>(sub.data(), n, w, static_cast<char*>(out) + b * Op::kBytes, len, vec, div, st);
    if (rc != DLSIM_OK) return rc;
  }
  return DLSIM_OK;
}

// ---- cross-task hazards of the batched entry points ---------------------------
// A batched launch runs its tasks concurrently; b separate calls run them in
// order. They agree unless one task writes bytes another task reads or
// writes. Detected in O((inputs + b) log b): the output spans are sorted (any
// overlap among them shows between neighbours), then each input span is
// looked up among them. A task's exact in-place alias of its own input is
// fine (one lane reads every term of an element before writing it).
struct Span {
  uintptr_t a, b;
  int task;
};

inline bool cross_task_overlap(int nt, const int* fan_in, const void* const* in, void* const* outs, const size_t* nelem,
                        size_t esz) {
  std::vector<Span> wr;
  wr.reserve(static_cast<size_t>(nt));
  for (int t = 0; t < nt; ++t) {
    if (nelem[t] == 0) continue;
    const uintptr_t a = reinterpret_cast<uintptr_t>(outs[t]);
    wr.push_back({a, a + nelem[t] * esz, t});
  }
  std::sort(wr.begin(), wr.end(), [](const Span& x, const Span& y) { return x.a < y.a; });
  for (size_t k = 1; k < wr.size(); ++k)
    if (wr[k].a < wr[k - 1].b) return true;  // two outputs overlap (disjoint otherwise: ends sorted too)
  size_t off = 0;
  for (int t = 0; t < nt; ++t) {
    const size_t bytes = nelem[t] * esz;
    for (int i = 0; i < fan_in[t]; ++i) {
      if (bytes == 0) continue;
      const uintptr_t a = reinterpret_cast<uintptr_t>(in[off + i]), b = a + bytes;
      auto it = std::upper_bound(wr.begin(), wr.end(), a, [](uintptr_t v, const Span& x) { return v < x.b; });
      for (; it != wr.end() && it->a < b; ++it)
        if (it->task != t) return true;
    }
    off += static_cast<size_t>(fan_in[t]);
  }
  return false;
}

// ---- batched launches ---------------------------------------------------------
// Lane map of the table batches' full tiles: the wave map (each wave sweeps
// VPT contiguous KiB per stream) where the single-task kernels use it, VPT 4
// tiles of 4/8-byte elements: 8 x 11.2 M fp32 cut into 8 / 32 tasks 64.47 ->
// 63.67 / 65.43 -> 64.46 us; the kernel-argument batches measured the same or
// 0.5 % slower with it and keep the block map
// (scripts/probes/probe_batch_vs_single.py, profiles/r03s3_batch_vs_single/).
template <class Op, int VPT> constexpr bool kBatchWave = VPT == 4 && wave_map<Op>();

template <class Op, int NF, int VPT>
hipError_t launch_batch_nf(const dlsim::BatchSlots& s, unsigned blocks, hipStream_t st) {
  hipLaunchKernelGGL((dlsim::k_wreduce_batch<Op, NF, group_size<Op>(), VPT, kNT, store_policy<Op>()>), dim3(blocks),
                     dim3(dlsim::kBlock), 0, st, s);
  return hipGetLastError();
}

template <class Op, int K, int VPT>
hipError_t launch_batch_fixed(const dlsim::BatchSlots& s, int n, unsigned blocks, hipStream_t st) {
  if constexpr (K > max_fixed_fan_in<Op>()) {
    return launch_batch_nf<Op, 0, VPT>(s, blocks, st);
  } else {
    if (n == K) return launch_batch_nf<Op, K, VPT>(s, blocks, st);
    return launch_batch_fixed<Op, K + 1, VPT>(s, n, blocks, st);
  }
}

// Fill and launch BatchSlots with tasks [t0, t1); all tasks vector-eligible.
// divs: per-task final divisor (the mean policies), nullptr = 1.
template <class Op>
hipError_t launch_batch(const int* fan_in, const size_t* in_off, const void* const* in, const float* w,
                        const float* divs, void* const* outs, const size_t* nelem, int t0, int t1,
                        hipStream_t st) {
  dlsim::BatchSlots s;
  std::memset(&s, 0, sizeof(s));
  const int vpt = batch_vpt<Op>(nelem, t0, t1);
  const size_t tile = static_cast<size_t>(dlsim::kBlock) * vpt;
  uint32_t blocks = 0;
  int ptrs = 0;
  bool uniform = true;
  for (int t = t0; t < t1; ++t) {
    const int k = t - t0;
    const size_t nvec = nelem[t] / Op::E;
    s.out[k] = outs[t];
    s.nvec[k] = nvec;
    s.nelem[k] = nelem[t];
    s.block_start[k] = blocks - static_cast<uint32_t>(k);  // full tiles before task k (ragged ends first)
    s.ptr_off[k] = static_cast<uint32_t>(ptrs);
    s.fan_in[k] = static_cast<uint32_t>(fan_in[t]);
    s.div[k] = divs ? divs[t] : 1.0f;
    for (int i = 0; i < fan_in[t]; ++i) {
      s.p[ptrs + i] = in[in_off[t] + i];
      s.w[ptrs + i] = w[in_off[t] + i];
    }
    ptrs += fan_in[t];
    blocks += static_cast<uint32_t>(nvec / tile + 1);
    uniform = uniform && fan_in[t] == fan_in[t0];
  }
  s.ntasks = t1 - t0;
  s.block_start[t1 - t0] = blocks - static_cast<uint32_t>(t1 - t0);
  if (vpt == 1) {
    if (uniform) return launch_batch_fixed<Op, 1, 1>(s, fan_in[t0], blocks, st);
    return launch_batch_nf<Op, 0, 1>(s, blocks, st);
  }
  if (uniform) return launch_batch_fixed<Op, 1, 4>(s, fan_in[t0], blocks, st);
  return launch_batch_nf<Op, 0, 4>(s, blocks, st);
}

template <class Op>
int run_batched(int b, const int* fan_in, const void* const* in, const float* w, void* const* outs,
                const size_t* nelem, hipStream_t st, const float* divs = nullptr) {
  std::vector<size_t> off(static_cast<size_t>(b) + 1, 0);
  for (int t = 0; t < b; ++t) off[t + 1] = off[t] + static_cast<size_t>(fan_in[t]);
  if (cross_task_overlap(b, fan_in, in, outs, nelem, Op::kBytes)) {
    // A task reads or writes another task's output: keep the semantics of b
    // separate calls by running the tasks one launch each, in order.
    for (int t = 0; t < b; ++t) {
      int rc = run<Op>(in + off[t], fan_in[t], w + off[t], outs[t], nelem[t], st, divs ? divs[t] : 1.0f);
      if (rc != DLSIM_OK) return rc;
    }
    return DLSIM_OK;
  }
  auto batchable = [&](int t) {
    if (nelem[t] == 0 || fan_in[t] > 16) return false;
    if (nelem[t] * Op::kBytes > kMaxLaunchOutBytes) return false;
    // a task the deferred-store kernel takes (>= 10 MB per stream) runs alone
    // through it: a launch that size amortises its own overhead, and the
    // batch kernel interleaves its stores
    if (use_defer<Op>(fan_in[t], nelem[t])) return false;
    if (!aligned16(outs[t])) return false;
    for (int i = 0; i < fan_in[t]; ++i)
      if (!aligned16(in[off[t] + i])) return false;
    return true;
  };
  // Tasks that cannot ride in a batch (large fan-in, misaligned, > 2 GiB) go
  // alone (no task touches another's output, so the order is free).
  std::vector<int> group;
  for (int t = 0; t < b; ++t) {
    if (batchable(t)) {
      group.push_back(t);
      continue;
    }
    if (nelem[t] == 0) continue;
    int rc = run<Op>(in + off[t], fan_in[t], w + off[t], outs[t], nelem[t], st, divs ? divs[t] : 1.0f);
    if (rc != DLSIM_OK) return rc;
  }
  // Pack the rest greedily into kernel-argument batches, in task order.
  std::vector<const void*> ins;
  std::vector<float> ws, dv;
  std::vector<void*> os;
  std::vector<size_t> ne, ioff;
  std::vector<int> fi;
  for (int t : group) {
    ioff.push_back(ins.size());
    for (int i = 0; i < fan_in[t]; ++i) {
      ins.push_back(in[off[t] + i]);
      ws.push_back(w[off[t] + i]);
    }
    os.push_back(outs[t]);
    ne.push_back(nelem[t]);
    fi.push_back(fan_in[t]);
    dv.push_back(divs ? divs[t] : 1.0f);
  }
  const int g = static_cast<int>(group.size());
  const size_t tile1 = dlsim::kBlock;  // the most blocks a task can need (VPT 1)
  int t0 = 0;
  while (t0 < g) {
    int t1 = t0, ptrs = 0;
    uint64_t blocks = 0;
    while (t1 < g && t1 - t0 < dlsim::kBatchMaxTasks && ptrs + fi[t1] <= dlsim::kBatchMaxPtrs &&
           blocks + ne[t1] / Op::E / tile1 + 1 < 0x7fffffffull) {
      ptrs += fi[t1];
      blocks += ne[t1] / Op::E / tile1 + 1;
      ++t1;
    }
    hipError_t e = launch_batch<Op>(fi.data(), ioff.data(), ins.data(), ws.data(), dv.data(), os.data(),
                                    ne.data(), t0, t1, st);
    if (e != hipSuccess) return hip_fail(e, "batched kernel launch");
    t0 = t1;
  }
  return DLSIM_OK;
}

// ---- descriptor-table batches ---------------------------------------------------
struct TableLayout {
  size_t tasks_off, map_off, ptrs_off, w_off, bytes;
  uint32_t nblocks;
  int vpt;  // batch_vpt of the tasks, kept in the header
};

inline size_t round8(size_t x) { return (x + 7) / 8 * 8; }

template <class Op>
uint32_t task_blocks(size_t nelem, int vpt) {
  const size_t tile = static_cast<size_t>(dlsim::kBlock) * vpt;
  return static_cast<uint32_t>(nelem / Op::E / tile + 1);
}

template <class Op>
bool table_layout(int b, const int* fan_in, const size_t* nelem, TableLayout* L) {
  uint64_t blocks = 0, ptrs = 0;
  L->vpt = batch_vpt<Op>(nelem, 0, b);
  for (int t = 0; t < b; ++t) {
    blocks += task_blocks<Op>(nelem[t], L->vpt);
    ptrs += static_cast<uint64_t>(fan_in[t]);
  }
  if (blocks >= 0x7fffffffull) return false;
  L->nblocks = static_cast<uint32_t>(blocks);
  L->tasks_off = round8(sizeof(dlsim::BatchTableHeader));
  L->map_off = round8(L->tasks_off + sizeof(dlsim::BatchTaskDesc) * static_cast<size_t>(b));
  L->ptrs_off = round8(L->map_off + sizeof(uint32_t) * static_cast<size_t>(blocks));
  L->w_off = round8(L->ptrs_off + sizeof(void*) * static_cast<size_t>(ptrs));
  L->bytes = round8(L->w_off + sizeof(float) * static_cast<size_t>(ptrs));
  return true;
}

template <class Op>
int table_fill(int b, const int* fan_in, const void* const* in, const float* w, void* const* outs,
               const size_t* nelem, void* h_table, size_t bytes) {
  TableLayout L;
  if (!table_layout<Op>(b, fan_in, nelem, &L)) return fail(DLSIM_E_ARG, "batch too large");
  if (bytes < L.bytes) return fail(DLSIM_E_ARG, "table buffer too small (%zu < %zu)", bytes, L.bytes);
  if (cross_task_overlap(b, fan_in, in, outs, nelem, Op::kBytes))
    return fail(DLSIM_E_ARG,
                "a task's output overlaps another task's input or output: one table launch runs all tasks "
                "concurrently (use separate calls, or dlsim_wreduce_batched, which orders them)");
  unsigned char* base = static_cast<unsigned char*>(h_table);
  std::memset(base, 0, L.bytes);
  auto* h = reinterpret_cast<dlsim::BatchTableHeader*>(base);
  auto* tasks = reinterpret_cast<dlsim::BatchTaskDesc*>(base + L.tasks_off);
  auto* map = reinterpret_cast<uint32_t*>(base + L.map_off);
  auto* ptrs = reinterpret_cast<const void**>(base + L.ptrs_off);
  auto* ws = reinterpret_cast<float*>(base + L.w_off);
  h->ntasks = static_cast<uint32_t>(b);
  h->nblocks = L.nblocks;
  h->vpt = static_cast<uint32_t>(L.vpt);
  h->tasks_off = L.tasks_off;
  h->map_off = L.map_off;
  h->ptrs_off = L.ptrs_off;
  h->w_off = L.w_off;
  // block order (k_wreduce_batch_table): the b ragged-end blocks, then every
  // task's full tiles; a task's block_start is one before its first full tile
  uint32_t blk = static_cast<uint32_t>(b), off = 0;
  bool uniform = true;
  for (int t = 0; t < b; ++t) {
    const size_t total = nelem[t] * Op::kBytes;
    if (fan_in[t] > DLSIM_MAX_FUSED_INPUTS || total > kMaxLaunchOutBytes || !aligned16(outs[t]))
      return fail(DLSIM_E_ARG, "task %d cannot be table-batched (fan-in <= %d, 16-B aligned, < 2 GiB)", t,
                  DLSIM_MAX_FUSED_INPUTS);
    const uint32_t nb = task_blocks<Op>(nelem[t], L.vpt);
    tasks[t].out = outs[t];
    tasks[t].nvec = nelem[t] / Op::E;
    tasks[t].nelem = nelem[t];
    tasks[t].block_start = blk - 1;
    tasks[t].ptr_off = off;
    tasks[t].fan_in = static_cast<uint32_t>(fan_in[t]);
    map[t] = static_cast<uint32_t>(t);  // its ragged end
    for (uint32_t k = 0; k + 1 < nb; ++k) map[blk + k] = static_cast<uint32_t>(t);
    for (int i = 0; i < fan_in[t]; ++i) {
      if (!aligned16(in[off + i]))
        return fail(DLSIM_E_ARG, "task %d input %d is not 16-byte aligned", t, i);
      ptrs[off + i] = in[off + i];
      ws[off + i] = w[off + i];
    }
    blk += nb - 1;
    off += static_cast<uint32_t>(fan_in[t]);
    uniform = uniform && fan_in[t] == fan_in[0];
  }
  h->uniform_fan_in = uniform ? static_cast<uint32_t>(fan_in[0]) : 0u;
  return DLSIM_OK;
}

template <class Op, int NF, int VPT>
hipError_t launch_table_nf(const void* d_table, uint32_t blocks, hipStream_t st) {
  hipLaunchKernelGGL((dlsim::k_wreduce_batch_table<Op, NF, group_size<Op>(), VPT, kNT, store_policy<Op>(),
                                                    kBatchWave<Op, VPT>>),
                     dim3(blocks), dim3(dlsim::kBlock), 0, st, static_cast<const unsigned char*>(d_table));
  return hipGetLastError();
}

template <class Op, int K, int VPT>
hipError_t launch_table_fixed(const void* d_table, int n, uint32_t blocks, hipStream_t st) {
  if constexpr (K > max_fixed_fan_in<Op>()) {
    return launch_table_nf<Op, 0, VPT>(d_table, blocks, st);
  } else {
    if (n == K) return launch_table_nf<Op, K, VPT>(d_table, blocks, st);
    return launch_table_fixed<Op, K + 1, VPT>(d_table, n, blocks, st);
  }
}

template <class Op>
int table_launch(const void* h_table, const void* d_table, hipStream_t st) {
  const auto* h = static_cast<const dlsim::BatchTableHeader*>(h_table);
  if (h->ntasks == 0) return DLSIM_OK;
  if (h->vpt != 1 && h->vpt != 4)
    return fail(DLSIM_E_ARG, "not a table written by dlsim_batch_table_fill (vectors per lane %u)", h->vpt);
  const int n = static_cast<int>(h->uniform_fan_in);
  hipError_t e;
  if (h->vpt == 1)
    e = n ? launch_table_fixed<Op, 1, 1>(d_table, n, h->nblocks, st) : launch_table_nf<Op, 0, 1>(d_table, h->nblocks, st);
  else
    e = n ? launch_table_fixed<Op, 1, 4>(d_table, n, h->nblocks, st) : launch_table_nf<Op, 0, 4>(d_table, h->nblocks, st);
  if (e != hipSuccess) return hip_fail(e, "table batch launch");
  return DLSIM_OK;
}


// ---- chunk mean in PyTorch's CPU order (chunk_mean_kernels.hpp) --------------
// First column that ATen's cascade_sum folds in row_sum (ilp) order, for an
// [m, n] fp32 reduction over dim 0 at `threads` intra-op threads
// (parallel_dim_reduction's column split, 32-column rounding; the 8-wide
// vectorized_outer_sum blocks of 32 columns; scalar_outer_sum's groups of 4
// under 8 columns). n == 1 is the inner reduction (all "ilp"/inner).
// esz / vw: the summed element's bytes and its Vectorized<> lanes (fp32 and
// the widened 16-bit types: 4 / 8; fp64: 8 / 4): ranges round to 128 B of
// columns, cascade blocks are 4 * vw columns, the vectorized path starts at
// vw columns (oracle/fedavg_oracle.c ilp_begin_gen).
inline size_t chunk_mean_ilp_begin(int m, size_t n, int threads, size_t esz = 4, size_t vw = 8) {
  if (n <= 1) return 0;
  const size_t rnd = 128 / esz;
  size_t b = 0, e = n;
  if (!(static_cast<unsigned long long>(m) * n < 32768ULL || threads <= 1)) {
    const size_t tp = static_cast<size_t>(threads) < n ? static_cast<size_t>(threads) : n;
    const size_t cs = (n + tp - 1) / tp;
    for (size_t t = 0; t < tp; ++t) {
      size_t tb = t * cs;
      if (tb >= n) break;
      size_t te = tb + cs < n ? tb + cs : n;
      tb -= tb % rnd;
      if (te != n) te -= te % rnd;
      if (tb < te) {
        b = tb;
        e = te;
      }
    }
  }
  const size_t s1 = e - b;
  return b + (s1 >= vw ? s1 / (4 * vw) * (4 * vw) : s1 / 4 * 4);
}

// Chunk mean tiles: VPT 4, wave map, 8 rows per load group (the kernel runs at
// its own memory-only probe from m = 6 up: profiles/r03_chunks_m/); a launch
// whose tasks all have m <= 6 contributors loads 4 rows per group instead:
// 26.5 against 29.3 us at m = 2, 36.2 against 38.0 at m = 4, 49.6 against
// 50.0 at m = 6 (ResNet-18 chunks, k = 10; RF 4 is slower from m = 7).
using CmDefault = dlsim::CmShape<4, true, 8>;
using CmFewRows = dlsim::CmShape<4, true, 4>;
constexpr int kCmFewRowsMax = 6;

// Deferred stores for the chunk means (dlsim::k_chunk_mean_defer, DESIGN.md
// §6b): fp32 launches of 16-B aligned tasks of m >= 16 contributors each, at
// least 20 MB per stream in all. ResNet-18 chunks, k = 10 (profiles/r05al_ab/,
// r05am/): m = 16 120.2 against 124.1 us; fewer contributors lose (m = 4
// 39.0 against 37.1, m = 10 80.8 against 78.5: the tiled kernel keeps more
// loads in flight per lane there, and U = 4 rows per group did not recover
// it). R: the fewest even rows per block with every row block of the launch
// resident at once beside the ragged blocks (up to 24 rows), else two rounds,
// else RMAX. DLSIM_CHUNK_DEFER=0 (read once): the tiled kernel;
// DLSIM_DEFER_R=r: that R.
constexpr int kCmDeferRMax = 32, kCmDeferU = kDeferU, kCmDeferMinRows = 16;
inline bool chunk_defer_on() {
  static const bool on = [] {
    const char* e = dlsim::ab_getenv("DLSIM_CHUNK_DEFER");
    return !(e && e[0] == '0');
  }();
  return on;
}
// DLSIM_CHUNK_DEFER_MIN_M=k (read once; A/B runs): defer from k contributors
inline int chunk_defer_min_m() {
  static const int k = [] {
    const char* e = dlsim::ab_getenv("DLSIM_CHUNK_DEFER_MIN_M");
    return e ? std::atoi(e) : kCmDeferMinRows;
  }();
  return k;
}
// Fixed-m deferral (dlsim::k_chunk_mean_defer_m, round 6): every task of the
// launch has the same m, 4 <= m < 16 (ResNet-18 chunks, k = 10, against the
// tiled kernel on one box, profiles/r06_chunk_ab6/: m = 4 36.7-36.8 against
// 37.8, m = 10 77.3 against 77.9, m = 15 110.9 against 112.8; m = 2 loses,
// 24.1 against 23.7). DLSIM_CHUNK_DEFER_FIXED=0 (read once; A/B runs, under
// DLSIM_AB=1): the tiled kernel there instead.
constexpr int kCmFixedMinM = 4, kCmFixedMaxM = 15;  // m = 2 measured slower than the tiled kernel (24.1 / 23.7 us)
inline bool chunk_defer_fixed_on() {
  static const bool on = [] {
    const char* e = dlsim::ab_getenv("DLSIM_CHUNK_DEFER_FIXED");
    return !(e && e[0] == '0');
  }();
  return on;
}
// results per lane beside MF x U loads, as the reduce's defer_rmax
constexpr int cm_defer_m_rmax(int mf) { return mf >= 12 ? 24 : kCmDeferRMax; }
// bpt: blocks of every task but the last when they are all equal (the
// kernel then maps a block to its task by a division), else 0 (a search).
template <class Op, int MF>
hipError_t launch_chunk_defer_m(const dlsim::ChunkMeanSlots& s, int m, int R, int bpt, unsigned grid,
                                hipStream_t st) {
  if constexpr (MF > kCmFixedMaxM || !std::is_same<Op, dlsim::F32Mean>::value) {
    return hipErrorInvalidValue;
  } else {
    if (m == MF) {
      hipLaunchKernelGGL((dlsim::k_chunk_mean_defer_m<Op, MF, cm_defer_m_rmax(MF), kCmDeferU>), dim3(grid),
                         dim3(dlsim::kDeferBlock), 0, st, bpt, s.ntasks, R, s);
      return hipGetLastError();
    }
    return launch_chunk_defer_m<Op, MF + 1>(s, m, R, bpt, grid, st);
  }
}
// R of the fixed-m form (k_chunk_mean_defer_m: no separate ragged blocks, at
// least one block per task): the fewest even rows per block with every block
// of the launch resident at once (up to 24 rows), else two rounds, else rmax.
inline size_t chunk_defer_m_blocks(size_t rows, size_t R) { return rows ? (rows + R - 1) / R : 1; }
inline int chunk_defer_m_rows(const std::vector<size_t>& rows, size_t cus, int rmax) {
  if (defer_r_override() > 0) return std::min(defer_r_override(), rmax);
  auto blocks = [&](size_t R) {
    size_t b = 0;
    for (size_t r : rows) b += chunk_defer_m_blocks(r, R);
    return b;
  };
  for (size_t R = 4; R <= static_cast<size_t>(std::min(rmax, kDeferOneRoundMax)); R += 2)
    if (blocks(R) <= cus) return static_cast<int>(R);
  for (size_t R = 4; R <= static_cast<size_t>(rmax); R += 2)
    if (blocks(R) <= 2 * cus) return static_cast<int>(R);
  return rmax;
}
inline int chunk_defer_rows(const std::vector<size_t>& rows, size_t cus, int rmax = kCmDeferRMax) {
  if (defer_r_override() > 0) return std::min(defer_r_override(), rmax);
  const size_t nt = rows.size();
  auto blocks = [&](size_t R) {
    size_t b = 0;
    for (size_t r : rows) b += (r + R - 1) / R;
    return b;
  };
  for (size_t R = 4; R <= static_cast<size_t>(std::min(rmax, kDeferOneRoundMax)); R += 2)
    if (blocks(R) + nt <= cus) return static_cast<int>(R);
  for (size_t R = 4; R <= static_cast<size_t>(rmax); R += 2)
    if (blocks(R) + nt <= 2 * cus) return static_cast<int>(R);
  return rmax;
}

template <class Op>
int run_chunk_mean(int b, const int* fan_in, const void* const* in, void* const* outs, const size_t* nelem,
                   int threads, hipStream_t st) {
  constexpr size_t tile = static_cast<size_t>(dlsim::kBlock) * CmDefault::VPT;
  std::vector<size_t> off(static_cast<size_t>(b) + 1, 0);
  for (int t = 0; t < b; ++t) off[t + 1] = off[t] + static_cast<size_t>(fan_in[t]);
  if (b > 1 && cross_task_overlap(b, fan_in, in, outs, nelem, Op::kBytes)) {
    // tasks touch each other's outputs: one launch per task, in order
    for (int t = 0; t < b; ++t) {
      int rc = run_chunk_mean<Op>(1, fan_in + t, in + off[t], outs + t, nelem + t, threads, st);
      if (rc != DLSIM_OK) return rc;
    }
    return DLSIM_OK;
  }
  auto task_flags = [&](int t) {
    bool vec = aligned16(outs[t]);
    for (int i = 0; i < fan_in[t] && vec; ++i) vec = aligned16(in[off[t] + i]);
    uint8_t f = vec ? dlsim::kCmVec : 0;
    if (nelem[t] == 1 && fan_in[t] >= dlsim::cm_lanes<Op>()) f |= dlsim::kCmInner;
    return f;
  };
  // Leading columns block 0 folds so the tiles start on a 128-B line (cm_task):
  // only when every input and the output share one misalignment (chunks cut
  // at the same offset of equally aligned rows, ChunkManager's layout) and the
  // task has whole tiles to align.
  auto task_head = [&](int t, size_t ib, uint8_t flags) -> uint32_t {
    if (!(flags & dlsim::kCmVec)) return 0;
    const uintptr_t mis = reinterpret_cast<uintptr_t>(outs[t]) & 127u;
    if (mis == 0) return 0;
    for (int i = 0; i < fan_in[t]; ++i)
      if ((reinterpret_cast<uintptr_t>(in[off[t] + i]) & 127u) != mis) return 0;
    const size_t h = (128u - mis) / Op::kBytes;  // mis is a multiple of 16: whole elements
    return ib >= h + 2 * tile * Op::E ? static_cast<uint32_t>(h) : 0u;
  };
  static_assert(128 / 2 <= dlsim::kCmTailCols, "a head fits block 0's scalar columns");
  auto task_blocks = [&](size_t ib, uint32_t head) { return (ib - head) / Op::E / tile + 1; };
  // RF by the call's largest contributor count (both shapes use VPT 4, so the
  // block layout is the same)
  int mmax = 0;
  for (int t = 0; t < b; ++t) mmax = fan_in[t] > mmax ? fan_in[t] : mmax;
  const bool few_rows = mmax <= kCmFewRowsMax;
  static_assert(CmFewRows::VPT == CmDefault::VPT, "one block layout for both tile shapes");
  // one launch's tasks (kernel-argument batch): index, ilp_begin, flags, head
  struct CmTask {
    int t;
    size_t ib;
    uint8_t flags;
    uint32_t head;
  };
  std::vector<CmTask> batch;
  int np = 0;
  size_t tiles = 0;  // the tiled kernel's grid for the batch so far
  auto flush = [&]() -> int {
    if (batch.empty()) return DLSIM_OK;
    dlsim::ChunkMeanSlots s;
    std::memset(&s, 0, sizeof(s));
    // deferred stores: fp32, every task vector-aligned with m >= 16 (or every
    // task with one m, 2 <= m < 16: the fixed-m form), >= 20 MB per stream
    bool defer = Op::kBytes == 4 && chunk_defer_on();
    bool fixed = std::is_same<Op, dlsim::F32Mean>::value && chunk_defer_on() && chunk_defer_fixed_on();
    const int m0 = fan_in[batch.front().t];
    size_t cols = 0;
    std::vector<size_t> rows;
    for (const CmTask& k : batch) {
      const bool vec = (k.flags & dlsim::kCmVec) != 0;
      defer = defer && vec && fan_in[k.t] >= chunk_defer_min_m();
      fixed = fixed && vec && fan_in[k.t] == m0;
      cols += nelem[k.t];
      rows.push_back((k.ib - k.head) / Op::E / dlsim::kDeferBlock);
    }
    fixed = fixed && m0 >= kCmFixedMinM && m0 <= kCmFixedMaxM && !defer;
    defer = (defer || fixed) && cols * Op::kBytes >= 20000000;
    fixed = fixed && defer;
    int R = 0;
    if (fixed)
      R = chunk_defer_m_rows(rows, static_cast<size_t>(device_cus()), cm_defer_m_rmax(m0));
    else if (defer)
      R = chunk_defer_rows(rows, static_cast<size_t>(device_cus()));
    size_t blocks = 0;
    int nt = 0, p = 0;
    for (const CmTask& k : batch) {
      const int m = fan_in[k.t];
      const size_t rt = rows[static_cast<size_t>(nt)];
      const size_t tb = fixed ? chunk_defer_m_blocks(rt, static_cast<size_t>(R))
                              : defer ? (rt + R - 1) / R + 1 : task_blocks(k.ib, k.head);
      // the fixed-m kernel: first block of task nt; the others: full blocks before it
      s.block_start[nt] = static_cast<uint32_t>(fixed ? blocks : blocks - static_cast<size_t>(nt));
      s.ptr_off[nt] = static_cast<uint32_t>(p);
      s.m[nt] = static_cast<uint32_t>(m);
      s.out[nt] = outs[k.t];
      s.nelem[nt] = nelem[k.t];
      s.ilp_begin[nt] = k.ib;
      s.flags[nt] = k.flags;
      s.head[nt] = k.head;
      for (int i = 0; i < m; ++i) s.p[p + i] = in[off[k.t] + i];
      p += m;
      blocks += tb;
      ++nt;
    }
    s.ntasks = nt;
    s.block_start[nt] = static_cast<uint32_t>(fixed ? blocks : blocks - static_cast<size_t>(nt));
    if (blocks > 0x7fffffffu) return fail(DLSIM_E_ARG, "chunk mean batch too large");
    if (defer) {
      if constexpr (Op::kBytes == 4) {
        const unsigned grid = static_cast<unsigned>(blocks);
        if (fixed) {
          int bpt = static_cast<int>(nt > 1 ? s.block_start[1] - s.block_start[0] : s.block_start[1]);
          for (int k = 1; bpt > 0 && k + 1 < nt; ++k)
            if (s.block_start[k + 1] - s.block_start[k] != static_cast<uint32_t>(bpt)) bpt = 0;
          const hipError_t e = launch_chunk_defer_m<Op, 2>(s, m0, R, bpt, grid, st);
          if (e != hipSuccess) return hip_fail(e, "chunk mean batch launch");
        } else if (few_rows)
          hipLaunchKernelGGL((dlsim::k_chunk_mean_defer<Op, CmFewRows::RF, kCmDeferRMax, kCmDeferU>), dim3(grid),
                             dim3(dlsim::kDeferBlock), 0, st, s, R);
        else
          hipLaunchKernelGGL((dlsim::k_chunk_mean_defer<Op, CmDefault::RF, kCmDeferRMax, kCmDeferU>), dim3(grid),
                             dim3(dlsim::kDeferBlock), 0, st, s, R);
      }
    } else if (few_rows) {
      hipLaunchKernelGGL((dlsim::k_chunk_mean_batch<Op, CmFewRows>), dim3(static_cast<unsigned>(blocks)),
                         dim3(dlsim::kBlock), 0, st, s);
    } else {
      hipLaunchKernelGGL((dlsim::k_chunk_mean_batch<Op, CmDefault>), dim3(static_cast<unsigned>(blocks)),
                         dim3(dlsim::kBlock), 0, st, s);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "chunk mean batch launch");
    batch.clear();
    np = 0;
    tiles = 0;
    return DLSIM_OK;
  };
  for (int t = 0; t < b; ++t) {
    const size_t n = nelem[t];
    if (n == 0) continue;
    const int m = fan_in[t];
    const size_t ib = chunk_mean_ilp_begin(m, n, threads, Op::kBytes == 8 ? 8 : 4, dlsim::cm_lanes<Op>());
    const uint8_t flags = task_flags(t);
    const uint32_t head = m > dlsim::kCmMaxPtrs ? 0u : task_head(t, ib, flags);
    const size_t tb = task_blocks(ib, head);
    if (m > dlsim::kCmMaxPtrs) {
      // input pointers through a stream-ordered device array (any m)
      void* d = nullptr;
      const size_t bytes = static_cast<size_t>(m) * sizeof(void*);
      hipError_t e = hipMallocAsync(&d, bytes, st);
      if (e != hipSuccess) return hip_fail(e, "chunk mean pointer table alloc");
      // pageable source: the copy is staged before the call returns
      e = hipMemcpyAsync(d, in + off[t], bytes, hipMemcpyHostToDevice, st);
      if (e == hipSuccess) {
        hipLaunchKernelGGL((dlsim::k_chunk_mean_table<Op, CmDefault>), dim3(static_cast<unsigned>(tb)),
                           dim3(dlsim::kBlock), 0, st, static_cast<const void* const*>(d), m, outs[t], n, ib,
                           flags);
        e = hipGetLastError();
      }
      hipError_t e2 = hipFreeAsync(d, st);
      if (e != hipSuccess) return hip_fail(e, "chunk mean table launch");
      if (e2 != hipSuccess) return hip_fail(e2, "chunk mean pointer table free");
      continue;
    }
    if (static_cast<int>(batch.size()) == dlsim::kCmMaxTasks || np + m > dlsim::kCmMaxPtrs ||
        tiles + tb > 0x7fffffffu) {
      int rc = flush();
      if (rc != DLSIM_OK) return rc;
    }
    batch.push_back({t, ib, flags, head});
    np += m;
    tiles += tb;
  }
  return flush();
}

}  // namespace dlsim_host

// ---- per-policy entry points, instantiated by the inst_*.hip units ----------------
#define DLSIM_REDUCE_ENTRIES(X, Op)                                                                      \
  X int dlsim_host::run<Op>(const void* const*, int, const float*, void*, size_t, hipStream_t, float);  \
  X int dlsim_host::run_batched<Op>(int, const int*, const void* const*, const float*, void* const*,    \
                                    const size_t*, hipStream_t, const float*);                          \
  X bool dlsim_host::table_layout<Op>(int, const int*, const size_t*, dlsim_host::TableLayout*);        \
  X int dlsim_host::table_fill<Op>(int, const int*, const void* const*, const float*, void* const*,     \
                                   const size_t*, void*, size_t);                                       \
  X int dlsim_host::table_launch<Op>(const void*, const void*, hipStream_t);
#define DLSIM_MEAN_ENTRIES(X, Op)                                                                        \
  X int dlsim_host::run<Op>(const void* const*, int, const float*, void*, size_t, hipStream_t, float);  \
  X int dlsim_host::run_batched<Op>(int, const int*, const void* const*, const float*, void* const*,    \
                                    const size_t*, hipStream_t, const float*);                          \
  X int dlsim_host::run_chunk_mean<Op>(int, const int*, const void* const*, void* const*, const size_t*, \
                                       int, hipStream_t);
#define DLSIM_PROBE_ENTRIES(X, Op) \
  X int dlsim_host::run<Op>(const void* const*, int, const float*, void*, size_t, hipStream_t, float);
#define DLSIM_F64_ENTRIES(X, Op) \
  X int dlsim_host::run<Op>(const void* const*, int, const double*, void*, size_t, hipStream_t, float);
#define DLSIM_CHUNK_ENTRIES(X, Op)                                                                       \
  X int dlsim_host::run_chunk_mean<Op>(int, const int*, const void* const*, void* const*, const size_t*, \
                                       int, hipStream_t);

// every policy's entries, with X = `extern template` (declare) or `template` (define)
#define DLSIM_ALL_ENTRIES(X)                  \
  DLSIM_REDUCE_ENTRIES(X, dlsim::F32Exact)    \
  DLSIM_REDUCE_ENTRIES(X, dlsim::F32Fast)     \
  DLSIM_REDUCE_ENTRIES(X, dlsim::BF16Exact)   \
  DLSIM_REDUCE_ENTRIES(X, dlsim::BF16Fast)    \
  DLSIM_REDUCE_ENTRIES(X, dlsim::F16Exact)    \
  DLSIM_REDUCE_ENTRIES(X, dlsim::F16Fast)     \
  DLSIM_MEAN_ENTRIES(X, dlsim::F32Mean)       \
  DLSIM_MEAN_ENTRIES(X, dlsim::BF16Mean)      \
  DLSIM_MEAN_ENTRIES(X, dlsim::F16Mean)       \
  DLSIM_PROBE_ENTRIES(X, dlsim::XorProbe<4>)  \
  DLSIM_PROBE_ENTRIES(X, dlsim::XorProbe<2>)  \
  DLSIM_F64_ENTRIES(X, dlsim::F64Exact)       \
  DLSIM_F64_ENTRIES(X, dlsim::F64Fast)        \
  DLSIM_CHUNK_ENTRIES(X, dlsim::F64Mean)
