// chunk_mean_kernels.hpp — gfx950 kernels for the chunk mean of the chunked
// algorithms (Conflux/Shatter): torch.mean(torch.stack(chunks), dim=0) per
// chunk index (reference simulation/conflux/chunk_manager.py:38-40), computed
// in PyTorch's own CPU summation order so the result is bit-identical to the
// reference's worker at settings.torch_threads threads (broker.py:31).
//
// PyTorch's CPU mean is a sum over dim 0 followed by one division (a bf16
// input is summed in fp32, divided, and rounded once). The sum is ATen's
// cascade_sum; the host (dlsim_abi.hip, chunk_mean_ilp_begin) classifies the
// columns of a chunk into two orders, restated in oracle/fedavg_oracle.c and
// pinned against torch.mean (tests/test_chunk_mean_order.py):
//
//   cascade  columns [0, ilp_begin): multi_row_sum — rows folded in order
//            into a level-0 accumulator from +0; after every 16 rows the
//            level-0 sum is added into level 1 (and level 1 into level 2
//            every 256 rows, ...); at the end level 0 + level 1 + ...
//   ilp      columns [ilp_begin, n) (< 32 of them): row_sum — four
//            interleaved cascades over rows k, k+4, k+8, ... (k = 0..3), the
//            m mod 4 remaining rows added to the first, then
//            ((p0 + p1) + p2) + p3;
//   inner    a one-element chunk with m >= 8 (vectorized_inner_sum): eight
//            lanes l, each the ilp order over rows l, l+8, ...; the m mod 8
//            remaining rows summed from +0, then the eight lanes added in turn.
//
// fp64 chunks (F64Mean) run the same orders in double with Vectorized<double>'s
// 4 lanes: 16-column cascade blocks and rounding, the inner order from m >= 4.
//
// Layout of the work: every chunk index is one task of a batched grid (the
// kernel-argument batches of k_wreduce_batch). The cascade columns stream in
// tiles of 256 lanes x VPT 16-byte vectors, one lane folding its elements'
// m terms in registers in row order (no cross-lane step: the order is per
// element). Block 0 of a task — dispatched first — takes the task's ragged
// end: the partial tile, then the < 40 scalar columns (the cascade columns
// past the last whole vector and the ilp/inner columns), whose rows it stages
// through LDS 64 at a time so one thread per column folds them at LDS speed.
#pragma once

#include <type_traits>

#include "wreduce_kernels.hpp"

#pragma clang fp contract(off)

namespace dlsim {

// Output stores of the chunk means: buffer stores with the nt bit for 4/8-byte
// elements (round 5; sc1 before, measured with outputs that stayed in the
// Infinity Cache, as the reduce's), global nt for 2-byte.
template <class Op> inline constexpr int kCmStore = Op::kBytes >= 4 ? 2 : kStNT;


constexpr int kCmMaxTasks = 32;
constexpr int kCmMaxPtrs = 192;
constexpr int kCmTailRows = 64;  // rows staged per LDS round in block 0
constexpr int kCmTailCols = 64;  // scalar columns of a task (< E + 32)

enum : uint8_t { kCmVec = 1, kCmInner = 2 };

// Per-task fields are 32-bit or wider (round 6): a block reads its task's
// fields at a run-time index, and 8- or 16-bit fields there compiled to
// vector global loads (scalar loads read whole dwords) on the path from the
// block's start to its first input load.
struct ChunkMeanSlots {
  const void* p[kCmMaxPtrs];
  void* out[kCmMaxTasks];
  size_t nelem[kCmMaxTasks];
  size_t ilp_begin[kCmMaxTasks];
  uint32_t block_start[kCmMaxTasks + 1];  // first full tile of each task (k_chunk_mean_batch)
  uint32_t ptr_off[kCmMaxTasks];
  uint32_t m[kCmMaxTasks];
  uint32_t flags[kCmMaxTasks];
  uint32_t head[kCmMaxTasks];  // leading columns folded by block 0 (see cm_task)
  int ntasks;
};

// The task of block-start entry f: the last t with block_start[t] <= f (the
// entries are non-decreasing over the ntasks tasks). A count over a
// compile-time range: the entries load with a few wide scalar loads and the
// compares are scalar ALU work, where a `while` scan waited on one dependent
// load per task passed (round 6: ~0.3 us each, on every block's start).
__device__ __forceinline__ int cm_find_task(const ChunkMeanSlots& s, uint32_t f) {
  int t = 0;
#pragma unroll
  for (int j = 1; j < kCmMaxTasks; ++j) t += (j < s.ntasks && f >= s.block_start[j]) ? 1 : 0;
  return t;
}

struct PtrArgs {
  const void* const* p;
  __device__ const void* ptr(int i) const { return p[i]; }
};

// The same inputs `off` bytes further on (the cascade tiles of a task whose
// leading columns are peeled off, cm_task).
template <class A>
struct ShiftArgs {
  A a;
  size_t off;
  __device__ const void* ptr(int i) const { return static_cast<const char*>(a.ptr(i)) + off; }
};

// The add of the cascade tiles: `a + b`, or for the memory-only probe
// (XorProbe, csrc/tune_wreduce.hip's chunk-mean pattern ceiling) its pinned
// XOR, so the probe runs exactly this dispatch with the arithmetic removed.
template <class Op> struct CmIsProbe : std::false_type {};
template <int B> struct CmIsProbe<XorProbe<B>> : std::true_type {};
template <class Op, class T>
__device__ __forceinline__ T cm_add(T a, T b) {
  if constexpr (CmIsProbe<Op>::value) return Op::step(a, 0.0f, b);
  else return a + b;
}

// Lanes of ATen's Vectorized<acc> in the sum kernel (the inner order and the
// column blocks): 8 floats, 4 doubles.
template <class Op> constexpr int cm_lanes() { return Op::kBytes == 8 ? 4 : 8; }

// One element's cascade (multi_row_sum with 16-value blocks and 4 levels),
// in the accumulator type T (float; double for fp64 chunks).
template <class T>
struct CascadeSum {
  T a[4];
  __device__ void init() { a[0] = a[1] = a[2] = a[3] = T(0); }
  // value number i (0-based) of the sequence, in order
  __device__ void add(long long i, T x) {
    a[0] = a[0] + x;
    if (((i + 1) & 15) == 0) flush(i + 1);
  }
  __device__ void flush(long long i) {
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      a[l] = a[l] + a[l - 1];
      a[l - 1] = T(0);
      if ((i & (15LL << (4 * l))) != 0) break;
    }
  }
  __device__ T result() const { return ((a[0] + a[1]) + a[2]) + a[3]; }
};

// One element's row_sum (ilp) order over a sequence of `len` values.
template <class T>
struct IlpSum {
  T a[4][4];  // [level][k]
  T p[4];
  long long s;    // values per interleaved cascade (len / 4)
  bool done;
  __device__ void init(long long len) {
    s = len / 4;
    done = false;
#pragma unroll
    for (int l = 0; l < 4; ++l)
#pragma unroll
      for (int k = 0; k < 4; ++k) a[l][k] = T(0);
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = T(0);
  }
  __device__ void add(long long idx, T x) {
    if (idx < 4 * s) {
      const int k = static_cast<int>(idx & 3);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)  // constant indices: the state stays in VGPRs
        if (kk == k) a[0][kk] = a[0][kk] + x;
      const long long i = (idx >> 2) + 1;  // groups of 4 completed
      if (k == 3 && (i & 15) == 0) {
#pragma unroll
        for (int l = 1; l < 4; ++l) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            a[l][kk] = a[l][kk] + a[l - 1][kk];
            a[l - 1][kk] = T(0);
          }
          if ((i & (15LL << (4 * l))) != 0) break;
        }
      }
    } else {
      if (!done) finish();
      p[0] = p[0] + x;
    }
  }
  __device__ void finish() {
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] = ((a[0][k] + a[1][k]) + a[2][k]) + a[3][k];
    done = true;
  }
  __device__ T result() {
    if (!done) finish();
    return ((p[0] + p[1]) + p[2]) + p[3];
  }
};

// Raw 16-byte slot of E elements from a buffer of unknown alignment (scalar
// loads; elements at or past `lim` read as 0).
template <class Op>
__device__ __forceinline__ u32x4 ld_slot_scalar(const void* base, size_t v, size_t lim) {
  u32x4 r = {0u, 0u, 0u, 0u};
  const size_t j0 = v * Op::E;
  if constexpr (Op::kBytes == 8) {
    const uint64_t* q = static_cast<const uint64_t*>(base);
#pragma unroll
    for (int e = 0; e < 2; ++e)
      if (j0 + e < lim) {
        r[2 * e] = static_cast<uint32_t>(q[j0 + e]);
        r[2 * e + 1] = static_cast<uint32_t>(q[j0 + e] >> 32);
      }
  } else if constexpr (Op::kBytes == 4) {
    const uint32_t* q = static_cast<const uint32_t*>(base);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (j0 + e < lim) r[e] = q[j0 + e];
  } else {
    const uint16_t* q = static_cast<const uint16_t*>(base);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (j0 + e < lim) r[e >> 1] |= static_cast<uint32_t>(q[j0 + e]) << (16 * (e & 1));
  }
  return r;
}

// Launch shape of the cascade tiles: VPT 16-byte slots per lane, lane map
// (WAVE: lane l of wave w owns slots w*64*VPT + l + k*64; else l' + k*256),
// RF rows loaded per group before they are folded (RF divides 16).
template <int VPT_, bool WAVE_, int RF_>
struct CmShape {
  static constexpr int VPT = VPT_;
  static constexpr bool WAVE = WAVE_;
  static constexpr int RF = RF_;
  static constexpr int VS = WAVE_ ? 64 : kBlock;  // slot stride of one lane
  __device__ static size_t lane_off() {
    return WAVE_ ? (threadIdx.x >> 6) * 64 * VPT_ + (threadIdx.x & 63) : threadIdx.x;
  }
};

// Cascade fold of m rows for the VPT slots v0 + k*VS of one lane.
// LV: accumulator levels in use (2 while m < 256, else 4).
// VEC: 16-B aligned task (vector loads, buffer stores); else scalar access.
template <class Op, class A, class SH, int LV, bool VEC, bool CHECK>
__device__ __forceinline__ void cm_tile(const A& a, int m, const OutRef& o, size_t v0, size_t nvec,
                                        size_t ncol, float div) {
  constexpr int VPT = SH::VPT, RF = SH::RF;
  using T = acc_t<Op>;
  T acc[LV][VPT][Op::E];
#pragma unroll
  for (int l = 0; l < LV; ++l)
#pragma unroll
    for (int v = 0; v < VPT; ++v)
#pragma unroll
      for (int e = 0; e < Op::E; ++e) acc[l][v][e] = T(0);
  for (int i0 = 0; i0 < m; i0 += 16) {
    const int cnt = m - i0 < 16 ? m - i0 : 16;
#pragma unroll
    for (int h = 0; h < 16; h += RF) {
      if (h < cnt) {
        u32x4 r[RF][VPT];
#pragma unroll
        for (int g = 0; g < RF; ++g) {
          if (h + g < cnt) {
            const void* src = a.ptr(i0 + h + g);
#pragma unroll
            for (int v = 0; v < VPT; ++v) {
              const size_t idx = v0 + static_cast<size_t>(v) * SH::VS;
              if constexpr (VEC) {
                if (!CHECK || idx < nvec) r[g][v] = ld16<1>(src, idx);
                else r[g][v] = u32x4{0u, 0u, 0u, 0u};
              } else {
                r[g][v] = (!CHECK || idx < nvec) ? ld_slot_scalar<Op>(src, idx, ncol) : u32x4{0u, 0u, 0u, 0u};
              }
            }
          }
        }
#pragma unroll
        for (int g = 0; g < RF; ++g) {
          if (h + g < cnt) {
#pragma unroll
            for (int v = 0; v < VPT; ++v) {
              T x[Op::E];
              unpack<Op>(r[g][v], x);
#pragma unroll
              for (int e = 0; e < Op::E; ++e) acc[0][v][e] = cm_add<Op>(acc[0][v][e], x[e]);
            }
          }
        }
      }
    }
    if (cnt == 16) {
      const int i = i0 + 16;
#pragma unroll
      for (int l = 1; l < LV; ++l) {
#pragma unroll
        for (int v = 0; v < VPT; ++v)
#pragma unroll
          for (int e = 0; e < Op::E; ++e) {
            acc[l][v][e] = cm_add<Op>(acc[l][v][e], acc[l - 1][v][e]);
            acc[l - 1][v][e] = T(0);
          }
        if ((i & (15 << (4 * l))) != 0) break;
      }
    }
  }
#pragma unroll
  for (int l = 1; l < LV; ++l)
#pragma unroll
    for (int v = 0; v < VPT; ++v)
#pragma unroll
      for (int e = 0; e < Op::E; ++e) acc[0][v][e] = cm_add<Op>(acc[0][v][e], acc[l][v][e]);
#pragma unroll
  for (int v = 0; v < VPT; ++v) {
    const size_t idx = v0 + static_cast<size_t>(v) * SH::VS;
    if (CHECK && idx >= nvec) continue;
    if constexpr (VEC) {
      store_vec<kCmStore<Op>>(o, idx, pack<Op>(acc[0][v], div));
    } else {
#pragma unroll
      for (int e = 0; e < Op::E; ++e) {
        const size_t j = idx * Op::E + e;
        if (j < ncol) store_elem<Op>(o.ptr, j, acc[0][v][e], div);
      }
    }
  }
}

// Block 0 of a task: the scalar columns [c0, n) — cascade order below
// ilp_begin, ilp order from it (or the inner order for a one-element chunk) —
// staged through LDS TR rows at a time (kCmTailRows, halved for 8-byte
// elements so the stage is 16 KiB for every policy: the static LDS of this
// function is reserved by every block of k_chunk_mean_batch).
template <class Op, class A>
__device__ __forceinline__ void cm_scalar_cols(const A& a, int m, void* out, size_t c0, size_t n,
                                               size_t ilp_begin, bool inner, float div) {
  using T = acc_t<Op>;
  constexpr int VW = cm_lanes<Op>();
  constexpr int TR = kCmTailRows * 4 / static_cast<int>(sizeof(T));
  static_assert(TR * kCmTailCols * sizeof(T) == 16384, "16 KiB tail stage");
  __shared__ T st[TR][kCmTailCols];
  const int W = static_cast<int>(n - c0);  // block-uniform, <= kCmTailCols
  const int tid = threadIdx.x;
  const size_t col = c0 + static_cast<size_t>(tid);
  const bool is_ilp = col >= ilp_begin;
  const long long vs = m / VW;  // inner: VW-lane vectors
  CascadeSum<T> cs;
  IlpSum<T> il;
  cs.init();
  il.init(inner ? vs : m);
  T fin = T(0);  // inner: the m mod VW trailing rows, from +0
  for (int r0 = 0; r0 < m; r0 += TR) {
    const int rc = m - r0 < TR ? m - r0 : TR;
    for (int idx = tid; idx < rc * W; idx += kBlock) {
      const int row = idx / W, c = idx - row * W;
      st[row][c] = load_elem<Op>(a.ptr(r0 + row), c0 + static_cast<size_t>(c));
    }
    __syncthreads();
    if (!inner) {
      if (tid < W) {
        for (int rr = 0; rr < rc; ++rr) {
          const T x = st[rr][tid];
          if (is_ilp) il.add(r0 + rr, x);
          else cs.add(r0 + rr, x);
        }
      }
    } else if (tid < VW) {
      for (int rr = 0; rr < rc; ++rr) {
        const long long i = r0 + rr;
        if (i < VW * vs && (i % VW) == tid) il.add(i / VW, st[rr][0]);
        if (tid == 0 && i >= VW * vs) fin = fin + st[rr][0];
      }
    }
    __syncthreads();
  }
  if (!inner) {
    if (tid < W) store_elem<Op>(out, col, is_ilp ? il.result() : cs.result(), div);
    return;
  }
  if (tid < VW) st[0][tid] = il.result();
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int l = 0; l < VW; ++l) fin = fin + st[0][l];
    store_elem<Op>(out, 0, fin, div);
  }
}

// One task's share of the grid: local block 0 does the ragged end, local
// block b >= 1 the full tile b - 1 of the cascade columns.
// `head` (< kCmTailCols, below ilp_begin) leading columns are folded by block
// 0 too, so that the tiles start on a 128-B line of every input and of the
// output: a chunk of a flat model starts wherever P / k puts it, and tiles
// laid from a misaligned start straddle lines (+1.2-1.4 % HBM traffic at
// ResNet-18 chunks, profiles/r03s3_chunk_pmc/). Every column keeps its own
// order (the cascade order does not depend on where a column sits).
template <class Op, class A, class SH, int LV>
__device__ __forceinline__ void cm_task(const A& a, int m, void* out, size_t n, size_t ilp_begin,
                                        uint8_t flags, uint32_t local, uint32_t head) {
  const float div = static_cast<float>(m);
  const size_t hb = static_cast<size_t>(head) * Op::kBytes;
  const ShiftArgs<A> sa{a, hb};
  const size_t nvec = (ilp_begin - head) / Op::E;  // whole vectors of cascade columns past the head
  constexpr size_t kTile = static_cast<size_t>(kBlock) * SH::VPT;
  const size_t full = nvec / kTile;
  const bool vec = (flags & kCmVec) != 0;
  const OutRef o = make_out<kCmStore<Op>>(static_cast<char*>(out) + hb, vec ? nvec : 0);
  const size_t ncol = ilp_begin - head;
  if (local == 0) {
    if (full * kTile < nvec) {  // the partial tile, block map (bounds-checked)
      using PT = CmShape<SH::VPT, false, SH::RF>;
      if (vec) cm_tile<Op, ShiftArgs<A>, PT, LV, true, true>(sa, m, o, full * kTile + threadIdx.x, nvec, ncol, div);
      else cm_tile<Op, ShiftArgs<A>, PT, LV, false, true>(sa, m, o, full * kTile + threadIdx.x, nvec, ncol, div);
    }
    if (head > 0) cm_scalar_cols<Op, A>(a, m, out, 0, head, ilp_begin, false, div);
    const size_t c0 = head + nvec * Op::E;
    if (c0 < n) cm_scalar_cols<Op, A>(a, m, out, c0, n, ilp_begin, (flags & kCmInner) != 0, div);
    return;
  }
  const size_t v0 = static_cast<size_t>(local - 1) * kTile + SH::lane_off();
  if (vec) cm_tile<Op, ShiftArgs<A>, SH, LV, true, false>(sa, m, o, v0, nvec, ncol, div);
  else cm_tile<Op, ShiftArgs<A>, SH, LV, false, false>(sa, m, o, v0, nvec, ncol, div);
}

// Kernel-argument batch: up to kCmMaxTasks tasks, kCmMaxPtrs inputs (so
// m < 256 and two accumulator levels suffice). Blocks 0 .. ntasks-1 are the
// tasks' ragged-end blocks (local block 0: a few dependent round trips), so
// all of them are dispatched first and finish under the full tiles instead of
// one of them trailing the grid; block ntasks + f is full tile f of the
// concatenated tasks (block_start: each task's first full tile).
template <class Op, class SH>
__global__ __launch_bounds__(kBlock) void k_chunk_mean_batch(const ChunkMeanSlots s) {
  const uint32_t bid = blockIdx.x;
  int t = 0;
  uint32_t local = 0;
  if (bid < static_cast<uint32_t>(s.ntasks)) {
    t = static_cast<int>(bid);
  } else {
    const uint32_t f = bid - static_cast<uint32_t>(s.ntasks);
    t = cm_find_task(s, f);
    local = f - s.block_start[t] + 1;
  }
  const PtrArgs a{s.p + s.ptr_off[t]};
  cm_task<Op, PtrArgs, SH, 2>(a, s.m[t], s.out[t], s.nelem[t], s.ilp_begin[t], s.flags[t], local, s.head[t]);
}

// One task whose input pointers live in device memory (any m).
template <class Op, class SH>
__global__ __launch_bounds__(kBlock) void k_chunk_mean_table(const void* const* __restrict__ ptrs, int m,
                                                             void* out, size_t n, size_t ilp_begin,
                                                             uint8_t flags) {
  const PtrArgs a{ptrs};
  cm_task<Op, PtrArgs, SH, 4>(a, m, out, n, ilp_begin, flags, blockIdx.x, 0);
}

// ---- deferred stores (round 5; the reduce's k_wreduce_defer) ----
// The cascade columns of every task cut into rows of kDeferBlock vectors; a
// 512-lane block folds up to R rows of one task (lane t: vector t of each
// row), keeps the packed means in registers and stores them together. The
// order per element is cm_tile's: rows of contributors folded in order into
// level 0 from +0, level 0 into level 1 after every 16, the levels summed at
// the end, one division.
//
// U rows' vectors v0 + u * kDeferBlock (a row past R re-reads row v0's,
// already in flight) over the m contributors, RF at a time.
template <class Op, class A, int RF, int U>
__device__ __forceinline__ void cm_rows_fold(const A& a, int m, size_t v0, int r0, int R, float div,
                                             u32x4 (&res)[U]) {
  using T = acc_t<Op>;
  T acc[2][U][Op::E];
#pragma unroll
  for (int l = 0; l < 2; ++l)
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int e = 0; e < Op::E; ++e) acc[l][u][e] = T(0);
  for (int i0 = 0; i0 < m; i0 += 16) {
    const int cnt = m - i0 < 16 ? m - i0 : 16;
#pragma unroll
    for (int h = 0; h < 16; h += RF) {
      if (h < cnt) {
        u32x4 r[RF][U];
#pragma unroll
        for (int g = 0; g < RF; ++g) {
          if (h + g < cnt) {
            const void* src = a.ptr(i0 + h + g);
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int row = r0 + u < R ? r0 + u : r0;
              r[g][u] = ld16<1>(src, v0 + static_cast<size_t>(row) * kDeferBlock);
            }
          }
        }
#pragma unroll
        for (int g = 0; g < RF; ++g) {
          if (h + g < cnt) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
              T x[Op::E];
              unpack<Op>(r[g][u], x);
#pragma unroll
              for (int e = 0; e < Op::E; ++e) acc[0][u][e] = cm_add<Op>(acc[0][u][e], x[e]);
            }
          }
        }
      }
    }
    if (cnt == 16) {  // m < 256 (kernel-argument batches): two levels
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < Op::E; ++e) {
          acc[1][u][e] = cm_add<Op>(acc[1][u][e], acc[0][u][e]);
          acc[0][u][e] = T(0);
        }
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
#pragma unroll
    for (int e = 0; e < Op::E; ++e) acc[0][u][e] = cm_add<Op>(acc[0][u][e], acc[1][u][e]);
    res[u] = pack<Op>(acc[0][u], div);
  }
}

// Kernel-argument batch of 16-B aligned tasks (kCmVec), m < 256: blocks
// 0 .. ntasks-1 are the tasks' ragged blocks (the partial row, the head and
// the scalar columns, on the first 256 lanes as cm_task's block 0 does them);
// block ntasks + f is row block f of the concatenated tasks (block_start),
// rows [j * R, min((j + 1) * R, rows of the task)) of its task.
template <class Op, int RF, int RMAX, int U>
__global__ __launch_bounds__(kDeferBlock) void k_chunk_mean_defer(const ChunkMeanSlots s, int R) {
  const uint32_t bid = blockIdx.x;
  int t = 0;
  uint32_t local = 0;
  if (bid < static_cast<uint32_t>(s.ntasks)) {
    t = static_cast<int>(bid);
  } else {
    const uint32_t f = bid - static_cast<uint32_t>(s.ntasks);
    t = cm_find_task(s, f);
    local = f - s.block_start[t] + 1;
  }
  const PtrArgs a{s.p + s.ptr_off[t]};
  const int m = s.m[t];
  const size_t n = s.nelem[t], ilp_begin = s.ilp_begin[t];
  const uint32_t head = s.head[t];
  const float div = static_cast<float>(m);
  const size_t hb = static_cast<size_t>(head) * Op::kBytes;
  const ShiftArgs<PtrArgs> sa{a, hb};
  const size_t nvec = (ilp_begin - head) / Op::E;
  const size_t rows = nvec / kDeferBlock;
  const OutRef o = make_out<kCmStore<Op>>(static_cast<char*>(s.out[t]) + hb, nvec);
  if (local == 0) {
    if (threadIdx.x >= kBlock) return;  // whole waves 4-7: the barriers below count the rest
    if (rows * kDeferBlock < nvec) {  // the partial row: 256 lanes x 2 vectors, bounds-checked
      using PT = CmShape<kDeferBlock / kBlock, false, RF>;
      cm_tile<Op, ShiftArgs<PtrArgs>, PT, 2, true, true>(sa, m, o, rows * kDeferBlock + threadIdx.x, nvec,
                                                         ilp_begin - head, div);
    }
    if (head > 0) cm_scalar_cols<Op, PtrArgs>(a, m, s.out[t], 0, head, ilp_begin, false, div);
    const size_t c0 = head + nvec * Op::E;
    if (c0 < n) cm_scalar_cols<Op, PtrArgs>(a, m, s.out[t], c0, n, ilp_begin, (s.flags[t] & kCmInner) != 0, div);
    return;
  }
  const size_t first = static_cast<size_t>(local - 1) * static_cast<size_t>(R);
  const int Rb = static_cast<int>(rows - first < static_cast<size_t>(R) ? rows - first : static_cast<size_t>(R));
  const size_t v0 = first * kDeferBlock + threadIdx.x;
  u32x4 res[RMAX];
#pragma unroll
  for (int r0 = 0; r0 < RMAX; r0 += U) {
    if (r0 < Rb) {
      u32x4 ru[U];
      cm_rows_fold<Op, ShiftArgs<PtrArgs>, RF, U>(sa, m, v0, r0, Rb, div, ru);
#pragma unroll
      for (int u = 0; u < U; ++u) res[r0 + u] = ru[u];
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int r = 0; r < RMAX; ++r)
    if (r < Rb) store_vec<kCmStore<Op>>(o, v0 + static_cast<size_t>(r) * kDeferBlock, res[r]);
}

// Fixed contributor count MF < 16 for every task of the launch (round 6;
// VERDICT r05 next #3). Conflux rebuilds every chunk index from the same m
// peers, and below 16 contributors the cascade is its level 0 alone: rows
// folded in order from +0, the (zero) upper levels added, one division --
// cm_rows_fold's order for m < 16. With MF known at compile time the U rows
// of all MF contributors load back to back and fold straight-line (the
// reduce's fixed fan-in form, defer_rows), and the stores run unguarded: a row
// past the block's count goes to vector nvec, past the task's output range,
// which the buffer store drops.
// Layout: task t owns blocks [block_start[t], block_start[t + 1]), at least
// one; block j of the task folds rows [j * R, min((j + 1) * R, rows)), and
// the task's LAST block then also does its ragged end (the partial row, the
// head and the scalar columns, on its first 256 lanes as cm_task's block 0).
// No block is spent on ragged ends alone: k_chunk_mean_defer's separate
// ragged blocks pushed Conflux's ten ResNet-18 chunks from R = 22 to 24 rows
// per block to fit one round (38.8 against 37.5 us tiled at m = 4,
// profiles/r06_chunk_ab/); here R = 22 fits, the reduce's grid.
// MF input pointers and the divisor in registers, as a reduce slot set
// (ptr / wt / divisor) for defer_rows
template <int MF>
struct FixedPtrs {
  const void* p[MF];
  float div;
  __device__ const void* ptr(int i) const { return p[i]; }
  __device__ float wt(int) const { return 1.0f; }
  __device__ float divisor() const { return div; }
};

//
// The scalars come first: they are preloaded into SGPRs at wave launch
// (-mllvm -amdgpu-kernarg-preload-count, __graft_entry__.HIP_FLAGS), so with
// bpt > 0 (every task but the last has bpt blocks; the host checks) a block
// finds its task with no load at all, and its first loads are its task's
// fields and pointers. Every deferred block of the launch starts at once, so
// each dependent load before the first input load is on the kernel's
// critical path (round 6: one task of 4 x 11.2 M, 36.9 against 35.3-35.6 us
// for dlsim_mean's deferred kernel on the same rows, profiles/r06_cvr/).
template <class Op, int MF, int RMAX, int U>
__global__ __launch_bounds__(kDeferBlock) void k_chunk_mean_defer_m(int bpt, int nt, int R, const ChunkMeanSlots s) {
  static_assert(MF >= 1 && MF < 16, "level 0 only");
  static_assert(std::is_same<Op, F32Mean>::value, "the input-order mean's fold is the cascade's below 16 rows");
  const uint32_t bid = blockIdx.x;
  const int t = bpt > 0 ? min(static_cast<int>(bid / static_cast<uint32_t>(bpt)), nt - 1) : cm_find_task(s, bid);
  const uint32_t local = bid - s.block_start[t];
  const bool last = bid + 1 == s.block_start[t + 1];
  const PtrArgs a{s.p + t * MF};  // every task has MF inputs, packed in task order (ptr_off[t] == t * MF)
  const size_t n = s.nelem[t], ilp_begin = s.ilp_begin[t];
  const uint32_t head = s.head[t];
  const float div = static_cast<float>(MF);
  const size_t hb = static_cast<size_t>(head) * Op::kBytes;
  const ShiftArgs<PtrArgs> sa{a, hb};
  const size_t nvec = (ilp_begin - head) / Op::E;
  const size_t rows = nvec / kDeferBlock;
  const OutRef o = make_out<kCmStore<Op>>(static_cast<char*>(s.out[t]) + hb, nvec);
  const size_t first = static_cast<size_t>(local) * static_cast<size_t>(R);
  const int Rb = first >= rows ? 0
                               : static_cast<int>(rows - first < static_cast<size_t>(R) ? rows - first
                                                                                        : static_cast<size_t>(R));
  const size_t v0 = first * kDeferBlock + threadIdx.x;
  // Below 16 contributors the cascade columns' order is the input-order
  // mean's (F32Mean: from +0, in order, one division; the level-1 add of +0
  // changes no bit), so the rows run the reduce's own deferred fold,
  // defer_rows, on the task's pointers held in registers.
  FixedPtrs<MF> fp;
#pragma unroll
  for (int i = 0; i < MF; ++i) fp.p[i] = sa.ptr(i);
  fp.div = div;
  defer_rows<Op, FixedPtrs<MF>, MF, 8, RMAX, U, kCmStore<Op>>(fp, MF, o, v0, Rb, nvec);
  if (!last || threadIdx.x >= kBlock) return;  // whole waves 4-7: the barriers below count the rest
  if (rows * kDeferBlock < nvec) {  // the partial row: 256 lanes x 2 vectors, bounds-checked
    using PT = CmShape<kDeferBlock / kBlock, false, (MF <= 6 ? 4 : 8)>;  // dispatch.hpp CmFewRows / CmDefault RF
    cm_tile<Op, ShiftArgs<PtrArgs>, PT, 2, true, true>(sa, MF, o, rows * kDeferBlock + threadIdx.x, nvec,
                                                       ilp_begin - head, div);
  }
  if (head > 0) cm_scalar_cols<Op, PtrArgs>(a, MF, s.out[t], 0, head, ilp_begin, false, div);
  const size_t c0 = head + nvec * Op::E;
  if (c0 < n) cm_scalar_cols<Op, PtrArgs>(a, MF, s.out[t], c0, n, ilp_begin, (s.flags[t] & kCmInner) != 0, div);
}

}  // namespace dlsim
