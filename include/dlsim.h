/*
 * dlsim.h — C ABI of the MI355X-native aggregation hot path.
 *
 * The reference (sacs-epfl/decentralized-learning-simulator) has no native
 * code: its hot path is the Python/PyTorch-CPU loop of
 *   dasklearn/gradient_aggregation/fedavg.py:12-26   FedAvg.aggregate(models, weights)
 * reached through
 *   dasklearn/model_manager.py:41-43                  ModelManager.aggregate_trained_models
 *   dasklearn/functions.py:89-106                     aggregate(settings, params)  (the "aggregate" task)
 *   dasklearn/worker.py:27-31                         globals()[func_name](settings, data)
 * Every entry point below replaces one piece of that loop; the Python host
 * package (dasklearn_amd) binds them with ctypes, and INTEGRATION.md shows the
 * binding a maintainer adds to the reference.
 *
 * Conventions
 *   - Plain pointers and sizes only. Device buffers are caller-owned
 *     (hipMalloc / torch CUDA tensors); host arrays (weights, pointer lists,
 *     sizes) are read during the call and may be freed when it returns.
 *   - Calls that take a `stream` (a hipStream_t, NULL = legacy default
 *     stream) are stream-ordered and asynchronous: they enqueue work and
 *     return; nothing synchronises the device.
 *   - Return value: 0 on success, a negative DLSIM_E* code otherwise;
 *     dlsim_last_error() gives a message (thread-local).
 *   - No global state besides a per-thread error string and the host pack
 *     thread pool of the host entry points (created on first use, idle
 *     between calls).
 */
#ifndef DLSIM_H_
#define DLSIM_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- element types and summation modes ---------------------------------- */
enum dlsim_dtype {
  DLSIM_F32 = 0,  /* IEEE binary32                                      */
  DLSIM_BF16 = 1, /* bfloat16 (upper 16 bits of binary32), RNE rounding  */
  DLSIM_F16 = 2,  /* IEEE binary16, RNE rounding                        */
  DLSIM_F64 = 3   /* IEEE binary64: dlsim_wreduce_f64 (double weights) and
                     the chunk means (dlsim_chunk_mean_batched,
                     dlsim_host_chunk_mean) only */
};

enum dlsim_mode {
  /* Bit-identical to FedAvg.aggregate (fedavg.py:20-25) on the same inputs:
   *   acc = x0 * 0;  for i in 0..n-1: acc = acc + fl32(w_i) * x_i
   * in that order, multiply and add rounded separately (no FMA); for bf16
   * and f16 the product and every partial sum are rounded to the element
   * type (PyTorch's CPU opmath semantics). NaN payloads are not part of the
   * contract. */
  DLSIM_EXACT = 0,
  /* Fused multiply-add, fp32 accumulation (bf16/f16: one final rounding).
   * Within n * 2^-23 relative (fp32) of EXACT; not bit-identical. */
  DLSIM_FAST = 1
};

/* ---- error codes --------------------------------------------------------- */
#define DLSIM_OK 0
#define DLSIM_E_ARG (-1)      /* null pointer, n < 1, overlapping out/in, ... */
#define DLSIM_E_DTYPE (-2)    /* dtype not in enum dlsim_dtype                */
#define DLSIM_E_MODE (-3)     /* mode not in enum dlsim_mode                  */
#define DLSIM_E_RCCL (-4)     /* RCCL not bound, or an RCCL call failed       */
#define DLSIM_E_PEER (-5)     /* another rank of the communicator failed its
                                 checks (dlsim_wreduce_sharded's agreement)   */
#define DLSIM_E_DISAGREE (-6) /* the ranks of a communicator passed different
                                 n_elems / fan-in / dtype / gather (agreement) */

/* How the sharded entry points materialise the whole output on every rank. */
enum dlsim_gather {
  DLSIM_GATHER_NONE = 0,      /* each rank keeps its own slice only            */
  DLSIM_GATHER_BCAST = 1,     /* every rank broadcasts its slice in place in
                                 d_out: W ncclBroadcast in one group            */
  DLSIM_GATHER_ALLGATHER = 2  /* one in-place ncclAllGather of equal-width
                                 (padded) segments in a scratch buffer, then one
                                 kernel moves them to their offsets in d_out;
                                 at most 64 ranks                               */
};
#define DLSIM_E_HIP (-100)    /* a HIP call failed: code = -100 - hipError_t  */

/* Fan-in carried in kernel arguments. Larger n (any n >= 1) reads its
 * pointer/weight table from a small device buffer the call allocates and
 * uploads on `stream` (hipMallocAsync / hipMemcpyAsync / hipFreeAsync; do not
 * capture such a call in a graph). Either way the reduce is ONE pass: every
 * output element is written once, after all n of its terms are folded. */
#define DLSIM_MAX_FUSED_INPUTS 128

/*
 * dlsim_wreduce — N-way weighted element-wise reduce of flat buffers.
 *
 *   d_out[j] = sum_{i=0..n-1} h_weights[i] * d_inputs[i][j],  j < n_elems
 *
 * Replaces the N x T loop of FedAvg.aggregate (fedavg.py:20-25) for one flat
 * parameter arena (all of a model's parameters() concatenated in order).
 *   d_inputs   host array of n device pointers (each n_elems elements of dtype)
 *   h_weights  host array of n fp32 weights (already rounded to fp32 — the
 *              reference's `w * p1` converts its Python float with RNE,
 *              fedavg.py:25); uniform 1/n is the caller's job (fedavg.py:14-15)
 *   d_out      device buffer of n_elems. It may BE an input (d_out ==
 *              d_inputs[i], any i: an in-place update; every term of an
 *              element is read before the element is written); any other
 *              overlap with an input is rejected (DLSIM_E_ARG)
 *   stream     hipStream_t
 * Any alignment is accepted; 16-byte-aligned buffers take the vector path.
 */
int dlsim_wreduce(const void* const* d_inputs, int n, const float* h_weights,
                  void* d_out, size_t n_elems, int dtype, int mode,
                  void* stream);

/*
 * dlsim_wreduce_f64 — dlsim_wreduce for fp64 (double) parameters.
 *
 * For a double model the reference's `w * p1` (fedavg.py:25) keeps the
 * Python-float weight exact as a double scalar, so the weights here are
 * doubles (no fp32 rounding), and every product and partial sum is rounded to
 * double, in input order, without FMA (DLSIM_EXACT; DLSIM_FAST is an fma
 * chain). Same buffer, aliasing, fan-in and stream rules as dlsim_wreduce.
 * The other entry points take float weights and reject DLSIM_F64.
 */
int dlsim_wreduce_f64(const void* const* d_inputs, int n, const double* h_weights, void* d_out, size_t n_elems,
                      int mode, void* stream);

/*
 * dlsim_wreduce_tensors — the same reduce over T separate tensors per model,
 * without packing them into an arena first: tensor k of every model is one
 * task of a batch (dlsim_wreduce_batched), so T tensors take a few launches.
 *
 * Replaces the inner `zip(center_model.parameters(), m.parameters())` loop
 * (fedavg.py:24-25) when the models' parameters already live on the device
 * as separate tensors (e.g. a device-resident model cache).
 *   d_inputs   host array of n*t device pointers, model-major:
 *              d_inputs[i*t + k] = tensor k of model i
 *   numels     host array of t element counts
 *   d_outs     host array of t device pointers (outputs)
 * Same weights, dtype and mode rules as dlsim_wreduce.
 */
int dlsim_wreduce_tensors(const void* const* d_inputs, int n, int t,
                          const size_t* numels, const float* h_weights,
                          void* const* d_outs, int dtype, int mode,
                          void* stream);

/*
 * dlsim_wreduce_batched — b independent weighted reduces (e.g. the aggregate
 * tasks of one simulated round, one per peer) in as few kernel launches as
 * possible.
 *
 * Task t has fan_in[t] inputs: d_inputs[o_t .. o_t + fan_in[t]) with weights
 * h_weights[o_t ..], o_t = fan_in[0] + ... + fan_in[t-1]; it writes
 * n_elems[t] elements to d_outs[t]. Every task follows dlsim_wreduce's rules
 * and rounding, and the results are bit-identical to b separate dlsim_wreduce
 * calls made in task order, also when tasks depend on each other: if any
 * task's output overlaps another task's input or output (task 1 reads what
 * task 0 writes), the tasks run one launch each, in order; otherwise up to
 * 32 tasks / 192 inputs share one launch and tasks with fan-in > 16 run
 * alone. Replaces b separate `aggregate` tasks scheduled by the broker
 * (broker.py:261-275 -> functions.py:89-106).
 */
int dlsim_wreduce_batched(int b, const int* fan_in, const void* const* d_inputs,
                          const float* h_weights, void* const* d_outs, const size_t* n_elems,
                          int dtype, int mode, void* stream);

/*
 * Descriptor-table batches: any number of tasks per launch.
 *
 * The kernel-argument form above carries at most 32 tasks / 192 inputs per
 * launch. For a whole round (hundreds of peers) the task descriptors go to a
 * caller-owned device buffer instead:
 *   dlsim_batch_table_bytes   size of the table for these tasks
 *   dlsim_batch_table_fill    write it into caller host memory h_table
 *                             (every task: fan-in <= 128, 16-B aligned
 *                             buffers, output < 2 GiB, and no task's output
 *                             overlapping another task's input or output —
 *                             the launch runs all tasks concurrently; else
 *                             DLSIM_E_ARG)
 *   (caller copies h_table to d_table, e.g. hipMemcpyAsync on `stream`)
 *   dlsim_batch_table_launch  one launch over every task; reads the grid size
 *                             from h_table and the descriptors from d_table
 * A filled table can be launched again as long as the buffers it names are
 * alive (a prepared round; graph-capturable: no allocation, no sync).
 * Results are bit-identical to separate dlsim_wreduce calls.
 */
int dlsim_batch_table_bytes(int b, const int* fan_in, const size_t* n_elems, int dtype,
                            size_t* bytes);
int dlsim_batch_table_fill(int b, const int* fan_in, const void* const* d_inputs,
                           const float* h_weights, void* const* d_outs, const size_t* n_elems,
                           int dtype, void* h_table, size_t table_bytes);
int dlsim_batch_table_launch(const void* h_table, const void* d_table, int dtype, int mode,
                             void* stream);

/*
 * dlsim_mean — element-wise mean of n flat buffers (no weights).
 *
 *   d_out[j] = (0 + d_inputs[0][j] + ... + d_inputs[n-1][j]) / n
 *
 * Replaces `torch.mean(torch.stack(chunks_at_idx), dim=0)` of
 * ChunkManager.reconstruct_model (simulation/conflux/chunk_manager.py:38-40),
 * which PyTorch computes as a sum over dim 0 followed by div_(n): here the
 * sum is folded in input order from +0 in fp32 and divided once (IEEE
 * division); bf16/f16 inputs are summed in fp32, divided and rounded once,
 * for every n. PyTorch's own CPU order (cascade_sum) is
 * dlsim_chunk_mean_batched; this input-order mean is off the reference path.
 * Same buffer and stream rules as dlsim_wreduce.
 */
int dlsim_mean(const void* const* d_inputs, int n, void* d_out, size_t n_elems, int dtype,
               void* stream);

/*
 * dlsim_mean_batched — b independent dlsim_mean calls in as few launches as
 * possible (the kernel-argument batches of dlsim_wreduce_batched, with a
 * per-task divisor): task t averages fan_in[t] buffers d_inputs[o_t ..
 * o_t + fan_in[t]) into d_outs[t] (n_elems[t] elements), o_t the prefix sum
 * of fan_in. Replaces the per-chunk-index loop of
 * ChunkManager.reconstruct_model (simulation/conflux/chunk_manager.py:38-40):
 * every chunk index of one reconstruction (or of many) in one launch.
 * Results are bit-identical to b separate dlsim_mean calls in task order
 * (cross-task overlaps are ordered as in dlsim_wreduce_batched).
 */
int dlsim_mean_batched(int b, const int* fan_in, const void* const* d_inputs, void* const* d_outs,
                       const size_t* n_elems, int dtype, void* stream);

/*
 * dlsim_chunk_mean_batched — b chunk means, each bit-identical to the
 * reference's CPU `torch.mean(torch.stack(chunks), dim=0)`
 * (simulation/conflux/chunk_manager.py:38-40) as PyTorch computes it at
 * `cpu_threads` intra-op threads (the worker's settings.torch_threads,
 * broker.py:31; torch.get_num_threads() in the calling process). Task t
 * averages fan_in[t] buffers d_inputs[o_t .. o_t + fan_in[t]) (o_t the prefix
 * sum of fan_in) into d_outs[t] (n_elems[t] elements, < 2 GiB). The order is
 * ATen's cascade_sum (chunk_mean_kernels.hpp); bf16 chunks are summed in
 * fp32, divided and rounded once; DLSIM_F64 chunks are summed and divided in
 * double in PyTorch's double order (Vectorized<double>'s 4 lanes: 16-column
 * blocks and rounding). Any fan-in up to 65535: up to 192 inputs
 * per launch travel as kernel arguments, larger ones through a stream-ordered
 * device array (hipMallocAsync / hipFreeAsync on `stream`). Tasks whose
 * outputs overlap another task's buffers run one launch each, in order.
 * Replaces the per-index loop of ChunkManager.reconstruct_model.
 */
int dlsim_chunk_mean_batched(int b, const int* fan_in, const void* const* d_inputs, void* const* d_outs,
                             const size_t* n_elems, int dtype, int cpu_threads, void* stream);

/*
 * dlsim_chunk_mean_ilp_begin — the first column of an [m, n_elems] chunk
 * stack that PyTorch's CPU sum folds in its row_sum order at cpu_threads
 * threads (host logic, no GPU; exposed for tests).
 */
size_t dlsim_chunk_mean_ilp_begin(int m, size_t n_elems, int cpu_threads);

/*
 * dlsim_rccl_bind — dlopen the RCCL library whose communicators will be
 * passed to dlsim_wreduce_sharded (the library does not link RCCL, so a
 * process keeps one RCCL instance: from PyTorch, torch/lib/librccl.so, whose
 * communicator ProcessGroupNCCL._comm_ptr() returns). Idempotent.
 */
int dlsim_rccl_bind(const char* librccl_path);

/*
 * dlsim_wreduce_sharded — the parameter-sharded aggregate across the ranks of
 * an RCCL communicator (one process per GPU, xGMI). SURVEY.md §8b's
 * `dlsim_wreduce_sharded(..., rcclComm)`; no reference counterpart (the
 * reference is single-process CPU, fedavg.py:12-26).
 * COST: every call agrees with its peers first (an all-reduce read back by
 * the host), so every call is a host round trip (81 us at W = 2 on the stub
 * communicator against 12 us for a plan run). For repeated
 * aggregates of one shape -- the steady state of a simulation -- create a
 * plan once (dlsim_sharded_plan_create, below) and run it
 * (dlsim_sharded_plan_run): stream-ordered, no agreement, no host wait.
 *   rank r of W (from the communicator) owns elements [b_r, e_r) =
 *   dlsim_shard_range(n_elems, W, r, 64); d_slices[i] points at that slice of
 *   model i (slice_elems elements, which must equal e_r - b_r, else
 *   DLSIM_E_ARG); d_out is a full n_elems buffer, and the
 *   exact reduce of the slices lands at d_out + b_r. gather (enum
 *   dlsim_gather; 1 = DLSIM_GATHER_BCAST for callers that pass a bool):
 *   every rank ends with the whole output, through grouped in-place
 *   broadcasts or one padded all-gather plus an unpad kernel, on `stream`.
 *   Each element's N terms stay on one GPU in input order: results are
 *   bit-identical to dlsim_wreduce on one GPU, with either gather.
 *   Errors are collective when W > 1: the rank-local checks (slice length,
 *   pointers, dtype, fan-in, weights, gather) and the local reduce's launch
 *   run first, then every rank joins one agreement all-reduce (int64 MAX of a
 *   failure slot per rank plus n_elems, dtype and gather, on `stream`, read
 *   back by the host: the call waits for the stream once). A rank whose own
 *   checks failed returns its own error; every other rank returns
 *   DLSIM_E_PEER naming the failed ranks, or DLSIM_E_DISAGREE if the ranks
 *   disagree on n_elems, dtype or gather; in both cases no rank enters the
 *   gather, so none is left waiting in it. Only a failure before the
 *   communicator can be queried (RCCL not bound, null communicator) is
 *   rank-local. For repeated aggregates of one shape, a plan
 *   (dlsim_sharded_plan_create) agrees once and skips the per-call
 *   agreement and its host wait.
 */
int dlsim_wreduce_sharded(const void* const* d_slices, size_t slice_elems, int n, const float* h_weights,
                          void* d_out, size_t n_elems, int dtype, int mode, void* rccl_comm, int gather,
                          void* stream);

/*
 * dlsim_wreduce_sharded_f64 — dlsim_wreduce_sharded for fp64 (double)
 * parameters: double weights and the arithmetic of dlsim_wreduce_f64 (a
 * double model's `w * p1` keeps the Python float exact, fedavg.py:25), the
 * gather in ncclFloat64. The agreement step is the same one, with
 * dtype DLSIM_F64, so ranks that call the fp32/bf16/fp16 entry with the same
 * communicator are told of the disagreement instead of left waiting.
 */
int dlsim_wreduce_sharded_f64(const void* const* d_slices, size_t slice_elems, int n, const double* h_weights,
                              void* d_out, size_t n_elems, int mode, void* rccl_comm, int gather, void* stream);

/*
 * dlsim_sharded_plan — dlsim_wreduce_sharded for a repeated shape, without
 * the per-call agreement.
 *
 * dlsim_sharded_plan_create is COLLECTIVE: every rank of the communicator
 * calls it with its own arguments; the ranks agree once on n_elems, the
 * fan-in n, dtype (DLSIM_F32/BF16/F16/F64) and gather (enum dlsim_gather), in
 * one int64 MAX all-reduce read back by the host, as dlsim_wreduce_sharded
 * does. A rank whose own checks failed gets its error, the others
 * DLSIM_E_PEER or DLSIM_E_DISAGREE, and *plan stays NULL on every rank.
 * DLSIM_GATHER_ALLGATHER plans own their padded segment buffer
 * (W x ceil64(max slice) elements, hipMalloc).
 *
 * dlsim_sharded_plan_run[_f64] reduces this rank's slices (dlsim_shard_range
 * of the plan's n_elems, n models; d_slices and h_weights must hold exactly
 * the plan's n entries: the run has no fan-in argument and reads n of each;
 * slice_elems must equal e_r - b_r) into
 * d_out + b_r (a full n_elems buffer) and runs the plan's gather:
 * stream-ordered, no host wait, no agreement. Every rank must run
 * the same sequence of plans, as with any collective. A rank whose local
 * checks or launch fail (null or overlapping pointers, mode, the f64 entry
 * on a non-f64 plan) still enters the plan's gather, so no peer is left
 * waiting, and returns its error. It sends its slice as all-ones bytes, a NaN
 * in every supported format, through a stand-in buffer when d_out is NULL.
 * Its peers get no error code, but that slice of their output is NaN, never
 * stale numbers. Agree again (dlsim_wreduce_sharded, or a new plan) when a
 * peer must learn of the failure.
 *
 * dlsim_sharded_plan_destroy frees the plan (rank-local; NULL is a no-op).
 * Plans are not thread-safe: one caller per plan at a time.
 */
typedef struct dlsim_sharded_plan dlsim_sharded_plan;

int dlsim_sharded_plan_create(void* rccl_comm, size_t n_elems, int n, int dtype, int gather, void* stream,
                              dlsim_sharded_plan** plan);
int dlsim_sharded_plan_run(dlsim_sharded_plan* plan, const void* const* d_slices, size_t slice_elems,
                           const float* h_weights, void* d_out, int mode, void* stream);
int dlsim_sharded_plan_run_f64(dlsim_sharded_plan* plan, const void* const* d_slices, size_t slice_elems,
                               const double* h_weights, void* d_out, int mode, void* stream);
int dlsim_sharded_plan_destroy(dlsim_sharded_plan* plan);

/*
 * dlsim_host_wreduce — the aggregate of N *host* models (the reference's own
 * case: CPU modules, fedavg.py:20-25 run by functions.py:89-106), staged
 * through pinned memory and reduced on the device, as one pipeline.
 *
 *   h_srcs[i * t + k]  host pointer of tensor k of model i (contiguous,
 *                      numels[k] elements of dtype; any alignment)
 *   h_staging, d_rows  n rows of row_stride elements each, page-locked host
 *                      memory and device memory; 16-B aligned, row_stride a
 *                      multiple of 8 elements, >= sum(numels)
 *   d_out              device result, sum(numels) elements: the exact or fast
 *                      reduce of the concatenated models (dlsim_wreduce rules)
 *   h_out              page-locked host copy of the result, or NULL
 *   chunk_elems        pipeline chunk of the parameter axis (rounded up to a
 *                      multiple of 1024; 0 = one chunk)
 *   threads            host threads packing the staging rows (the caller's
 *                      own thread included; <= 1: the caller's thread only)
 *   stream             the reduce; h2d_stream / d2h_stream the copies (may be
 *                      `stream` itself or NULL = `stream`; with one chunk
 *                      the copies go on `stream`, as there is nothing to
 *                      overlap)
 * Model i's share of chunk c is packed (memcpy, several threads) into its
 * staging row and copied H2D on h2d_stream as soon as it is packed; once
 * every model's share of chunk c is on the device, the chunk is reduced on
 * `stream` and (h_out) copied back on d2h_stream, while later chunks are
 * still being packed and copied. Returns after the pack and the queueing:
 * the copies and kernels are stream-ordered and asynchronous, `stream` is
 * ordered after all of them (synchronise it before reading h_out), and the
 * staging buffers must not be reused before then. Results are bit-identical
 * to dlsim_wreduce over the packed rows.
 */
int dlsim_host_wreduce(int n, int t, const void* const* h_srcs, const size_t* numels,
                       const float* h_weights, void* h_staging, void* d_rows, size_t row_stride,
                       void* d_out, void* h_out, int dtype, int mode, size_t chunk_elems, int threads,
                       void* stream, void* h2d_stream, void* d2h_stream);

/*
 * dlsim_host_wreduce_zc — dlsim_host_wreduce for SMALL host models with no
 * DMA in either direction (round 5): the models are
 * packed into page-locked staging rows on `threads` host threads as above,
 * then the reduce kernel reads those rows in place over PCIe and writes the
 * result straight into h_out. h_staging (n rows of row_stride elements,
 * 16-B aligned, row_stride a multiple of 8 and >= sum(numels)) and h_out
 * (sum(numels) elements) must be page-locked memory the device maps
 * (hipHostMalloc, torch's pin_memory); anything else is refused with
 * DLSIM_E_ARG before any launch. Below 1 MiB of rows: one launch after the
 * pack. From 1 MiB: the parameter range is cut into up to 8 chunks (at least
 * 128 KiB per model each; DLSIM_AB=1 DLSIM_ZC_CHUNK_KB=k for A/B runs), and
 * each chunk's launch is queued as soon as its rows are packed, so the PCIe
 * reads of chunk c overlap the pack of chunk c + 1. Returns after queueing
 * the last launch: synchronise `stream` before reading h_out or reusing the
 * rows. Results are bit-identical to dlsim_wreduce over the packed rows.
 * The library sets no size cap: the caller chooses when to use it (the
 * package routes tasks of up to 4 MiB of rows here, arena.py ZC_MAX_BYTES;
 * for a 2 x GNLeNet task, 683 KB of rows, the kernel's PCIe reads cost less
 * than the two DMAs' setup); larger models are better served
 * by dlsim_host_wreduce.
 */
int dlsim_host_wreduce_zc(int n, int t, const void* const* h_srcs, const size_t* numels, const float* h_weights,
                          void* h_staging, size_t row_stride, void* h_out, int dtype, int mode, int threads,
                          void* stream);

/*
 * dlsim_host_wreduce_resident — dlsim_host_wreduce when some models are
 * already on the device (a per-worker cache of host models it has uploaded
 * before, dasklearn_amd/device_cache.py).
 *   resident[i] != 0  d_rows[i] already holds model i (sum(numels) elements)
 *   resident[i] == 0  model i's tensors h_srcs[i * t + k] are packed into
 *                     staging row j (the j-th such model; rows of
 *                     staging_stride elements, page-locked, 16-B aligned)
 *                     and sent to d_rows[i], which keeps them for later calls
 * then the reduce of d_rows[0..n) into d_out (dlsim_wreduce rules, input
 * order i) and, if h_out, the D2H of the result; one chunk, all on `stream`,
 * asynchronous (h_out page-locked). Device rows must not overlap d_out; a
 * non-resident model's row must not overlap any other row (resident rows may
 * alias each other: the same model twice). Consecutive non-resident models whose device rows lie one staging stride
 * apart go H2D in runs of >= 1 MiB (DLSIM_H2D_MIN_KB).
 */
int dlsim_host_wreduce_resident(int n, int t, const void* const* h_srcs, const size_t* numels,
                                const float* h_weights, const int* resident, void* const* d_rows, void* h_staging,
                                size_t staging_stride, void* d_out, void* h_out, int dtype, int mode, int threads,
                                void* stream);

/*
 * dlsim_host_chunk_mean — dlsim_chunk_mean_batched for *host* chunks (the
 * reference's case: ChunkManager.reconstruct_model over chunks received from
 * peers, chunk_manager.py:38-40), staged and pipelined like
 * dlsim_host_wreduce.
 *   h_inputs       the host chunks, task by task (fan_in[t] each, n_elems[t]
 *                  elements; contiguous, any alignment)
 *   h_staging,     page-locked host / device staging of staging_elems
 *   d_staging      elements, 16-B aligned; the library puts input row r at a
 *                  256-B aligned offset, so staging_elems must be at least
 *                  sum_t fan_in[t] * round_up(n_elems[t], 256 / sizeof(elem))
 *   d_outs[t]      device mean of task t (16-B aligned for the vector path)
 *   h_outs         NULL, or per task a page-locked host destination (or NULL)
 * Rows are packed on `threads` host threads; each row goes H2D as soon as it
 * is packed, each task's mean runs on `stream` once its rows are on the
 * device (in PyTorch's CPU order at cpu_threads, as dlsim_chunk_mean_batched),
 * and its result goes back on d2h_stream (with b == 1 every copy goes on
 * `stream`). Returns after packing and queueing; `stream` is ordered after
 * everything.
 */
int dlsim_host_chunk_mean(int b, const int* fan_in, const void* const* h_inputs, const size_t* n_elems,
                          void* h_staging, void* d_staging, size_t staging_elems, void* const* d_outs,
                          void* const* h_outs, int dtype, int cpu_threads, int threads, void* stream,
                          void* h2d_stream, void* d2h_stream);

/*
 * dlsim_host_pack — host-only gather: copy t host buffers (h_srcs[j],
 * nbytes[j] bytes) to h_dst + dst_off[j] on `threads` host threads (the
 * caller's included), with the pack of dlsim_host_wreduce (streaming stores).
 * Synchronous; no GPU call. Used to stage many host models for one H2D (the
 * round executor's upload of a wave's host-trained models; worker.py:24 ->
 * functions.py:89-106 receive them as CPU modules).
 */
int dlsim_host_pack(int t, const void* const* h_srcs, const size_t* nbytes, const size_t* dst_off, void* h_dst,
                    int threads);

/*
 * dlsim_shard_range — parameter-axis partition used by the sharded path.
 *
 * Splits [0, n_elems) into `world` contiguous slices whose boundaries are
 * multiples of `align_elems` (except the end) and writes rank's slice to
 * [*begin, *end). Every rank of a job must call it with the same arguments
 * so shard boundaries agree. Host-only; no device work.
 * (New: the reference has no multi-device path)
 */
int dlsim_shard_range(size_t n_elems, int world, int rank, size_t align_elems,
                      size_t* begin, size_t* end);

/*
 * dlsim_probe_pattern — memory-only probe of dlsim_wreduce's access pattern:
 * the same dispatch for these buffers (kernel, launch shape, fan-in form,
 * load and store policies) with the weighted fold replaced by a bitwise XOR
 * of the inputs (n = 1: a bit-exact copy). Its time is what the memory
 * system allows for exactly the reduce's read/write mix; bench.py times the
 * reduce against it. dtype DLSIM_F32, DLSIM_BF16 or DLSIM_F16 (16-bit types
 * share one probe); same buffer and stream rules as dlsim_wreduce.
 */
int dlsim_probe_pattern(const void* const* d_inputs, int n, void* d_out, size_t n_elems, int dtype,
                        void* stream);

/*
 * dlsim_wreduce_mixed — one output parameter whose inputs differ in dtype
 * (fedavg.py:20-25 when a model's parameter at this position has another
 * dtype than models[0]'s). d_out has out_dtype, which is
 * input 0's (models[0] defines c1). d_out = input 0 * 0, then per input i in
 * order the reference's `c1.add_(w_i * p1)` with torch's type promotion: the
 * product in dtypes[i] (float(w_i) * x rounded to fp32 and then to dtypes[i]
 * for DLSIM_F32 / BF16 / F16, the exact double w_i times x for DLSIM_F64), the
 * add in the promoted dtype (fp32 for any pair of fp32 / bf16 / fp16, fp64
 * with a double on either side), cast back into out_dtype as c10 casts (a
 * double to bf16 / fp16 goes through float). h_weights are the Python-float
 * weights as doubles. Exact only; one element per lane (a rare path), in
 * passes of 32 inputs for larger n, so the output must not overlap any input.
 * Bit-exact to the reference (tests/golden/mixed_*.npz). Stream-ordered.
 */
int dlsim_wreduce_mixed(const void* const* d_inputs, const int* dtypes, int n, const double* h_weights,
                        void* d_out, int out_dtype, size_t n_elems, void* stream);

/*
 * dlsim_device_alloc / dlsim_device_free — device memory for long-lived
 * large buffers (staging rows, resident model blocks) on the calling
 * thread's current device. flags DLSIM_ALLOC_CONTIGUOUS asks the driver for
 * physically contiguous memory (hipExtMallocWithFlags with
 * hipDeviceMallocContiguous): the HBM channel and page placement of a
 * buffer's rows is then the same in every process (DESIGN.md §5b measured
 * 1-3 % between allocations of the default kind). If the driver cannot
 * provide it, the call falls back to hipMalloc and sets *contiguous = 0.
 * dlsim_device_free synchronises the device (hipFree): for buffers that
 * live long, not per call. (New: the reference allocates nothing on a GPU.)
 */
#define DLSIM_ALLOC_CONTIGUOUS 1
int dlsim_device_alloc(size_t nbytes, int flags, void** d_out, int* contiguous);
int dlsim_device_free(void* d_ptr);

/*
 * dlsim_pool_alloc / dlsim_pool_free — the same physically contiguous
 * blocks, in the signature of a PyTorch pluggable allocator
 * (torch.cuda.memory.CUDAPluggableAllocator: alloc(size, device, stream),
 * free(ptr, size, device, stream)). dasklearn_amd hands them to a
 * torch.cuda.MemPool and allocates large aggregate outputs inside it
 * (arena.OUTPUT_POOL), so torch's caching allocator owns the blocks:
 * Tensor.record_stream, torch.cuda.memory_allocated / memory_reserved,
 * per-stream reuse and the pool's release all behave as for any torch
 * tensor. Blocks are 2 MiB-aligned;
 * a request the driver cannot serve contiguously falls back to hipMalloc;
 * out of memory returns NULL (torch then frees its cache and retries, or
 * raises its OutOfMemoryError). Called by torch's allocator with `device`
 * current; `stream` is unused (the caching allocator orders reuse).
 * dlsim_pool_stats: segments made contiguous, made by the fallback, and the
 * bytes the pool's segments hold now (any argument may be NULL).
 */
void* dlsim_pool_alloc(size_t nbytes, int device, void* stream);
void dlsim_pool_free(void* d_ptr, size_t nbytes, int device, void* stream);
void dlsim_pool_stats(unsigned long long* contiguous, unsigned long long* fallback, unsigned long long* live_bytes);

/*
 * dlsim_kernel_name — the kernel dlsim_wreduce (mode DLSIM_EXACT or
 * DLSIM_FAST) or dlsim_mean (mode -1) launches for n 16-byte-aligned inputs
 * of n_elems elements of dtype on the current device: "dlsim::k_wreduce_defer"
 * (fp32, n >= 3, >= 10 MB per stream; for 11 <= n <= 14 from 8.4 M elements),
 * "dlsim::k_wreduce_tiles" otherwise (misaligned buffers take
 * "dlsim::k_wreduce_scalar"), "" for no launch (n_elems == 0) or bad
 * arguments. A static string, for profilers and benches that look a kernel up
 * by name. (New: no reference counterpart.)
 */
const char* dlsim_kernel_name(int n, size_t n_elems, int dtype, int mode);

/* Message for the last failing call on this thread ("" if none). */
const char* dlsim_last_error(void);

/* ABI version: (major << 16) | minor. */
int dlsim_version(void);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* DLSIM_H_ */
