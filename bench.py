"""bench.py — device-resident GB/s of the N-way weighted model-tensor reduce.

Metric (BASELINE.json): "device-resident GB/s, N-way weighted model-tensor
reduce; 1/2/4/8 MI355X". A step is one aggregate: one launch of the fused HIP
reduce over N flat parameter arenas already resident in HBM (the arithmetic of
FedAvg.aggregate, dasklearn/gradient_aggregation/fedavg.py:12-26).

Workload (default, --config north_star): 8 models x 11,181,642 fp32 params
(ResNet-18/CIFAR-10 size), Dirichlet(1) weights, DLSIM_EXACT (bit-identical to
the reference).

Multi-GPU (one process per GPU). `python bench.py --gpus N` spawns its N rank
processes itself (fresh interpreters started before anything touches the GPU,
127.0.0.1 rendezvous); under torchrun the ranks come from the environment
instead. The default is STRONG scaling of the named config: the parameter axis
of the same aggregate is split into N contiguous 64-element-aligned slices
(dlsim_shard_range), rank r reduces slice r of all N models with no data-path
collective. `value` = the config's bytes x K / the max over ranks of each
rank's HIP-event time around its K launches; the barriers that line the ranks
up sit outside that window. The line carries the speed-up over the same
config on one GPU (rank 0 times it alone, same K, same timing) and, in their
own fields, the RCCL all-gather that would materialise the full output and
the C ABI's sharded entry points (local reduce + grouped in-place broadcasts
or a padded all-gather, agreed per call or once through a plan).
--weak instead gives every rank the config's full parameter count.

Bytes per step per rank = (N_models + 1) * P_rank * sizeof(dtype) (read N,
write 1). Input sets rotate, with enough sets that their footprint is >= 1 GiB,
so the 256 MiB Infinity Cache cannot serve re-reads (small slices included).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME] [--weak]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(ROOT, "decentralized-learning-simulator_amd")
for _p in (ROOT, PKG_ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (importing torch does not initialise the GPU)
import torch.distributed as dist  # noqa: E402

METRIC = "device-resident GB/s, N-way weighted model-tensor reduce; 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
RESNET18_P = 11_181_642
MIN_SET_FOOTPRINT = 1 << 30  # rotate >= 1 GiB of inputs: 4x the 256 MiB Infinity Cache
MIN_OUT_FOOTPRINT = 1 << 30  # and >= 1 GiB of outputs (round 5)
PRIME_LAUNCHES = 8  # launches on a decoy set before the warm-up (ReduceWorkload._prime)

GNLENET_SHAPES = [(32, 3, 5, 5), (32,), (32,), (32,), (32, 32, 5, 5), (32,), (32,), (32,),
                  (64, 32, 5, 5), (64,), (64,), (64,), (10, 576), (10,)]


def resnet18_shapes():
    """parameters() shapes of torchvision resnet18(num_classes=10), the
    reference's create_model("cifar10", "resnet18") (models/__init__.py:27-29):
    62 tensors, 11,181,642 params."""
    shapes = [(64, 3, 7, 7), (64,), (64,)]
    cin = 64
    for cout, stride in ((64, 1), (128, 2), (256, 2), (512, 2)):
        for b in range(2):
            shapes += [(cout, cin, 3, 3), (cout,), (cout,), (cout, cout, 3, 3), (cout,), (cout,)]
            if b == 0 and (stride != 1 or cin != cout):
                shapes += [(cout, cin, 1, 1), (cout,), (cout,)]
            cin = cout
    return shapes + [(10, 512), (10,)]


# parameter layout the CPU baseline runs on (what the reference would iterate)
LAYOUTS = {"north_star": resnet18_shapes, "cfg3": resnet18_shapes, "cfg5": resnet18_shapes,
           "cfg2_gnlenet": lambda: GNLENET_SHAPES}

# name: (n_models, params, dtype, weights, description)
CONFIGS = {
    "north_star": (8, RESNET18_P, "f32", "dirichlet",
                   "8-way Dirichlet-weighted fp32 reduce, 11,181,642 params (ResNet-18/CIFAR-10)"),
    "cfg2": (8, 1_048_576, "f32", "uniform",
             "8-way unweighted fp32 average, 1,048,576 params (CIFAR-10 model, ~1 M label)"),
    "cfg2_gnlenet": (8, 85_354, "f32", "uniform",
                     "8-way unweighted fp32 average of GNLeNet (85,354 params)"),
    "cfg3": (17, RESNET18_P, "f32", "dirichlet",
             "D-PSGD k=16 weighted neighbour mix, 17 x 11,181,642 fp32"),
    "cfg4": (2, 125_000_000, "bf16", "age",
             "gossip 2-way bf16 merge, 125,000,000 params, age weights [3/8, 5/8]"),
    "cfg5": (100, RESNET18_P, "f32", "dirichlet",
             "FedAvg 100-client weighted fp32 reduce, 11,181,642 params"),
    # not a BASELINE.json config: fp16 models through the same path
    "cfg4_f16": (2, 125_000_000, "f16", "age",
                 "gossip 2-way fp16 merge, 125,000,000 params, age weights [3/8, 5/8]"),
}

TORCH_DTYPE = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}
ELEM_BYTES = {"f32": 4, "bf16": 2, "f16": 2}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="north_star", choices=sorted(CONFIGS))
    ap.add_argument("--shape", default=None,
                    help="n:params[:dtype] instead of --config (launch-shape studies; the line's "
                         "config.workload is then 'custom', not a BASELINE.json config)")
    ap.add_argument("--mode", default="exact", choices=["exact", "fast"])
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling: every rank reduces the config's full parameter count "
                         "(default: strong scaling, the config's parameters split over the ranks)")
    ap.add_argument("--strong", action="store_true", help="strong scaling (the default; kept for old scripts)")
    ap.add_argument("--slice-of", type=int, default=1,
                    help="1 GPU only: run rank 0's slice of a strong split over this many ranks "
                         "(the per-rank work of the strong split at that world size, without the other ranks)")
    ap.add_argument("--batch", type=int, default=1,
                    help="B independent aggregates of the config per step, in batched launches "
                         "(a simulated round's per-peer tasks)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend: nccl (= RCCL over xGMI, the real path); gloo only "
                         "to rehearse the multi-process flow on a box with fewer GPUs than ranks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--two-streams", action="store_true",
                    help="diagnostic: also time the K steps alternating over two streams (field two_streams); "
                         "off by default because those overlapping dispatches would enter a rocprof average "
                         "of the same command")
    ap.add_argument("--xor-probe", action="store_true",
                    help="diagnostic: also time dlsim_probe_pattern (the step's dispatch with an XOR fold; "
                         "field xor_probe; not a bound)")
    ap.add_argument("--no-single-gpu-reference", action="store_true",
                    help="N > 1: skip rank 0's timing of the whole config alone (the speed-up base)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget for the CPU baseline sample (rank 0, N=1 only)")
    return ap.parse_args(argv)


# ---- process launch ----------------------------------------------------------------

def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv, script: str = None) -> int:
    """Start N rank processes of this script (fresh interpreters: this parent
    never touches the GPU, and nothing is exec'd over it), wait for them and
    return the first failing exit code (0 if all succeed). If one rank fails,
    the others are stopped after a grace period instead of waiting forever in
    a collective."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__), *argv], env=env))
    rc, failed_at = 0, None
    while True:
        codes = [p.poll() for p in procs]
        for c in codes:
            if c not in (None, 0) and rc == 0:
                rc, failed_at = c, time.monotonic()
        if all(c is not None for c in codes):
            return rc
        if failed_at is not None and time.monotonic() - failed_at > 30:
            for p in procs:
                if p.poll() is None:
                    p.kill()
            for p in procs:
                p.wait()
            return rc
        time.sleep(0.05)


# ---- timing ----------------------------------------------------------------------

def time_steps(launch, k_steps: int, sync, barrier, new_event):
    """Time exactly k_steps launches. The barrier that lines the ranks up and
    a device sync come BEFORE the window; the window is two events on the
    launch stream around the launches (plus a host clock from the first
    launch to the sync after the last); the closing barrier comes AFTER the
    window is read. Returns (event_ms, wall_ms) for all k_steps. (Round 4
    measured a GPU-side gate before the start event, so the window would not
    hold the host's enqueue of launch 0: no difference at K = 20 or 400,
    profiles/r04a/placement.jsonl; not kept.)"""
    barrier()
    sync()
    e0, e1 = new_event(), new_event()
    t0 = time.perf_counter()
    e0.record()
    for k in range(k_steps):
        launch(k)
    e1.record()
    sync()
    wall_ms = (time.perf_counter() - t0) * 1e3
    ev_ms = e0.elapsed_time(e1)
    barrier()
    return ev_ms, wall_ms


def _rows_alloc() -> str:
    """How the input rows were allocated (arena.resident_empty)."""
    from dasklearn_amd.arena import RESIDENT_BLOCKS
    if RESIDENT_BLOCKS["contiguous"] and not RESIDENT_BLOCKS["fallback"]:
        return "physically contiguous (dlsim_device_alloc)"
    if RESIDENT_BLOCKS["fallback"]:
        return "hipMalloc (the driver had no contiguous block)"
    return "torch caching allocator"


def _outputs_alloc() -> str:
    """Where the aggregate outputs came from (arena.arena_empty)."""
    from dasklearn_amd import _native
    from dasklearn_amd.arena import OUTPUT_POOL
    if OUTPUT_POOL.made:
        st = _native.pool_stats()
        return (f"torch.cuda.MemPool over dlsim_pool_alloc (arena.OUTPUT_POOL: {OUTPUT_POOL.made} outputs, "
                f"{st['contiguous']} contiguous segments, {st['fallback']} hipMalloc fallbacks)")
    return "torch caching allocator"


def n_sets(bytes_per_set: int) -> int:
    return max(3, min(256, math.ceil(MIN_SET_FOOTPRINT / max(1, bytes_per_set))))


def weights_for(kind: str, n: int) -> list:
    if kind == "dirichlet":
        return [float(w) for w in np.random.default_rng(7).dirichlet(np.ones(n))]
    if kind == "age":
        return [3.0 / 8.0, 5.0 / 8.0][:n] if n == 2 else [1.0 / n] * n
    return [float(1.0 / n)] * n  # fedavg.py:14-15


def _out_alloc(p, tdt, dev):
    """An aggregate output as the product allocates it (arena_empty: the
    output pool), or for placement A/B runs (DLSIM_BENCH_OUT_ALLOC) a
    separate contiguous library block ("resident") or torch's allocator
    ("torch"), 2 MiB-aligned."""
    from dasklearn_amd.arena import aligned_empty, arena_empty, resident_empty
    kind = os.environ.get("DLSIM_BENCH_OUT_ALLOC", "pool")
    if kind == "resident":
        return resident_empty(p, tdt, dev, 2 << 20)
    if kind == "torch":
        return aligned_empty(p, tdt, dev, 2 << 20)
    return arena_empty(p, tdt, dev)


class ReduceWorkload:
    """Rotating input sets and outputs, and prepared launches of one
    config's aggregate on one device: `launch(k)` runs step k (input set
    k mod S into output k mod O; S and O each >= 1 GiB, O a multiple of S)."""

    def __init__(self, n, p, dtype, w32, mode, batch, dev, seed, stream):
        from dasklearn_amd import _native
        from dasklearn_amd.arena import aligned_empty, arena_empty, base_align, resident_empty, row_stride
        tdt = TORCH_DTYPE[dtype]
        esz = ELEM_BYTES[dtype]
        self.stream = stream
        self.bytes_per_step = (n + 1) * p * esz * batch
        # DLSIM_BENCH_MIN_SETS / DLSIM_BENCH_SET_ALLOC=per_set: A/B knobs for
        # the placement study, not for bench lines
        self.sets = max(n_sets(self.bytes_per_step), int(os.environ.get("DLSIM_BENCH_MIN_SETS", "0")))
        per_set = os.environ.get("DLSIM_BENCH_SET_ALLOC") == "per_set"
        g = torch.Generator(device=dev).manual_seed(seed)
        # the models are rows of one arena laid out as the product's staging
        # and round uploads lay them out (arena.row_stride / base_align: 256 B
        # rows, or 2 MiB-aligned rows for >= 16 MiB of 4/8-byte elements), the
        # outputs as the product allocates aggregate outputs (arena_empty)
        p_pad = row_stride(p, esz)
        al = base_align(p * esz, esz)
        self.plans, self.probe_plans, self.outs, self._keep = [], [], [], []
        # every set's rows in ONE allocation, as the staging buffer holds a
        # call's rows, and allocated as the staging is (arena.resident_empty:
        # physically contiguous from 64 MiB on): rows in separate per-set
        # allocations measured 0.5-2.5 % slower and varied with where the
        # driver placed them (profiles/r03_bench_gap.jsonl)
        if per_set:
            rows = [resident_empty(batch * n * p_pad, tdt, dev, al).view(batch, n, p_pad) for _ in range(self.sets)]
        else:
            rows = resident_empty(self.sets * batch * n * p_pad, tdt, dev, al).view(self.sets, batch, n, p_pad)
        self._keep.append(rows)
        # the outputs rotate too, over >= 1 GiB (round 5): outputs that rotate
        # over a few buffers (rounds 1-4: one per input set, 134 MB for the
        # north star) stay in the 256 MiB Infinity Cache and their rewrites
        # never reach HBM -- 5-8 % of a north-star step. A
        # multiple of the input sets, so step k reads set k mod S.
        # DLSIM_BENCH_OUT_SETS=k overrides (A/B runs of that study only).
        out_bytes = batch * p * esz
        need = max(self.sets, math.ceil(MIN_OUT_FOOTPRINT / max(1, out_bytes)))
        self.out_sets = int(os.environ.get("DLSIM_BENCH_OUT_SETS", "0")) or \
            -(-need // self.sets) * self.sets
        for s in range(self.sets):
            if batch == 1:
                x = rows[s][0]
                x[:, :p].copy_((torch.randn((n, p), generator=g, device=dev) * 0.05).to(tdt))
            else:
                x = rows[s]
                x[:, :, :p].copy_((torch.randn((batch, n, p), generator=g, device=dev) * 0.05).to(tdt))
            self._keep.append(x)
        for j in range(self.out_sets):
            x = rows[j % self.sets][0] if batch == 1 else rows[j % self.sets]
            if batch == 1:
                out = _out_alloc(p, tdt, dev)
                plan = _native.ReducePlan([x[i, :p] for i in range(n)], w32, out, mode)
                assert all(t.data_ptr() % 16 == 0 for t in plan._keep[0]), "arena rows must be 16-B aligned"
                self.outs.append(out)
                if j < self.sets:
                    self.probe_plans.append(_native.ReducePlan([x[i, :p] for i in range(n)], w32, out, mode,
                                                               probe=True))
            else:
                ob = aligned_empty(batch * p_pad, tdt, dev, al).view(batch, p_pad)
                plan = _native.BatchPlan([([x[b, i, :p] for i in range(n)], w32, ob[b, :p]) for b in range(batch)],
                                         mode)
                self.outs.append(ob[0, :p])
                self._keep.append(ob)
            self.plans.append(plan)
        self.kernel = _native.kernel_name(n, p, tdt, mode) if batch == 1 else "dlsim::k_wreduce_batch_table"
        self._prime(n, p, p_pad, tdt, al, w32, mode, batch, dev, g)

    def _prime(self, n, p, p_pad, tdt, al, w32, mode, batch, dev, g):
        """Read a decoy set, never timed, before the first warm-up launch (round
        6): the first set the reduce reads after the caches were flushed by
        ordinary stores (here: the sets' fill) stays in the Infinity Cache
        while the rotating sets stream past it, and ran ~20 % faster than
        the others for the whole run (set 0: 7.96 against 9.6-10.0 us in the
        8-rank slice, 60.1 against 61.7-62.1 in the north star;
        scripts/probes/probe_slice_sets.py). The decoy takes
        that place, so every timed set streams from HBM."""
        from dasklearn_amd import _native
        from dasklearn_amd.arena import aligned_empty, resident_empty
        if os.environ.get("DLSIM_BENCH_PRIME", "1") == "0":  # A/B of the study only
            return
        rows = resident_empty(batch * n * p_pad, tdt, dev, al).view(batch, n, p_pad)
        rows[:, :, :p].copy_((torch.randn((batch, n, p), generator=g, device=dev) * 0.05).to(tdt))
        if batch == 1:
            out = _out_alloc(p, tdt, dev)
            plan = _native.ReducePlan([rows[0, i, :p] for i in range(n)], w32, out, mode)
        else:
            out = aligned_empty(batch * p_pad, tdt, dev, al).view(batch, p_pad)  # the timed outputs' layout
            plan = _native.BatchPlan([([rows[b, i, :p] for i in range(n)], w32, out[b, :p]) for b in range(batch)],
                                     mode)
        for _ in range(PRIME_LAUNCHES):
            plan.launch(self.stream)
        torch.cuda.synchronize(dev)
        self._keep.append((rows, out, plan))

    def launch(self, k):
        self.plans[k % self.out_sets].launch(self.stream)

    def launch_probe(self, k):
        self.probe_plans[k % len(self.probe_plans)].launch(self.stream)


def xor_probe(wl, k_steps: int, sync, new_event, achieved_gbps: float):
    """dlsim_probe_pattern over the same rotating sets: the reduce's own
    dispatch (kernel, launch shape, nt loads, store policy) with the weighted
    fold replaced by a bitwise XOR. Opt-in (--xor-probe), and NOT a bound:
    rounds 1-3 read it as the memory system's ceiling for this read/write
    mix, but at round 4's HEAD it ran 3-4 % slower than the reduce it was
    meant to bound, so the line no longer carries it."""
    for k in range(10):
        wl.launch_probe(k)
    ev_ms, _ = time_steps(wl.launch_probe, k_steps, sync, lambda: None, new_event)
    us = ev_ms * 1e3 / k_steps
    gbps = wl.bytes_per_step / (us * 1e-6) / 1e9
    return {"GBps": round(gbps, 1), "frac": round(gbps / HBM_PEAK_GBPS, 4), "us_per_launch": round(us, 3),
            "reduce_over_probe": round(achieved_gbps / gbps, 4),
            "kernel": "dlsim_probe_pattern: same dispatch and shapes, XOR fold",
            "note": "diagnostic only, not a bound (the reduce has run faster than it)"}


def launch_floor(wl, n, dtype, w32, mode, dev, k_steps: int, sync, new_event, step_us: float):
    """GPU-side per-launch floor of back-to-back launches on one stream: the
    step's dispatch (as dlsim_probe_pattern) with one 256-element tile per
    input (fan-in min(n, 8)). A host
    launch through ctypes takes a few µs, about as long as such a kernel, so
    the K tiny launches are queued behind a backlog of the step's own
    launches (enough GPU time to cover the host's enqueue of all of them):
    the events around them then see the GPU run them back to back. What
    remains of a step after this floor is what its bytes take; at the 8-rank
    slices the floor is a large part of a ~10 µs step (MI355X_MICROARCH.md,
    price table row 'boundary': 1.7-1.9 µs between streaming kernels).
    Diagnostic only: `value` is the full step time."""
    from dasklearn_amd import _native
    tdt = TORCH_DTYPE[dtype]
    # at most 8 inputs: with more, one 256-element tile is a chain of
    # dependent load groups in a single block (latency, not launch cost)
    nf = min(n, 8)
    x = torch.randn((nf, 256), device=dev).to(tdt)
    out = torch.empty(256, dtype=tdt, device=dev)
    # the memory-only probe's entry (same dispatch, XOR fold): its kernel name
    # differs from the reduce's, so rocprof's per-kernel averages of the step
    # stay clean of these tiny launches
    plan = _native.ReducePlan([x[i] for i in range(nf)], w32[:nf], out, mode, probe=True)
    stream = wl.stream
    for _ in range(10):
        plan.launch(stream)
    sync()
    t0 = time.perf_counter()
    for _ in range(k_steps):
        plan.launch(stream)
    host_us = (time.perf_counter() - t0) * 1e6 / k_steps
    sync()
    # GPU time of the backlog >= 2x the host time to enqueue it and the K launches
    backlog = min(4000, math.ceil(2.0 * k_steps * host_us / max(step_us - 2.0 * host_us, 0.5)) + 10)
    e0, e1 = new_event(), new_event()
    for k in range(backlog):
        wl.launch(k)
    e0.record()
    for _ in range(k_steps):
        plan.launch(stream)
    e1.record()
    sync()
    floor_us = e0.elapsed_time(e1) * 1e3 / k_steps
    res = {"us_per_launch": round(floor_us, 3), "host_enqueue_us_per_launch": round(host_us, 3),
           "backlog_launches": backlog,
           "note": f"{k_steps} back-to-back launches of dlsim_probe_pattern (the step's dispatch; n={nf}, 256 elements per input) "
                   f"queued behind {backlog} launches of the step; HIP events on the launch stream"}
    body_us = step_us - floor_us
    if body_us > 0:
        res["step_minus_floor_us"] = round(body_us, 3)
        res["bytes_frac_of_peak_excl_floor"] = round(wl.bytes_per_step / (body_us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
    return res


def two_streams(wl, k_steps: int, sync, dev):
    """The same K steps with consecutive steps on two streams (independent
    aggregates: distinct inputs and outputs), so one launch's ramp overlaps
    the previous one's drain instead of waiting behind the launch boundary.
    A D-PSGD or gossip round has many such independent aggregates in flight
    (the reference runs them in parallel worker processes, broker.py:137-149).
    Diagnostic only: `value` is one aggregate after another on one stream."""
    a = wl.stream
    b = torch.cuda.Stream(dev)
    for k in range(10):
        wl.plans[k % wl.out_sets].launch(a if k % 2 == 0 else b)
    sync()
    e0, e1, eb = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(a)
    b.wait_event(e0)
    for k in range(k_steps):
        wl.plans[k % wl.out_sets].launch(a if k % 2 == 0 else b)
    eb.record(b)
    a.wait_event(eb)
    e1.record(a)
    sync()
    us = e0.elapsed_time(e1) * 1e3 / k_steps
    gbps = wl.bytes_per_step / (us * 1e-6) / 1e9
    return {"us_per_step": round(us, 3), "GBps": round(gbps, 1), "frac": round(gbps / HBM_PEAK_GBPS, 4),
            "note": "steps alternate between two streams (independent aggregates in flight); not in value"}


def pmc_traffic(config: str, mode: str, split: int):
    """Per-launch HBM bytes for this config (and strong split) from the
    committed PMC summaries (profiles/*pmc*.json, scripts/pmc_summary.py over
    rocprofv3 --pmc runs of this same command; FETCH_SIZE doubled per the
    gfx950 rule). Returns (bytes, source file) or (None, reason)."""
    import glob
    import re
    best, src = None, None
    key = config if split <= 1 else f"{config}@slice{split}"

    def newest_last(path):  # r01 < r01_s4 < r02 < r02s2 < r03 ...: round, then session, then name
        m = re.match(r"r(\d+)(?:_?s(\d+))?", os.path.basename(path))
        return (int(m.group(1)), int(m.group(2) or 0), path) if m else (-1, 0, path)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*pmc*.json"), recursive=True),
                       key=newest_last):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        ent = d.get(key, {}).get(mode)
        if ent and "hbm_bytes_per_launch" in ent:
            best, src = ent["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    if best is None:
        return None, f"no committed rocprofv3 --pmc summary for {key}/{mode}"
    return best, src + " (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, separate passes; not measured in this run)"


def _host_threads() -> int:
    """Host cores this process may use: the affinity set, capped by
    OMP_NUM_THREADS (the GPU box sets it to the job's CPU share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def box_info() -> dict:
    """The host the CPU baseline ran on (its numbers move with the box's CPU
    share and memory)."""
    info = {"host_cpus": os.cpu_count(), "threads_usable": _host_threads(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    if hasattr(os, "sched_getaffinity"):
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()
        info["cgroup_cpu_quota"] = None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        info["cgroup_cpu_quota"] = None
    try:
        with open("/proc/cpuinfo") as f:
            info["cpu_model"] = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        pass
    return info


def cpu_baseline(config, n, p, dtype, weights, budget_s):
    """The reference's aggregate as it runs in the simulator's worker: the
    op-for-op PyTorch-CPU restatement of FedAvg.aggregate (oracle/, validated
    bit-identical to the reference and timed against it, profiles/r02_cpu_port_vs_reference.json)
    on N host modules with the workload's real parameter layout (ResNet-18: 62
    tensors), including the deepcopy of models[0], at the worker's 4 threads
    (broker.py:31, session_settings.py:52). A second, shorter sample at every
    host core this job may use goes under "all_cores" (SURVEY.md §8d)."""
    from torch import nn
    from oracle import fedavg_torch
    tdt = TORCH_DTYPE[dtype]
    shapes = LAYOUTS[config]() if config in LAYOUTS else [(p,)]
    assert sum(int(torch.Size(sh).numel()) for sh in shapes) == p

    class Shaped(nn.Module):
        def __init__(self, seed):
            super().__init__()
            g = torch.Generator().manual_seed(seed)
            self.ps = nn.ParameterList(
                [nn.Parameter((torch.randn(sh, generator=g) * 0.05).to(tdt)) for sh in shapes])

    models = [Shaped(1234 + i) for i in range(n)]
    bytes_ = (n + 1) * p * ELEM_BYTES[dtype]

    def timed(threads, budget):
        prev = torch.get_num_threads()
        torch.set_num_threads(threads)
        try:
            fedavg_torch.aggregate_modules(models, weights)  # warm
            reps, t0 = 0, time.perf_counter()
            while True:
                fedavg_torch.aggregate_modules(models, weights)
                reps += 1
                el = time.perf_counter() - t0
                if el >= budget or reps >= 2000:
                    return reps, el
        finally:
            torch.set_num_threads(prev)

    threads = 4
    reps, el = timed(threads, budget_s)
    per = el / reps
    layout = f"{len(shapes)} parameter tensors" if len(shapes) > 1 else "one flat parameter"
    out = {"value": round(bytes_ / per / 1e9, 3), "unit": "GB/s", "cores": threads,
           "kind": "port",
           "ms_per_step": round(per * 1e3, 3),
           "sample": f"{reps} x FedAvg.aggregate of {n} host modules ({layout}, {p} {dtype} params) "
                     f"in {el:.1f} s: the reference's torch CPU op sequence at {threads} threads"}
    all_t = _host_threads()
    if all_t != threads:
        reps2, el2 = timed(all_t, budget_s / 2)
        out["all_cores"] = {"value": round(bytes_ * reps2 / el2 / 1e9, 3), "unit": "GB/s", "cores": all_t,
                            "ms_per_step": round(el2 / reps2 * 1e3, 3),
                            "sample": f"{reps2} x the same aggregate in {el2:.1f} s at {all_t} threads"}
    out["box"] = box_info()
    return out


# ---- one rank -------------------------------------------------------------------

def run_rank(args, rank: int, world: int, local: int):
    from dasklearn_amd import _native

    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and world > ndev:
        print(f"bench.py: {world} ranks but {ndev} GPUs visible (use --backend gloo to rehearse)", file=sys.stderr)
        return 2
    local_dev = local % max(1, ndev)  # a gloo rehearsal may share a GPU
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    backend_note = None
    if world > 1:
        if args.backend == "nccl":
            try:
                dist.init_process_group("nccl", device_id=dev)
            except Exception as e:  # the data path has no collective: keep measuring
                backend_note = f"gloo control plane (RCCL init failed: {type(e).__name__}: {e})"[:300]
                print(f"bench.py: {backend_note}", file=sys.stderr)
                args.backend = "gloo"
                dist.init_process_group("gloo")
        else:
            dist.init_process_group("gloo")
    cdev = dev if args.backend == "nccl" else torch.device("cpu")  # control-plane tensors
    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)

    n, p_cfg, dtype, wkind, desc = CONFIGS[args.config]
    if args.shape:
        f = args.shape.split(":")
        n, p_cfg = int(f[0]), int(f[1])
        dtype = f[2] if len(f) > 2 else "f32"
        wkind, desc = "dirichlet", f"custom {n}-way Dirichlet-weighted {dtype} reduce, {p_cfg:,} params"
        args.config = "custom"
    strong = world > 1 and not args.weak
    split = world if strong else (args.slice_of if world == 1 else 1)
    b0, e0 = _native.shard_range(p_cfg, split, rank if strong else 0, 64) if split > 1 else (0, p_cfg)
    p = e0 - b0
    esz = ELEM_BYTES[dtype]
    mode = _native.DLSIM_EXACT if args.mode == "exact" else _native.DLSIM_FAST
    weights = weights_for(wkind, n)
    w32 = _native.fp32_weights(weights)
    B = max(1, args.batch)
    stream = torch.cuda.current_stream(dev)
    new_event = lambda: _StreamEvent(stream)  # noqa: E731
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731

    wl = ReduceWorkload(n, p, dtype, w32, mode, B, dev, 1234 + rank, stream)
    for k in range(args.warmup):
        wl.launch(k)
    K = args.steps
    ev_ms, wall_ms = time_steps(wl.launch, K, sync, barrier, new_event)

    stats = torch.tensor([ev_ms, wall_ms, float(wl.bytes_per_step) * K], dtype=torch.float64, device=cdev)
    per_rank_us = torch.tensor([ev_ms / K * 1e3], dtype=torch.float64, device=cdev)
    if world > 1:
        mx = stats[:2].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot = stats[2:].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        gathered = [torch.zeros_like(per_rank_us) for _ in range(world)]
        dist.all_gather(gathered, per_rank_us)
        max_ev, max_wall, total_bytes = float(mx[0]), float(mx[1]), float(tot[0])
        rank_us = [round(float(t.item()), 3) for t in gathered]
    else:
        max_ev, max_wall, total_bytes = ev_ms, wall_ms, float(wl.bytes_per_step) * K
        rank_us = [round(ev_ms / K * 1e3, 3)]
    value = total_bytes / (max_ev * 1e-3) / 1e9

    # ---- N > 1: the output all-gather, in its own fields -----------------------
    gather = None
    if world > 1:
        gather = _time_gathers(args, wl, rank, world, p_cfg, p, n, w32, mode, dtype, dev, cdev, stream, strong, barrier)

    # ---- N > 1 strong: the same config on one GPU (rank 0 alone) ----------------
    single = None
    if strong and not args.no_single_gpu_reference:
        barrier()
        if rank == 0:
            full = ReduceWorkload(n, p_cfg, dtype, w32, mode, B, dev, 99, stream)
            for k in range(args.warmup):
                full.launch(k)
            t1_ms, _ = time_steps(full.launch, K, sync, lambda: None, new_event)
            single = {"ms_per_step": round(t1_ms / K, 6),
                      "speedup": round((t1_ms / K) / (max_ev / K), 3),
                      "note": f"T1 = the whole {args.config} aggregate on rank 0's GPU alone, {K} launches, "
                              f"same event timing; speedup = T1 / T{world} (max over ranks)"}
            del full
        barrier()

    result = None
    if rank == 0:
        achieved = wl.bytes_per_step / (ev_ms / K * 1e-3) / 1e9
        traffic, traffic_src = (pmc_traffic(args.config, args.mode, split) if B == 1
                                else (None, "no committed PMC summary for batched launches"))
        probe = xor_probe(wl, K, sync, new_event, achieved) if B == 1 and args.xor_probe else None
        floor = launch_floor(wl, n, dtype, w32, mode, dev, K, sync, new_event, ev_ms / K * 1e3) \
            if B == 1 else None
        # opt-in: its concurrent launches share the reduce's kernel name, so
        # they would skew rocprof's per-dispatch average of the same command
        overlap = two_streams(wl, K, sync, dev) if B == 1 and args.two_streams else None
        scaling = "weak" if args.weak and world > 1 else "strong"
        workload = args.config + ": " + desc
        if B > 1:
            workload += f" x {B} tasks per launch"
        if strong:
            workload += f" (strong scaling: {p_cfg} params split over {world} ranks)"
        elif args.weak and world > 1:
            workload += f" (weak scaling: {p_cfg} params per rank)"
        elif split > 1:
            workload += f" (rank 0's slice of a {split}-rank strong split, alone on 1 GPU)"
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(max_ev / K, 6),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": dtype,
            "data": f"synthetic: torch.randn*0.05 on device, {wl.sets} rotating input sets "
                    f"(>= 1 GiB) into {wl.out_sets} rotating outputs "
                    f"({wl.out_sets * wl.bytes_per_step // (n + 1) / 1e9:.2f} GB: none stays in the "
                    f"256 MiB Infinity Cache; a decoy set read first takes the one set the cache "
                    f"would keep, DESIGN.md §5f); {wkind} weights",
            "config": {"workload": workload,
                       "backend": (backend_note or args.backend) if world > 1 else None,
                       "n_models": n, "params_total": p_cfg if strong or split > 1 else p * world,
                       "params_rank0": p, "tasks_per_step": B, "mode": args.mode,
                       "parallelism": f"param-shard x{world}",
                       "bytes_per_step_rank0": wl.bytes_per_step,
                       "rows_alloc": _rows_alloc(), "outputs_alloc": _outputs_alloc()},
            "timing": {"value_from": "HIP events around the K launches on each rank's launch stream; "
                                     "value = all ranks' bytes / max over ranks; barriers outside the window",
                       "kernel_avg_us_per_rank": rank_us,
                       "wall_ms_per_step_max": round(max_wall / K, 6)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": wl.kernel, "kernel_avg_us": round(ev_ms / K * 1e3, 3),
                         "timing": "rank 0: HIP events around the K timed launches on the launch stream"},
            "launch_floor": floor,
            "two_streams": overlap,
        }
        if probe:
            result["xor_probe"] = probe
        if single:
            result["single_gpu_reference"] = single
        if gather:
            result["allgather"] = gather
    barrier()
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args.config, n, p, dtype, weights, args.cpu_seconds)
        else:
            result["cpu_baseline"] = None
    if world > 1 and args.backend == "nccl" and strong:
        # last, and under a watchdog: RCCL calls made by the library itself
        def on_timeout():
            if rank == 0:
                result["allgather"]["dlsim_wreduce_sharded_error"] = \
                    f"timed out after {SHARDED_TIMEOUT_S:.0f} s; line printed without it"
                print(json.dumps(result), file=_RESULT_OUT or sys.stdout, flush=True)
        sharded = _guarded(lambda: _time_sharded(wl, n, p_cfg, w32, mode, dtype, dev, cdev, stream, barrier),
                           SHARDED_TIMEOUT_S, on_timeout)
        if rank == 0:
            result["allgather"].update(sharded)
    if rank == 0:
        print(json.dumps(result), file=_RESULT_OUT or sys.stdout, flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


class _StreamEvent:
    """A timing event recorded on a given stream (torch.cuda.Event.record()
    without an argument would use the current stream)."""

    def __init__(self, stream):
        self.stream = stream
        self.ev = torch.cuda.Event(enable_timing=True)

    def record(self):
        self.ev.record(self.stream)

    def elapsed_time(self, other):
        return self.ev.elapsed_time(other.ev)


def _time_gathers(args, wl, rank, world, p_cfg, p, n, w32, mode, dtype, dev, cdev, stream, strong, barrier):
    """The collective that would materialise the full output, timed apart
    from `value`: RCCL all_gather_into_tensor of width-padded slices (torch).
    The C ABI's own gather (dlsim_wreduce_sharded) is timed at the end of the
    run, under a watchdog (_time_sharded, _guarded)."""
    from dasklearn_amd import _native
    tdt = TORCH_DTYPE[dtype]
    esz = ELEM_BYTES[dtype]
    width = max(e - b for b, e in (_native.shard_range(p_cfg, world, r, 64) for r in range(world))) \
        if strong else p
    shard = torch.zeros(width, dtype=tdt, device=dev)
    shard[:p].copy_(wl.outs[0])
    if args.backend != "nccl":
        shard = shard.cpu()
    full = torch.empty(width * world, dtype=tdt, device=shard.device)
    reps = 20
    for _ in range(3):
        dist.all_gather_into_tensor(full, shard)
    torch.cuda.synchronize(dev)
    barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_gather_into_tensor(full, shard)
    torch.cuda.synchronize(dev)
    ag_ms = (time.perf_counter() - t0) / reps * 1e3
    out = {"all_gather_into_tensor_ms": ag_ms,
           "bytes_out_per_rank": width * esz * world,
           "note": ("RCCL" if args.backend == "nccl" else "gloo (rehearsal)")
                   + " collectives of the reduced slices; host clock over 20 back-to-back ops after a sync; "
                     "not in value"}
    t = torch.tensor([out["all_gather_into_tensor_ms"]], dtype=torch.float64, device=cdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out["all_gather_into_tensor_ms"] = round(float(t[0]), 4)
    return out


SHARDED_TIMEOUT_S = 90.0


def _time_sharded(wl, n, p_cfg, w32, mode, dtype, dev, cdev, stream, barrier, reps: int = 20):
    """The C ABI's sharded aggregate end to end on the group's own RCCL
    communicator, four ways, HIP events on the launch stream, max over ranks:
    dlsim_wreduce_sharded (agreement all-reduce + host wait every call) and a
    dlsim_sharded_plan (agreed once), each with the grouped in-place
    ncclBroadcast gather and with the padded ncclAllGather + unpad kernel."""
    from dasklearn_amd import _native
    out = {"sharded_note": "this rank's reduce + the gather on the group's RCCL communicator; agreed = "
                           "dlsim_wreduce_sharded (agreement all-reduce and host wait per call), plan = "
                           "dlsim_sharded_plan_run (agreed once); HIP events on the launch stream, max over ranks"}
    pg = dist.distributed_c10d._get_default_group()
    comm = int(pg._get_backend(dev)._comm_ptr())
    slices = [wl.plans[0]._keep[0][i] for i in range(n)]
    fullout = torch.empty(p_cfg, dtype=TORCH_DTYPE[dtype], device=dev)
    plans = {}
    for gather in ("bcast", "allgather"):
        try:  # collective: the agreement makes a failure every rank's
            plans[gather] = _native.ShardedPlan(comm, p_cfg, n, TORCH_DTYPE[dtype], gather, device=dev,
                                                stream=stream)
        except Exception as e:  # noqa: BLE001 - reported in the line
            plans[gather] = None
            out[f"plan_{gather}_create_error"] = f"{type(e).__name__}: {e}"[:300]

    def run_plan(gather):
        if plans[gather] is None:
            raise RuntimeError("no plan")
        plans[gather].run(slices, w32, fullout, mode, stream)
    runs = {
        "dlsim_wreduce_sharded_gather_ms": lambda: _native.wreduce_sharded(slices, w32, fullout, comm, "bcast",
                                                                         mode, stream),
        "dlsim_wreduce_sharded_allgather_ms": lambda: _native.wreduce_sharded(slices, w32, fullout, comm,
                                                                            "allgather", mode, stream),
        "plan_bcast_ms": lambda: run_plan("bcast"),
        "plan_allgather_ms": lambda: run_plan("allgather"),
    }
    for key, fn in runs.items():
        try:
            for _ in range(3):
                fn()
            torch.cuda.synchronize(dev)
            barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / reps
        except Exception as e:  # report, do not fail the bench line
            ms = -1.0
            out[key.replace("_ms", "_error")] = f"{type(e).__name__}: {e}"[:300]
        t = torch.tensor([ms], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if ms >= 0:
            out[key] = round(float(t[0]), 4)
    for pl in plans.values():
        if pl is not None:
            pl.close()
    return out


WATCHDOG_EXIT = 3  # exit code of a rank whose guarded collective timed out


def _guarded(fn, timeout_s: float, on_timeout):
    """fn() with a watchdog: a collective issued outside torch's own watchdog
    (the C ABI's RCCL calls) must not hold the bench line hostage. If fn has
    not returned after timeout_s, on_timeout() runs (rank 0 prints the line
    it has, with the timeout recorded in it) and the process exits with
    WATCHDOG_EXIT, so spawn_ranks and the driver see the run as failed
    (a hung collective must not read as a successful bench)."""
    import threading
    done = threading.Event()

    def fire():
        if not done.is_set():
            try:
                on_timeout()
            finally:
                os._exit(WATCHDOG_EXIT)
    timer = threading.Timer(timeout_s, fire)
    timer.daemon = True
    timer.start()
    try:
        return fn()
    finally:
        done.set()
        timer.cancel()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # self-launch: one fresh process per GPU, started before any GPU call
        return spawn_ranks(args.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    _stdout_for_result_only()
    return run_rank(args, rank, world, local)


_RESULT_OUT = None


def _stdout_for_result_only():
    """Keep this process's stdout for the one JSON line: libraries that write
    to file descriptor 1 themselves (gloo's "[Gloo] Rank r is connected ..."
    at rendezvous, RCCL warnings) go to stderr instead, so a multi-rank run
    still prints exactly one parseable line."""
    global _RESULT_OUT
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


if __name__ == "__main__":
    sys.exit(main())
