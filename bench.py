"""bench.py — device-resident GB/s of the N-way weighted model-tensor reduce.

Metric (BASELINE.json): "device-resident GB/s, N-way weighted model-tensor
reduce; 1/2/4/8 MI355X". A step is one aggregate of one batch: one launch of
the fused HIP reduce over N flat parameter arenas already resident in HBM
(the arithmetic of FedAvg.aggregate, dasklearn/gradient_aggregation/fedavg.py:12-26).

Workload (default, --config north_star): 8 models x 11,181,642 fp32 params
(ResNet-18/CIFAR-10 size), Dirichlet(1) weights, DLSIM_EXACT (bit-identical
to the reference). Multi-GPU: one process per GPU (torchrun); the parameter
axis is sharded — each rank owns an 11,181,642-element slice of every model
(weak scaling: the global parameter count grows with N) and reduces it with
no data-path collective; `value` = bytes all ranks processed / max-over-ranks
time. The RCCL all-gather that would materialise the full output is timed
separately (`allgather`), never inside `value`.

Bytes per step per rank = (N_models + 1) * P * sizeof(dtype) (read N, write 1).
Inputs rotate over 3 disjoint sets so the 256 MiB Infinity Cache cannot serve
re-reads.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(ROOT, "decentralized-learning-simulator_amd")
for _p in (ROOT, PKG_ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "device-resident GB/s, N-way weighted model-tensor reduce; 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
RESNET18_P = 11_181_642

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

# name: (n_models, params per rank, dtype, weights, description)
CONFIGS = {
    "north_star": (8, RESNET18_P, "f32", "dirichlet",
                   "8-way Dirichlet-weighted fp32 reduce, 11,181,642 params/rank (ResNet-18/CIFAR-10)"),
    "cfg2": (8, 1_048_576, "f32", "uniform",
             "8-way unweighted fp32 average, 1,048,576 params (CIFAR-10 model, ~1 M label)"),
    "cfg2_gnlenet": (8, 85_354, "f32", "uniform",
                     "8-way unweighted fp32 average of GNLeNet (85,354 params)"),
    "cfg3": (17, RESNET18_P, "f32", "dirichlet",
             "D-PSGD k=16 weighted neighbour mix, 17 x 11,181,642 fp32"),
    "cfg4": (2, 125_000_000, "bf16", "age",
             "gossip 2-way bf16 merge, 125,000,000 params/rank, age weights [3/8, 5/8]"),
    "cfg5": (100, RESNET18_P, "f32", "dirichlet",
             "FedAvg 100-client weighted fp32 reduce, 11,181,642 params/rank"),
    # not a BASELINE.json config: fp16 models through the same path
    "cfg4_f16": (2, 125_000_000, "f16", "age",
                 "gossip 2-way fp16 merge, 125,000,000 params/rank, age weights [3/8, 5/8]"),
}

TORCH_DTYPE = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}
ELEM_BYTES = {"f32": 4, "bf16": 2, "f16": 2}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="north_star", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="exact", choices=["exact", "fast"])
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: split the config's params over ranks instead of per rank")
    ap.add_argument("--slice-of", type=int, default=1,
                    help="1 GPU only: run rank 0's slice of a strong split over this many ranks "
                         "(the per-rank work of --strong at that world size, without the other ranks)")
    ap.add_argument("--batch", type=int, default=1,
                    help="B independent aggregates of the config per step, in batched launches "
                         "(dlsim_wreduce_batched; a simulated round's per-peer tasks)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend: nccl (= RCCL over xGMI, the real path); gloo only "
                         "to rehearse the multi-process flow on a box with fewer GPUs than ranks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="budget for the CPU baseline sample (rank 0, N=1 only)")
    return ap.parse_args()


def weights_for(kind: str, n: int) -> list:
    if kind == "dirichlet":
        return [float(w) for w in np.random.default_rng(7).dirichlet(np.ones(n))]
    if kind == "age":
        return [3.0 / 8.0, 5.0 / 8.0][:n] if n == 2 else [1.0 / n] * n
    return [float(1.0 / n)] * n  # fedavg.py:14-15


def pmc_traffic(config: str, mode: str):
    """Per-launch HBM bytes for this config from the committed PMC summary
    (profiles/*pmc*.json, made by scripts/pmc_summary.py from rocprofv3 --pmc
    runs of this same command; FETCH_SIZE doubled per the gfx950 rule)."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        ent = d.get(config, {}).get(mode)
        if ent and "hbm_bytes_per_launch" in ent:
            best = ent["hbm_bytes_per_launch"]
    return best


def _host_threads() -> int:
    """Host cores this process may use: the affinity set, capped by
    OMP_NUM_THREADS (the GPU box sets it to the job's CPU share)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def cpu_baseline(config, n, p, dtype, weights, budget_s):
    """The reference's aggregate as it runs in the simulator's worker: the
    op-for-op PyTorch-CPU restatement of FedAvg.aggregate (oracle/, validated
    bit-identical to the reference) on N host modules with the workload's real
    parameter layout (ResNet-18: 62 tensors), including the deepcopy of
    models[0], at the worker's 4 threads (broker.py:31, session_settings.py:52).
    A second, shorter sample at every host core this job may use goes under
    "all_cores" (SURVEY.md §8d asks for both)."""
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
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus != 1:
            print(f"bench.py: --gpus {args.gpus} needs torchrun with that many ranks", file=sys.stderr)
            sys.exit(2)
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and world > ndev:
        print(f"bench.py: {world} ranks but {ndev} GPUs visible", file=sys.stderr)
        sys.exit(2)
    local_dev = local % max(1, ndev)  # gloo rehearsal may share a GPU
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
    # small control-plane tensors live where the backend can reduce them
    cdev = dev if args.backend == "nccl" else torch.device("cpu")

    from dasklearn_amd import _native

    n, p_cfg, dtype, wkind, desc = CONFIGS[args.config]
    if args.strong and world > 1:
        b, e = _native.shard_range(p_cfg, world, rank, 64)
        p = e - b
    elif args.slice_of > 1 and world == 1:
        b, e = _native.shard_range(p_cfg, args.slice_of, 0, 64)
        p = e - b
    else:
        p = p_cfg
    tdt = TORCH_DTYPE[dtype]
    esz = ELEM_BYTES[dtype]
    mode = _native.DLSIM_EXACT if args.mode == "exact" else _native.DLSIM_FAST
    weights = weights_for(wkind, n)
    w32 = _native.fp32_weights(weights)

    # 3 rotating input sets (each > 256 MiB Infinity Cache for the large configs)
    sets = 3
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    arenas = []
    # rows padded to 256 B so every model's arena starts 16-byte aligned
    # (the vector kernel's requirement; unaligned rows would take the scalar
    # path), at the staging arena's stride (4 KiB more at power-of-two strides)
    from dasklearn_amd.arena import row_stride
    p_pad = row_stride(p, esz)
    for s in range(sets):
        x = torch.empty((n, p_pad), dtype=tdt, device=dev)
        for i in range(n):
            x[i, :p].copy_(torch.randn(p, generator=g, device=dev) * 0.05)
        arenas.append(x)
    B = max(1, args.batch)
    if B == 1:
        outs = [torch.empty(p, dtype=tdt, device=dev) for _ in range(sets)]
        plans = [_native.ReducePlan([arenas[s][i, :p] for i in range(n)], w32, outs[s], mode)
                 for s in range(sets)]
        assert all(t.data_ptr() % 16 == 0 for t in plans[0]._keep[0]), "arena rows must be 16-B aligned"
    else:
        # B tasks per step, each with its own N input models (rows of a bigger
        # arena block) and output; sets rotate as above
        blocks = []
        for s in range(sets):
            x = torch.empty((B, n, p_pad), dtype=tdt, device=dev)
            x.copy_(arenas[s].unsqueeze(0).expand(B, n, p_pad))
            x.add_(torch.randn((B, 1, 1), generator=g, device=dev).to(tdt) * 0.01)
            blocks.append(x)
        del arenas
        outs_b = [torch.empty((B, p_pad), dtype=tdt, device=dev) for _ in range(sets)]
        plans = [_native.BatchPlan([([blocks[s][b, i, :p] for i in range(n)], w32, outs_b[s][b, :p])
                                    for b in range(B)], mode) for s in range(sets)]
        outs = [o[0, :p] for o in outs_b]
    stream = torch.cuda.current_stream(dev)

    for k in range(args.warmup):
        plans[k % sets].launch(stream)
    torch.cuda.synchronize(dev)

    K = args.steps
    # HIP events on the launch stream bracket the whole timed region: the
    # per-launch kernel time is (elapsed / K), which includes the ~1-2 us
    # launch boundaries between back-to-back kernels (so it is an upper bound
    # of the rocprofv3 per-dispatch duration).
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(K):
        plans[k % sets].launch(stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_avg_ms = ev0.elapsed_time(ev1) / K

    bytes_per_launch = (n + 1) * p * esz * B
    el_t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    tot_b = torch.tensor([bytes_per_launch * K], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot_b, op=dist.ReduceOp.SUM)
    max_el = float(el_t.item())
    total_bytes = float(tot_b.item())
    value = total_bytes / max_el / 1e9

    # copy ceiling on this device (same footprint as one step), reported beside
    cb = min(bytes_per_launch // 2, 1 << 30) & ~15
    src = torch.empty(cb, dtype=torch.uint8, device=dev).fill_(1)
    dst = torch.empty_like(src)
    for _ in range(5):
        _native.probe_copy(src, dst)
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0.record(stream)
    for _ in range(20):
        _native.probe_copy(src, dst)
    c1.record(stream)
    torch.cuda.synchronize(dev)
    copy_gbps = 2 * cb * 20 / (c0.elapsed_time(c1) * 1e-3) / 1e9
    del src, dst

    allgather = None
    if world > 1:
        # slices can differ by one 64-element unit under --strong: pad to the widest
        width = p
        if args.strong:
            width = max(e - b for b, e in (_native.shard_range(p_cfg, world, r, 64) for r in range(world)))
        shard = torch.zeros(width, dtype=tdt, device=dev)
        shard[:p].copy_(outs[0])
        if args.backend != "nccl":
            shard = shard.cpu()
        full = torch.empty(width * world, dtype=tdt, device=shard.device)
        for _ in range(3):
            dist.all_gather_into_tensor(full, shard)
        torch.cuda.synchronize(dev)
        dist.barrier()
        a0 = time.perf_counter()
        reps = 10
        for _ in range(reps):
            dist.all_gather_into_tensor(full, shard)
        torch.cuda.synchronize(dev)
        ag_ms = (time.perf_counter() - a0) / reps * 1e3
        agt = torch.tensor([ag_ms], dtype=torch.float64, device=cdev)
        dist.all_reduce(agt, op=dist.ReduceOp.MAX)
        allgather = {"ms": round(float(agt.item()), 4),
                     "bytes_out_per_rank": width * esz * world,
                     "note": ("RCCL" if args.backend == "nccl" else "gloo (rehearsal)")
                             + " all_gather_into_tensor of the reduced shards (not in value)"}

    result = None
    if rank == 0:
        achieved = bytes_per_launch / (kern_avg_ms * 1e-3) / 1e9
        # PMC bytes were profiled for the plain single-task, per-rank-shard run
        traffic = pmc_traffic(args.config, args.mode) if (B == 1 and not args.strong and args.slice_of <= 1) \
            else None
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(max_el / K * 1e3, 5),
            "higher_is_better": True,
            "scaling": "strong" if (args.strong and world > 1) else "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic: torch.randn*0.05 on device, 3 rotating input sets; "
                    f"{wkind} weights",
            "config": {"workload": args.config + ": " + desc + (f" x {B} tasks per launch" if B > 1 else "")
                       + (f" (strong scaling: {p_cfg} params split over {world} ranks)" if args.strong and world > 1 else "")
                       + (f" (rank 0's slice of a {args.slice_of}-rank strong split, alone on 1 GPU)"
                          if args.slice_of > 1 and world == 1 else ""),
                       "backend": (backend_note or args.backend) if world > 1 else None,
                       "n_models": n, "params_per_rank": p, "tasks_per_step": B,
                       "mode": args.mode, "parallelism": f"param-shard x{world}",
                       "bytes_per_step_per_rank": bytes_per_launch},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic,
                         "kernel": "dlsim::k_wreduce_tiles" if B == 1 else "dlsim::k_wreduce_batch",
                         "kernel_avg_us": round(kern_avg_ms * 1e3, 2),
                         "timing": "HIP events around the K timed launches on the launch stream"},
            "copy_ceiling_GBps": round(copy_gbps, 1),
        }
        if allgather:
            result["allgather"] = allgather
    if world > 1:
        dist.barrier()
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args.config, n, p, dtype, weights, args.cpu_seconds)
        else:
            result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
