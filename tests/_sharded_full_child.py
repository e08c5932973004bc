"""One rank of tests/test_gpu_sharded_multiproc.py's full-size cases (TEST
INFRASTRUCTURE).

BASELINE.json's two parameter-sharded configurations at their real geometry:
  cfg4  W = 4: gossip 2-way bf16 merge of 125,000,000 params, age weights [3/8, 5/8]
  cfg5  W = 8: FedAvg 100-client Dirichlet(1)-weighted fp32 reduce of 11,181,642 params
Every rank generates the same models on the GPU (one seeded device
generator), keeps its contiguous 64-element-aligned slice of each
(ShardedAggregator.bounds), reduces it with the product's HIP
kernel (ShardedAggregator's default local reduce) and all-gathers the slices
(gloo: every rank shares the box's one MI355X). Each rank checks its own
slice against the oracle's ordered fold over that slice; rank 0 also checks
the assembled full output against the oracle's fold over the full models
(fedavg.py:23-25). Prints one JSON line of named checks.

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/_sharded_full_child.py cfg4|cfg5
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {  # name: (models, params, dtype, weights) -- bench.py CONFIGS / weights_for
    "cfg4": (2, 125_000_000, torch.bfloat16, [3.0 / 8.0, 5.0 / 8.0]),
    "cfg5": (100, 11_181_642, torch.float32, [float(w) for w in np.random.default_rng(7).dirichlet(np.ones(100))]),
}


def host_bits(t):
    t = t.detach().cpu()
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()


def main():
    cfg = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dasklearn_amd import sharded
    from dasklearn_amd.sharded import ShardedAggregator
    from oracle import oracle as orc

    t0 = time.perf_counter()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    n, p, dt, ws = CONFIGS[cfg]
    agg = ShardedAggregator()
    b, e = agg.bounds(p)
    checks = {"hip_local_reduce": agg.local_reduce is sharded._hip_reduce,
              "slices_tile_the_axis": agg.all_bounds(p)[0][0] == 0 and agg.all_bounds(p)[-1][1] == p
              and all(agg.all_bounds(p)[r][1] == agg.all_bounds(p)[r + 1][0] for r in range(world - 1))}
    kind = "bf16" if dt == torch.bfloat16 else "f32"
    g = torch.Generator(device=dev).manual_seed(1234)
    shards = []
    full_rows = np.empty((n, p), dtype=np.uint16 if kind == "bf16" else np.float32) if rank == 0 else None
    for i in range(n):  # model by model: one full model on the device at a time
        x = (torch.randn(p, generator=g, device=dev) * 0.05).to(dt)
        shards.append(x[b:e].clone())
        if rank == 0:
            full_rows[i] = host_bits(x)
        del x
    full = agg.aggregate_param_sharded(shards, ws, p)  # HIP reduce of this slice + the gather
    torch.cuda.synchronize()
    w32 = orc.reference_weights(n, ws)
    mine = [host_bits(s) for s in shards]
    exp_slice = orc.wreduce(mine, w32, kind)
    got = host_bits(full)
    checks["full_is_on_device"] = bool(full.is_cuda and full.numel() == p and full.dtype == dt)
    checks["own_slice_bit_exact"] = orc.same_bits(got[b:e], exp_slice)
    if rank == 0:
        exp = orc.wreduce_rows_f32(full_rows, w32) if kind == "f32" else orc.wreduce(list(full_rows), w32, kind)
        checks["assembled_full_bit_exact"] = orc.same_bits(got, exp)
        checks["not_trivial"] = bool(np.any(got != 0))
    print(json.dumps({"rank": rank, "world": world, "config": cfg, "slice": [b, e],
                      "seconds": round(time.perf_counter() - t0, 1), "checks": checks}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
