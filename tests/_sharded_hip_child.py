"""One rank of tests/test_gpu_sharded_multiproc.py (TEST INFRASTRUCTURE).

A fresh interpreter per rank, started before it touches the GPU; every rank
shares the one MI355X (cuda:0) and a gloo control plane on 127.0.0.1. The
local reduce is the product's HIP kernel (ShardedAggregator's default), not
the oracle; the oracle only checks the assembled outputs. Prints one JSON
line of named checks.

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/_sharded_hip_child.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dasklearn_amd import sharded
    from dasklearn_amd.sharded import ShardedAggregator
    from oracle import oracle as orc

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    agg = ShardedAggregator()
    checks = {"hip_local_reduce": agg.local_reduce is sharded._hip_reduce}
    n, p = 6, 64 * 1000 * world + 37  # ragged last slice
    ws = [float(v) for v in np.random.default_rng(5).dirichlet(np.ones(n))]
    w32 = orc.reference_weights(n, ws)
    g = torch.Generator().manual_seed(77)
    x32 = [(torch.randn(p, generator=g) * 0.05) for _ in range(n)]
    exp32 = orc.wreduce([x.numpy() for x in x32], w32, "f32")
    xb = [x.to(torch.bfloat16) for x in x32]
    rows_b = [x.view(torch.int16).numpy().view(np.uint16) for x in xb]
    expb = orc.wreduce(rows_b, w32, "bf16")

    def bits32(t):
        return t.detach().cpu().numpy()

    def bitsb(t):
        return t.detach().cpu().view(torch.int16).numpy().view(np.uint16)

    b, e = agg.bounds(p)
    for name, xs, exp, bits in (("f32", x32, exp32, bits32), ("bf16", xb, expb, bitsb)):
        shards = [x[b:e].contiguous().to(dev) for x in xs]
        full = agg.aggregate_param_sharded(shards, ws, p)
        checks[f"param_sharded_{name}"] = bool(full.is_cuda and orc.same_bits(bits(full), exp))
        mine = agg.aggregate_param_sharded(shards, ws, p, gather=False)
        checks[f"param_slice_{name}"] = orc.same_bits(bits(mine), exp[b:e])
        plan = agg.plan(p, n, shards[0].dtype)
        out1 = plan.run(shards, ws)
        out2 = plan.run(shards, ws)
        checks[f"plan_{name}"] = orc.same_bits(bits(out1), exp) and orc.same_bits(bits(out2), exp)
        # whole models on different ranks: all-to-all into slices, ordered fold, all-gather
        counts = [n // world + (1 if r < n % world else 0) for r in range(world)]
        first = sum(counts[:rank])
        local = [x.to(dev) for x in xs[first:first + counts[rank]]]
        full2 = agg.aggregate_model_sharded(local, counts, ws, exact=True)
        checks[f"model_sharded_exact_{name}"] = bool(full2.is_cuda and orc.same_bits(bits(full2), exp))
        # FAST: local partial sums with the HIP fma
        # reduce, reduce-scatter, all-gather; within SURVEY §8e's tolerance of
        # the exact sum: (n + W) * 2^-23 of sum|w_i x_i| for fp32; the per-rank
        # bf16 rounding of the partial and the final cast, (W + 2) * 2^-8, for bf16
        full3 = agg.aggregate_model_sharded(local, counts, ws, exact=False)
        xf = np.stack([x.float().numpy().astype(np.float64) for x in xs])
        wf = np.asarray(w32, dtype=np.float64)[:, None]
        truth = (wf * xf).sum(0)
        mag = (np.abs(wf * xf)).sum(0)
        tol = (n + world) * 2.0 ** -23 if name == "f32" else (world + 2) * 2.0 ** -8
        got = full3.detach().float().cpu().numpy().astype(np.float64)
        err = np.abs(got - truth)
        checks[f"model_sharded_fast_{name}"] = bool(full3.is_cuda and full3.dtype == xs[0].dtype
                                                    and np.all(err <= tol * mag + 1e-30))
        checks[f"model_sharded_fast_{name}_not_trivial"] = bool(np.any(got != 0.0))
    torch.cuda.synchronize()
    print(json.dumps({"rank": rank, "world": world, "checks": checks}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
