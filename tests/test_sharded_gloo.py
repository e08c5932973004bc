"""Multi-process (world 2 and 3, gloo, CPU) tests of the sharded path's
collective logic. The local reduce is the CPU oracle, injected — test
infrastructure standing in for the GPU kernel, which tests/test_gpu_*.py
check separately; the product default is the HIP kernel."""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PATHS = [ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd"), HERE]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def oracle_reduce(inputs, w32, out, mode):
    from oracle import oracle as orc
    bf16 = inputs[0].dtype == torch.bfloat16
    if inputs[0].dtype == torch.float64:  # exact double weights (weights_for_dtype)
        rows = [t.contiguous().numpy() for t in inputs]
        out.copy_(torch.from_numpy(orc.wreduce(rows, np.asarray(w32, np.float64), "f64",
                                               "exact" if mode == 0 else "fast")))
    elif bf16:
        rows = [t.contiguous().view(torch.int16).numpy().view(np.uint16) for t in inputs]
        res = orc.wreduce(rows, w32, "bf16", "exact" if mode == 0 else "fast")
        out.copy_(torch.from_numpy(res.view(np.int16).copy()).view(torch.bfloat16))
    else:
        rows = [t.contiguous().numpy() for t in inputs]
        out.copy_(torch.from_numpy(orc.wreduce(rows, w32, "f32", "exact" if mode == 0 else "fast")))


def models(n, p, dtype):
    g = torch.Generator().manual_seed(42)
    xs = [torch.randn(p, generator=g) * 0.05 for _ in range(n)]
    return [x.to(dtype) for x in xs]


def _worker(rank, world, port, p, dtype_name, q, n=5):
    for path in PATHS:
        sys.path.insert(0, path)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dasklearn_amd.sharded import ShardedAggregator
        from oracle import oracle as orc
        dtype = {"bf16": torch.bfloat16, "f64": torch.float64}.get(dtype_name, torch.float32)
        agg = ShardedAggregator(local_reduce=oracle_reduce)
        xs = models(n, p, dtype)
        weights = [0.1, 0.3, 0.2, 0.15, 0.25][:n]
        w32 = orc.reference_weights(n, weights)
        if dtype == torch.bfloat16:
            rows = [x.view(torch.int16).numpy().view(np.uint16) for x in xs]
            expect = torch.from_numpy(orc.wreduce(rows, w32, "bf16").view(np.int16).copy()).view(torch.bfloat16)
        elif dtype == torch.float64:  # the Python floats kept exact (fedavg.py:25)
            w32 = orc.reference_weights_f64(n, weights)
            expect = torch.from_numpy(orc.wreduce([x.numpy() for x in xs], w32, "f64"))
        else:
            expect = torch.from_numpy(orc.wreduce([x.numpy() for x in xs], w32, "f32"))

        def same(a, b):
            if a.dtype != b.dtype:
                return False
            if a.dtype == torch.bfloat16:
                return torch.equal(a.view(torch.int16), b.view(torch.int16))
            return torch.equal(a.view(torch.int64 if a.dtype == torch.float64 else torch.int32),
                               b.view(torch.int64 if b.dtype == torch.float64 else torch.int32))

        res = {}
        # 1) parameter-sharded: each rank holds its slice of every model
        b, e = agg.bounds(p)
        full = agg.aggregate_param_sharded([x[b:e].contiguous() for x in xs], weights, p)
        res["param_sharded_exact"] = same(full, expect)
        res["aligned_start"] = (b % 64 == 0)
        shard_only = agg.aggregate_param_sharded([x[b:e].contiguous() for x in xs], weights, p, gather=False)
        res["shard_only"] = same(shard_only, expect[b:e])
        # 2) model-sharded, exact (all-to-all into slices, then the ordered fold)
        counts = [n // world + (1 if r < n % world else 0) for r in range(world)]
        first = sum(counts[:rank])
        mine = xs[first:first + counts[rank]]
        full2 = agg.aggregate_model_sharded(mine, counts, weights, exact=True)
        res["model_sharded_exact"] = same(full2, expect)
        # 3) model-sharded, fast (partial sums + reduce-scatter): tolerance only
        full3 = agg.aggregate_model_sharded(mine, counts, weights, exact=False)
        scale = sum(abs(w) * x.double().abs() for w, x in zip(w32, xs))
        ulp = {torch.bfloat16: 2.0 ** -8, torch.float64: 2.0 ** -52}.get(dtype, 2.0 ** -23)
        res["model_sharded_fast_tol"] = bool(torch.all(
            (full3.double() - expect.double()).abs() <= (n + 2) * ulp * scale + 1e-300))
        # 4) uniform weights (None) path
        full4 = agg.aggregate_param_sharded([x[b:e].contiguous() for x in xs], None, p)
        w_u = orc.reference_weights(n, None)
        if dtype == torch.bfloat16:
            exp4 = torch.from_numpy(orc.wreduce(rows, w_u, "bf16").view(np.int16).copy()).view(torch.bfloat16)
        elif dtype == torch.float64:
            exp4 = torch.from_numpy(orc.wreduce([x.numpy() for x in xs], orc.reference_weights_f64(n, None), "f64"))
        else:
            exp4 = torch.from_numpy(orc.wreduce([x.numpy() for x in xs], w_u, "f32"))
        res["param_sharded_uniform"] = same(full4, exp4)
        # 5) a plan (agreed once): repeated runs, gathered and not
        plan = agg.plan(p, n, dtype)
        res["plan_run_1"] = same(plan.run([x[b:e].contiguous() for x in xs], weights), expect)
        res["plan_run_2"] = same(plan.run([x[b:e].contiguous() for x in xs], weights), expect)
        plan_s = agg.plan(p, n, dtype, gather=False)
        res["plan_shard_only"] = same(plan_s.run([x[b:e].contiguous() for x in xs], weights), expect[b:e])
        q.put((rank, res))
    except Exception as exc:  # surface worker failures to the parent
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,p,dtype,n", [(2, 10_003, "f32", 5), (3, 4_097, "f32", 5), (2, 5_001, "bf16", 5),
                                             (3, 130, "f32", 5), (2, 3_001, "f64", 5),
                                             (3, 1_000, "bf16", 2)])  # rank 2 holds no model
def test_sharded_paths_gloo(world, p, dtype, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, p, dtype, q, n)) for r in range(world)]
    for pr in procs:
        pr.start()
    results = {}
    for _ in range(world):
        r, res = q.get(timeout=300)
        results[r] = res
    for pr in procs:
        pr.join(timeout=60)
    for r in range(world):
        assert "error" not in results[r], results[r].get("error")
        assert all(results[r].values()), (r, results[r])


def _err_worker(rank, world, port, case, q):
    """One rank misbehaves; every rank must raise the same error promptly
    (no rank left waiting inside a collective), and the group stays usable."""
    import datetime
    import time
    for path in PATHS:
        sys.path.insert(0, path)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    try:
        from dasklearn_amd.sharded import ShardedAggregator
        agg = ShardedAggregator(local_reduce=oracle_reduce)
        n, p = 3, 1000
        xs = models(n, p, torch.float32)
        b, e = agg.bounds(p)
        shards = [x[b:e].contiguous() for x in xs]
        counts = [2, 1] if world == 2 else [1] * world
        first = sum(counts[:rank])
        mine = xs[first:first + counts[rank]]
        t0 = time.perf_counter()
        err = None
        try:
            if case == "bad_shard":
                agg.aggregate_param_sharded(shards if rank != 1 else [s[:-1] for s in shards], None, p)
            elif case == "bad_weights":
                agg.aggregate_param_sharded(shards, [0.5, 0.5] if rank == 1 else None, p)
            elif case == "gather_mismatch":
                agg.aggregate_param_sharded(shards, None, p, gather=(rank == 0))
            elif case == "bad_counts":
                agg.aggregate_model_sharded(mine, counts if rank != 1 else counts[::-1] + [0], None)
            elif case == "size_mismatch":
                agg.aggregate_model_sharded([m[:-64] for m in mine] if rank == 1 else mine, counts, None)
            elif case == "int64_shard":  # a dtype error joins the agreement too
                agg.aggregate_param_sharded(shards if rank != 1 else [s.to(torch.int64) for s in shards], None, p)
            elif case == "plan_mismatch":
                agg.plan(p, n if rank == 0 else n + 1, torch.float32)
        except Exception as ex:  # noqa: BLE001 - the error is the result
            err = (type(ex).__name__, str(ex))
        secs = time.perf_counter() - t0
        # the group is still usable afterwards
        ok = agg.aggregate_param_sharded(shards, None, p)
        q.put((rank, {"err": err, "secs": secs, "after_ok": ok.numel() == p}))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,kind,text", [
    ("bad_shard", "ValueError", "rank 1 of 2: rank 1: shard has"),
    ("bad_weights", "AssertionError", "rank 1 of 2"),
    ("gather_mismatch", "ValueError", "disagree"),
    ("bad_counts", "ValueError", "rank 1 of 2: counts must list"),
    ("size_mismatch", "ValueError", "differ in size"),
    ("int64_shard", "TypeError", "rank 1 of 2: aggregation supports"),
    ("plan_mismatch", "ValueError", "disagree"),
])
def test_sharded_errors_are_collective_gloo(case, kind, text):
    """a rank-local argument error (a wrong-length shard,
    a weight-count mismatch, disagreeing arguments) makes every rank raise the
    same error, with no rank left inside a collective."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_err_worker, args=(r, world, port, case, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    results = {}
    for _ in range(world):
        r, res = q.get(timeout=120)
        results[r] = res
    for pr in procs:
        pr.join(timeout=60)
    for r in range(world):
        assert "error" not in results[r], results[r].get("error")
        assert results[r]["err"] is not None, (r, case)
        assert results[r]["err"][0] == kind and text in results[r]["err"][1], (r, results[r]["err"])
        assert results[r]["secs"] < 20, (r, results[r]["secs"])
        assert results[r]["after_ok"]
    assert results[0]["err"] == results[1]["err"]  # the same error on every rank


def _plan_fail_worker(rank, world, port, q):
    """A plan run whose local checks fail on rank 1 (wrong-length shards):
    rank 1 raises after entering the gather, rank 0 completes with rank 1's
    slice as NaN, nobody hangs, and the plan keeps working."""
    import datetime
    import time
    for path in PATHS:
        sys.path.insert(0, path)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    try:
        from dasklearn_amd.sharded import ShardedAggregator
        from oracle import oracle as orc
        agg = ShardedAggregator(local_reduce=oracle_reduce)
        n, p = 3, 1000
        xs = models(n, p, torch.float32)
        b, e = agg.bounds(p)
        shards = [x[b:e].contiguous() for x in xs]
        plan = agg.plan(p, n, torch.float32)
        t0 = time.perf_counter()
        err, peer_nan = None, None
        try:
            got = plan.run(shards if rank != 1 else [s[:-1] for s in shards], None)
            b1, e1 = agg.bounds(p, 1)
            peer_nan = bool(torch.isnan(got[b1:e1]).all())
        except Exception as ex:  # noqa: BLE001
            err = type(ex).__name__
        secs = time.perf_counter() - t0
        again = plan.run(shards, None)
        expect = torch.from_numpy(orc.wreduce([x.numpy() for x in xs], orc.reference_weights(n, None), "f32"))
        q.put((rank, {"err": err, "secs": secs, "peer_nan": peer_nan,
                      "again": torch.equal(again.view(torch.int32), expect.view(torch.int32))}))
    except Exception:
        import traceback
        q.put((rank, {"error": traceback.format_exc()}))
    finally:
        dist.destroy_process_group()


def test_plan_run_failure_does_not_hang_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_fail_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
    for r in range(world):
        assert "error" not in results[r], results[r].get("error")
        assert results[r]["secs"] < 20 and results[r]["again"], (r, results[r])
    assert results[0]["err"] is None and results[1]["err"] == "ValueError"
    assert results[0]["peer_nan"] is True  # rank 1's slice arrived as NaN
