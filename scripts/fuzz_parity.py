"""Randomised parity soak (GPU): every entry point against the oracle on random
shapes, dtypes, alignments, weights and special values, for a time budget.

  reduce      dlsim_wreduce / dlsim_wreduce_f64 (flat; exact bit-for-bit, FAST
              against its own oracle; any fan-in; sometimes in place, the
              output being one of the inputs)
  tensors     dlsim_wreduce_tensors (one model split into random tensors)
  batched     dlsim_wreduce_batched (random tasks, mixed fan-in and sizes; some
              tasks read earlier tasks' outputs or overwrite their inputs, which
              must give the results of the calls made in task order)
  chunk_mean  dlsim_chunk_mean_batched (random m, n, threads) vs PyTorch's CPU order
  modules     FedAvg.aggregate on random module trees (mixed fp32/bf16/fp16
              parameters, buffers, host or device) vs the oracle per dtype group
  reconstruct ChunkManager.reconstruct_model on random models and chunkings vs
              the reference's own arithmetic (torch.mean of torch.stack on the CPU)
  host_reduce dlsim_host_wreduce (random host tensors at odd offsets, pipeline
              chunks, pack threads, side streams or not) vs the oracle
  host_chunk  dlsim_host_chunk_mean (random tasks, threads) vs PyTorch's CPU order
  executor    RoundExecutor on random DAGs of random module trees, each train
              output on the device or the host at random (in-place tensors,
              registered arenas, uploaded host models, fp64 groups in one
              wave), random release/in-place settings, vs an oracle replay
  sharded     dlsim_wreduce_sharded and dlsim_sharded_plan (both gathers) as
              rank r of W on the stub RCCL (tests/native/stub_rccl.hip: the
              peers' slices come from buffers the case fills): random W, sizes
              (empty shards included), dtypes, repeated plan runs, vs one GPU
  cached      FedAvg.aggregate on host modules in file_system shared memory
              with the per-worker device cache on (random capacity: hits,
              misses, evictions, duplicates within a task, non-contiguous
              parameters) vs the oracle per dtype group

Prints one JSON line with the case counts and the first failures (if any).

    python scripts/fuzz_parity.py [--seconds 120] [--seed 0] [--only cached,modules]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dasklearn_amd import _native  # noqa: E402
from oracle import oracle as orc  # noqa: E402

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}


def rand_values(rng, n, p, dtype):
    if dtype == "f64":
        x = rng.standard_normal((n, p)) * np.exp(rng.uniform(-20, 20))
        if rng.random() < 0.3 and p > 0:
            k = max(1, p // 50)
            specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -1e-310, 1.7e308, 0.1, 1e-300])
            x[rng.integers(0, n, size=k), rng.integers(0, p, size=k)] = rng.choice(specials, size=k)
        return x
    scale = np.exp(rng.uniform(-6, 6)) if dtype == "f32" else np.exp(rng.uniform(-4, 4))
    x = (rng.standard_normal((n, p)) * scale).astype(np.float32)
    if rng.random() < 0.3 and p > 0:  # sprinkle special values
        k = max(1, p // 50)
        specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 3e38, 6e4, 1e-7],
                            dtype=np.float32)
        idx = rng.integers(0, p, size=k)
        rows = rng.integers(0, n, size=k)
        x[rows, idx] = rng.choice(specials, size=k)
    if dtype == "bf16":
        return orc.f32_to_bf16_bits(x)
    if dtype == "f16":
        return orc.f32_to_f16_bits(x)
    return x


def to_dev(rows, dtype, offset):
    out = []
    for r in rows:
        h = torch.from_numpy(np.ascontiguousarray(r).view(np.int16).copy()).view(DT[dtype]) if dtype in ("bf16", "f16") \
            else torch.from_numpy(np.ascontiguousarray(r).copy())
        buf = torch.empty(h.numel() + offset, dtype=h.dtype, device="cuda")
        buf[offset:].copy_(h)
        out.append(buf[offset:])
    return out


def to_host(rows, dtype):
    """Host tensors of the rows, every other one at an odd element offset."""
    out = []
    for i, r in enumerate(rows):
        h = torch.from_numpy(np.ascontiguousarray(r).view(np.int16).copy()).view(DT[dtype]) \
            if dtype in ("bf16", "f16") else torch.from_numpy(np.ascontiguousarray(r).copy())
        if i % 2:
            buf = torch.empty(h.numel() + 1, dtype=h.dtype)
            buf[1:].copy_(h)
            h = buf[1:]
        out.append(h)
    return out


def bits(t):
    t = t.cpu()
    return t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()


def first_diff(got, exp, rows, w):
    """Details of the first element where got and exp differ (for a report)."""
    g = np.asarray(got)
    e = np.asarray(exp)
    gi = g.view(np.uint16) if g.dtype == np.float16 else g.view(np.uint32) if g.dtype == np.float32 else g
    ei = e.view(np.uint16) if e.dtype == np.float16 else e.view(np.uint32) if e.dtype == np.float32 else e
    d = np.nonzero(gi != ei)[0]
    if len(d) == 0:
        return None
    j = int(d[0])
    col = [np.asarray(r).view(np.uint16)[j] if np.asarray(r).dtype != np.float32 else np.asarray(r).view(np.uint32)[j]
           for r in rows]
    return dict(idx=j, ndiff=int(len(d)), got=hex(int(gi[j])), exp=hex(int(ei[j])),
                inputs=[hex(int(c)) for c in col[:8]], weights=[float(x) for x in np.asarray(w)[:8]])


def rand_weights(rng, n, dtype="f32"):
    """Random weights as the reference's op sees them for this dtype (fp32-
    rounded; exact doubles for f64)."""
    kind = rng.integers(0, 4)
    raw = None
    if kind == 1:
        raw = [float(v) for v in rng.dirichlet(np.ones(n))]
    elif kind == 2:
        raw = [float(v) for v in rng.standard_normal(n)]  # negative weights
    elif kind == 3:
        raw = [float(v) for v in rng.choice([0.0, 1.0, 1e-39, -2.5, 0.5, 0.1], size=n)]
    return orc.reference_weights_f64(n, raw) if dtype == "f64" else orc.reference_weights(n, raw)


def rand_module(rng, seed, odd=False):
    """A random nn.Module tree: nested submodules, parameters of random shapes
    and dtypes, a BatchNorm (buffers incl. an int64 counter), a frozen
    parameter; sometimes a tied parameter and a shared submodule; with `odd`,
    sometimes a transposed (non-contiguous) parameter and a submodule without
    parameters."""
    from torch import nn
    g = torch.Generator().manual_seed(int(seed))
    n_leaf = int(rng.integers(1, 6))
    dts = [DT[str(d)] for d in rng.choice(["f32", "f32", "bf16", "f16", "f64"], size=n_leaf)]
    shapes = [tuple(int(v) for v in rng.integers(1, 40, size=int(rng.integers(1, 4)))) for _ in range(n_leaf)]
    share = bool(rng.random() < 0.3)  # a tied parameter and a shared submodule
    strided = odd and bool(rng.random() < 0.3)
    tshape = (int(rng.integers(1, 9)), int(rng.integers(2, 9)))

    class Leaf(nn.Module):
        def __init__(self, shape, dt):
            super().__init__()
            self.w = nn.Parameter((torch.randn(shape, generator=g) * 0.1).to(dt))

    class Tree(nn.Module):
        def __init__(self):
            super().__init__()
            self.leaves = nn.ModuleList([Leaf(sh, dt) for sh, dt in zip(shapes, dts)])
            self.bn = nn.BatchNorm1d(7)
            self.frozen = nn.Parameter(torch.randn(5, generator=g), requires_grad=False)
            if share:
                self.tied = Leaf(shapes[0], dts[0])
                self.tied.w = self.leaves[0].w  # one parameter, two attributes
                self.alias = self.leaves  # a shared submodule
            if strided:
                self.tw = nn.Parameter(torch.randn(tshape, generator=g).t())  # non-contiguous
                self.act = nn.ReLU()  # no parameters

    return Tree()


def executor_case(rng):
    """RoundExecutor on a random D-PSGD-like DAG against a host replay with the
    oracle aggregate (the reference's op sequence). Training computes its
    update on the host, so both sides train to the same bits; where each train
    output lives (device or host) is drawn per task."""
    import copy
    from dasklearn_amd.rounds import RoundExecutor
    from oracle import fedavg_torch
    n = int(rng.integers(2, 7))
    rounds = int(rng.integers(1, 3))
    base = int(rng.integers(0, 1 << 30))
    init = rand_module(np.random.default_rng(base), base, odd=True)
    place = {(p, r): str(rng.choice(["cuda", "cpu"])) for p in range(n) for r in range(1, rounds + 1)}
    tasks = []
    for r in range(1, rounds + 1):
        for p in range(n):
            src = ("init", 0) if r == 1 else (f"agg_{p}_{r - 1}", 0)
            tasks.append((f"train_{p}_{r}", "train", {"model": src, "round": r, "peer": p}))
        for p in range(n):
            nb = sorted({int(q) for q in rng.choice(n, size=int(rng.integers(1, n + 1)))} - {p})
            models = [(f"train_{q}_{r}", 0) for q in nb] + [(f"train_{p}_{r}", 0)]
            if r > 1 and rng.random() < 0.3:
                models.append((f"agg_{p}_{r - 1}", 0))  # a registered arena output too
            data = {"models": models, "round": r, "peer": p}
            if rng.random() < 0.6:
                data["weights"] = [float(v) for v in rng.standard_normal(len(models))]
            tasks.append((f"agg_{p}_{r}", "aggregate", data))

    def make_train(host_only):
        def train(settings, params):
            r, p = params["round"], params["peer"]
            out = copy.deepcopy(params["model"]).to("cpu" if host_only else place[(p, r)])
            g = torch.Generator().manual_seed(1000 * r + p)
            with torch.no_grad():
                for q in out.parameters():
                    q.copy_((q.detach().cpu() + (torch.randn(q.shape, generator=g) * 0.01).to(q.dtype)).to(q.device))
            return [out]
        return train

    class S:
        pass
    ex = RoundExecutor({"train": make_train(False)}, S(), release_early=bool(rng.random() < 0.7),
                       tensors_in_place=bool(rng.random() < 0.8))
    got = ex.run(tasks, seed={"init": [copy.deepcopy(init).to(str(rng.choice(["cuda", "cpu"])))]})
    results = {"init": [init]}
    tr = make_train(True)
    for name, func, data in tasks:
        d = {k: ([results[x[0]][x[1]] for x in v] if k == "models" else
                 (results[v[0]][v[1]] if isinstance(v, tuple) else v)) for k, v in data.items()}
        results[name] = tr(None, d) if func == "train" else [fedavg_torch.aggregate_modules(d["models"],
                                                                                            d.get("weights"))]
    ok = True
    for name, res in got.items():
        if not name.startswith("agg_"):
            continue
        a, b = res[0], results[name][0]
        for x, y in zip(a.parameters(), b.parameters()):
            ok = ok and x.dtype == y.dtype and orc.same_bits(bits(x.detach().reshape(-1).cpu()),
                                                             bits(y.detach().reshape(-1)))
    return ok, dict(kind="executor", n=n, rounds=rounds, release_early=ex.release_early,
                    in_place=ex.tensors_in_place)


def _check_modules(models, weights, out):
    """FedAvg.aggregate's result against the oracle, per dtype group."""
    n = len(models)
    ok = True
    for dt, code in ((torch.float32, "f32"), (torch.bfloat16, "bf16"), (torch.float16, "f16"),
                     (torch.float64, "f64")):
        w = orc.reference_weights_f64(n, weights) if code == "f64" else orc.reference_weights(n, weights)
        rows = []
        for m in models:
            ps = [p.detach().reshape(-1).cpu() for p in m.parameters() if p.dtype == dt]
            if ps:
                t = torch.cat(ps)
                rows.append(t.view(torch.int16).numpy().view(np.uint16) if dt in (torch.bfloat16, torch.float16)
                            else t.numpy())
        if rows:
            got = torch.cat([p.detach().reshape(-1).cpu() for p in out.parameters() if p.dtype == dt])
            ok = ok and orc.same_bits(bits(got), orc.wreduce(rows, w, code))
    return ok


STUB = os.path.join(ROOT, "tests", "native", "_build", "libstub_rccl.so")
_STUB = None


def _stub():
    global _STUB
    if _STUB is None:
        lib = ctypes.CDLL(STUB)
        vp = ctypes.c_void_p
        lib.stub_comm_create.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(vp)]
        lib.stub_comm_create.restype = vp
        lib.stub_comm_destroy.argtypes = [vp]
        lib.stub_comm_set_gather_sources.argtypes = [vp, ctypes.POINTER(vp)]
        lib.stub_comm_set_out_bytes.argtypes = [vp, ctypes.c_size_t]
        _STUB = lib
    return _STUB


def sharded_case(rng, dtype):
    """Rank r of W on the stub RCCL: its slices reduced locally, the other
    ranks' slices delivered by the stub's broadcast / all-gather from buffers
    holding what those ranks would send; the assembled output must equal the
    one-GPU reduce bit for bit."""
    stub = _stub()
    world = int(rng.choice([1, 2, 3, 4, 5, 7, 8, 12]))
    p = int(rng.choice([1, 63, 64, 100, 64 * world, 64 * world + 1, 4099, 70_001]))
    n = int(rng.choice([1, 2, 3, 8, 17]))
    gather = str(rng.choice(["bcast", "allgather"]))
    how = str(rng.choice(["agreed", "plan"]))
    r = int(rng.integers(0, world))
    rows = rand_values(rng, n, p, dtype)
    xs = to_dev(rows, dtype, 0)
    w = rand_weights(rng, n, dtype)
    full = torch.empty_like(xs[0])
    _native.wreduce(xs, w, full)
    bounds = [_native.shard_range(p, world, q, 64) for q in range(world)]
    nan = float("nan")
    peers = []
    for b, e in bounds:
        buf = torch.full_like(full, nan)
        buf[b:e].copy_(full[b:e])
        peers.append(buf)
    width = (max(e - b for b, e in bounds) + 63) // 64 * 64
    srcs = []
    for b, e in bounds:
        seg = torch.full((max(width, 1),), nan, dtype=full.dtype, device=full.device)
        seg[:e - b].copy_(full[b:e])
        srcs.append(seg)
    out = torch.full_like(full, nan)
    vp = ctypes.c_void_p
    comm = stub.stub_comm_create(world, r, out.data_ptr(), (vp * world)(*[t.data_ptr() for t in peers]))
    stub.stub_comm_set_out_bytes(comm, out.numel() * out.element_size())
    stub.stub_comm_set_gather_sources(comm, (vp * world)(*[t.data_ptr() for t in srcs]))
    _native.rccl_bind(STUB)
    try:
        b, e = bounds[r]
        shards = [x[b:e] for x in xs]
        if how == "agreed":
            _native.wreduce_sharded(shards, w, out, comm, gather)
            runs = 1
        else:
            plan = _native.ShardedPlan(comm, p, n, DT[dtype], gather, device=torch.device("cuda", 0))
            runs = int(rng.integers(1, 4))
            for _ in range(runs):
                out.fill_(nan)
                plan.run(shards, w, out)
            plan.close()
        torch.cuda.synchronize()
        ok = orc.same_bits(bits(out), bits(full))
    finally:
        _native.rccl_bind()
        stub.stub_comm_destroy(comm)
    return ok, dict(kind="sharded", dtype=dtype, world=world, rank=r, p=p, n=n, gather=gather, how=how, runs=runs)


def cached_case(rng):
    """The device cache (dasklearn_amd/device_cache.py) on a pool of shm host
    modules: several tasks draw random subsets (duplicates allowed), so models
    hit, miss and get evicted; every result exact."""
    import torch.multiprocessing as tmp
    from dasklearn_amd import arena, device_cache
    from dasklearn_amd.gradient_aggregation.fedavg import FedAvg
    prev_strategy = tmp.get_sharing_strategy()
    prev_cache = device_cache.active()
    tmp.set_sharing_strategy("file_system")
    try:
        base = int(rng.integers(0, 1 << 30))
        pool = [rand_module(np.random.default_rng(base), base + i, odd=True) for i in range(int(rng.integers(2, 10)))]
        for m in pool:
            m.share_memory()
        biggest = max(sum(p.numel() for p in m.parameters() if p.dtype == d) * torch.empty((), dtype=d).element_size()
                      for m in pool for d in (torch.float32, torch.bfloat16, torch.float16))
        rows = int(rng.integers(1, 9))
        c = device_cache.enable(rows * (arena.row_stride(max(1, biggest), 1) + 4096))
        ok, tasks = True, int(rng.integers(2, 7))
        for _ in range(tasks):
            k = int(rng.integers(1, 9))
            models = [pool[int(i)] for i in rng.integers(0, len(pool), size=k)]
            weights = None if rng.random() < 0.4 else [float(v) for v in rng.standard_normal(k)]
            out = FedAvg.aggregate(models, weights)
            ok = ok and not any(p.is_cuda for p in out.parameters()) and _check_modules(models, weights, out)
        st = dict(c.stats)
        return ok, dict(kind="cached", pool=len(pool), tasks=tasks, cap_rows=rows, hits=st["hits"],
                        misses=st["misses"], evictions=st["evictions"])
    finally:
        device_cache._CACHE = prev_cache
        tmp.set_sharing_strategy(prev_strategy)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--only", default=None, help="comma-separated families (default: all, weighted)")
    a = ap.parse_args()
    only = a.only.split(",") if a.only else None
    rng = np.random.default_rng(a.seed)
    counts = {"reduce": 0, "reduce_fast": 0, "tensors": 0, "batched": 0, "chunk_mean": 0, "modules": 0,
              "reconstruct": 0, "host_reduce": 0, "host_chunk": 0, "executor": 0, "cached": 0, "sharded": 0}
    fails = []
    t_end = time.time() + a.seconds
    t_note = time.time() + 20
    while time.time() < t_end and len(fails) < 10:
        if time.time() > t_note:  # progress (long runs must keep writing)
            print(json.dumps({"progress": counts, "failures": len(fails)}), file=sys.stderr, flush=True)
            t_note = time.time() + 20
        dtype = str(rng.choice(["f32", "bf16", "f16", "f64"]))
        which = rng.choice(["reduce", "tensors", "batched", "chunk_mean", "modules", "reconstruct",
                            "host_reduce", "host_chunk", "executor", "cached", "sharded"],
                           p=[0.18, 0.1, 0.1, 0.15, 0.1, 0.1, 0.1, 0.05, 0.05, 0.04, 0.03])
        if only:
            which = str(rng.choice(only))
        if dtype == "f64" and which not in ("reduce", "chunk_mean", "host_chunk", "sharded"):
            dtype = "f32"  # fp64 reduces are the single-task entry (dlsim_wreduce_f64); chunk means take fp64
        try:
            if which == "reduce":
                n = int(rng.choice([1, 2, 3, 5, 8, 9, 14, 15, 16, 17, 33, 128, 129, 200]))
                p = int(rng.choice([1, 2, 7, 8, 9, 63, 1000, 4099, 65537, 300_001]))
                rows = rand_values(rng, n, p, dtype)
                off = int(rng.choice([0, 0, 0, 1]))
                xs = to_dev(rows, dtype, off)
                w = rand_weights(rng, n, dtype)
                fast = rng.random() < 0.2  # one pass for every n: one final rounding
                in_place = rng.random() < 0.15
                if in_place:
                    out = xs[int(rng.integers(0, n))]
                else:
                    zero = np.zeros(p, dtype={"f32": np.float32, "f64": np.float64}.get(dtype, np.uint16))
                    out = to_dev([zero], dtype, int(rng.choice([0, 0, 1])))[0]
                _native.wreduce(xs, w, out, _native.DLSIM_FAST if fast else _native.DLSIM_EXACT)
                exp = orc.wreduce(list(rows), w, dtype, "fast" if fast else "exact")
                ok = orc.same_bits(bits(out), exp)
                counts["reduce_fast" if fast else "reduce"] += 1
                case = dict(kind="reduce", dtype=dtype, n=n, p=p, off=off, fast=bool(fast), in_place=bool(in_place))
                if not ok:
                    case["diff"] = first_diff(bits(out), exp, rows, w)
            elif which == "tensors":
                n = int(rng.choice([1, 2, 4, 8, 17, 130]))
                sizes = [int(s) for s in rng.integers(1, 5000, size=int(rng.integers(1, 12)))]
                p = sum(sizes)
                rows = rand_values(rng, n, p, dtype)
                flat = to_dev(rows, dtype, 0)
                by_model = [[t[o:o + s].clone() for o, s in zip(np.cumsum([0] + sizes[:-1]), sizes)]
                            for t in flat]
                outs = [torch.empty(s, dtype=DT[dtype], device="cuda") for s in sizes]
                w = rand_weights(rng, n)
                _native.wreduce_tensors(by_model, w, outs)
                got = np.concatenate([bits(o) for o in outs])
                ok = orc.same_bits(got, orc.wreduce(list(rows), w, dtype))
                counts["tensors"] += 1
                case = dict(kind="tensors", dtype=dtype, n=n, sizes=len(sizes))
            elif which == "batched":
                tasks, exps = [], []
                chain = rng.random() < 0.3
                p_chain = int(rng.choice([1, 5, 100, 4097]))
                for _ in range(int(rng.integers(1, 60))):
                    n = int(rng.choice([1, 2, 3, 7, 8, 16, 17, 40]))
                    p = p_chain if chain else int(rng.choice([1, 5, 100, 4097, 85_354]))
                    rows = rand_values(rng, n, p, dtype)
                    xs = to_dev(rows, dtype, int(rng.choice([0, 0, 0, 1])))
                    rows = list(rows)
                    w = rand_weights(rng, n)
                    out = torch.empty(p, dtype=DT[dtype], device="cuda")
                    if chain and tasks and rng.random() < 0.5:
                        # read an earlier task's output (its result, in task order)
                        j = int(rng.integers(0, len(tasks)))
                        i = int(rng.integers(0, n))
                        xs[i], rows[i] = tasks[j][2], exps[j][0]
                    if chain and tasks and rng.random() < 0.2:
                        # overwrite an input of an earlier task (after it was read);
                        # never one of this task's own inputs or an earlier output
                        j = int(rng.integers(0, len(tasks)))
                        cand = tasks[j][0][0]
                        if all(cand is not x for x in xs) and all(cand is not t[2] for t in tasks):
                            out = cand
                    tasks.append((xs, w, out))
                    exps.append((orc.wreduce(rows, w, dtype), rows, n, p))
                _native.wreduce_batched(tasks)
                # a buffer written by a later task holds that task's result
                final = {}
                for t, e in zip(tasks, exps):
                    final[id(t[2])] = (t[2], e[0])
                oks = [orc.same_bits(bits(t[2]), e[0]) if final[id(t[2])][1] is e[0] else True
                       for t, e in zip(tasks, exps)]
                ok = all(oks)
                counts["batched"] += 1
                case = dict(kind="batched", dtype=dtype, tasks=len(tasks))
                if not ok:
                    i = oks.index(False)
                    e, rows, n, p = exps[i]
                    case.update(task=i, n=n, p=p, diff=first_diff(bits(tasks[i][2]), e, rows, tasks[i][1]))
            elif which == "modules":
                from dasklearn_amd.gradient_aggregation.fedavg import FedAvg
                n = int(rng.choice([1, 2, 3, 8, 17]))
                base = int(rng.integers(0, 1 << 30))
                models = [rand_module(np.random.default_rng(base), base + i, odd=True) for i in range(n)]
                on_dev = bool(rng.random() < 0.5)
                if on_dev:
                    models = [m.to("cuda") for m in models]
                weights = None if rng.random() < 0.4 else [float(v) for v in rng.standard_normal(n)]
                out = FedAvg.aggregate(models, weights)
                ok = all(p.is_cuda == on_dev for p in out.parameters())
                for dt, code in ((torch.float32, "f32"), (torch.bfloat16, "bf16"), (torch.float16, "f16"),
                                 (torch.float64, "f64")):
                    w = orc.reference_weights_f64(n, weights) if code == "f64" else orc.reference_weights(n, weights)
                    rows = []
                    for m in models:
                        ps = [p.detach().reshape(-1).cpu() for p in m.parameters() if p.dtype == dt]
                        if ps:
                            t = torch.cat(ps)
                            rows.append(t.view(torch.int16).numpy().view(np.uint16) if dt == torch.bfloat16
                                        else t.numpy())
                    if rows:
                        got = torch.cat([p.detach().reshape(-1).cpu() for p in out.parameters() if p.dtype == dt])
                        ok = ok and orc.same_bits(bits(got), orc.wreduce(rows, w, code))
                ok = ok and all(torch.equal(a.cpu(), b.cpu()) for a, b in zip(out.buffers(), models[0].buffers()))
                ok = ok and [p.requires_grad for p in out.parameters()] == [p.requires_grad for p in models[0].parameters()]
                # deepcopy(models[0])'s layouts (preserve_format: a transposed weight stays
                # transposed); strides of size-1 dimensions carry no layout
                ok = ok and all(
                    all(sa == sb for sa, sb, k in zip(q.stride(), q0.stride(), q.shape) if k > 1)
                    for q, q0 in zip(out.parameters(),
                                     (torch.empty_like(t, memory_format=torch.preserve_format)
                                      for t in models[0].parameters())))
                if hasattr(models[0], "tied"):  # deepcopy(models[0]) keeps the sharing (fedavg.py:20)
                    ok = ok and out.tied.w is out.leaves[0].w and out.alias is out.leaves
                counts["modules"] += 1
                case = dict(kind="modules", n=n, device=on_dev, weighted=weights is not None)
            elif which == "reconstruct":
                from torch import nn
                from dasklearn_amd.chunk_manager import ChunkManager
                k = int(rng.integers(1, 12))
                n_peers = int(rng.integers(1, 12))
                base = int(rng.integers(0, 1 << 30))
                shape_rng = np.random.default_rng(base)
                models = [rand_module(np.random.default_rng(base), base + i) for i in range(n_peers)]
                models = [m.float() for m in models]  # chunk_model cats the state_dict (one dtype)
                chunked = [ChunkManager.chunk_model(m, k) for m in models]
                # each chunk index gets a random non-empty subset of the peers
                by_index = []
                for c in range(k):
                    who = [i for i in range(n_peers) if shape_rng.random() < 0.6] or [0]
                    by_index.append([chunked[i][c] for i in who])
                threads = int(rng.choice([1, 4, 8]))
                prev = torch.get_num_threads()
                torch.set_num_threads(threads)
                try:
                    # the reference's reconstruct_model (chunk_manager.py:34-53) on a CPU
                    # target: means, cat, copied in state_dict() order (a tied tensor
                    # appears there twice: the later copy wins), then get_flat_params
                    flat = torch.cat([torch.mean(torch.stack(cs), dim=0) for cs in by_index])
                    ref_target = rand_module(np.random.default_rng(base), base).float()
                    ptr = 0
                    with torch.no_grad():
                        for prm in ref_target.state_dict().values():
                            prm.data.copy_(flat[ptr:ptr + prm.numel()].view(prm.shape))
                            ptr += prm.numel()
                    expect = torch.cat([t.data.view(-1) for t in ref_target.state_dict().values()])
                    # every chunk on the device or every chunk on the host (the
                    # reference's stack and cat need one device), the target model
                    # on either (its copy_ crosses devices)
                    place = str(rng.choice(["device", "host"]))
                    chunks = [[c.to("cuda") if place == "device" else c for c in cs] for cs in by_index]
                    target = rand_module(np.random.default_rng(base), base).float()
                    if rng.random() < 0.5:
                        target = target.to("cuda")
                    ChunkManager.reconstruct_model(chunks, target)
                finally:
                    torch.set_num_threads(prev)
                got = ChunkManager.get_flat_params(target).cpu()
                ok = orc.same_bits(got.numpy(), expect.numpy())
                counts["reconstruct"] += 1
                case = dict(kind="reconstruct", k=k, peers=n_peers, threads=threads, place=place,
                            target=str(next(target.parameters()).device))
            elif which == "host_reduce":
                from dasklearn_amd.arena import _side_streams
                n = int(rng.choice([1, 2, 3, 8, 9, 17]))
                sizes = [int(s) for s in rng.integers(0, int(rng.choice([10, 5000, 200_000])),
                                                     size=int(rng.integers(1, 30)))]
                p = sum(sizes)
                rows = rand_values(rng, n, p, dtype)
                offs = np.cumsum([0] + sizes[:-1])
                by_model = [[t[o:o + s].clone() for o, s in zip(offs, sizes)] for t in
                            [torch.from_numpy(np.ascontiguousarray(r).view(np.int16).copy()).view(DT[dtype])
                             if dtype != "f32" else torch.from_numpy(np.ascontiguousarray(r).copy()) for r in rows]]
                for i, ts in enumerate(by_model):  # odd host offsets
                    if i % 2:
                        by_model[i] = [torch.cat([t.new_zeros(1), t])[1:] for t in ts]
                stride = (p + 63) // 64 * 64 + 64
                stage = torch.empty((n, stride), dtype=DT[dtype], pin_memory=True)
                d_rows = torch.empty((n, stride), dtype=DT[dtype], device="cuda")
                out = torch.empty(max(p, 1), dtype=DT[dtype], device="cuda")[:p]
                host = torch.empty(p, dtype=DT[dtype], pin_memory=True) if rng.random() < 0.7 else None
                chunk = int(rng.choice([0, 1024, 5000, 65536]))
                threads = int(rng.choice([1, 2, 4, 8]))
                side = bool(rng.random() < 0.5)
                h2d, d2h = _side_streams(torch.device("cuda", 0)) if side else (None, None)
                w = rand_weights(rng, n)
                _native.host_wreduce(by_model, w, stage, d_rows, out, host, _native.DLSIM_EXACT, chunk, threads,
                                     None, h2d, d2h)
                torch.cuda.current_stream().synchronize()
                exp = orc.wreduce(list(rows), w, dtype)
                ok = p == 0 or orc.same_bits(bits(out), exp)
                ok = ok and (host is None or p == 0 or orc.same_bits(bits(host), exp))
                counts["host_reduce"] += 1
                case = dict(kind="host_reduce", dtype=dtype, n=n, p=p, tensors=len(sizes), chunk=chunk,
                            threads=threads, side=side)
            elif which == "executor":
                ok, case = executor_case(rng)
                counts["executor"] += 1
            elif which == "cached":
                ok, case = cached_case(rng)
                counts["cached"] += 1
            elif which == "sharded":
                ok, case = sharded_case(rng, dtype)
                counts["sharded"] += 1
            elif which == "host_chunk":
                from dasklearn_amd.arena import _side_streams
                cpu_threads = int(rng.choice([1, 2, 4, 8, 16]))
                tasks, exps, hosts = [], [], []
                for _ in range(int(rng.integers(1, 16))):
                    m = int(rng.choice([1, 2, 3, 4, 9, 16, 17, 33, 100]))
                    n = int(rng.choice([0, 1, 2, 7, 8, 33, 1000, 8193, 100_003]))
                    if m * n > 1_000_000:
                        n = int(rng.choice([1, 7, 33, 1000]))
                    rows = rand_values(rng, m, n, dtype)
                    tasks.append((to_host(rows, dtype), torch.empty(n + 8, dtype=DT[dtype], device="cuda")[:n]))
                    hosts.append(torch.empty(n, dtype=DT[dtype], pin_memory=True))
                    exps.append(orc.chunk_mean(list(rows), dtype, cpu_threads) if n else None)
                esz = tasks[0][1].element_size()
                need = _native.staged_rows_elems([t[1].numel() for t in tasks], [len(t[0]) for t in tasks], esz)
                stage = torch.empty(max(need, 1), dtype=DT[dtype], pin_memory=True)
                d_in = torch.empty(max(need, 1), dtype=DT[dtype], device="cuda")
                side = bool(rng.random() < 0.5)
                h2d, d2h = _side_streams(torch.device("cuda", 0)) if side else (None, None)
                threads = int(rng.choice([1, 2, 4, 8]))
                _native.host_chunk_mean(tasks, stage, d_in, host_outs=hosts, threads=threads,
                                        cpu_threads=cpu_threads, h2d_stream=h2d, d2h_stream=d2h)
                torch.cuda.current_stream().synchronize()
                ok = all(e is None or (orc.same_bits(bits(t[1]), e) and orc.same_bits(bits(h), e))
                         for t, h, e in zip(tasks, hosts, exps))
                counts["host_chunk"] += 1
                case = dict(kind="host_chunk", dtype=dtype, tasks=len(tasks), threads=threads,
                            cpu_threads=cpu_threads, side=side)
            else:
                threads = int(rng.choice([1, 2, 4, 8, 16]))
                tasks, exps = [], []
                for _ in range(int(rng.integers(1, 24))):
                    m = int(rng.choice([1, 2, 3, 4, 5, 8, 9, 15, 16, 17, 31, 33, 64, 100, 250]))
                    n = int(rng.choice([1, 2, 3, 4, 7, 8, 9, 31, 32, 33, 95, 1000, 8193, 100_003]))
                    if m * n > 1_000_000:  # keeps one case's oracle work to well under a second
                        n = int(rng.choice([1, 7, 33, 1000]))
                    rows = rand_values(rng, m, n, dtype)
                    xs = to_dev(rows, dtype, int(rng.choice([0, 0, 0, 1])))
                    out = torch.empty(n, dtype=DT[dtype], device="cuda")
                    tasks.append((xs, out))
                    exps.append(orc.chunk_mean(list(rows), dtype, threads))
                _native.chunk_mean_batched(tasks, threads=threads)
                ok = all(orc.same_bits(bits(t[1]), e) for t, e in zip(tasks, exps))
                counts["chunk_mean"] += 1
                case = dict(kind="chunk_mean", dtype=dtype, tasks=len(tasks), threads=threads)
        except Exception as e:  # an unexpected exception is a failure too
            ok, case = False, dict(kind=str(which), dtype=str(dtype), error=f"{type(e).__name__}: {e}"[:300])
        if not ok:
            fails.append(case)
    torch.cuda.synchronize()
    print(json.dumps({"seconds": a.seconds, "seed": a.seed, "cases": counts, "failures": fails}), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
