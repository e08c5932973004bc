"""The reference's own deployment, timed: a broker process and W worker
processes (broker.py:137-149, 227-236; worker.py:21-38) running a D-PSGD DAG
whose models cross processes through torch.multiprocessing file_system
shared memory (broker.py:26, worker.py:6). The workers run the aggregate task
three ways, one run each:

  cpu_ref    the reference's FedAvg.aggregate op sequence (oracle restatement)
             on the host models, at the worker's 4 threads (broker.py:31)
  hip        dasklearn_amd.functions.aggregate (the drop-in hook)
  hip_cache  the same with the per-worker device model cache
             (DLSIM_DEVICE_CACHE_MB, dasklearn_amd/device_cache.py)

The train task is a synthetic CPU perturbation that returns a fresh host
model, as the reference's trainer does after training (model_trainer.py:129,
functions.py:70-77); real training needs network datasets (out of scope).
Each worker reports, like the reference's task statistics (broker.py:194-200),
the execution time of every task it ran; the line gives the median and mean
aggregate task time per way, the run's wall time, and the cache's counters.
The broker is a fresh interpreter that never touches the GPU; workers are
forked from it (the reference's start method) and initialise HIP themselves.

    python scripts/bench_workers.py [--peers 100] [--workers 4] [--rounds 6] [--model gnlenet|resnet18]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def worker_proc(way, shared, results, index, model_kind="gnlenet", profile=False):
    import copy

    import torch
    torch.multiprocessing.set_sharing_strategy("file_system")
    torch.set_num_threads(4)  # broker.py:31
    if way != "cpu_ref":
        from dasklearn_amd import device_cache
        if way == "hip_cache":
            device_cache.enable(2 << 30)
        else:
            device_cache.disable()
    if way == "cpu_ref":
        from oracle import fedavg_torch

        def aggregate(settings, params):
            return [fedavg_torch.aggregate_modules(params["models"], params.get("weights"))]
    else:
        from dasklearn_amd.functions import aggregate

    def train(settings, params):
        model = params["model"]
        out = copy.deepcopy(model)
        with torch.no_grad():
            for q in out.parameters():
                q.add_(1e-3 * (params["peer"] + 1))
        return [out]

    class Settings:
        gradient_aggregation = 1

    funcs = {"aggregate": aggregate, "train": train}

    def cache_hits():
        if way != "hip_cache":
            return 0
        from dasklearn_amd import device_cache
        return device_cache.active().stats["hits"]
    settings = Settings()
    # one untimed aggregate first: the worker's one-time start-up (HIP
    # context, library and kernel loads, staging buffers) is not a task cost
    from bench_rounds import make_model
    warm = make_model(model_kind)
    for _ in range(2):
        aggregate(settings, {"models": [warm, warm], "round": 0, "peer": 0})
    del warm
    results.put(("__ready__", index))
    stats = []
    prof = None
    if profile:  # --profile: cProfile around the aggregate calls only
        import cProfile
        prof = cProfile.Profile()
    while True:
        item = shared.get()
        if item is None:
            break
        name, fn, data = item
        h0 = cache_hits()
        if prof is not None and fn == "aggregate":
            prof.enable()
        t0 = time.perf_counter()
        res = funcs[fn](settings, data)
        stats.append((fn, time.perf_counter() - t0, cache_hits() - h0))
        if prof is not None and fn == "aggregate":
            prof.disable()
        results.put((name, res))
        del data, res
    cache = None
    if way == "hip_cache":
        from dasklearn_amd import device_cache
        c = device_cache.active()
        cache = None if c is None else dict(c.stats, entries=len(c))
    top = None
    if prof is not None:
        import io
        import pstats
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(12)
        top = buf.getvalue()
    results.put(("__stats__", (index, stats, cache, top)))


def run(way, peers, workers, rounds, model, profile=False):
    import torch
    import torch.multiprocessing as mp
    from bench_rounds import dag, make_model
    tasks, fan = dag(peers, rounds)
    by_name = {n: (f, d) for n, f, d in tasks}
    deps, consumers = {}, {}
    for n, f, d in tasks:
        refs = [m[0] for m in d["models"]] if f == "aggregate" else [d["model"][0]]
        deps[n] = refs
        for r in refs:
            consumers.setdefault(r, []).append(n)
    shared, results = mp.Queue(), mp.Queue()
    procs = [mp.Process(target=worker_proc, args=(way, shared, results, i, model, profile))
             for i in range(workers)]
    for pr in procs:
        pr.start()
    for _ in procs:  # every worker has warmed up
        tag, _i = results.get(timeout=300)
        assert tag == "__ready__"
    # the initial model is made after the fork: a parallel torch op in the
    # broker before it would leave the forked workers' OpenMP runtime locked
    # (the reference's broker makes no model either)
    torch.manual_seed(0)
    init = make_model(model)
    data = {"init": init}
    waiting = {n: sum(1 for r in deps[n] if r != "init") for n in deps}
    left = {r: len(c) for r, c in consumers.items()}

    def resolve(n):
        f, d = by_name[n]
        if f == "aggregate":
            return dict(d, models=[data[m[0]] for m in d["models"]])
        return dict(d, model=data[d["model"][0]])

    t0 = time.perf_counter()
    for n in deps:
        if waiting[n] == 0:
            shared.put((n, by_name[n][0], resolve(n)))
    done = 0
    while done < len(tasks):
        name, res = results.get(timeout=600)
        done += 1
        data[name] = res[0]
        for r in deps[name]:  # the broker clears a task's inputs once read by all (broker.py:221)
            left[r] -= 1
            if left[r] == 0 and r != "init":
                data.pop(r, None)
        for c in consumers.get(name, []):
            waiting[c] -= 1
            if waiting[c] == 0:
                shared.put((c, by_name[c][0], resolve(c)))
    wall = time.perf_counter() - t0
    for _ in procs:
        shared.put(None)
    agg, train, caches = [], [], []
    for _ in procs:
        name, (idx, stats, cache, top) = results.get(timeout=120)
        assert name == "__stats__"
        if top is not None and idx == 0:  # worker 0's profile
            print(f"== {way}: worker 0 aggregate profile\n{top}", file=sys.stderr, flush=True)
        agg += [(t, h) for f, t, h in stats if f == "aggregate"]
        train += [t for f, t, _ in stats if f == "train"]
        if cache is not None:
            caches.append(cache)
    for pr in procs:
        pr.join(timeout=60)
    times = [t for t, _ in agg]
    line = {"way": way, "model": model, "peers": peers, "workers": workers, "rounds": rounds, "fan_in": fan,
            "aggregate_tasks": len(agg), "aggregate_us_median": round(statistics.median(times) * 1e6, 1),
            "aggregate_us_mean": round(statistics.mean(times) * 1e6, 1),
            "train_us_median": round(statistics.median(train) * 1e6, 1), "wall_s": round(wall, 3)}
    if way == "hip_cache":  # median task time by the number of its inputs read from the cache
        by = {}
        for t, h in agg:
            by.setdefault(h, []).append(t)
        line["aggregate_us_median_by_hits"] = {str(h): [len(v), round(statistics.median(v) * 1e6, 1)]
                                              for h, v in sorted(by.items())}
    if caches:
        tot = {k: sum(c[k] for c in caches) for k in ("hits", "misses", "uncacheable", "bytes_not_sent")}
        tot["hit_fraction"] = round(tot["hits"] / max(1, tot["hits"] + tot["misses"] + tot["uncacheable"]), 4)
        line["device_cache"] = tot
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=100)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--ways", nargs="+", default=["cpu_ref", "hip", "hip_cache"])
    ap.add_argument("--model", choices=("gnlenet", "resnet18"), default="gnlenet")
    ap.add_argument("--profile", action="store_true", help="cProfile the aggregate calls (worker 0, stderr)")
    ap.add_argument("--one", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()
    if not a.one:
        # one fresh broker process per way: a broker that has run parallel
        # torch ops (the previous way's models) would fork workers whose
        # OpenMP runtime is left locked
        import subprocess
        rc = 0
        for way in a.ways:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", "--ways", way, "--peers",
                                str(a.peers), "--workers", str(a.workers), "--rounds", str(a.rounds), "--model",
                                a.model] + (["--profile"] if a.profile else []), timeout=900)
            rc = rc or r.returncode
        return rc
    import torch.multiprocessing as mp
    mp.set_sharing_strategy("file_system")  # broker.py:26
    from bench import box_info
    box = box_info()
    for way in a.ways:
        print(json.dumps(dict(run(way, a.peers, a.workers, a.rounds, a.model, a.profile), box=box)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
