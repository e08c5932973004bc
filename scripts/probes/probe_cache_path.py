"""Probe (round 4): the device cache's host path against the normal one.

In the 4-worker deployment (scripts/bench_workers.py, profiles/r04h/) tasks
whose models all missed the cache took 711 us against 472 us for the same
task without the cache. Here, in one process, GNLeNet models in file_system
shared memory, fan-in 7, medians of FedAvg.aggregate: the normal pipeline
(cache off) on 7 new models per call, the cache with 7 new models per call
(all miss), 7 resident models (all hit), and 3 resident + 4 new. New models
are made and moved to shared memory before each timed call.

Then, with cProfile, 100 calls each of the normal pipeline and the cache on
7 new models (inputs built before profiling): the functions with the most
own time, to place the cache path's extra cost (Python or the library call).

    python scripts/probes/probe_cache_path.py [reps]
"""
import cProfile
import io
import pstats
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import torch.multiprocessing as tmp  # noqa: E402

from bench_rounds import GNLeNetTree  # noqa: E402
from dasklearn_amd import device_cache  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402


def shm_model():
    m = GNLeNetTree()
    m.share_memory()
    return m


def med(make_inputs, reps):
    ts = []
    for r in range(reps + 10):
        ms = make_inputs()
        t = time.perf_counter()
        FedAvg.aggregate(ms, None)
        if r >= 10:
            ts.append(time.perf_counter() - t)
        del ms
    return round(statistics.median(ts) * 1e6, 1)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    tmp.set_sharing_strategy("file_system")
    torch.set_num_threads(4)
    torch.cuda.set_device(0)
    torch.manual_seed(0)
    fixed = [shm_model() for _ in range(7)]
    res = {"reps": reps}
    for rnd in range(2):
        device_cache.disable()
        res.setdefault("normal_7_new", []).append(med(lambda: [shm_model() for _ in range(7)], reps))
        res.setdefault("normal_7_same", []).append(med(lambda: fixed, reps))
        c = device_cache.enable(2 << 30)
        res.setdefault("cache_7_new_all_miss", []).append(med(lambda: [shm_model() for _ in range(7)], reps))
        FedAvg.aggregate(fixed, None)
        res.setdefault("cache_7_same_all_hit", []).append(med(lambda: fixed, reps))
        res.setdefault("cache_3_same_4_new", []).append(med(lambda: fixed[:3] + [shm_model() for _ in range(4)],
                                                            reps))
        res.setdefault("cache_stats", []).append(dict(c.stats, slab_bytes=c.slab_bytes))
        # a cache of 32 rows: every miss reuses an evicted slot (device memory
        # the cache has written before) instead of a never-used one
        row = sum(q.numel() for q in fixed[0].parameters()) * 4
        c = device_cache.enable(32 * (row + 4096))
        res.setdefault("small_cache_7_new_all_miss", []).append(med(lambda: [shm_model() for _ in range(7)], reps))
        res.setdefault("small_cache_stats", []).append(dict(c.stats, slab_bytes=c.slab_bytes))
    device_cache.disable()
    print(json.dumps(res), flush=True)
    for name in ("normal", "cache"):
        if name == "cache":
            device_cache.enable(2 << 30)
        else:
            device_cache.disable()
        for _ in range(10):
            FedAvg.aggregate([shm_model() for _ in range(7)], None)
        inputs = [[shm_model() for _ in range(7)] for _ in range(100)]
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        for ms in inputs:
            FedAvg.aggregate(ms, None)
        pr.disable()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(14)
        print("== profile", name, "(100 calls)\n" + buf.getvalue(), flush=True)
        del inputs
    device_cache.disable()


if __name__ == "__main__":
    main()
