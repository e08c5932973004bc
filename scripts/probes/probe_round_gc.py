"""A/B inside one process: RoundExecutor host-model rounds (scripts/bench_rounds.py
--host workload) with Python's cyclic GC as is, and with GC paused around each
wave's aggregate, to see how much of the per-task cost is collector time driven
by the objects the simulation keeps alive. Prints JSON lines."""
from __future__ import annotations

import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning-simulator_amd"))

import torch  # noqa: E402

import bench_rounds as br  # noqa: E402
from dasklearn_amd import rounds as rmod  # noqa: E402


def run(peers, nrounds, pause_gc):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    init = br.Shaped(br.GNLENET)
    tasks, fan = br.dag(peers, nrounds)
    ex = rmod.RoundExecutor({"train": br.train_host}, br.Settings(), device=dev, timing=True)
    orig = ex._aggregate_wave
    t_up = [0.0]

    def wave(aggs, *rest):
        if pause_gc:
            gc.disable()
        try:
            return orig(aggs, *rest)
        finally:
            if pause_gc:
                gc.enable()
    ex._aggregate_wave = wave
    up = ex._upload_host_models

    def timed_up(models, cache):
        t0 = time.perf_counter()
        up(models, cache)
        torch.cuda.synchronize()
        t_up[0] += time.perf_counter() - t0
    ex._upload_host_models = timed_up
    ex.run(tasks, seed={"init": [init]})
    n = ex.stats["aggregate_tasks"]
    return {"pause_gc": pause_gc, "us_per_task": round(ex.stats["aggregate"] / n * 1e6, 1),
            "upload_us_per_task": round(t_up[0] / n * 1e6, 1), "tasks": n, "fan_in": fan,
            "gc_counts": gc.get_count()}


def main():
    run(100, 1, False)  # warm-up
    for rep in range(2):
        for pause in (False, True):
            print(json.dumps(run(100, 4, pause)), flush=True)


if __name__ == "__main__":
    main()
