"""Probe: one RoundExecutor wave of device-trained ResNet-18 models (100
peers, fan-in 7), with the inputs' last references dropped once the launches
are queued (what release_early does inside a round) or kept until after the
wave. Median wall ms of the synchronised wave over fresh inputs each rep.

    python scripts/probes/probe_wave_drop.py [--model resnet18] [--peers 100]
"""
from __future__ import annotations

import argparse
import copy
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from bench_rounds import Settings, make_model, ring  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18", choices=("resnet18", "gnlenet", "flat"))
    ap.add_argument("--peers", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from dasklearn_amd import rounds
    dev = torch.device("cuda", 0)
    base = make_model(a.model).to(dev)
    k = min(max(1, math.floor(math.log2(a.peers))), a.peers - 1)
    nb = ring(a.peers, k)
    ex = rounds.RoundExecutor({}, Settings(), device=dev)

    def wave(drop: bool):
        holder = {"models": [copy.deepcopy(base) for _ in range(a.peers)]}
        ms = holder["models"]
        tasks = [(f"agg_{p}", "aggregate", {"models": [ms[q] for q in nb[p]] + [ms[p]]}) for p in range(a.peers)]
        del ms
        torch.cuda.synchronize()

        def on_launched():
            if drop:
                holder.clear()
                tasks.clear()
        t0 = time.perf_counter()
        outs = ex._aggregate_wave(tasks, on_launched)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        t1 = time.perf_counter()
        holder.clear()
        tasks.clear()
        torch.cuda.synchronize()
        after = time.perf_counter() - t1
        del outs
        return t, after

    res = {"model": a.model, "peers": a.peers}
    for drop in (False, True, False, True):
        wave(drop)
    for drop in (False, True):
        ts = [wave(drop) for _ in range(a.reps)]
        res[f"wave_ms_drop{int(drop)}"] = round(statistics.median(t for t, _ in ts) * 1e3, 2)
        res[f"free_after_ms_drop{int(drop)}"] = round(statistics.median(f for _, f in ts) * 1e3, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
