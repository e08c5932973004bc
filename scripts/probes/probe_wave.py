"""Probe: where the time of one RoundExecutor aggregate wave goes, for a
D-PSGD wave of device models that are not arenas (what a device train task
returns: deepcopies of the previous outputs, separate parameter storages).

Stages, each timed with a device sync on both sides (median of reps):
  arena_of      per model, its flat arena or (separate device tensors) the
                tensors themselves, read in place
  launch        the batched reduce launches (outputs allocated, weights)
  modules       the output modules (clone of models[0] + parameter views)
and the whole wave as RoundExecutor._aggregate_wave runs it.

    python scripts/probes/probe_wave.py [--model resnet18|gnlenet] [--peers 16]
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
    ap.add_argument("--peers", type=int, default=16)
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    from dasklearn_amd import batch, rounds

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    base = make_model(a.model).to(dev)
    k = min(max(1, math.floor(math.log2(a.peers))), a.peers - 1)
    nb = ring(a.peers, k)
    models = []
    for p in range(a.peers):
        m = copy.deepcopy(base)
        with torch.no_grad():
            for q in m.parameters():
                q.add_(1e-3 * (p + 1))
        models.append(m)
    tasks = [(f"agg_{p}", "aggregate", {"models": [models[q] for q in nb[p]] + [models[p]], "round": 1, "peer": p})
             for p in range(a.peers)]
    ex = rounds.RoundExecutor({}, Settings(), device=dev)
    sync = torch.cuda.synchronize

    def stage_times():
        sync()
        t0 = time.perf_counter()
        cache = {}
        prepared = []
        for _, _, d in tasks:
            ms = d["models"]
            ents = [ex._arena_of(m, cache) for m in ms]
            views = {dt: [e[1][dt] for e in ents] for dt in ents[0][0].groups}
            prepared.append((ms[0], ents[0][0], views, batch._resolve(ms, None), [e[0].params for e in ents]))
        t_host_arena = time.perf_counter()
        sync()
        t1 = time.perf_counter()
        launched = {}

        def mark():
            launched["t"] = time.perf_counter()
        outs = batch.aggregate_arena_tasks(prepared, on_launched=mark)
        t_host_mod = time.perf_counter()
        sync()
        t2 = time.perf_counter()
        del outs
        return {"arena_of_host": t_host_arena - t0, "arena_of_sync": t1 - t0,
                "launch_host": launched["t"] - t1, "modules_host": t_host_mod - launched["t"],
                "launch_modules_sync": t2 - t1}

    def whole():
        sync()
        t0 = time.perf_counter()
        outs = ex._aggregate_wave(tasks)
        sync()
        t = time.perf_counter() - t0
        del outs
        return t

    for _ in range(2):
        stage_times()
        whole()
    recs = [stage_times() for _ in range(a.reps)]
    w = [whole() for _ in range(a.reps)]
    out = {"model": a.model, "peers": a.peers, "fan_in": k + 1,
           "wave_us_median": round(statistics.median(w) * 1e6, 1),
           "per_task_us": round(statistics.median(w) * 1e6 / a.peers, 1)}
    for key in recs[0]:
        out[key + "_us"] = round(statistics.median(r[key] for r in recs) * 1e6, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
