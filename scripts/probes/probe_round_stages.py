"""Probe: the stages of RoundExecutor's aggregate waves inside a real round
(train waves between them), to set against scripts/probes/probe_wave.py's wave in
isolation. Per aggregate wave, with a device sync at each boundary:
  resolve    inputs resolved to arenas / in-place tensors (_arena_of)
  launch     the batched reduce launches queued (host)
  release    the results no later task reads dropped (release_early)
  modules    the output modules built (host)
  drain      the wait for the GPU after that
Prints the median over waves, in µs per task.

    python scripts/probes/probe_round_stages.py [--model resnet18] [--peers 16] [--rounds 6]
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from bench_rounds import Settings, dag, make_model, train  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18", choices=("resnet18", "gnlenet", "flat"))
    ap.add_argument("--peers", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--release-late", action="store_true", help="RoundExecutor(release_early=False)")
    ap.add_argument("--nogc", action="store_true", help="collector disabled inside the waves (diagnostic)")
    ap.add_argument("--freeze", action="store_true", help="gc.freeze() once the models exist (application-level)")
    a = ap.parse_args()
    from dasklearn_amd import batch, rounds

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    init = copy.deepcopy(make_model(a.model)).to(dev)
    tasks, fan = dag(a.peers, a.rounds)
    sync = torch.cuda.synchronize
    rec = []
    orig_wave = rounds.RoundExecutor._aggregate_wave
    orig_arena_tasks = batch.aggregate_arena_tasks

    def timed_arena_tasks(prepared, mode=0, on_launched=None):
        marks = {}

        def launched():
            marks["launched"] = time.perf_counter()
            if on_launched is not None:
                on_launched()
            marks["released"] = time.perf_counter()
        t0 = time.perf_counter()
        mods = orig_arena_tasks(prepared, mode, launched)
        t1 = time.perf_counter()
        sync()
        t2 = time.perf_counter()
        rec[-1].update(resolve=t0 - rec[-1]["t0"], launch=marks["launched"] - t0,
                       release=marks["released"] - marks["launched"], modules=t1 - marks["released"],
                       drain=t2 - t1)
        return mods

    def timed_wave(self, aggs, on_launched=None):
        import gc
        sync()
        rec.append({"t0": time.perf_counter(), "n": len(aggs)})
        if a.nogc:
            gc.disable()
        try:
            return orig_wave(self, aggs, on_launched)
        finally:
            gc.enable()

    rounds.aggregate_arena_tasks = timed_arena_tasks
    rounds.RoundExecutor._aggregate_wave = timed_wave
    if a.freeze:
        import gc
        gc.collect()
        gc.freeze()  # everything alive now moves to the permanent generation
    try:
        for _ in range(2):
            rec.clear()
            rounds.RoundExecutor({"train": train}, Settings(), device=dev,
                                 release_early=not a.release_late).run(tasks, seed={"init": [init]})
    finally:
        rounds.aggregate_arena_tasks = orig_arena_tasks
        rounds.RoundExecutor._aggregate_wave = orig_wave
    out = {"model": a.model, "peers": a.peers, "fan_in": fan, "waves": len(rec), "release_early": not a.release_late,
           "gc_in_waves": not a.nogc, "gc_freeze": a.freeze}
    for k in ("resolve", "launch", "release", "modules", "drain"):
        out[k + "_us_per_task"] = round(statistics.median(r[k] / r["n"] for r in rec) * 1e6, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
