"""Probe: where the time of one `functions.aggregate` task with device models
goes (the reference worker's loop, worker.py:27-31, with models resident on
the GPU), for the reference's GNLeNet module tree and the flat 14-tensor
model, fan-in 7.

Inputs are what a device train task returns (deepcopy of an aggregate
output: separate parameter storages, so the tensor-list entry reads them in
place). Prints JSON lines: the median wall time of the whole call, the
stage breakdown of aggregate_modules (timing dict: layout, kernel, module;
synchronising), and a cProfile of the top functions.

    python scripts/probes/probe_device_task.py
"""
from __future__ import annotations

import copy
import cProfile
import gc
import io
import json
import os
import pstats
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench_rounds import Settings, make_model  # noqa: E402
from dasklearn_amd import _native, arena, functions  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for kind in ("gnlenet", "flat"):
        torch.manual_seed(0)
        base = make_model(kind).to(dev)
        models = [copy.deepcopy(base) for _ in range(7)]
        params = {"models": models, "round": 1, "peer": 0}
        sync = torch.cuda.synchronize
        for _ in range(50):
            functions.aggregate(Settings(), params)
        sync()
        gc.collect()
        gc.disable()
        ts = []
        for _ in range(500):
            t0 = time.perf_counter()
            functions.aggregate(Settings(), params)
            sync()
            ts.append(time.perf_counter() - t0)
        # back to back without a sync per call (one at the end): the rate a
        # worker's loop sustains when nothing waits on each result
        bb = []
        for _ in range(5):
            sync()
            t0 = time.perf_counter()
            for _ in range(200):
                functions.aggregate(Settings(), params)
            sync()
            bb.append((time.perf_counter() - t0) / 200)
        stages = {}
        for _ in range(300):
            st = {}
            arena.aggregate_modules(models, None, _native.DLSIM_EXACT, timing=st)
            for k, v in st.items():
                stages.setdefault(k, []).append(v)
        gc.enable()
        prof = cProfile.Profile()
        prof.enable()
        for _ in range(300):
            functions.aggregate(Settings(), params)
            sync()
        prof.disable()
        s = io.StringIO()
        pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(18)
        print(json.dumps({"model": kind, "us_call_median": round(statistics.median(ts) * 1e6, 1),
                          "us_call_min": round(min(ts) * 1e6, 1),
                          "us_call_back_to_back": round(statistics.median(bb) * 1e6, 1),
                          "stages_us_median": {k: round(statistics.median(v) * 1e6, 1) for k, v in stages.items()}}),
              flush=True)
        print(s.getvalue(), file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
