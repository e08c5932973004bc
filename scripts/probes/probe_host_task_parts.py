"""Probe (round 4): where one host-model aggregate task's
time goes outside the library pipeline.

7 x GNLeNet (the reference's module tree, fan-in 7 = its 100-peer D-PSGD
default), host tensors in, host module out, at the worker's 4 torch threads
(broker.py:31). The task's steps are replayed one by one as
FedAvg.aggregate -> arena.aggregate_modules runs them (input_arenas, the
device output arena, the host result, the data pointers, the staging rows,
dlsim_host_wreduce, the wait, the release, the output module), each timed
with perf_counter and NO extra synchronisation (the one wait is the path's
own), medians over REPS tasks; then the whole FedAvg.aggregate call alone.
Prints one JSON line.

    python scripts/probes/probe_host_task_parts.py [reps]
    python scripts/probes/probe_host_task_parts.py [reps] --fresh

--fresh: the shipped path's steps on the same 7 models every task against 7
models made just before each task as a train task makes them (a deepcopy of
the previous aggregate, updated in place: model_trainer.py's in-place
optimiser steps), to place the ~100 us a task costs more in a round than
isolated.
"""
from __future__ import annotations

import copy

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench_rounds import GNLeNetTree  # noqa: E402
from dasklearn_amd import _native, arena  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402


def parts_once(models, dev, stream):
    n = len(models)
    marks = []
    t0 = time.perf_counter()

    def mark(name):
        nonlocal t0
        now = time.perf_counter()
        marks.append((name, now - t0))
        t0 = now

    weights = [float(1. / n) for _ in range(n)]
    w32 = _native.fp32_weights(weights)
    mark("weights")
    layout, all_params, _ = arena.input_arenas(models)
    mark("input_arenas")
    (dt, idx), = layout.groups.items()
    total = layout.totals[dt]
    out = arena.arena_empty(total, dt, dev)
    mark("device_out_alloc")
    pinned_result = arena.HOST_RESULT_PINNED or total * 4 >= arena.PAGEABLE_RESULT_BYTES
    host = torch.empty(total, dtype=dt, pin_memory=pinned_result)
    mark("host_result_alloc")
    keep, ptrs = arena._data_ptrs(all_params, idx)
    mark("data_ptrs")
    rows, pinned = arena.STAGING.acquire(dev, dt, n, total, stream)
    mark("staging_acquire")
    _native.host_wreduce_raw(ptrs, n, layout.split_sizes[dt], w32, pinned, rows, out, host, _native.dtype_code(dt),
                             _native.DLSIM_EXACT, 0, torch.get_num_threads(), stream.cuda_stream, None, None)
    mark("native_call")
    if not pinned_result:  # round 3: wait, then build the module
        stream.synchronize()
        mark("stream_wait")
    arena.STAGING.release(dev, dt, stream, not pinned_result)
    mark("staging_release")
    res = arena.module_from_arenas(models[0], layout, {dt: host})
    mark("output_module")
    if pinned_result:  # round 4: the module is built while the copies run
        stream.synchronize()
        mark("stream_wait")
    return marks, res


def fedavg_us(models, reps):
    for _ in range(20):
        FedAvg.aggregate(models, None)
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        FedAvg.aggregate(models, None)
        ts.append(time.perf_counter() - t)
    ts.sort()
    return round(statistics.median(ts) * 1e6, 1), [round(ts[len(ts) // 10] * 1e6, 1), round(ts[len(ts) * 9 // 10] * 1e6, 1)]


def fresh_parts(reps, dev, stream):
    torch.manual_seed(0)
    base = GNLeNetTree()
    same = [GNLeNetTree() for _ in range(7)]
    arena.HOST_RESULT_PINNED = True
    os.environ["DLSIM_H2D_MIN_KB"] = "1024"

    def trained(m, i):
        out = copy.deepcopy(m)
        with torch.no_grad():
            for q in out.parameters():
                q.add_(1e-3 * (i + 1))
        return out
    res = {"model": "gnlenet_tree", "n": 7, "threads": torch.get_num_threads(), "reps": reps}
    for rnd in range(2):
        for kind in ("same", "fresh"):
            acc, totals = {}, []
            agg = base
            for r in range(reps + 20):
                models = same if kind == "same" else [trained(agg, i) for i in range(7)]
                t = time.perf_counter()
                marks, out = parts_once(models, dev, stream)
                dt = time.perf_counter() - t
                if kind == "fresh":
                    agg = out  # the next task's models are trained from this result
                if r >= 20:
                    totals.append(dt)
                    for k, v in marks:
                        acc.setdefault(k, []).append(v)
            res.setdefault(f"parts_us_median_{kind}", []).append(
                {k: round(statistics.median(v) * 1e6, 1) for k, v in acc.items()})
            res.setdefault(f"parts_sum_us_median_{kind}", []).append(round(statistics.median(totals) * 1e6, 1))
    print(json.dumps(res), flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    torch.set_num_threads(4)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    if "--fresh" in sys.argv:
        return fresh_parts(reps, dev, stream)
    torch.manual_seed(0)
    models = [GNLeNetTree() for _ in range(7)]
    res = {"model": "gnlenet_tree", "n": 7, "threads": torch.get_num_threads(), "reps": reps}
    for pinned in (False, True):
        arena.HOST_RESULT_PINNED = pinned
        os.environ["DLSIM_H2D_MIN_KB"] = "1024" if pinned else "0"  # round 4's path / round 3's
        for _ in range(20):
            parts_once(models, dev, stream)
        acc, totals = {}, []
        for _ in range(reps):
            t = time.perf_counter()
            marks, _ = parts_once(models, dev, stream)
            totals.append(time.perf_counter() - t)
            for k, v in marks:
                acc.setdefault(k, []).append(v)
        key = "pinned_deferred" if pinned else "pageable_r03"
        res[f"parts_us_median_{key}"] = {k: round(statistics.median(v) * 1e6, 1) for k, v in acc.items()}
        res[f"parts_sum_us_median_{key}"] = round(statistics.median(totals) * 1e6, 1)
    # the whole call, interleaved variants: result memory x smallest H2D run
    # (DLSIM_H2D_MIN_KB, read per call by the library: 0 = every packed run at
    # once, as round 3; 4096 = one DMA for the task's 2.4 MB)
    for rnd in range(2):
        for pinned in (False, True):
            for kb in ("0", "512", "1024", "4096"):
                arena.HOST_RESULT_PINNED = pinned
                os.environ["DLSIM_H2D_MIN_KB"] = kb
                med, p1090 = fedavg_us(models, reps)
                k = f"fedavg_us_{'pinned' if pinned else 'pageable'}_h2dmin{kb}k"
                res.setdefault(k, []).append(med)
                res.setdefault(k + "_p10_p90", []).append(p1090)
    os.environ.pop("DLSIM_H2D_MIN_KB")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
