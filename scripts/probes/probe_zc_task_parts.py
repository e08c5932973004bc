"""Probe (round 6): where a small zero-copy host task's
time goes. cfg1 (2 x GNLeNet) and the 100-peer round's fan-in 7, host models
made fresh before every task as bench_rounds.py's train_host makes them
(deepcopy of the previous aggregate, updated in place), at the worker's 4
torch threads. The zero-copy path's steps (arena.reduce_modules_to_arenas ->
_host_pipeline(out=None) -> module_from_arenas) are replayed one by one with
perf_counter marks and no extra synchronisation; then the whole
functions.aggregate call on the same kind of models. Medians over REPS tasks.
Prints one JSON line per fan-in.

    python scripts/probes/probe_zc_task_parts.py [reps]
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

from bench_rounds import GNLeNetTree, Settings  # noqa: E402
from dasklearn_amd import _native, arena, functions  # noqa: E402


def trained(m, i):
    out = copy.deepcopy(m)
    with torch.no_grad():
        for q in out.parameters():
            q.add_(1e-3 * (i + 1))
    return out


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
    host = torch.empty(total, dtype=dt, pin_memory=arena.pinned_result(total * 4))
    mark("host_result_alloc")
    keep, ptrs = arena._data_ptrs(all_params, idx)
    mark("data_ptrs")
    _, rows = arena.STAGING.acquire(dev, dt, n, total, stream, device_rows=False)
    mark("staging_acquire")
    _native.host_wreduce_zc_raw(ptrs, n, layout.split_sizes[dt], w32, rows, host, _native.dtype_code(dt),
                                _native.DLSIM_EXACT, torch.get_num_threads(), stream.cuda_stream)
    mark("zc_call_pack_launch")
    res = arena.module_from_arenas(models[0], layout, {dt: host})
    mark("output_module")
    stream.synchronize()
    mark("stream_wait")
    arena.STAGING.release(dev, dt, stream, True, device_rows=False)
    mark("staging_release")
    return marks, res


def run(n, reps, dev, stream):
    torch.manual_seed(0)
    agg = GNLeNetTree()
    res = {"model": "gnlenet_tree", "n": n, "threads": torch.get_num_threads(), "reps": reps}
    settings = Settings()
    for rnd in range(2):
        acc, totals = {}, []
        for r in range(reps + 20):
            models = [trained(agg, i) for i in range(n)]
            t = time.perf_counter()
            marks, out = parts_once(models, dev, stream)
            dt = time.perf_counter() - t
            agg = out
            if r >= 20:
                totals.append(dt)
                for k, v in marks:
                    acc.setdefault(k, []).append(v)
        res.setdefault("parts_us_median", []).append({k: round(statistics.median(v) * 1e6, 1) for k, v in acc.items()})
        res.setdefault("parts_sum_us_median", []).append(round(statistics.median(totals) * 1e6, 1))
        ts = []
        for r in range(reps + 20):
            models = [trained(agg, i) for i in range(n)]
            t = time.perf_counter()
            agg = functions.aggregate(settings, {"models": models, "round": r, "peer": 0})[0]
            if r >= 20:
                ts.append(time.perf_counter() - t)
        res.setdefault("functions_aggregate_us_median", []).append(round(statistics.median(ts) * 1e6, 1))
    print(json.dumps(res), flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    torch.set_num_threads(4)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    for n in (2, 7):
        run(n, reps, dev, stream)


if __name__ == "__main__":
    main()
