"""Probe: each piece of one device-model aggregate task timed alone (median
over many calls, collector off), for the flat and the GNLeNet-tree model,
fan-in 7: the Python entry layers, input_arenas, the weight arrays, the
pointer collection, the library call (ctypes with a Python pointer list, and
the C path of the product, csrc/pyhost.cpp: launch only, and launch + sync), and
the output module build. Prints one JSON line per model.

    python scripts/probes/probe_task_parts.py
"""
from __future__ import annotations

import copy
import gc
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench_rounds import Settings, make_model  # noqa: E402
from dasklearn_amd import _native, arena, functions  # noqa: E402


def med(f, reps=400, sync=False):
    for _ in range(30):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        if sync:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    return round(statistics.median(ts) * 1e6, 2)


def main():
    dev = torch.device("cuda", 0)
    gc.disable()
    for kind in ("flat", "gnlenet"):
        torch.manual_seed(0)
        base = make_model(kind).to(dev)
        models = [copy.deepcopy(base) for _ in range(7)]
        params = {"models": models, "round": 1, "peer": 0}
        layout, all_params, views = arena.input_arenas(models)
        dt = torch.float32
        idx = layout.groups[dt]
        out = torch.empty(layout.totals[dt], device=dev)
        w32 = _native.fp32_weights([1 / 7] * 7)
        keep, ptrs = arena._data_ptrs(all_params, idx)
        base_ptr, esz = out.data_ptr(), out.element_size()
        outs = [base_ptr + layout.offsets[k] * esz for k in idx]
        stream = torch.cuda.current_stream(dev)
        arenas = {dt: out}

        def call():
            _native.wreduce_tensors_raw(ptrs, 7, layout.split_sizes[dt], w32, outs, _native.DLSIM_F32,
                                        _native.DLSIM_EXACT, stream.cuda_stream)

        def rows_call():
            _native.wreduce_rows(all_params, idx, layout.split_sizes[dt], w32, out.data_ptr(),
                                 layout.byte_offsets[dt], _native.DLSIM_F32, _native.DLSIM_EXACT, stream.cuda_stream)

        r = {"model": kind,
             "task_total_sync": med(lambda: functions.aggregate(Settings(), params), sync=True),
             "aggregate_modules_sync": med(lambda: arena.aggregate_modules(models, None, _native.DLSIM_EXACT),
                                           sync=True),
             "input_arenas": med(lambda: arena.input_arenas(models)),
             "fp32_weights+f64_weights": med(lambda: (_native.fp32_weights([1 / 7] * 7),
                                                      _native.f64_weights([1 / 7] * 7))),
             "data_ptrs": med(lambda: arena._data_ptrs(all_params, idx)),
             "torch.empty(out)": med(lambda: torch.empty(layout.totals[dt], device=dev)),
             "current_stream": med(lambda: torch.cuda.current_stream(dev)),
             "ctypes_call_launch_only": med(call),
             "ctypes_call_plus_sync": med(call, sync=True),
             "wreduce_rows_launch_only": med(rows_call),
             "wreduce_rows_plus_sync": med(rows_call, sync=True),
             "sync_only": med(lambda: None, sync=True),
             "module_from_arenas": med(lambda: arena.module_from_arenas(models[0], layout, arenas)),
             "layout_of": med(lambda: arena.layout_of(models[0]))}
        print(json.dumps(r), flush=True)

        # host models (the reference worker's case): the same task with every
        # model on the host and the result back on the host
        hmodels = [copy.deepcopy(m).cpu() for m in models]
        hparams = {"models": hmodels, "round": 1, "peer": 0}
        hlayout, hall, _ = arena.input_arenas(hmodels)
        hidx = hlayout.groups[dt]
        total = hlayout.totals[dt]

        def pipeline():
            arena._host_pipeline(hall, hidx, hlayout, dt, dev, out, w32, _native.DLSIM_EXACT, stream, True)[0]

        def stage_cycle():
            arena.STAGING.acquire(dev, dt, 7, total, stream)
            arena.STAGING.release(dev, dt, stream)

        host_arena = {dt: torch.empty(total)}
        h = {"model": kind + "_host",
             "task_total_sync": med(lambda: functions.aggregate(Settings(), hparams), sync=True),
             "input_arenas": med(lambda: arena.input_arenas(hmodels)),
             "host_pipeline_plus_sync": med(pipeline, sync=True),
             "staging_acquire_release": med(stage_cycle),
             "host_result_alloc_pageable": med(lambda: torch.empty(total)),
             "module_from_arenas": med(lambda: arena.module_from_arenas(hmodels[0], hlayout, host_arena))}
        st = {}
        for _ in range(200):
            arena.aggregate_modules(hmodels, None, _native.DLSIM_EXACT, timing=st)
        h["stages_us_mean"] = {k: round(v / 200 * 1e6, 1) for k, v in st.items()}
        print(json.dumps(h), flush=True)
    gc.enable()


if __name__ == "__main__":
    main()
