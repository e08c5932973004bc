"""Probe: the chunk-mean kernel against the weighted reduce on the SAME bytes.

Both read 4 rows of 11,181,642 fp32 and write one: the reduce (n = 4,
dlsim_wreduce) and the chunk mean (m = 4) as Conflux runs it (k = 10 chunk
tasks in one dlsim_chunk_mean_batched launch), as ONE task over the whole rows,
and the input-order mean (dlsim_mean_batched, one task). Same arena rows as
bench.py / bench_chunks.py (2 MiB-aligned rows, >= 1 GiB rotating), HIP events
around back-to-back launches, three interleaved rounds in one process.

    python scripts/probes/probe_chunk_vs_reduce.py [--m 4]
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning-simulator_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dasklearn_amd import _native  # noqa: E402
from dasklearn_amd.arena import aligned_empty, arena_empty, base_align, row_stride  # noqa: E402

P = 11_181_642


def main():
    m = int(sys.argv[sys.argv.index("--m") + 1]) if "--m" in sys.argv else 4
    k = 10
    dev = torch.device("cuda", 0)
    byts = (m + 1) * P * 4
    sets = max(3, -(-(1 << 30) // byts))
    stride = row_stride(P, 4)
    rows = aligned_empty(sets * m * stride, torch.float32, dev, base_align(P * 4, 4)).view(sets, m, stride)
    g = torch.Generator(device=dev).manual_seed(1)
    rows[:, :, :P].copy_(torch.randn((sets, m, P), generator=g, device=dev) * 0.05)
    # round 6: the outputs rotate over >= 1 GiB too (a multiple of the input
    # sets), as bench.py and bench_chunks.py since round 5
    nout = -(-max(sets, -(-(1 << 30) // (P * 4))) // sets) * sets
    outs = [arena_empty(P, torch.float32, dev) for _ in range(nout)]
    bounds = [(c * (P // k), (c + 1) * (P // k) if c < k - 1 else P) for c in range(k)]
    w = _native.fp32_weights([1.0 / m] * m)
    plans = [_native.ReducePlan([rows[j % sets, i, :P] for i in range(m)], w, outs[j]) for j in range(nout)]
    chunk_tasks = [[([rows[j % sets, i, b:e] for i in range(m)], outs[j][b:e]) for b, e in bounds]
                   for j in range(nout)]
    one_task = [[([rows[j % sets, i, :P] for i in range(m)], outs[j])] for j in range(nout)]
    mean_in = [[rows[j % sets, i, :P] for i in range(m)] for j in range(nout)]
    legs = {
        "reduce_n%d" % m: lambda s: plans[s].launch(),
        "mean_n%d (dlsim_mean, deferred)" % m: lambda s: _native.mean(mean_in[s], outs[s]),
        "chunk_mean_k10": lambda s: _native.chunk_mean_batched(chunk_tasks[s], threads=4),
        "chunk_mean_one_task": lambda s: _native.chunk_mean_batched(one_task[s], threads=4),
        "input_order_mean_one_task": lambda s: _native.mean_batched(one_task[s]),
    }
    reps = 200
    res = {name: [] for name in legs}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        for name, fn in legs.items():
            for r in range(10):
                fn(r % nout)
            torch.cuda.synchronize()
            e0.record()
            for r in range(reps):
                fn(r % nout)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / reps)
    for name, ts in res.items():
        us = sorted(ts)[1]
        print(json.dumps({"leg": name, "m": m, "sets": sets, "us": round(us, 2), "all_us": [round(t, 2) for t in ts],
                          "frac": round(byts / us / 1e3 / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
