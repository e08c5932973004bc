"""Probe (round 4): does bench.py's way of building its inputs cost time?

On one box the same layout ran at 61.1 us per launch in
probe_layout_placements.py (20 allocations, all 60.9-61.5) and at 62.6-63.0
us in five fresh bench.py processes (profiles/r04e/). The two build their
rotating sets differently: bench.py's ReduceWorkload fills each set from one
(n, P) randn temporary (358 MB, freed to torch's cache) and then allocates
that set's output, which torch's caching allocator carves out of the freed
temporary; the layout probe allocates the outputs first and fills row by row.
Here both constructions, PLACEMENTS allocations each, in one process,
interleaved: 'bench' is bench.ReduceWorkload itself, 'outs_first' the same
code with every output allocated before any fill. K launches per timing.

    python scripts/probes/probe_bench_setup.py [placements] [K]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from dasklearn_amd import _native  # noqa: E402

N, P = 8, bench.RESNET18_P
dev = torch.device("cuda", 0)


def build(kind, stream, seed):
    w32 = _native.fp32_weights(bench.weights_for("dirichlet", N))
    if kind == "bench":
        return bench.ReduceWorkload(N, P, "f32", w32, _native.DLSIM_EXACT, 1, dev, seed, stream)
    os.environ["DLSIM_BENCH_OUTS_FIRST"] = "1"
    try:
        return bench.ReduceWorkload(N, P, "f32", w32, _native.DLSIM_EXACT, 1, dev, seed, stream)
    finally:
        os.environ.pop("DLSIM_BENCH_OUTS_FIRST")


def timed(wl, k_steps):
    for k in range(10):
        wl.launch(k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(wl.stream)
    for k in range(k_steps):
        wl.launch(k)
    e1.record(wl.stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k_steps


def main():
    placements = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    k_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    stream = torch.cuda.current_stream(dev)
    kinds = ("bench", "outs_first")
    built = {(k, pl): build(k, stream, 1234) for pl in range(placements) for k in kinds}
    res = {k: [] for k in kinds}
    keys = list(built)
    for rnd in range(2):
        for key in (keys if rnd == 0 else keys[::-1]):
            us = timed(built[key], k_steps)
            res[key[0]].append(us)
            wl = built[key]
            print(json.dumps({"round": rnd, "kind": key[0], "placement": key[1], "us_per_launch": round(us, 3),
                              "out_mod_2MiB": wl.outs[0].data_ptr() % (2 << 20)}), flush=True)
    for k, v in res.items():
        print(json.dumps({"summary": k, "mean_us": round(statistics.mean(v), 3), "min_us": round(min(v), 3),
                          "max_us": round(max(v), 3),
                          "mean_frac": round(9 * P * 4 / (statistics.mean(v) * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
