"""Probe (round 3, second step): with the bench's sets already in one
allocation (62.2-62.3 us) the tuning harness still runs the same kernel on
the same rows at 61.3-61.5 us. Vary where the outputs live: one arena_empty
per set after its inputs are filled (bench.py), all outputs allocated before
the inputs, the outputs as rows of one output arena (row rule), and the
outputs as extra rows of the input allocation; plus data filled by randn
through a temporary (bench) or in place. Two rounds, rotating order.

    python scripts/probes/probe_bench_gap2.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dasklearn_amd import _native  # noqa: E402
from dasklearn_amd.arena import aligned_empty, arena_empty, base_align, row_stride  # noqa: E402

N, P, K, SETS = 8, 11_181_642, 400, 3
dev = torch.device("cuda", 0)
w32 = _native.fp32_weights([float(w) for w in np.random.default_rng(7).dirichlet(np.ones(N))])
stride = row_stride(P, 4)
al = base_align(P * 4, 4)


def build(kind):
    g = torch.Generator(device=dev).manual_seed(1234)
    keep = []
    if kind == "outs_first":
        outs = [arena_empty(P, torch.float32, dev) for _ in range(SETS)]
    if kind == "outs_arena":
        ob = aligned_empty(SETS * stride, torch.float32, dev, al).view(SETS, stride)
        keep.append(ob)
        outs = [ob[s, :P] for s in range(SETS)]
    rows_n = N + 1 if kind == "outs_in_rows" else N
    rows = aligned_empty(SETS * rows_n * stride, torch.float32, dev, al).view(SETS, rows_n, stride)
    keep.append(rows)
    plans = []
    for s in range(SETS):
        x = rows[s]
        if kind == "inplace_fill":
            for i in range(N):
                x[i, :P].normal_(0.0, 0.05, generator=g)
        else:
            x[:N, :P].copy_(torch.randn((N, P), generator=g, device=dev) * 0.05)
        if kind in ("bench", "inplace_fill"):
            out = arena_empty(P, torch.float32, dev)
        elif kind == "outs_in_rows":
            out = x[N, :P]
        else:
            out = outs[s]
        keep.append(out)
        plans.append(_native.ReducePlan([x[i, :P] for i in range(N)], w32, out))
    return plans, keep


def run(stream, ps):
    for k in range(20):
        ps[k % SETS].launch(stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for k in range(K):
        ps[k % SETS].launch(stream)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / K


def main():
    stream = torch.cuda.current_stream(dev)
    kinds = ["bench", "outs_first", "outs_arena", "outs_in_rows", "inplace_fill"]
    for rnd in range(2):
        for kind in (kinds if rnd == 0 else kinds[::-1]):
            ps, keep = build(kind)
            us = run(stream, ps)
            print(json.dumps({"round": rnd, "outputs": kind, "us_per_launch": round(us, 3),
                              "frac": round(9 * P * 4 / (us * 1e-6) / 8e12, 4)}), flush=True)
            del ps, keep
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
