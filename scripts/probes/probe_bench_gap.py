"""Probe (round 3): why bench.py's north-star step (62.8-63.6 us) is slower
than the tuning harness's same kernel on the same 2 MiB rows (61.2-61.4 us).
Times K = 400 back-to-back ReducePlan launches (bench's launch path) with
HIP events, varying one thing at a time: the launch stream (torch's current
= the null stream, or a created stream), the input sets (one allocation per
set, or all sets in one allocation like the harness) and the data (randn *
0.05, or the harness's random bit patterns). Prints one JSON line per
variant, two rounds in rotating order.

    python scripts/probes/probe_bench_gap.py
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
p_pad = row_stride(P, 4)
al = base_align(P * 4, 4)


def fill(x, how, g):
    if how == "randn":
        x.copy_(torch.randn(x.shape, generator=g, device=dev) * 0.05)
    else:  # exponent 120..127, random sign and mantissa (the harness's k_fill)
        r = torch.randint(0, 2 ** 31, x.shape, generator=g, device=dev, dtype=torch.int64)
        bits = (r & 0x807FFFFF) | ((120 + (r >> 24) % 8) << 23)
        x.copy_(bits.to(torch.int32).view(torch.float32))


def plans(layout, how):
    g = torch.Generator(device=dev).manual_seed(1234)
    ps, keep = [], []
    if layout == "one_arena":
        big = aligned_empty(SETS * N * p_pad, torch.float32, dev, al).view(SETS, N, p_pad)
        keep.append(big)
    for s in range(SETS):
        x = big[s] if layout == "one_arena" else aligned_empty(N * p_pad, torch.float32, dev, al).view(N, p_pad)
        fill(x[:, :P], how, g)
        out = arena_empty(P, torch.float32, dev)
        ps.append(_native.ReducePlan([x[i, :P] for i in range(N)], w32, out))
        keep.append((x, out))
    return ps, keep


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
    created = torch.cuda.Stream(dev)
    variants = [(s, lay, how) for s in ("null", "created") for lay in ("per_set", "one_arena")
                for how in ("randn", "bits")]
    built = {}
    for rnd in range(2):
        order = variants if rnd == 0 else variants[::-1]
        for s, lay, how in order:
            key = (lay, how)
            if key not in built:
                built[key] = plans(lay, how)
            stream = torch.cuda.current_stream(dev) if s == "null" else created
            us = run(stream, built[key][0])
            print(json.dumps({"round": rnd, "stream": s, "layout": lay, "data": how, "us_per_launch": round(us, 3),
                              "frac": round(9 * P * 4 / (us * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
