"""Sweep the shipped library (dlsim_wreduce through ctypes) over fan-in n and
dtype: device-resident GB/s per configuration, timed with HIP events around
back-to-back launches on 3 rotating input sets. Prints one JSON line per case.

    python scripts/sweep_fanin.py [--p 11181642] [--reps 30]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning-simulator_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dasklearn_amd import _native  # noqa: E402


def run_case(n, p, dtype, mode, reps, dev):
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    esz = 2 if dtype == "bf16" else 4
    p_pad = (p + 127) // 128 * 128
    sets = 3
    xs = [torch.randn((n, p_pad), device=dev).to(tdt) for _ in range(sets)]
    outs = [torch.empty(p, dtype=tdt, device=dev) for _ in range(sets)]
    w = _native.fp32_weights(np.random.default_rng(n).dirichlet(np.ones(n)))
    plans = [_native.ReducePlan([xs[s][i, :p] for i in range(n)], w, outs[s], mode) for s in range(sets)]
    for k in range(20):
        plans[k % sets].launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for k in range(reps):
        plans[k % sets].launch()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    gb = (n + 1) * p * esz / (us * 1e-6) / 1e9
    del xs, outs, plans
    return {"n": n, "p": p, "dtype": dtype, "mode": "exact" if mode == 0 else "fast",
            "us": round(us, 2), "GBps": round(gb, 1), "frac": round(gb / 8000.0, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=int, default=11_181_642)
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ns = list(range(1, 21)) + [24, 33, 64, 100, 128, 129]
    for dtype in ("f32", "bf16"):
        for n in ns:
            if n > 64 and dtype == "bf16":
                continue
            print(json.dumps(run_case(n, a.p, dtype, _native.DLSIM_EXACT, a.reps, dev)), flush=True)
    for n in (2, 8, 17):
        print(json.dumps(run_case(n, a.p, "f32", _native.DLSIM_FAST, a.reps, dev)), flush=True)
        print(json.dumps(run_case(n, a.p, "bf16", _native.DLSIM_FAST, a.reps, dev)), flush=True)


if __name__ == "__main__":
    main()
