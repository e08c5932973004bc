"""Probe: dlsim_wreduce_batched over b ResNet-18-sized tasks (fan-in 7, 11,181,642
fp32 each: RoundExecutor's waves of device models) -- with the deferred-store
kernel each such task runs alone through it (dispatch.hpp run_batched), with
DLSIM_DEFER=0 they ride one kernel-argument batch. Run it once per setting in
fresh processes (scripts/gpu_batched_large_ab.sh). Outputs rotate over >= 1 GiB.

    DLSIM_DEFER=0|1 python scripts/probes/probe_batched_large.py [b]
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
N = 7


def main():
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    stride = row_stride(P, 4)
    sets = 2  # 2 x b x 7 x 44.7 MB of inputs
    rows = aligned_empty(sets * b * N * stride, torch.float32, dev, base_align(P * 4, 4)).view(sets, b, N, stride)
    g = torch.Generator(device=dev).manual_seed(1)
    for s in range(sets):
        rows[s, :, :, :P].copy_(torch.randn((b, N, P), generator=g, device=dev) * 0.05)
    out_sets = max(sets, -(-(1 << 30) // (b * P * 4)))
    outs = [[arena_empty(P, torch.float32, dev) for _ in range(b)] for _ in range(out_sets)]
    w = np.random.default_rng(7).dirichlet(np.ones(N))
    w32 = _native.fp32_weights(w)

    def call(k):
        s = k % sets
        tasks = [([rows[s, t, i, :P] for i in range(N)], w32, outs[k % out_sets][t]) for t in range(b)]
        _native.wreduce_batched(tasks)
    for k in range(5):
        call(k)
    torch.cuda.synchronize()
    K = 40
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(K):
        call(k)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / K
    byts = b * (N + 1) * P * 4
    print(json.dumps({"b": b, "defer": os.environ.get("DLSIM_DEFER", "1"), "kernel": _native.kernel_name(N, P, torch.float32),
                      "us_per_call": round(us, 2), "us_per_task": round(us / b, 2),
                      "frac": round(byts / (us * 1e-6) / 8e12, 4)}))


if __name__ == "__main__":
    main()
