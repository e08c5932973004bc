"""Probe (round 4): the north star's row layouts, each averaged over several
physical placements.

Round 3 chose the row rule (arena.row_stride: 2 MiB-aligned rows of k 2 MiB
units, k + 1 when k is a multiple of 4) from one allocation per variant; round
4 found that two allocations of the same layout differ by 1-2 % with the
pages the driver hands out. Here every layout is allocated
PLACEMENTS times (all held at once, so each gets other physical pages), and
the layouts are compared on their mean over placements. One process,
interleaved, >= 1 GiB rotating per placement, dlsim_wreduce (the bench's
launch), K launches per timing, two rounds in alternating order.

    python scripts/probes/probe_layout_placements.py [placements] [K]
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dasklearn_amd import _native  # noqa: E402
from dasklearn_amd.arena import aligned_empty, arena_empty, row_stride  # noqa: E402

N, P, SETS, ESZ = 8, 11_181_642, 3, 4
MIB2 = 2 << 20
dev = torch.device("cuda", 0)
W32 = _native.fp32_weights([float(w) for w in np.random.default_rng(7).dirichlet(np.ones(N))])
BYTES = (N + 1) * P * ESZ


def layouts():
    row = P * ESZ
    k = (row + MIB2 - 1) // MIB2
    pad256 = (P + 63) // 64 * 64
    if (pad256 * ESZ) % 65536 == 0:
        pad256 += 1024
    return {
        "shipped_2MiB_k": (MIB2, row_stride(P, ESZ) * ESZ),         # k = 22 here (not a multiple of 4)
        "2MiB_k_plus1": (MIB2, (k + 1) * MIB2),
        "256B_rows": (256, pad256 * ESZ),                              # round 1-2's rule
        "2MiB_k_stagger64K": (MIB2, k * MIB2 + (64 << 10)),
        "2MiB_k_stagger1M": (MIB2, k * MIB2 + (1 << 20)),
    }


class Sets:
    def __init__(self, align, stride_bytes, seed):
        g = torch.Generator(device=dev).manual_seed(seed)
        stride = stride_bytes // ESZ
        self.rows = aligned_empty(SETS * N * stride, torch.float32, dev, align)
        base = self.rows.data_ptr()
        self.outs = [arena_empty(P, torch.float32, dev) for _ in range(SETS)]
        for s in range(SETS):
            for i in range(N):
                off = (s * N + i) * stride
                self.rows[off:off + P].copy_(torch.randn(P, generator=g, device=dev) * 0.05)
        self.ptrs = [(ctypes.c_void_p * N)(*[base + ((s * N + i) * stride) * ESZ for i in range(N)])
                     for s in range(SETS)]
        self.wp = W32.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        self.lib = _native.load()
        self.addr_mod = base % MIB2

    def launch(self, k, stream):
        s = k % SETS
        assert self.lib.dlsim_wreduce(self.ptrs[s], N, self.wp, ctypes.c_void_p(self.outs[s].data_ptr()), P,
                                      _native.DLSIM_F32, _native.DLSIM_EXACT, stream) == 0


def timed(sets, stream, k_steps):
    h = stream.cuda_stream
    for k in range(10):
        sets.launch(k, h)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for k in range(k_steps):
        sets.launch(k, h)
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k_steps


def main():
    placements = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    k_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    stream = torch.cuda.current_stream(dev)
    lay = layouts()
    built = {(name, pl): Sets(a, sb, 1234) for pl in range(placements) for name, (a, sb) in lay.items()}
    res = {name: [] for name in lay}
    keys = list(built)
    for rnd in range(2):
        for key in (keys if rnd == 0 else keys[::-1]):
            us = timed(built[key], stream, k_steps)
            res[key[0]].append(us)
            print(json.dumps({"round": rnd, "layout": key[0], "placement": key[1], "us_per_launch": round(us, 3),
                              "frac": round(BYTES / (us * 1e-6) / 8e12, 4)}), flush=True)
    for name, v in res.items():
        print(json.dumps({"summary": name, "stride_bytes": lay[name][1], "align": lay[name][0],
                          "mean_us": round(statistics.mean(v), 3), "min_us": round(min(v), 3),
                          "max_us": round(max(v), 3), "mean_frac": round(BYTES / (statistics.mean(v) * 1e-6) / 8e12, 4)}),
              flush=True)


if __name__ == "__main__":
    main()
