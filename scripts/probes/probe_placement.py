"""Probe (round 4): is the north star's 1-2 % spread
between bench.py's process and the tuning harness placement, data or the
timing window?

One process, interleaved rounds, >= 1 GiB rotating (3 sets of 8 x 11,181,642
fp32 rows at bench.py's row stride, 2 MiB-aligned):

  placement  torch_a / torch_b   rows from torch's caching allocator
                                 (arena.aligned_empty, as bench.py), two
                                 separate allocations held at once
             hip_a / hip_b       rows from a raw hipMalloc (the harness's
                                 allocator) through the HIP runtime torch
                                 loaded, outputs too
  data       torch_a_bits        torch_a's placement refilled with the
                                 harness's bit patterns (k_fill: exponent
                                 120..127, random sign and mantissa)
  window     K = 400 launches, and bench.py's driver shape K = 20 after 5
             warm-up launches, each with and without a GPU-side gate
             (torch.cuda._sleep before the start event, so the event does
             not time the host's enqueue of the first launch)

Every variant launches dlsim_wreduce (bench.py's entry point) with the
bench's Dirichlet weights. Prints one JSON line per (round, variant, window).

    python scripts/probes/probe_placement.py [rounds]
"""
import ctypes
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

N, P, SETS = 8, 11_181_642, 3
ESZ = 4
dev = torch.device("cuda", 0)
W32 = _native.fp32_weights([float(w) for w in np.random.default_rng(7).dirichlet(np.ones(N))])
P_PAD = row_stride(P, ESZ)
AL = base_align(P * ESZ, ESZ)
BYTES = (N + 1) * P * ESZ
GATE_CYCLES = 200_000  # ~80-100 us of GPU spin: covers the host's enqueue of e0 and the first launches

_hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
_hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
_hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
HIP_D2D = 3


def hip_malloc(nbytes):
    p = ctypes.c_void_p()
    rc = _hip.hipMalloc(ctypes.byref(p), nbytes)
    assert rc == 0, f"hipMalloc({nbytes}) -> {rc}"
    return p.value


def fill(x, how, g):
    if how == "randn":
        x.copy_(torch.randn(x.shape, generator=g, device=dev) * 0.05)
    else:
        r = torch.randint(0, 2 ** 31, x.shape, generator=g, device=dev, dtype=torch.int64)
        bits = (r & 0x807FFFFF) | ((120 + (r >> 24) % 8) << 23)
        x.copy_(bits.to(torch.int32).view(torch.float32))


class Sets:
    """SETS x N rows plus SETS outputs; ptrs[s] = row pointers of set s."""

    def __init__(self, alloc, seed, how="randn"):
        g = torch.Generator(device=dev).manual_seed(seed)
        self.keep = []
        row_bytes = P_PAD * ESZ
        if alloc == "torch":
            rows = aligned_empty(SETS * N * P_PAD, torch.float32, dev, AL).view(SETS, N, P_PAD)
            self.keep.append(rows)
            base = rows.data_ptr()
            outs = [arena_empty(P, torch.float32, dev) for _ in range(SETS)]
            self.keep += outs
            out_ptrs = [o.data_ptr() for o in outs]
            for s in range(SETS):
                fill(rows[s, :, :P], how, g)
        else:  # raw hipMalloc, 2 MiB-aligned like aligned_empty
            raw = hip_malloc(SETS * N * row_bytes + AL)
            base = (raw + AL - 1) // AL * AL
            out_ptrs = [hip_malloc(P * ESZ + 256) for _ in range(SETS)]
            tmp = torch.empty((N, P), dtype=torch.float32, device=dev)
            for s in range(SETS):
                fill(tmp, how, g)
                torch.cuda.synchronize()
                for i in range(N):
                    dst = base + (s * N + i) * row_bytes
                    assert _hip.hipMemcpy(dst, tmp[i].data_ptr(), P * ESZ, HIP_D2D) == 0
            del tmp
        torch.cuda.synchronize()
        self.base, self.out_ptrs = base, out_ptrs
        self.ptrs = [(ctypes.c_void_p * N)(*[base + (s * N + i) * row_bytes for i in range(N)])
                     for s in range(SETS)]
        self.wp = W32.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        self.lib = _native.load()

    def launch(self, k, stream):
        s = k % SETS
        rc = self.lib.dlsim_wreduce(self.ptrs[s], N, self.wp, ctypes.c_void_p(self.out_ptrs[s]), P,
                                    _native.DLSIM_F32, _native.DLSIM_EXACT, stream)
        assert rc == 0


def timed(sets, stream_obj, k_steps, warm, gate):
    stream = stream_obj.cuda_stream
    for k in range(warm):
        sets.launch(k, stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if gate:
        with torch.cuda.stream(stream_obj):
            torch.cuda._sleep(GATE_CYCLES)
    e0.record(stream_obj)
    for k in range(k_steps):
        sets.launch(k, stream)
    e1.record(stream_obj)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k_steps


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    stream = torch.cuda.current_stream(dev)
    variants = {"torch_a": Sets("torch", 1234), "hip_a": Sets("hip", 1234), "torch_b": Sets("torch", 1234),
                "hip_b": Sets("hip", 1234), "torch_a_bits": None}
    variants["torch_a_bits"] = Sets("torch", 1234, how="bits")
    print(json.dumps({"addr_mod_2MiB": {k: v.base % (2 << 20) for k, v in variants.items()},
                      "out_mod_2MiB": {k: v.out_ptrs[0] % (2 << 20) for k, v in variants.items()}}), flush=True)
    windows = [("K400", 400, 20, True), ("K400_nogate", 400, 20, False),
               ("K20w5", 20, 5, True), ("K20w5_nogate", 20, 5, False)]
    names = list(variants)
    for rnd in range(rounds):
        order = names if rnd % 2 == 0 else names[::-1]
        for name in order:
            for wname, k, warm, gate in windows:
                us = timed(variants[name], stream, k, warm, gate)
                print(json.dumps({"round": rnd, "variant": name, "window": wname, "us_per_launch": round(us, 3),
                                  "frac": round(BYTES / (us * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
