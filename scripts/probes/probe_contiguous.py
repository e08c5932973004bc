"""Probe (round 4, session 2): does physically contiguous device memory
(hipExtMallocWithFlags(..., hipDeviceMallocContiguous)) take the north star
out of the page lottery of DESIGN §5b, and does it recover the 9-10 % that a
12-set (4.3 GB) rotation loses against 3 sets (the address-translation
suspect)?

One process, interleaved rounds. Each variant holds its own rotating sets of
8 x 11,181,642 fp32 rows at bench.py's row stride (2 MiB-aligned) plus one
output per set:

  torch_a / torch_b       torch's caching allocator (arena.aligned_empty, as
                          bench.py), two allocations held at once
  contig_a / contig_b     one hipExtMallocWithFlags(hipDeviceMallocContiguous)
                          block for rows and outputs
  torch12 / contig12      the same with 12 sets instead of 3

Every variant launches dlsim_wreduce (bench.py's entry point) with the
bench's Dirichlet weights and randn*0.05 rows. Prints one JSON line per
(round, variant, window).

    python scripts/probes/probe_contiguous.py [rounds]
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

N, P = 8, 11_181_642
ESZ = 4
dev = torch.device("cuda", 0)
W32 = _native.fp32_weights([float(w) for w in np.random.default_rng(7).dirichlet(np.ones(N))])
P_PAD = row_stride(P, ESZ)
AL = base_align(P * ESZ, ESZ)
BYTES = (N + 1) * P * ESZ
HIP_CONTIGUOUS = 0x4

_hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
_hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
_hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
HIP_D2D = 3


def hip_malloc_contig(nbytes):
    p = ctypes.c_void_p()
    rc = _hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, HIP_CONTIGUOUS)
    return p.value, rc


class Sets:
    def __init__(self, alloc, n_sets, seed):
        g = torch.Generator(device=dev).manual_seed(seed)
        self.n_sets = n_sets
        row_bytes = P_PAD * ESZ
        out_bytes = row_stride(P, ESZ) * ESZ
        self.keep, self.rc = [], 0
        if alloc == "contig_rows":  # rows in a contiguous block, outputs from torch (the product's split)
            total = n_sets * N * row_bytes + AL
            raw, self.rc = hip_malloc_contig(total)
            if self.rc != 0:
                raise RuntimeError(f"hipExtMallocWithFlags(contiguous, {total}) -> {self.rc}")
            base = (raw + AL - 1) // AL * AL
            outs = [arena_empty(P, torch.float32, dev) for _ in range(n_sets)]
            self.keep += outs
            out_ptrs = [o.data_ptr() for o in outs]
        elif alloc == "contig_outs":  # rows from torch, outputs in a contiguous block
            rows = aligned_empty(n_sets * N * P_PAD, torch.float32, dev, AL)
            self.keep.append(rows)
            base = rows.data_ptr()
            raw, self.rc = hip_malloc_contig(n_sets * out_bytes + AL)
            if self.rc != 0:
                raise RuntimeError(f"hipExtMallocWithFlags(contiguous) -> {self.rc}")
            ob = (raw + AL - 1) // AL * AL
            out_ptrs = [ob + s * out_bytes for s in range(n_sets)]
        elif alloc == "torch":
            rows = aligned_empty(n_sets * N * P_PAD, torch.float32, dev, AL)
            self.keep.append(rows)
            base = rows.data_ptr()
            outs = [arena_empty(P, torch.float32, dev) for _ in range(n_sets)]
            self.keep += outs
            out_ptrs = [o.data_ptr() for o in outs]
        else:
            total = n_sets * N * row_bytes + n_sets * out_bytes + AL
            raw, self.rc = hip_malloc_contig(total)
            if self.rc != 0:
                raise RuntimeError(f"hipExtMallocWithFlags(contiguous, {total}) -> {self.rc}")
            base = (raw + AL - 1) // AL * AL
            out_ptrs = [base + n_sets * N * row_bytes + s * out_bytes for s in range(n_sets)]
        tmp = torch.empty((N, P), dtype=torch.float32, device=dev)
        for s in range(n_sets):
            tmp.copy_(torch.randn((N, P), generator=g, device=dev) * 0.05)
            torch.cuda.synchronize()
            for i in range(N):
                dst = base + (s * N + i) * row_bytes
                assert _hip.hipMemcpy(dst, tmp[i].data_ptr(), P * ESZ, HIP_D2D) == 0
        del tmp
        torch.cuda.synchronize()
        self.base, self.out_ptrs = base, out_ptrs
        self.ptrs = [(ctypes.c_void_p * N)(*[base + (s * N + i) * row_bytes for i in range(N)])
                     for s in range(n_sets)]
        self.wp = W32.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        self.lib = _native.load()

    def launch(self, k, stream):
        s = k % self.n_sets
        rc = self.lib.dlsim_wreduce(self.ptrs[s], N, self.wp, ctypes.c_void_p(self.out_ptrs[s]), P,
                                    _native.DLSIM_F32, _native.DLSIM_EXACT, stream)
        assert rc == 0


def timed(sets, stream_obj, k_steps, warm):
    stream = stream_obj.cuda_stream
    for k in range(warm):
        sets.launch(k, stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream_obj)
    for k in range(k_steps):
        sets.launch(k, stream)
    e1.record(stream_obj)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k_steps


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    stream = torch.cuda.current_stream(dev)
    variants = {}
    only12 = os.environ.get("PROBE_NO12") is None
    specs = [("torch_a", "torch", 3), ("contig_a", "contig", 3), ("rows_a", "contig_rows", 3),
             ("outs_a", "contig_outs", 3), ("torch_b", "torch", 3), ("contig_b", "contig", 3),
             ("rows_b", "contig_rows", 3), ("outs_b", "contig_outs", 3)]
    if only12:
        specs += [("torch12", "torch", 12), ("contig12", "contig", 12)]
    for name, alloc, n_sets in specs:
        try:
            variants[name] = Sets(alloc, n_sets, 1234)
        except RuntimeError as e:
            print(json.dumps({"variant": name, "error": str(e)}), flush=True)
    print(json.dumps({"addr_mod_2MiB": {k: v.base % (2 << 20) for k, v in variants.items()}}), flush=True)
    windows = [("K400", 400, 20), ("K20w5", 20, 5)]
    names = list(variants)
    for rnd in range(rounds):
        order = names if rnd % 2 == 0 else names[::-1]
        for name in order:
            for wname, k, warm in windows:
                us = timed(variants[name], stream, k, warm)
                print(json.dumps({"round": rnd, "variant": name, "window": wname, "us_per_launch": round(us, 3),
                                  "frac": round(BYTES / (us * 1e-6) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
