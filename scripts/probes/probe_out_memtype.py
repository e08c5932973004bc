"""Probe (round 6, session 4): does the memory type of the outputs (or the
inputs) change the north star's time? The outputs are written with
non-temporal stores; whether a line stays in L2 / the Infinity Cache before it
reaches HBM is also set by the page's memory type, which hipExtMallocWithFlags
chooses: default (coarse-grained), uncached (0x3), contiguous (0x4),
fine-grained (0x1).

The bench's workload (8 x 11,181,642 fp32, Dirichlet, exact; 3 input sets in
one contiguous block, 27 outputs >= 1 GiB, a decoy set read first) with the
outputs, or the input block, allocated through hipExtMallocWithFlags (ctypes on
libamdhip64); each leg times K launches with HIP events and checks that its
outputs match the default leg's bit for bit. Legs alternate over two passes.

    python scripts/probes/probe_out_memtype.py [K]
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

import bench  # noqa: E402
from dasklearn_amd import _native  # noqa: E402
from dasklearn_amd.arena import resident_empty, row_stride  # noqa: E402

FLAGS = {"default": 0x0, "finegrained": 0x1, "uncached": 0x3, "contiguous": 0x4}
N, P = 8, bench.RESNET18_P
dev = torch.device("cuda", 0)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]


def raw_alloc(nbytes, flag):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flag)
    if rc != 0 or not p.value:
        raise RuntimeError(f"hipExtMallocWithFlags({nbytes}, {flag:#x}) -> {rc}")
    return p.value


def main():
    k_steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    lib = _native.load()
    w32 = _native.fp32_weights(bench.weights_for("dirichlet", N))
    wp = w32.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    stride = row_stride(P, 4)
    sets = 3
    n_out = 27
    stream = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev).manual_seed(3)
    src = torch.randn((sets + 1, N, P), generator=g, device=dev) * 0.05

    def make_inputs(kind):
        nbytes = (sets + 1) * N * stride * 4
        if kind == "torch":
            blk = resident_empty((sets + 1) * N * stride, torch.float32, dev, 2 << 20)
            base = blk.data_ptr()
            keep = blk
        else:
            base = raw_alloc(nbytes + (2 << 20), FLAGS[kind])
            keep = base
            base = (base + (2 << 20) - 1) // (2 << 20) * (2 << 20)
        for s in range(sets + 1):
            for i in range(N):
                hip.hipMemcpy(base + (s * N + i) * stride * 4, src[s, i].data_ptr(), P * 4, 3)
        ptrs = [(ctypes.c_void_p * N)(*[base + (s * N + i) * stride * 4 for i in range(N)]) for s in range(sets + 1)]
        return keep, ptrs

    def make_outputs(kind):
        return [raw_alloc(P * 4 + 256, FLAGS[kind]) for _ in range(n_out + 1)]

    def run(in_kind, out_kind):
        torch.cuda.synchronize()
        keep, ptrs = make_inputs(in_kind)
        outs = make_outputs(out_kind)
        launch = lambda s, o: lib.dlsim_wreduce(ptrs[s], N, wp, ctypes.c_void_p(o), P, _native.DLSIM_F32,  # noqa: E731
                                                _native.DLSIM_EXACT, ctypes.c_void_p(stream))
        for _ in range(8):  # the decoy (set `sets`), as bench.py reads it first
            launch(sets, outs[n_out])
        torch.cuda.synchronize()
        for k in range(20):
            launch(k % sets, outs[k % n_out])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for k in range(k_steps):
            launch(k % sets, outs[k % n_out])
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / k_steps
        res = np.empty(P, dtype=np.float32)
        hip.hipMemcpy(res.ctypes.data, outs[1], P * 4, 2)
        for o in outs:
            hip.hipFree(o)
        if in_kind != "torch":
            hip.hipFree(keep)
        del keep
        return us, res

    legs = [("torch", "default"), ("torch", "uncached"), ("torch", "contiguous"), ("torch", "finegrained"),
            ("uncached", "default"), ("contiguous", "contiguous")]
    ref = None
    for rep in range(2):
        for in_kind, out_kind in legs:
            us, res = run(in_kind, out_kind)
            if ref is None:
                ref = res
            same = bool(np.array_equal(res.view(np.uint32), ref.view(np.uint32)))
            print(json.dumps({"rep": rep, "inputs": in_kind, "outputs": out_kind, "us_per_launch": round(us, 3),
                              "frac": round((N + 1) * P * 4 / us / 1e3 / 8000, 4), "same_bits": same}),
                  flush=True)


if __name__ == "__main__":
    main()
