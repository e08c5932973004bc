"""Probe (round 5): a zero-copy host task for small
models. The shipped host path packs the models into page-locked staging rows,
copies them H2D, reduces, copies the result D2H (dlsim_host_wreduce). Here
the reduce kernel reads the packed page-locked rows in place over PCIe and
writes the page-locked result directly: no DMA setup in either direction.

GNLeNet host models (the reference's default; the cfg1 2-peer task and the
fan-in-7 D-PSGD task) at the worker's 4 torch threads; medians of REPS
synchronised calls, one process, interleaved:
  fedavg        the whole FedAvg.aggregate (shipped path)
  lib           dlsim_host_wreduce alone (pack, H2D, reduce, D2H) + sync
  pack          dlsim_host_pack into the page-locked rows alone
  zc            pack + dlsim_wreduce on the page-locked rows into a
                page-locked result + sync
  zc_kernel     the zero-copy reduce alone (rows already packed) + sync
  dev_kernel    the same reduce on device rows into a device result + sync
Results of zc are checked bit for bit against the shipped path's.

    python scripts/probes/probe_zero_copy.py [reps]
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench_rounds import GNLeNetTree  # noqa: E402
from dasklearn_amd import _native, arena  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402


def med(fn, reps):
    for _ in range(20):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 2)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    torch.set_num_threads(4)
    dev = torch.device("cuda", 0)
    lib = _native.load()
    stream = torch.cuda.current_stream(dev)
    out = {"threads": torch.get_num_threads()}
    for n in (2, 7):
        torch.manual_seed(n)
        models = [GNLeNetTree() for _ in range(n)]
        params = [[p.detach() for p in m.parameters()] for m in models]
        numels = [p.numel() for p in params[0]]
        total = sum(numels)
        stride = arena.row_stride(total, 4)
        pinned = torch.empty(n * stride, dtype=torch.float32, pin_memory=True)
        rows = torch.empty(n * stride, dtype=torch.float32, device=dev)
        hout = torch.empty(total, dtype=torch.float32, pin_memory=True)
        dout = torch.empty(total, dtype=torch.float32, device=dev)
        w32 = _native.fp32_weights([float(1. / n)] * n)
        wp = w32.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        srcs, offs = [], []
        for i, ps in enumerate(params):
            o = 0
            for q in ps:
                srcs.append(q)
                offs.append((i * stride + o) * 4)
                o += q.numel()
        zc_ptrs = (ctypes.c_void_p * n)(*[pinned.data_ptr() + i * stride * 4 for i in range(n)])
        dev_ptrs = (ctypes.c_void_p * n)(*[rows.data_ptr() + i * stride * 4 for i in range(n)])
        sh = stream.cuda_stream

        def fedavg():
            FedAvg.aggregate(models, None)

        def libcall():
            _native.host_wreduce(params, w32, pinned.view(n, stride), rows.view(n, stride), dout, hout)
            stream.synchronize()

        def pack():
            _native.host_pack(srcs, offs, pinned)

        def zc_kernel():
            _native._check("dlsim_wreduce", lib.dlsim_wreduce(zc_ptrs, n, wp, hout.data_ptr(), total,
                                                              _native.DLSIM_F32, _native.DLSIM_EXACT, sh))
            stream.synchronize()

        def zc():
            pack()
            zc_kernel()

        def dev_kernel():
            _native._check("dlsim_wreduce", lib.dlsim_wreduce(dev_ptrs, n, wp, dout.data_ptr(), total,
                                                              _native.DLSIM_F32, _native.DLSIM_EXACT, sh))
            stream.synchronize()

        ref = torch.cat([p.detach().reshape(-1) for p in FedAvg.aggregate(models, None).parameters()])
        zc()
        ok = bool(torch.equal(hout.view(torch.int32), ref.view(torch.int32)))
        libcall()
        rows.copy_(pinned.to(dev))  # device rows for dev_kernel
        torch.cuda.synchronize()
        res = {"n": n, "params": total, "zc_bit_exact": ok}
        for _ in range(2):  # two interleaved rounds
            for name, fn in (("fedavg", fedavg), ("lib", libcall), ("pack", pack), ("zc", zc),
                             ("zc_kernel", zc_kernel), ("dev_kernel", dev_kernel)):
                res.setdefault(name + "_us", []).append(med(fn, reps))
        out[f"gnlenet_n{n}"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
