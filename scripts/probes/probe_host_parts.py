"""Probe: the parts of one host-model aggregate task's native pipeline
(dlsim_host_wreduce) for 7 x GNLeNet (the reference worker's default task),
each timed alone with a sync, median wall µs:
  pack_t1 / pack_t16   dlsim_host_pack of the 98 parameter tensors into the
                       pinned staging rows, 1 or 16 threads
  h2d                  one H2D of the packed rows (2.4 MB) + sync
  reduce               the reduce of the rows on the device + sync
  d2h_pageable         D2H of the 85,354-float result into pageable memory
  d2h_pinned           the same into page-locked memory
  sync_empty           a sync of an idle stream
  pipeline_t16         the whole dlsim_host_wreduce call + sync (pageable result)

    python scripts/probes/probe_host_parts.py
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench_rounds import GNLeNetTree  # noqa: E402
from dasklearn_amd import _native, arena  # noqa: E402


def med(f, reps=300):
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 1)


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n = 7
    torch.manual_seed(0)
    models = [GNLeNetTree() for _ in range(n)]
    by_model = [[p.detach() for p in m.parameters()] for m in models]
    sizes = [t.numel() for t in by_model[0]]
    total = sum(sizes)
    stride = arena.row_stride(total, 4)
    stage = torch.empty((n, stride), pin_memory=True)
    rows = torch.empty((n, stride), device=dev)
    out = torch.empty(total, device=dev)
    host_pg = torch.empty(total)
    host_pin = torch.empty(total, pin_memory=True)
    w = _native.fp32_weights([1.0 / n] * n)
    srcs = [t for ts in by_model for t in ts]
    offs = []
    for i in range(n):
        o = i * stride * 4
        for sz in sizes:
            offs.append(o)
            o += sz * 4
    flat_stage = stage.view(-1).view(torch.uint8)
    ptrs = [t.data_ptr() for t in srcs]
    res = {"model": "gnlenet", "n": n, "params": total, "bytes_in": n * total * 4}
    for th in (1, 16):
        res[f"pack_t{th}"] = med(lambda: _native.host_pack(srcs, offs, flat_stage, threads=th))
    res["h2d"] = med(lambda: (rows.copy_(stage, non_blocking=True), st.synchronize()))
    views = [rows[i, :total] for i in range(n)]
    res["reduce"] = med(lambda: (_native.wreduce(views, w, out, _native.DLSIM_EXACT), st.synchronize()))
    res["d2h_pageable"] = med(lambda: (host_pg.copy_(out, non_blocking=True), st.synchronize()))
    res["d2h_pinned"] = med(lambda: (host_pin.copy_(out, non_blocking=True), st.synchronize()))
    res["sync_empty"] = med(lambda: st.synchronize())
    res["pipeline_t16"] = med(lambda: (_native.host_wreduce_raw(
        ptrs, n, sizes, w, stage[:, :total], rows[:, :total], out, host_pg, _native.DLSIM_F32,
        _native.DLSIM_EXACT, 0, 16, st.cuda_stream), st.synchronize()))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
