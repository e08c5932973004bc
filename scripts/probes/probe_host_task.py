"""Probe: one aggregate task of host models (the reference worker's case) on
the native pipeline, by pack threads and host-result memory.

7 x GNLeNet (the reference's 16-module tree, 14 tensors, 85,354 fp32; fan-in 7 = the reference's 100-peer
D-PSGD default) and 8 x ResNet-18 (62 tensors, 11,181,642 fp32), host tensors
in, host result out: `_native.host_wreduce` (dlsim_host_wreduce) alone with
1/2/4/8/16 pack threads and a pageable or page-locked result, then the whole
`FedAvg.aggregate` call; median wall time of synchronised calls (us).

    python scripts/probes/probe_host_task.py
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

from bench import resnet18_shapes  # noqa: E402
from bench_rounds import GNLeNetTree, Shaped  # noqa: E402
from dasklearn_amd import _native, arena  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402


def med(f, reps):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 1)


def main():
    dev = torch.device("cuda", 0)
    for name, n, reps in (("gnlenet", 7, 300), ("resnet18", 8, 30)):
        torch.manual_seed(0)
        models = [GNLeNetTree() if name == "gnlenet" else Shaped(resnet18_shapes()) for _ in range(n)]
        by_model = [[p.detach() for p in m.parameters()] for m in models]
        total = sum(t.numel() for t in by_model[0])
        stride = arena.row_stride(total, 4)
        stage = torch.empty((n, stride), pin_memory=True)[:, :total]
        rows = torch.empty((n, stride), device=dev)[:, :total]
        out = torch.empty(total, device=dev)
        w = _native.fp32_weights([1.0 / n] * n)
        chunk = arena.pipeline_chunk_elems(total, 4)
        h2d, d2h = arena._side_streams(dev) if chunk else (None, None)
        res = {"model": name, "n": n, "params": total}
        for pinned in (False, True):
            host = torch.empty(total, pin_memory=pinned)
            for th in (1, 2, 4, 8, 16):
                res[f"native_us_t{th}_{'pinned' if pinned else 'pageable'}"] = med(
                    lambda: _native.host_wreduce(by_model, w, stage, rows, out, host, _native.DLSIM_EXACT, chunk, th,
                                                 None, h2d, d2h), reps)
        for th in (4, 16):
            torch.set_num_threads(th)
            res[f"fedavg_us_t{th}"] = med(lambda: FedAvg.aggregate(models, None), reps)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
