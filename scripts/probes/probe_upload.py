"""Probe: uploading one wave of host-trained models (100 GNLeNets, 14 tensors
each) to the device, the RoundExecutor's step before a batched aggregate
(DESIGN.md §6a). Median wall ms per wave:

  per_tensor   torch.cat of per-tensor .to(dev) per model (the first version)
  upload       RoundExecutor._upload_host_models (dlsim_host_pack + one H2D)
  pack_only    dlsim_host_pack of the same tensors into a reused pinned buffer
  alloc_only   torch.empty(pin_memory=True) of the wave's size

    python scripts/probes/probe_upload.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd"), os.path.join(ROOT, "scripts")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from bench_rounds import GNLENET, Settings, Shaped  # noqa: E402
from dasklearn_amd import _native  # noqa: E402
from dasklearn_amd.rounds import RoundExecutor  # noqa: E402


def med(f, reps=15):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e3, 3)


def main():
    dev = torch.device("cuda", 0)
    models = [Shaped(GNLENET) for _ in range(100)]
    ex = RoundExecutor({}, Settings(), device=dev)
    res = {"models": len(models)}

    def per_tensor():
        for m in models:
            torch.cat([p.detach().reshape(-1).to(dev, non_blocking=True) for p in m.parameters()])
    res["per_tensor_ms"] = med(per_tensor)
    res["upload_ms"] = med(lambda: ex._upload_host_models(models, {}))
    srcs = [p.detach() for m in models for p in m.parameters()]
    offs, o = [], 0
    for t in srcs:
        offs.append(o)
        o += t.numel() * 4
    dst = torch.empty(o, dtype=torch.uint8, pin_memory=True)
    for th in (1, 4, torch.get_num_threads()):
        res[f"pack_only_t{th}_ms"] = med(lambda: _native.host_pack(srcs, offs, dst, threads=th))
    res["alloc_only_ms"] = med(lambda: torch.empty(o, dtype=torch.uint8, pin_memory=True))
    res["h2d_ms"] = med(lambda: torch.empty(o, dtype=torch.uint8, device=dev).copy_(dst, non_blocking=True))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
