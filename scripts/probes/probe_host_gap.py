"""Probe: where the 8 x ResNet-18 host aggregate spends its time, all on one
box in one process, median wall ms, 4 torch threads:

  pack_h2d_model   per model: torch.cat into a pinned row, H2D (no kernel)
  pack_h2d_chunk   the same per pipeline chunk (3 chunks), H2D on a side stream
  h2d_only         H2D of already packed rows
  pack_only        the packing alone
  aggregate        FedAvg.aggregate (the product: pack/H2D/kernel/D2H, module)
  stages           its stage breakdown (synchronising; slightly slower)

    python scripts/probes/probe_host_gap.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from torch import nn  # noqa: E402

from dasklearn_amd import arena  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402
from inputs import resnet18_cifar10_shapes  # noqa: E402


class Shaped(nn.Module):
    def __init__(self, shapes, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.ps = nn.ParameterList([nn.Parameter(torch.randn(*s, generator=g) * 0.05) for s in shapes])


def chunk_plan(layout, dt, esz, chunk_bytes=16 << 20, max_chunks=8, align=1024):
    """[(c0, c1, [(j, a, b)])]: the round-1 Python pipeline's chunks of the
    dtype group's arena and the tensor pieces [a, b) that fill each."""
    total = layout.totals[dt]
    k = max(1, min(max_chunks, round(total * esz / chunk_bytes)))
    bounds = [0]
    for c in range(1, k):
        b = (total * c // k) // align * align
        if b > bounds[-1]:
            bounds.append(b)
    bounds.append(total)
    offs, sizes = layout._group_offsets[dt], layout.split_sizes[dt]
    plan = []
    for c0, c1 in zip(bounds, bounds[1:]):
        pieces = [(j, max(c0, off) - off, min(c1, off + sz) - off)
                  for j, (off, sz) in enumerate(zip(offs, sizes)) if max(c0, off) < min(c1, off + sz)]
        plan.append((c0, c1, pieces))
    return plan


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
    torch.set_num_threads(4)
    dev = torch.device("cuda", 0)
    n = 8
    models = [Shaped(resnet18_cifar10_shapes(), i) for i in range(n)]
    flats = [[p.detach().reshape(-1) for p in m.parameters()] for m in models]
    P = sum(t.numel() for t in flats[0])
    stride = arena.row_stride(P, 4)
    pinned = torch.empty((n, stride), pin_memory=True)
    d = torch.empty((n, stride), device=dev)
    h2d = torch.cuda.Stream(dev)
    res = {"n": n, "GB_in": round(n * P * 4 / 1e9, 4)}

    def pack_h2d_model():
        for i in range(n):
            torch.cat(flats[i], out=pinned[i, :P])
            d[i, :P].copy_(pinned[i, :P], non_blocking=True)
    res["pack_h2d_model"] = med(pack_h2d_model)

    layout = arena.ParamLayout(models[0])
    plan = chunk_plan(layout, torch.float32, 4)
    sizes = layout.split_sizes[torch.float32]
    res["chunks"] = len(plan)

    def pack_h2d_chunk():
        for c0, c1, pieces in plan:
            for i in range(n):
                fl = flats[i]
                src = [fl[j] if (a == 0 and b == sizes[j]) else fl[j][a:b] for j, a, b in pieces]
                torch.cat(src, out=pinned[i, c0:c1])
                with torch.cuda.stream(h2d):
                    d[i, c0:c1].copy_(pinned[i, c0:c1], non_blocking=True)
        torch.cuda.current_stream(dev).wait_stream(h2d)
    res["pack_h2d_chunk"] = med(pack_h2d_chunk)
    res["h2d_only"] = med(lambda: d.copy_(pinned, non_blocking=True))
    res["pack_only"] = med(lambda: [torch.cat(flats[i], out=pinned[i, :P]) for i in range(n)])
    res["aggregate"] = med(lambda: FedAvg.aggregate(models, None))
    st = {}
    reps = 10
    for _ in range(reps):
        arena.aggregate_modules(models, None, 0, timing=st)
    res["stages"] = {k: round(v / reps * 1e3, 3) for k, v in st.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
