"""Probe: staging small host models (8 x GNLeNet, 14 tensors, 85,354 fp32)
into device rows — the single-chunk host path of arena._host_pipeline.

  cat_each      torch.cat per model into a pinned row, H2D per row (shipped)
  cat_one_h2d   torch.cat per model into a pinned row, one H2D of all rows
  foreach_h2d   one torch._foreach_copy_ into pinned views, one H2D

wall ms per call (synchronised), at the box's default threads and at 4.

    python scripts/probes/probe_small_host.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402
from bench_rounds import GNLENET  # noqa: E402


def med(f, reps=200):
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
    return round(ts[len(ts) // 2] * 1e3, 4)


def main():
    dev = torch.device("cuda", 0)
    for n in (8, 2):
        models = [[torch.randn(s).reshape(-1) for s in GNLENET] for _ in range(n)]
        sizes = [t.numel() for t in models[0]]
        P = sum(sizes)
        stride = (P + 63) // 64 * 64
        pinned = torch.empty((n, stride), pin_memory=True)
        d = torch.empty((n, stride), device=dev)
        offs = [0]
        for s in sizes:
            offs.append(offs[-1] + s)

        def cat_each():
            for i in range(n):
                torch.cat(models[i], out=pinned[i, :P])
                d[i].copy_(pinned[i], non_blocking=True)

        def cat_one_h2d():
            for i in range(n):
                torch.cat(models[i], out=pinned[i, :P])
            d.copy_(pinned, non_blocking=True)

        def foreach_h2d():
            dst = [pinned[i, offs[k]:offs[k + 1]] for i in range(n) for k in range(len(sizes))]
            src = [models[i][k] for i in range(n) for k in range(len(sizes))]
            torch._foreach_copy_(dst, src)
            d.copy_(pinned, non_blocking=True)

        res = {"n": n, "params": P}
        for th in (torch.get_num_threads(), 4):
            torch.set_num_threads(th)
            for f in (cat_each, cat_one_h2d, foreach_h2d):
                res[f"{f.__name__}_t{th}_ms"] = med(f)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
