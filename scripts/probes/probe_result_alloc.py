"""Probe: host result buffers that stay alive (the aggregate output kept by
its caller) vs recycled: fresh pinned allocation, recycled pinned block, and
pageable memory, for a GNLeNet and a ResNet-18 sized result; us per result
(allocation + D2H). DESIGN.md §6a.

    python scripts/probes/probe_result_alloc.py
"""
import json
import time

import torch

dev = torch.device("cuda", 0)
res = {}
for label, n in (("gnlenet", 85354), ("resnet18", 11181642)):
    d = torch.randn(n, device=dev)
    keep = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        h = torch.empty(n, pin_memory=True)
        h.copy_(d, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        keep.append(h)
    res[f"{label}_pinned_retained_us"] = round((time.perf_counter() - t0) / 50 * 1e6, 1)
    keep = []
    t0 = time.perf_counter()
    for _ in range(50):
        h = torch.empty(n, pin_memory=True)
        h.copy_(d, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        del h
    res[f"{label}_pinned_recycled_us"] = round((time.perf_counter() - t0) / 50 * 1e6, 1)
    t0 = time.perf_counter()
    for _ in range(50):
        h = torch.empty(n)
        h.copy_(d)
        keep.append(h)
    res[f"{label}_pageable_retained_us"] = round((time.perf_counter() - t0) / 50 * 1e6, 1)
    keep = []
print(json.dumps(res))
