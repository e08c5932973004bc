"""Probe of the host -> device staging costs on the GPU box (for the host
path design): pinned H2D bandwidth, packing 62 ResNet-18
tensors into pinned memory (torch.cat) at 1..16 threads, and both overlapped
as FedAvg's host path does."""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402
from inputs import resnet18_cifar10_shapes  # noqa: E402


def t(f, reps=10):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    dev = torch.device("cuda", 0)
    shapes = resnet18_cifar10_shapes()
    n = 8
    models = [[torch.randn(s) for s in shapes] for _ in range(n)]
    P = sum(x.numel() for x in models[0])
    nb = P * 4
    pinned = torch.empty((n, P), pin_memory=True)
    pageable = torch.empty((n, P))
    d = torch.empty((n, P), device=dev)
    res = {"bytes_per_model": nb, "threads_avail": torch.get_num_threads()}
    res["h2d_pinned_GBps"] = round(n * nb / t(lambda: [d[i].copy_(pinned[i], non_blocking=True) for i in range(n)]) / 1e9, 1)
    res["h2d_pageable_GBps"] = round(n * nb / t(lambda: [d[i].copy_(pageable[i], non_blocking=True) for i in range(n)]) / 1e9, 1)
    res["d2h_pinned_GBps"] = round(n * nb / t(lambda: [pinned[i].copy_(d[i], non_blocking=True) for i in range(n)]) / 1e9, 1)
    flat = [[x.reshape(-1) for x in m] for m in models]
    for th in (1, 4, 16):
        torch.set_num_threads(th)
        res[f"cat_pinned_t{th}_GBps"] = round(n * nb / t(lambda: [torch.cat(flat[i], out=pinned[i]) for i in range(n)]) / 1e9, 1)
    torch.set_num_threads(4)
    offs = [0]
    for x in flat[0]:
        offs.append(offs[-1] + x.numel())

    def pack_one(i):
        row = pinned[i]
        for k, x in enumerate(flat[i]):
            row[offs[k]:offs[k + 1]].copy_(x)
        return i

    for workers in (2, 4, 8):
        pool = ThreadPoolExecutor(workers)
        res[f"pack_pool{workers}_GBps"] = round(n * nb / t(lambda: list(pool.map(pack_one, range(n)))) / 1e9, 1)

        def pipelined():
            s = torch.cuda.current_stream(dev)
            for i in pool.map(pack_one, range(n)):
                d[i].copy_(pinned[i], non_blocking=True)
        res[f"pack_pool{workers}_h2d_GBps"] = round(n * nb / t(pipelined) / 1e9, 1)
        pool.shutdown()

    def serial_pipeline():
        for i in range(n):
            torch.cat(flat[i], out=pinned[i])
            d[i].copy_(pinned[i], non_blocking=True)
    res["cat_serial_h2d_GBps"] = round(n * nb / t(serial_pipeline) / 1e9, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
