"""Probe: the host pack of dlsim_host_wreduce, A/B in one process
(DESIGN.md §6). FedAvg.aggregate of 8 host ResNet-18-shaped models; the copy
mode (DLSIM_PACK_COPY stream|memcpy), the pipeline chunk and the thread count
vary, interleaved over rounds so box noise hits every variant alike; median
wall ms per aggregate.

    python scripts/probes/probe_host_pack.py [n]
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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    models = [Shaped(resnet18_cifar10_shapes(), i) for i in range(n)]
    variants = [(mode, cb, th) for mode in ("memcpy", "stream") for cb in (16 << 20, 8 << 20, 4 << 20)
                for th in (4, 8, 16)]
    times = {v: [] for v in variants}
    arena.PIPELINE_MAX_CHUNKS = 64
    for rnd in range(6):
        for mode, cb, th in variants:
            os.environ["DLSIM_PACK_COPY"] = mode
            arena.PIPELINE_CHUNK_BYTES = cb
            torch.set_num_threads(th)
            FedAvg.aggregate(models, None)
            for _ in range(3):
                t0 = time.perf_counter()
                FedAvg.aggregate(models, None)
                times[(mode, cb, th)].append(time.perf_counter() - t0)
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    out = {"n": n}
    for (mode, cb, th), ts in times.items():
        ts.sort()
        out[f"{mode}_chunk{cb >> 20}M_t{th}_ms"] = round(ts[len(ts) // 2] * 1e3, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
