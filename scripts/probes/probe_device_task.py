"""Probe (round 4): where one device-model aggregate task's host time goes.

7 x GNLeNet (the reference's module tree, fan-in 7) already on the GPU, as a
device train task leaves them; FedAvg.aggregate (the plugin call the worker
makes through functions.aggregate) timed per call, medians of REPS, and a
cProfile of 300 calls (functions with the most own time).

    python scripts/probes/probe_device_task.py [reps]
"""
import cProfile
import io
import json
import os
import pstats
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "scripts"), os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from bench_rounds import GNLeNetTree  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    torch.set_num_threads(4)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    models = [GNLeNetTree().to(dev) for _ in range(7)]
    for _ in range(50):
        FedAvg.aggregate(models, None)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        out = FedAvg.aggregate(models, None)
        ts.append(time.perf_counter() - t)
        del out
    torch.cuda.synchronize()
    # back to back, one sync at the end: the GPU is not the limit
    t = time.perf_counter()
    for _ in range(reps):
        FedAvg.aggregate(models, None)
    torch.cuda.synchronize()
    b2b = (time.perf_counter() - t) / reps
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(300):
        FedAvg.aggregate(models, None)
    pr.disable()
    torch.cuda.synchronize()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(16)
    print(json.dumps({"per_call_us_median": round(statistics.median(ts) * 1e6, 1),
                      "back_to_back_us": round(b2b * 1e6, 1), "reps": reps}), flush=True)
    print(buf.getvalue(), flush=True)


if __name__ == "__main__":
    main()
