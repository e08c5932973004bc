"""Host-boundary rates of the module-level aggregate (for DESIGN.md).

The reference's aggregate starts and ends in host memory: models reach the
worker as CPU nn.Modules (model_trainer.py:129, worker.py:24) and the result
goes back as one. This measures, for N ResNet-18/CIFAR-10-shaped models
(62 tensors, 11,181,642 fp32 params) and for GNLeNet-shaped ones:

  host      FedAvg.aggregate(cpu models) -> cpu module (pack into pinned
            staging, H2D, kernel, D2H): the PCIe-inclusive rate
  host_shm  the same with the models' storages in shared memory (torch-mp
            file_system strategy, how models reach the reference's worker)
  dev_list  CUDA models with separate parameter tensors (tensor-list ABI)
  dev_arena CUDA models whose parameters are views of one arena (one launch)
  cpu_ref   the reference's own op sequence on the CPU (oracle restatement),
            4 threads (the worker default, broker.py:31)

GB/s is algorithmic: (N+1) * P * 4 bytes / wall time of one aggregate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402
from torch import nn  # noqa: E402

from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402
from inputs import resnet18_cifar10_shapes  # noqa: E402
from oracle import fedavg_torch  # noqa: E402

GNLENET = [(32, 3, 5, 5), (32,), (32,), (32,), (32, 32, 5, 5), (32,), (32,), (32,), (64, 32, 5, 5),
           (64,), (64,), (64,), (10, 576), (10,)]


class Shaped(nn.Module):
    def __init__(self, shapes, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.ps = nn.ParameterList([nn.Parameter(torch.randn(*s, generator=g) * 0.05) for s in shapes])


def timed(fn, reps, sync=True):
    fn()
    if sync:
        torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        if sync:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name, shapes, n in (("resnet18", resnet18_cifar10_shapes(), 8), ("resnet18", resnet18_cifar10_shapes(), 2),
                            ("gnlenet", GNLENET, 8), ("gnlenet", GNLENET, 2)):
        P = sum(int(torch.Size(s).numel()) for s in shapes)
        byts = (n + 1) * P * 4
        cpu_models = [Shaped(shapes, i) for i in range(n)]
        res = {"model": name, "n": n, "params": P, "tensors": len(shapes)}
        t = timed(lambda: FedAvg.aggregate(cpu_models, None), a.reps)
        res["host_ms"] = round(t * 1e3, 3)
        res["host_GBps"] = round(byts / t / 1e9, 2)
        from dasklearn_amd import _native
        from dasklearn_amd.arena import aggregate_modules
        stages = {}
        for _ in range(3):
            aggregate_modules(cpu_models, None, _native.DLSIM_EXACT, timing=stages)
        res["host_stages_ms"] = {k: round(v / 3 * 1e3, 3) for k, v in stages.items()}
        # shm-backed host models, as they reach the reference's worker through
        # torch.multiprocessing's file_system strategy (worker.py:6)
        import copy
        import torch.multiprocessing as tmp
        tmp.set_sharing_strategy("file_system")
        shm_models = [copy.deepcopy(m).share_memory() for m in cpu_models]
        t = timed(lambda: FedAvg.aggregate(shm_models, None), a.reps)
        res["host_shm_ms"] = round(t * 1e3, 3)
        res["host_shm_GBps"] = round(byts / t / 1e9, 2)
        del shm_models
        dev_models = [Shaped(shapes, i).to(dev) for i in range(n)]
        t = timed(lambda: FedAvg.aggregate(dev_models, None), a.reps)
        res["dev_list_ms"] = round(t * 1e3, 3)
        res["dev_list_GBps"] = round(byts / t / 1e9, 1)
        arena_models = [FedAvg.aggregate([m], None) for m in dev_models]  # arena-backed copies
        t = timed(lambda: FedAvg.aggregate(arena_models, None), a.reps)
        res["dev_arena_ms"] = round(t * 1e3, 3)
        res["dev_arena_GBps"] = round(byts / t / 1e9, 1)
        torch.set_num_threads(4)
        t = timed(lambda: fedavg_torch.aggregate_modules(cpu_models, None), a.reps, sync=False)
        res["cpu_ref_4t_ms"] = round(t * 1e3, 3)
        res["cpu_ref_4t_GBps"] = round(byts / t / 1e9, 2)
        if n == 8:  # wire format vs the reference's pickle, one model's state_dict
            import pickle
            from dasklearn_amd import wire
            sd = cpu_models[0].state_dict()
            nbytes = P * 4
            t = timed(lambda: pickle.dumps(sd), a.reps, sync=False)
            blob = pickle.dumps(sd)
            res["pickle_dumps_GBps"] = round(nbytes / t / 1e9, 2)
            t = timed(lambda: pickle.loads(blob), a.reps, sync=False)
            res["pickle_loads_GBps"] = round(nbytes / t / 1e9, 2)
            t = timed(lambda: wire.encode_state_dict(sd), a.reps, sync=False)
            buf = wire.encode_state_dict(sd)
            res["dlsw_encode_GBps"] = round(nbytes / t / 1e9, 2)
            t = timed(lambda: wire.decode_state_dict(buf), a.reps, sync=False)
            res["dlsw_decode_host_GBps"] = round(nbytes / t / 1e9, 2)
            t = timed(lambda: wire.decode_state_dict(buf, dev), a.reps)
            res["dlsw_decode_device_GBps"] = round(nbytes / t / 1e9, 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
