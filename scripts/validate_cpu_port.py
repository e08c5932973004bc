"""the CPU baseline bench.py times on the GPU box is the repo's
op-for-op restatement (oracle/fedavg_torch.aggregate_modules) because the
reference cannot travel there. This script, run in the BUILD container where
/root/reference exists, validates that stand-in against the reference's own
FedAvg.aggregate (dasklearn/gradient_aggregation/fedavg.py:12-26):

* bit-identical outputs on the same host modules;
* timing within +-15 %: the two are timed interleaved (A B A B ...) in one
  process at torch.set_num_threads(4) (the worker's default, broker.py:31,
  session_settings.py:52), on the north star's parameter layout (8 x
  ResNet-18/CIFAR-10, 62 tensors, 11,181,642 fp32 params) and on cfg1/cfg2's
  GNLeNet layout (2 and 8 models).

Writes a JSON summary (default profiles/r02_cpu_port_vs_reference.json).
Nothing of the reference is copied: it is imported read-only
(PYTHONDONTWRITEBYTECODE=1). Skips when /root/reference is absent.

    PYTHONDONTWRITEBYTECODE=1 python scripts/validate_cpu_port.py [--reps 15]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_cpu_port_vs_reference.json"))
    a = ap.parse_args()
    if not os.path.isdir(REF):
        print("reference absent; nothing to do")
        return 0
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import torch
    from torch import nn
    from dasklearn.gradient_aggregation.fedavg import FedAvg
    from bench import GNLENET_SHAPES, resnet18_shapes
    from oracle import fedavg_torch

    torch.set_num_threads(a.threads)

    class Shaped(nn.Module):
        def __init__(self, shapes, seed):
            super().__init__()
            g = torch.Generator().manual_seed(seed)
            self.ps = nn.ParameterList([nn.Parameter(torch.randn(sh, generator=g) * 0.05) for sh in shapes])

    def flat(m):
        return torch.cat([p.detach().reshape(-1) for p in m.parameters()])

    cases = [("north_star_resnet18_n8_dirichlet", resnet18_shapes(), 8, True),
             ("cfg1_gnlenet_n2_none", GNLENET_SHAPES, 2, False),
             ("cfg2_gnlenet_n8_none", GNLENET_SHAPES, 8, False)]
    import numpy as np
    results = []
    for name, shapes, n, weighted in cases:
        models = [Shaped(shapes, 1234 + i) for i in range(n)]
        weights = [float(w) for w in np.random.default_rng(7).dirichlet(np.ones(n))] if weighted else None
        ref_out = FedAvg.aggregate(models, weights)
        port_out = fedavg_torch.aggregate_modules(models, weights)
        same = bool(torch.equal(flat(ref_out).view(torch.int32), flat(port_out).view(torch.int32)))
        # warm both, then interleave
        for _ in range(2):
            FedAvg.aggregate(models, weights)
            fedavg_torch.aggregate_modules(models, weights)
        t_ref, t_port = [], []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            FedAvg.aggregate(models, weights)
            t1 = time.perf_counter()
            fedavg_torch.aggregate_modules(models, weights)
            t2 = time.perf_counter()
            t_ref.append(t1 - t0)
            t_port.append(t2 - t1)
        mr, mp = statistics.median(t_ref), statistics.median(t_port)
        ent = {"case": name, "n_models": n, "tensors": len(shapes),
               "params": int(sum(torch.Size(s).numel() for s in shapes)),
               "bit_identical": same,
               "reference_ms_median": round(mr * 1e3, 3), "port_ms_median": round(mp * 1e3, 3),
               "port_over_reference": round(mp / mr, 4),
               "within_15_percent": abs(mp / mr - 1.0) <= 0.15,
               "reference_ms_all": [round(t * 1e3, 3) for t in t_ref],
               "port_ms_all": [round(t * 1e3, 3) for t in t_port]}
        results.append(ent)
        print(f"{name}: bit_identical={same} reference {mr * 1e3:.2f} ms, port {mp * 1e3:.2f} ms "
              f"(ratio {mp / mr:.3f})", flush=True)
    summary = {"what": "oracle/fedavg_torch.aggregate_modules (bench.py cpu_baseline) vs the reference's "
                       "FedAvg.aggregate, interleaved, same host modules",
               "threads": a.threads, "reps": a.reps, "torch": torch.__version__,
               "cpu_capability": torch.backends.cpu.get_cpu_capability(),
               "machine": platform.processor() or platform.machine(), "cores_visible": os.cpu_count(),
               "results": results,
               "all_bit_identical": all(r["bit_identical"] for r in results),
               "all_within_15_percent": all(r["within_15_percent"] for r in results)}
    with open(a.out, "w") as f:
        json.dump(summary, f, indent=1)
    print("wrote", a.out)
    return 0 if summary["all_bit_identical"] and summary["all_within_15_percent"] else 1


if __name__ == "__main__":
    sys.exit(main())
