"""Batched aggregation: many independent `aggregate` tasks in few launches.

In a simulated round every peer aggregates its neighbours' models
(dasklearn/simulation/dpsgd/client.py:142-151); the broker schedules those
tasks one by one (broker.py:261-275), so each is one call of
functions.aggregate (functions.py:89-106). For small models (GNLeNet: 3 MB
per 8-way task) one launch per task is launch-bound; `aggregate_batch` runs
the tasks that are ready together through `dlsim_wreduce_batched` (up to 32
tasks / 192 inputs per launch). Results are bit-identical to calling
FedAvg.aggregate on each task.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
from torch import nn

from . import _native
from .arena import ParamLayout, aggregate_modules, arenas_to_host, module_from_arenas


def _resolve(models, weights):
    # fedavg.py:14-17 rules, same exceptions
    if not weights:
        weights = [float(1. / len(models)) for _ in range(len(models))]
    else:
        assert len(weights) == len(models)
    return _native.fp32_weights(weights)


def aggregate_batch(tasks: Sequence[Tuple[List[nn.Module], Optional[Sequence[float]]]],
                    mode: int = _native.DLSIM_EXACT) -> List[nn.Module]:
    """tasks: [(models, weights)] -> one aggregated module per task.

    Tasks whose models are device-resident arenas (what this package returns
    for device inputs) are reduced together in batched launches; any other
    task goes through the single-task path. Output placement follows
    FedAvg.aggregate (where models[0] lives)."""
    results: List[Optional[nn.Module]] = [None] * len(tasks)
    batched = []  # (task index, layout, views per dtype, w32, host_out)
    for ti, (models, weights) in enumerate(tasks):
        w32 = _resolve(models, weights)
        model0 = models[0]  # IndexError for an empty task, as the reference
        layout = ParamLayout(model0)
        params = [layout.check_compatible(m) for m in models]
        views = {}
        ok = all(p.is_cuda for ps in params for p in ps) and len(layout.groups) > 0
        if ok:
            dev = params[0][0].device
            for dt in layout.groups:
                vs = [layout.arena_view(ps, dt) for ps in params]
                if any(v is None for v in vs) or any(v.device != dev for v in vs):
                    ok = False
                    break
                views[dt] = vs
        if not ok:
            results[ti] = aggregate_modules(models, weights, mode)
            continue
        batched.append((ti, layout, views, w32))
    # one batched call per dtype present; outputs are fresh arenas per task
    by_dtype = {}
    outs = {}
    for ti, layout, views, w32 in batched:
        dev = next(iter(views.values()))[0].device
        outs[ti] = {}
        for dt, vs in views.items():
            out = torch.empty(layout.totals[dt], dtype=dt, device=dev)
            outs[ti][dt] = out
            by_dtype.setdefault((dt, dev), []).append((vs, w32, out))
    for (dt, dev), group in by_dtype.items():
        _native.wreduce_batched(group, mode, torch.cuda.current_stream(dev))
    for ti, layout, views, w32 in batched:
        results[ti] = module_from_arenas(tasks[ti][0][0], layout, outs[ti])
    return results
