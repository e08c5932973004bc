"""TEST INFRASTRUCTURE ONLY — CPU baseline and module-level checker.

An op-for-op PyTorch-CPU restatement of the reference aggregation
(dasklearn/gradient_aggregation/fedavg.py:12-26, ``FedAvg.aggregate``):
the same tensor operations in the same order on the same modules, so that
bench.py can time "what the reference does" on the GPU box (where the
reference source does not exist) and tests can check module-level semantics
(buffers carried over from models[0], output type, requires_grad).

Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import copy
from typing import List, Optional, Sequence

import torch
from torch import nn


def resolve_weights(n: int, weights: Optional[Sequence[float]]) -> List[float]:
    # fedavg.py:14-17
    if not weights:
        return [float(1.0 / n)] * n
    assert len(weights) == n
    return list(weights)


def aggregate_modules(models: List[nn.Module], weights: Optional[Sequence[float]] = None) -> nn.Module:
    """fedavg.py:13-26 restated: deepcopy model 0, zero its parameters, then
    add each model's parameters scaled by its weight, model by model."""
    ws = resolve_weights(len(models), weights)
    with torch.no_grad():
        out = copy.deepcopy(models[0])                   # fedavg.py:20
        params = list(out.parameters())
        for p in params:                                 # fedavg.py:21-22
            p.mul_(0)
        for model, w in zip(models, ws):                 # fedavg.py:23
            for dst, src in zip(params, model.parameters()):  # fedavg.py:24
                dst.add_(w * src)                        # fedavg.py:25
    return out


def aggregate_flat(xs: Sequence[torch.Tensor], weights: Optional[Sequence[float]] = None) -> torch.Tensor:
    """The same op sequence on flat CPU tensors (one parameter per model)."""
    ws = resolve_weights(len(xs), weights)
    with torch.no_grad():
        acc = xs[0].clone()
        acc.mul_(0)
        for x, w in zip(xs, ws):
            acc.add_(w * x)
    return acc
