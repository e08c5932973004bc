"""What the simulator does with an aggregate next: train it (the reference's
train task, model_trainer.py:60-131, on the aggregate's output) and aggregate
again. The output's parameters are views of one device arena (built in C,
csrc/pyhost.cpp fill_param_views); training them must behave exactly like
training the reference's `deepcopy(models[0])` output with separately
allocated parameters, and the next aggregate must read the trained values.

Deterministic ops only (Linear, ReLU, MSE, SGD with momentum and weight
decay, foreach updates), so both sides can be compared bit for bit on the
same device."""
from __future__ import annotations

import copy

import pytest
import torch
from torch import nn

from oracle import fedavg_torch

pytestmark = pytest.mark.gpu

from dasklearn_amd import arena  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402


class MLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.body = nn.Sequential(nn.Linear(32, 64), nn.ReLU(), nn.Linear(64, 64), nn.ReLU())
        self.head = nn.Linear(64, 10)
        self.head.bias.requires_grad_(False)  # a frozen parameter rides along

    def forward(self, x):
        return self.head(self.body(x))


def bits(m):
    return [p.detach().clone() for p in m.parameters()]


def train(model, steps, seed):
    """A few SGD steps (momentum, weight decay; torch's foreach path on CUDA)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    opt = torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=0.05, momentum=0.9,
                          weight_decay=1e-4, foreach=True)
    for _ in range(steps):
        x = torch.randn(16, 32, device="cuda", generator=g)
        y = torch.randn(16, 10, device="cuda", generator=g)
        opt.zero_grad(set_to_none=True)
        loss = nn.functional.mse_loss(model(x), y)
        loss.backward()
        opt.step()
    return model


def test_training_the_output_matches_training_a_deepcopy_and_feeds_the_next_aggregate():
    torch.manual_seed(5)
    models = [MLP().cuda() for _ in range(5)]
    w = [0.1, 0.3, 0.2, 0.25, 0.15]

    out = FedAvg.aggregate(models, w)                      # HIP path: parameters are arena views
    ref = fedavg_torch.aggregate_modules(models, w)        # the reference's op sequence (deepcopy)
    assert arena.registered_arenas(out) is not None
    assert all(torch.equal(a, b) for a, b in zip(bits(out), bits(ref)))
    assert [p.requires_grad for p in out.parameters()] == [p.requires_grad for p in ref.parameters()]

    train(out, 4, seed=11)
    train(ref, 4, seed=11)
    for (name, a), b in zip(out.named_parameters(), ref.parameters()):
        assert torch.equal(a, b), name
        assert a.grad is None or a.requires_grad
    # the optimizer updated the arena in place: the views still are the arena
    assert arena.registered_arenas(out) is not None

    # round 2: the trained output is read in place, with the trained values
    others = [train(copy.deepcopy(m), 1, seed=20 + i) for i, m in enumerate(models[1:])]
    out2 = FedAvg.aggregate([out] + others, None)
    ref2 = fedavg_torch.aggregate_modules([ref] + others, None)
    assert all(torch.equal(a, b) for a, b in zip(bits(out2), bits(ref2)))

    # state_dict round trip and a move to the host, as the trainer does (model_trainer.py:129)
    sd = out.state_dict()
    back = MLP().cuda()
    back.load_state_dict(sd)
    assert all(torch.equal(a, b) for a, b in zip(bits(back), bits(out)))
    host = copy.deepcopy(out).to("cpu")
    assert all(torch.equal(a.cpu(), b) for a, b in zip(bits(out), bits(host)))


def test_replacing_a_parameter_invalidates_the_arena_fast_path():
    """`p.data = t` (or assigning a new Parameter) moves a parameter off the
    arena: the next aggregate must read the new tensor, not the stale arena."""
    torch.manual_seed(6)
    models = [MLP().cuda() for _ in range(3)]
    out = FedAvg.aggregate(models, None)
    with torch.no_grad():
        out.head.weight.data = torch.full_like(out.head.weight, 2.0)
        out.body[0].bias = nn.Parameter(torch.full_like(out.body[0].bias, -1.0))
    assert arena.registered_arenas(out) is None
    res = FedAvg.aggregate([out, models[1]], [1.0, 0.0])
    ref = fedavg_torch.aggregate_modules([out, models[1]], [1.0, 0.0])
    assert all(torch.equal(a, b) for a, b in zip(bits(res), bits(ref)))
    assert torch.all(res.head.weight == 2.0) and torch.all(res.body[0].bias == -1.0)
