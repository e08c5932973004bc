"""Round executor (dasklearn_amd/rounds.py): a D-PSGD DAG executed in waves,
every wave's aggregate tasks batched into one GPU launch over device-resident
arenas — bit-identical to the sequential oracle replay (the broker/worker
path of the reference, broker.py:261-290, worker.py:21-38)."""
from __future__ import annotations

import copy

import pytest
import torch

from oracle import oracle as orc
from test_gpu_dag_replay import GNLENET, Settings, Shaped, build_dag, flat, oracle_aggregate, replay

pytestmark = pytest.mark.gpu

from dasklearn_amd.rounds import RoundExecutor  # noqa: E402


def device_agnostic_train(settings, params):
    """synthetic_train that keeps the model where it lives (host or device)."""
    model = params["model"]
    out = copy.deepcopy(model)
    g = torch.Generator().manual_seed(1000 * params["round"] + params["peer"])
    with torch.no_grad():
        for p in out.parameters():
            p.add_((torch.randn(p.shape, generator=g) * 0.01).to(p.device))
    return [out]


@pytest.mark.parametrize("n,rounds", [(4, 2), (10, 3)])
def test_round_executor_matches_sequential_replay(n, rounds):
    torch.manual_seed(21)
    init = Shaped(GNLENET)
    with torch.no_grad():
        for p in init.parameters():
            p.copy_(torch.randn(p.shape) * 0.05)
    tasks, nb = build_dag(n, rounds)
    ex = RoundExecutor({"train": device_agnostic_train}, Settings())
    got = ex.run(tasks, seed={"init": [init]})
    exp = replay(tasks, {"aggregate": oracle_aggregate, "train": device_agnostic_train}, init)
    # waves: all trains of a round, then all aggregates of that round
    assert len(ex.waves) == 2 * rounds
    assert all(len(w) == n for w in ex.waves)
    for p in range(n):
        a = got[f"agg_{p}_{rounds}"][0]
        assert all(q.is_cuda for q in a.parameters())  # stayed resident
        b = exp[f"agg_{p}_{rounds}"][0]
        assert orc.same_bits(torch.cat([q.detach().reshape(-1).cpu() for q in a.parameters()]).numpy(),
                             flat(b))


def test_round_executor_reports_unresolvable_inputs():
    ex = RoundExecutor({}, Settings())
    with pytest.raises(RuntimeError, match="unresolvable"):
        ex.run([("agg_0", "aggregate", {"models": [("missing", 0)], "round": 1, "peer": 0})])


def host_train(settings, params):
    """device_agnostic_train that always returns a host model (the reference's
    CPU training): every wave's aggregates read host models."""
    return [device_agnostic_train(settings, {**params, "model": params["model"].cpu()})[0].cpu()]


class MixedShaped(torch.nn.Module):
    """GNLeNet shapes with some tensors in bf16 and fp16 (three dtype groups)."""

    def __init__(self):
        super().__init__()
        dts = [torch.float32, torch.bfloat16, torch.float16]
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(*s).to(dts[i % 3]) * 0.05)
                                          for i, s in enumerate(GNLENET)])


@pytest.mark.parametrize("mixed", [False, True])
def test_round_executor_host_trained_models(mixed):
    """Host models in every wave go to the device in one dlsim_host_pack + H2D
    per wave (one arena per model and dtype): bit-identical to the sequential
    oracle replay, for one and for three dtype groups."""
    from dasklearn_amd.arena import module_params
    torch.manual_seed(23)
    init = MixedShaped() if mixed else Shaped(GNLENET)
    tasks, nb = build_dag(6, 2)
    ex = RoundExecutor({"train": host_train}, Settings())
    got = ex.run(tasks, seed={"init": [init]})
    exp = replay(tasks, {"aggregate": oracle_aggregate, "train": host_train}, init)
    for p in range(6):
        a = got[f"agg_{p}_2"][0]
        b = exp[f"agg_{p}_2"][0]
        assert all(q.is_cuda for q in a.parameters())
        for dt in (torch.float32, torch.bfloat16, torch.float16):
            ga = [q.detach().reshape(-1).cpu() for q in module_params(a) if q.dtype == dt]
            gb = [q.detach().reshape(-1).cpu() for q in module_params(b) if q.dtype == dt]
            if ga:
                x, y = torch.cat(ga), torch.cat(gb)
                assert torch.equal(x.view(torch.int16) if x.element_size() == 2 else x.view(torch.int32),
                                   y.view(torch.int16) if y.element_size() == 2 else y.view(torch.int32)), (p, dt)
