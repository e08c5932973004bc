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
