"""DAG replay: D-PSGD rounds executed the way the reference's worker executes
tasks — `globals()[func_name](settings, data)` over a star-import of the task
module (dasklearn/worker.py:3,27-31) — with the HIP `aggregate` task, against
the same replay with the oracle's op-for-op restatement of FedAvg.aggregate.

The DAG shape follows the reference's D-PSGD client: each round every peer
trains its model, then aggregates its neighbours' trained models followed by
its own (dasklearn/simulation/dpsgd/client.py:142-151, fan-in k+1), with no
explicit weights (simulation/client.py:88-95 only adds "weights" when given).
Training is a synthetic, seeded perturbation (the real train task needs
datasets from the network and is out of scope); models come back on the host
as after ModelTrainer.train (model_trainer.py:129).
"""
from __future__ import annotations

import copy
import math

import pytest
import torch
from torch import nn

from oracle import fedavg_torch
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

GNLENET = [(32, 3, 5, 5), (32,), (32,), (32,), (32, 32, 5, 5), (32,), (32,), (32,), (64, 32, 5, 5),
           (64,), (64,), (64,), (10, 576), (10,)]


class Shaped(nn.Module):
    def __init__(self, shapes):
        super().__init__()
        self.ps = nn.ParameterList([nn.Parameter(torch.zeros(*s)) for s in shapes])


class Settings:
    from dasklearn_amd.gradient_aggregation import GradientAggregationMethod
    gradient_aggregation = GradientAggregationMethod.FEDAVG
    torch_threads = 4


def synthetic_train(settings, params):
    """Deterministic stand-in for the train task: host model in, host model out."""
    model = params["model"]
    peer, rnd = params["peer"], params["round"]
    out = copy.deepcopy(model)
    g = torch.Generator().manual_seed(1000 * rnd + peer)
    with torch.no_grad():
        for p in out.parameters():
            p.add_(torch.randn(p.shape, generator=g) * 0.01)
    return [out]


def oracle_aggregate(settings, params):
    return [fedavg_torch.aggregate_modules(params["models"], params.get("weights"))]


def ring_neighbours(n, k):
    """k-regular ring: k//2 on each side (plus one more clockwise if k is odd)."""
    nb = {}
    for p in range(n):
        s = set()
        for d in range(1, k // 2 + 1):
            s.add((p + d) % n)
            s.add((p - d) % n)
        if k % 2:
            s.add((p + k // 2 + 1) % n)
        s.discard(p)
        nb[p] = sorted(s)
    return nb


def build_dag(n, rounds):
    """[(task_name, func_name, data)] in topological order; model inputs are
    ("task", output_index) placeholders, as in Task.data (tasks/task.py:26-51)."""
    k = max(1, math.floor(math.log2(n)))
    nb = ring_neighbours(n, min(k, n - 1))
    tasks = []
    for r in range(1, rounds + 1):
        for p in range(n):
            model = ("init", 0) if r == 1 else (f"agg_{p}_{r - 1}", 0)
            tasks.append((f"train_{p}_{r}", "train", {"model": model, "round": r, "peer": p}))
        for p in range(n):
            models = [(f"train_{q}_{r}", 0) for q in nb[p]] + [(f"train_{p}_{r}", 0)]
            tasks.append((f"agg_{p}_{r}", "aggregate", {"models": models, "round": r, "peer": p}))
    return tasks, nb


def replay(tasks, funcs, init_model):
    results = {"init": [init_model]}

    def resolve(v):
        if isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], str):
            return results[v[0]][v[1]]
        if isinstance(v, list):
            return [resolve(x) for x in v]
        return v

    for name, func_name, data in tasks:
        f = funcs[func_name]  # worker.py:29: globals()[func_name]
        res = f(Settings(), {k: resolve(v) for k, v in data.items()})
        assert isinstance(res, (list, tuple))  # broker.py:282-283
        results[name] = res
    return results


def flat(m):
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy()


@pytest.mark.parametrize("n,rounds", [(2, 5), (4, 3), (10, 2)])
def test_dpsgd_replay_bit_identical(n, rounds):
    ns = {}
    exec("from dasklearn_amd.functions import *", ns)  # what worker.py does with dasklearn.functions
    hip_funcs = {"aggregate": ns["aggregate"], "train": synthetic_train}
    ref_funcs = {"aggregate": oracle_aggregate, "train": synthetic_train}
    torch.manual_seed(3)
    init = Shaped(GNLENET)
    with torch.no_grad():
        for p in init.parameters():
            p.copy_(torch.randn(p.shape) * 0.05)
    tasks, nb = build_dag(n, rounds)
    k = len(nb[0])
    for name, f, data in tasks:  # fan-in as the reference's test_dpsgd.py checks (k+1)
        if f == "aggregate":
            assert len(data["models"]) == k + 1
    got = replay(tasks, hip_funcs, init)
    exp = replay(tasks, ref_funcs, init)
    for p in range(n):
        a = got[f"agg_{p}_{rounds}"][0]
        b = exp[f"agg_{p}_{rounds}"][0]
        assert all(not q.is_cuda for q in a.parameters())
        assert orc.same_bits(flat(a), flat(b)), (n, p)


def oracle_reconstruct(settings, params):
    """The reference's reconstruct arithmetic (chunk_manager.py:38-53) with
    torch CPU ops: per chunk index torch.mean(torch.stack(...)), cat, copy."""
    chunks = params["chunks"]
    means = [torch.mean(torch.stack(list(cs)), dim=0) for cs in chunks]
    flat = torch.cat(means)
    model = Shaped(GNLENET)
    off = 0
    with torch.no_grad():
        for t in model.state_dict().values():
            t.copy_(flat[off:off + t.numel()].view(t.shape))
            off += t.numel()
    return [model]


def test_conflux_style_chunk_replay_bit_identical():
    """4 peers, k = 4 chunks: every peer chunks its trained model; chunk c of
    peer p goes to peers p+1 and p+2; each peer reconstructs from its own and
    the received chunks (3 contributors per index: PyTorch's mean is
    sequential there, so the GPU path must match bit for bit)."""
    ns = {}
    exec("from dasklearn_amd.functions import *", ns)
    n, k, rounds = 4, 4, 2
    torch.manual_seed(11)
    init = Shaped(GNLENET)
    with torch.no_grad():
        for p in init.parameters():
            p.copy_(torch.randn(p.shape) * 0.05)

    def run(reconstruct):
        models = {p: init for p in range(n)}
        for r in range(1, rounds + 1):
            trained = {p: synthetic_train(Settings(), {"model": models[p], "round": r, "peer": p})[0]
                       for p in range(n)}
            chunked = {p: ns["chunk"](Settings(), {"model": trained[p], "n": k}) for p in range(n)}
            for p in range(n):
                got = [[chunked[p][c]] + [chunked[(p - d) % n][c] for d in (1, 2)] for c in range(k)]
                models[p] = reconstruct(Settings(), {"chunks": got, "round": r, "peer": p})[0]
        return models

    import dasklearn_amd.functions as fn
    old = fn.model_factory
    fn.model_factory = lambda dataset, architecture=None: Shaped(GNLENET)
    try:
        Settings.dataset, Settings.model = "cifar10", "gnlenet"
        got = run(ns["reconstruct_from_chunks"])
    finally:
        fn.model_factory = old
    exp = run(oracle_reconstruct)
    for p in range(n):
        assert orc.same_bits(flat(got[p]), flat(exp[p])), p
