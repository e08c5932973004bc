"""The reference's process model around the HIP aggregate (GPU).

The broker hands tasks to worker processes over torch.multiprocessing queues
with the file_system sharing strategy (dasklearn/worker.py:6,21-38,
broker.py:142-143, 227-236): host models cross the process boundary through
shared memory, the worker runs globals()[func_name](settings, data), and the
result models travel back the same way. Here one spawned worker process runs
that loop (tests/_worker_child.py) with the HIP task functions; the parent
checks every result against the oracle bit for bit, and that a failing task
comes back as ("error", task, None) and ends the worker, as in the reference."""
from __future__ import annotations

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp
from torch import nn

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


class Net(nn.Module):
    """GNLeNet-sized convolutional model with GroupNorm-free BN buffers."""

    def __init__(self, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.conv = nn.Conv2d(3, 32, 5)
        self.bn = nn.BatchNorm2d(32)
        self.fc = nn.Linear(576, 10)
        with torch.no_grad():
            for p in self.parameters():
                p.copy_(torch.randn(p.shape, generator=g) * 0.05)
            self.bn.running_mean.copy_(torch.randn(32, generator=g))


def _flat(m):
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy()


def test_worker_process_round_trip():
    torch.multiprocessing.set_sharing_strategy("file_system")
    ctx = mp.get_context("spawn")
    shared, results = ctx.Queue(), ctx.Queue()
    from _worker_child import worker_main
    proc = ctx.Process(target=worker_main, args=(shared, results, 0), daemon=True)
    proc.start()
    try:
        models = [Net(s) for s in range(6)]
        w = [0.1, 0.3, 0.2, 0.15, 0.05, 0.2]
        shared.put(("agg_0", "aggregate", {"models": models[:4], "round": 1, "peer": 0}))
        shared.put(("agg_1", "aggregate", {"models": models, "round": 1, "peer": 1, "weights": w}))
        shared.put(("agg_bad", "aggregate", {"models": models[:3], "round": 1, "peer": 2, "weights": w}))
        got = {}
        for _ in range(3):
            name, res, info = results.get(timeout=90)
            got[name] = (res, info)
        # aggregate tasks: [model] on the host, bit-identical to the oracle,
        # buffers from models[0] (fedavg.py:20)
        for name, ms, weights in (("agg_0", models[:4], None), ("agg_1", models, w)):
            res, info = got[name]
            assert isinstance(res, list) and len(res) == 1 and info["worker"] == 0
            out = res[0]
            assert all(not p.is_cuda for p in out.parameters())
            exp = orc.wreduce([_flat(m) for m in ms], orc.reference_weights(len(ms), weights), "f32")
            assert orc.same_bits(_flat(out), exp), name
            assert torch.equal(out.bn.running_mean, ms[0].bn.running_mean)
        # a weight-count mismatch fails the task: ("error", task, None), worker exits
        assert got["error"][0] == "agg_bad" and got["error"][1] is None
        proc.join(timeout=30)
        assert not proc.is_alive()
    finally:
        if proc.is_alive():
            shared.put(None)
            proc.join(timeout=10)
        if proc.is_alive():
            proc.kill()
