"""Models whose parameter lists differ, on the GPU: the reference's `zip`
pairing (fedavg.py:23-24 — truncation at the shorter list, extra parameters
ignored, `add_` broadcasting, RuntimeError where torch's add_ raises) through
FedAvg.aggregate and aggregate_batch, against the reference's own outputs
(tests/golden/mismatch_*.npz, make_golden_mismatch.py) and the oracle."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch
from torch import nn

from conftest import load_mismatch, mismatch_paths
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

from dasklearn_amd import arena  # noqa: E402
from dasklearn_amd.batch import aggregate_batch  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402

TDT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}


class Shaped(nn.Module):
    def __init__(self, arrays, dtype):
        super().__init__()
        ps = []
        for a in arrays:
            if dtype in (torch.bfloat16, torch.float16):
                t = torch.from_numpy(np.ascontiguousarray(a).view(np.int16).copy()).view(dtype)
            else:
                t = torch.from_numpy(np.ascontiguousarray(a).copy())
            ps.append(nn.Parameter(t))
        self.ps = nn.ParameterList(ps)


def build(params, dtype, where):
    models = [Shaped(ps, TDT[dtype]) for ps in params]
    if where == "device":
        models = [m.cuda() for m in models]
    elif where == "arena":
        models = [arena.to_device_arena(m.cuda()) for m in models]
    return models


def flat_bits(model, dtype):
    ps = [p.detach().reshape(-1).cpu() for p in model.parameters()]
    if not ps:
        return np.zeros(0)
    t = torch.cat(ps)
    if dtype in ("bf16", "f16"):
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def check(out, models, meta, expected):
    assert type(out) is type(models[0])
    shapes0 = [p.shape for p in models[0].parameters()]
    assert [p.shape for p in out.parameters()] == shapes0
    got = flat_bits(out, meta["dtype"])
    if meta["dtype"] == "f16":
        got, expected = got.view(np.float16), expected.view(np.float16)
    assert orc.same_bits(got, expected), meta["case"]


@pytest.mark.parametrize("where", ["host", "device", "arena"])
@pytest.mark.parametrize("path", mismatch_paths(), ids=lambda p: os.path.basename(p)[:-4])
def test_fedavg_zip_matches_reference(path, where):
    meta, params, w, expected = load_mismatch(path)
    models = build(params, meta["dtype"], where)
    if meta["error"]:
        with pytest.raises(RuntimeError):
            FedAvg.aggregate(models, w)
        return
    out = FedAvg.aggregate(models, w)
    torch.cuda.synchronize()
    on_host = where == "host"
    assert all(p.is_cuda != on_host for p in out.parameters())
    check(out, models, meta, expected)
    # inputs are only read
    again = FedAvg.aggregate(models, w)
    torch.cuda.synchronize()
    check(again, models, meta, expected)


@pytest.mark.parametrize("path", [p for p in mismatch_paths() if "broadcast" not in p and "samenumel" not in p],
                         ids=lambda p: os.path.basename(p)[:-4])
def test_batch_zip_beside_same_signature_tasks(path):
    """aggregate_batch: a zip task among ordinary arena tasks keeps its
    place; every result as the reference's."""
    meta, params, w, expected = load_mismatch(path)
    dt = TDT[meta["dtype"]]
    ragged = build(params, meta["dtype"], "arena")
    same = [arena.to_device_arena(Shaped(params[0], dt).cuda()) for _ in range(3)]
    same_w = [0.5, 0.25, 0.25]
    outs = aggregate_batch([(same, same_w), (ragged, w), (same, None)])
    torch.cuda.synchronize()
    check(outs[1], ragged, meta, expected)
    for o, ww in ((outs[0], same_w), (outs[2], None)):
        ref = FedAvg.aggregate(same, ww)
        torch.cuda.synchronize()
        assert np.array_equal(flat_bits(o, meta["dtype"]), flat_bits(ref, meta["dtype"]))


def test_zip_dtype_mismatch_is_refused():
    """A parameter of another dtype at the same position: the reference would
    add a product rounded in that dtype; this path raises ValueError
    (INTEGRATION.md §3)."""
    a = nn.Linear(4, 3).cuda()
    b = nn.Linear(4, 3).cuda().to(torch.bfloat16)
    with pytest.raises(ValueError, match="dtype"):
        FedAvg.aggregate([a, b], None)


def test_zip_noncontiguous_model0_keeps_its_strides():
    """deepcopy(models[0]) keeps a transposed parameter transposed
    (fedavg.py:20); the zip path too."""
    torch.manual_seed(3)
    m0 = nn.Module()
    m0.w = nn.Parameter(torch.randn(6, 5).t())
    m0.b = nn.Parameter(torch.randn(7))
    m1 = nn.Module()
    m1.w = nn.Parameter(torch.randn(5, 6))
    out = FedAvg.aggregate([m0, m1], [0.25, 0.75])
    assert out.w.stride() == m0.w.stride()
    p0 = [m0.w.detach().numpy(), m0.b.detach().numpy()]
    p1 = [m1.w.detach().numpy()]
    ref = orc.wreduce_zip([p0, p1], [0.25, 0.75])
    assert orc.same_bits(out.w.detach().numpy(), ref[0])
    assert orc.same_bits(out.b.detach().numpy(), ref[1])


@pytest.mark.parametrize("path", [p for p in mismatch_paths() if "fewer_f32" in p or "mixed" in p or "more" in p],
                         ids=lambda p: os.path.basename(p)[:-4])
def test_round_executor_zip_task_in_a_wave(path):
    """RoundExecutor: a zip task and an ordinary task in one wave; the zip
    task's result is the reference's, the other one FedAvg's."""
    from test_gpu_dag_replay import Settings
    from dasklearn_amd.rounds import RoundExecutor

    meta, params, w, expected = load_mismatch(path)
    dt = TDT[meta["dtype"]]
    ragged = build(params, meta["dtype"], "device")
    same = [Shaped(params[0], dt).cuda() for _ in range(2)]
    n = len(ragged)
    tasks = [("agg_same", "aggregate", {"models": [("same", 0), ("same", 1)], "round": 1, "peer": 0}),
             ("agg_zip", "aggregate", {"models": [("ragged", i) for i in range(n)], "weights": w,
                                       "round": 1, "peer": 1})]
    ex = RoundExecutor({}, Settings())
    got = ex.run(tasks, seed={"ragged": ragged, "same": same})
    torch.cuda.synchronize()
    check(got["agg_zip"][0], ragged, meta, expected)
    ref = FedAvg.aggregate(same, None)
    torch.cuda.synchronize()
    assert np.array_equal(flat_bits(got["agg_same"][0], meta["dtype"]), flat_bits(ref, meta["dtype"]))
