"""Batched launches (dlsim_wreduce_batched / dasklearn_amd.batch): every task
bit-identical to its own reduce (oracle), across the kernel-argument limits
(32 tasks, 192 inputs), uniform and mixed fan-in, and tasks that must run
alone (fan-in > 16, misaligned)."""
from __future__ import annotations

import numpy as np
import pytest
import torch
from torch import nn

from oracle import oracle as orc
from oracle import fedavg_torch

pytestmark = pytest.mark.gpu

from dasklearn_amd import _native  # noqa: E402
from dasklearn_amd.batch import aggregate_batch  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402


def dev():
    return torch.device("cuda", 0)


def make_task(rng, n, p, dtype, misalign=False):
    x = rng.standard_normal((n, p + 1)).astype(np.float32) * np.float32(0.05)
    rows = orc.f32_to_bf16_bits(x) if dtype == "bf16" else orc.f32_to_f16_bits(x) if dtype == "f16" else x
    if dtype in ("bf16", "f16"):
        tdt = torch.bfloat16 if dtype == "bf16" else torch.float16
        t = [torch.from_numpy(r.view(np.int16).copy()).view(tdt).to(dev()) for r in rows]
    else:
        t = [torch.from_numpy(r.copy()).to(dev()) for r in rows]
    s = 1 if misalign else 0
    ins = [a[s:s + p] for a in t]
    host = [r[s:s + p] for r in rows]
    w = orc.reference_weights(n, list(rng.dirichlet(np.ones(n))))
    out = torch.empty(p, dtype=ins[0].dtype, device=dev())
    return ins, host, w, out


def check(tasks, dtype, mode=_native.DLSIM_EXACT):
    _native.wreduce_batched([(t[0], t[2], t[3]) for t in tasks], mode)
    for ins, host, w, out in tasks:
        got = out.cpu()
        got = got.view(torch.int16).numpy().view(np.uint16) if dtype == "bf16" else got.numpy()
        exp = orc.wreduce(host, w, dtype, "exact" if mode == 0 else "fast")
        assert orc.same_bits(got, exp)


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
def test_uniform_fan_in_batch(dtype):
    rng = np.random.default_rng(1)
    tasks = [make_task(rng, 4, 85_354 + k, dtype) for k in range(10)]
    check(tasks, dtype)


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
def test_mixed_fan_in_and_sizes(dtype):
    rng = np.random.default_rng(2)
    tasks = [make_task(rng, n, p, dtype) for n, p in [(2, 1), (3, 17), (9, 4096), (16, 100_003),
                                                        (1, 5000), (5, 0 + 3)]]
    check(tasks, dtype)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("sizes", [[262_143, 1000, 77], [262_144 * 2 // 2 + 1, 1000, 77], [600_001, 3]])
def test_batch_vectors_per_lane_either_side_of_1_mb(dtype, sizes):
    """A batch launch lays its tiles out for VPT 1 when every task is under
    1 MB per stream, else VPT 4 (dispatch.hpp batch_vpt): both layouts, in
    the kernel-argument batch and the descriptor table, bit-exact."""
    esz = 2 if dtype == "bf16" else 4
    sizes = [p * 4 // esz if p > 100_000 else p for p in sizes]  # the same byte sizes in bf16
    rng = np.random.default_rng(sum(sizes))
    tasks = [make_task(rng, 4, p, dtype) for p in sizes]
    check(tasks, dtype)
    for t in tasks:
        t[3].zero_()
    _native.BatchPlan([(t[0], t[2], t[3]) for t in tasks]).launch()
    for ins, host, w, out in tasks:
        got = out.cpu()
        got = got.view(torch.int16).numpy().view(np.uint16) if dtype == "bf16" else got.numpy()
        assert orc.same_bits(got, orc.wreduce(host, w, dtype))


def test_batch_split_by_limits_and_solo_tasks():
    rng = np.random.default_rng(3)
    tasks = [make_task(rng, 8, 1000 + 37 * k, "f32") for k in range(40)]  # > 32 tasks, 320 ptrs
    tasks += [make_task(rng, 20, 3333, "f32")]                            # fan-in > 16: alone
    tasks += [make_task(rng, 3, 2222, "f32", misalign=True)]               # scalar path: alone
    check(tasks, "f32")


def test_fast_mode_batch():
    rng = np.random.default_rng(4)
    tasks = [make_task(rng, 6, 50_000, "f32") for _ in range(5)]
    check(tasks, "f32", _native.DLSIM_FAST)


def test_module_level_batch_matches_per_task():
    torch.manual_seed(0)
    base = [nn.Sequential(nn.Linear(40, 30), nn.ReLU(), nn.Linear(30, 10)).to(dev()) for _ in range(6)]
    arenas = [FedAvg.aggregate([m], None) for m in base]  # arena-backed device models
    tasks = [([arenas[(p + i) % 6] for i in range(3)], None) for p in range(6)]
    tasks.append(([arenas[0], arenas[1]], [0.25, 0.75]))
    tasks.append(([base[0], base[1]], None))  # not arenas: single-task path
    res = aggregate_batch(tasks)
    for (models, w), out in zip(tasks, res):
        ref = fedavg_torch.aggregate_modules([m.cpu() if False else _cpu(m) for m in models], w)
        a = torch.cat([p.detach().reshape(-1).cpu() for p in out.parameters()]).numpy()
        b = torch.cat([p.detach().reshape(-1) for p in ref.parameters()]).numpy()
        assert orc.same_bits(a, b)


def _cpu(m):
    import copy
    return copy.deepcopy(m).cpu()


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
def test_table_plan_whole_round(dtype):
    """100 peers x fan-in 8 (one D-PSGD round of GNLeNet-sized tasks) in one
    table launch, launched twice (the table is reusable)."""
    rng = np.random.default_rng(7)
    tasks = [make_task(rng, 8, 85_354, dtype) for _ in range(100)]
    plan = _native.BatchPlan([(t[0], t[2], t[3]) for t in tasks])
    for _ in range(2):
        for t in tasks:
            t[3].zero_()
        plan.launch()
        for ins, host, w, out in tasks:
            got = out.cpu()
            got = got.view(torch.int16).numpy().view(np.uint16) if dtype == "bf16" else got.numpy()
            assert orc.same_bits(got, orc.wreduce(host, w, dtype))


def test_table_plan_mixed_fan_in_up_to_128():
    rng = np.random.default_rng(8)
    tasks = [make_task(rng, n, p, "f32") for n, p in [(1, 7), (17, 3000), (40, 70_001), (128, 4097),
                                                        (2, 1), (9, 100_000)]]
    plan = _native.BatchPlan([(t[0], t[2], t[3]) for t in tasks], _native.DLSIM_EXACT)
    plan.launch()
    for ins, host, w, out in tasks:
        assert orc.same_bits(out.cpu().numpy(), orc.wreduce(host, w, "f32"))


def test_table_plan_rejects_misaligned_task():
    rng = np.random.default_rng(9)
    t = make_task(rng, 3, 1000, "f32", misalign=True)
    with pytest.raises(_native.DlsimError):
        _native.BatchPlan([(t[0], t[2], t[3])])
