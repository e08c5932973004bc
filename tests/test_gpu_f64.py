"""fp64 parameters (dlsim_wreduce_f64) against the oracle (GPU).

For a double model the reference's `c1.add_(w * p1)` (fedavg.py:25) keeps the
Python-float weight exact and rounds every product and sum to double, in input
order; the C oracle restates that (oracle_wreduce_f64) and is pinned by the
reference's own fp64 fixtures (tests/golden/*f64*, test_oracle_golden.py).
Bit-exact is the bar."""
from __future__ import annotations

import copy

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
from test_gpu_parity import dev, from_dev, make_rows, to_dev  # noqa: E402


def w64(n, seed):
    return orc.reference_weights_f64(n, list(np.random.default_rng(seed).dirichlet(np.ones(n))))


def hip_f64(rows, w, mode=_native.DLSIM_EXACT):
    xs = to_dev(list(rows), "f64")
    out = torch.empty_like(xs[0])
    _native.wreduce(xs, w, out, mode)
    return from_dev(out)


@pytest.mark.parametrize("n", [1, 2, 3, 8, 9, 14, 15, 17, 100, 129, 200])
def test_f64_exact_vs_oracle_across_n(n):
    p = 4099 + n
    rows = make_rows(n, p, 40 + n, "f64")
    w = w64(n, n)
    assert orc.same_bits(hip_f64(rows, w), orc.wreduce(list(rows), w, "f64"))


@pytest.mark.parametrize("p", [1, 2, 3, 5, 1023, 65536 + 7, 999_999, 1_000_003, 2_499_999, 2_500_001])
def test_f64_exact_vs_oracle_across_sizes_and_shape_classes(p):
    """Tails of every width, and either side of the fp64 size classes (the
    fp32 shapes by bytes per stream: 8 MB and 20 MB)."""
    n = 8
    rows = make_rows(n, p, p, "f64")
    w = orc.reference_weights_f64(n, None)
    assert orc.same_bits(hip_f64(rows, w), orc.wreduce(list(rows), w, "f64"))


def test_f64_weights_are_not_rounded_to_fp32():
    """1/3 and 0.1 as doubles: a reduce with fp32-rounded weights differs."""
    rows = make_rows(2, 10_000, 3, "f64")
    w = orc.reference_weights_f64(2, [0.1, 1.0 / 3.0])
    got = hip_f64(rows, w)
    assert orc.same_bits(got, orc.wreduce(list(rows), w, "f64"))
    w32 = orc.reference_weights(2, [0.1, 1.0 / 3.0]).astype(np.float64)
    assert not orc.same_bits(got, orc.wreduce(list(rows), w32, "f64"))


def test_f64_misaligned_and_in_place():
    n, p = 5, 7001
    rows = make_rows(n, p + 1, 9, "f64")
    xs = [t[1:] for t in to_dev(list(rows), "f64")]
    w = w64(n, 2)
    out = torch.empty(p, dtype=torch.float64, device=dev())
    _native.wreduce(xs, w, out)
    assert orc.same_bits(from_dev(out), orc.wreduce([r[1:] for r in rows], w, "f64"))
    ys = to_dev(list(rows), "f64")
    _native.wreduce(ys, w, ys[3])
    assert orc.same_bits(from_dev(ys[3]), orc.wreduce(list(rows), w, "f64"))


@pytest.mark.parametrize("n", [2, 17, 150])
def test_f64_fast_is_the_fma_chain(n):
    rows = make_rows(n, 20_003, 60 + n, "f64")
    w = w64(n, 5)
    got = hip_f64(rows, w, _native.DLSIM_FAST)
    assert orc.same_bits(got, orc.wreduce(list(rows), w, "f64", mode="fast"))
    exact = orc.wreduce(list(rows), w, "f64")
    scale = np.abs(w[:, None] * rows).sum(axis=0)
    assert np.all(np.abs(got - exact) <= n * 2.0 ** -52 * scale + 1e-300)


def test_f64_north_star_size():
    n, p = 8, 11_181_642
    g = torch.Generator(device=dev()).manual_seed(8)
    xs = [torch.randn(p, generator=g, device=dev(), dtype=torch.float64) * 0.05 for _ in range(n)]
    w = w64(n, 7)
    out = torch.empty_like(xs[0])
    _native.wreduce(xs, w, out)
    assert orc.same_bits(from_dev(out), orc.wreduce([from_dev(x) for x in xs], w, "f64"))
    del xs, out
    torch.cuda.empty_cache()


class _Mixed(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Parameter(torch.randn(1001, dtype=torch.float64))
        self.b = nn.Parameter(torch.randn(333))
        self.c = nn.Parameter(torch.randn(7, 3, dtype=torch.float64))
        self.register_buffer("steps", torch.tensor(3))


@pytest.mark.parametrize("where", ["host", "device", "device_arena"])
def test_f64_modules_match_the_torch_restatement(where):
    """FedAvg.aggregate on modules with fp64 (and fp32) parameters, on the
    host (the reference's case), on the device and as device arenas."""
    torch.manual_seed(4)
    models = [_Mixed() for _ in range(3)]
    ws = [0.1, 1.0 / 3.0, 0.5]
    ref = fedavg_torch.aggregate_modules(models, ws)
    if where == "device":
        ins = [copy.deepcopy(m).to(dev()) for m in models]
    elif where == "device_arena":
        from dasklearn_amd.arena import to_device_arena
        ins = [to_device_arena(m, dev()) for m in models]
    else:
        ins = models
    out = FedAvg.aggregate(ins, ws)
    for p, q in zip(out.parameters(), ref.parameters()):
        assert p.dtype == q.dtype
        assert orc.same_bits(p.detach().cpu().numpy().reshape(-1), q.detach().numpy().reshape(-1))
    assert int(out.steps) == 3


def test_f64_tasks_in_a_batch():
    """aggregate_batch: fp64 groups run one dlsim_wreduce_f64 per task, next
    to the batched fp32 groups; results equal the per-task restatement."""
    from dasklearn_amd.arena import to_device_arena
    torch.manual_seed(5)
    models = [to_device_arena(_Mixed(), dev()) for _ in range(5)]
    tasks = [(models[0:3], None), (models[2:5], [0.2, 0.3, 0.5]), (models[1:3], [1.0 / 3.0, 2.0 / 3.0])]
    outs = aggregate_batch(tasks)
    for (ms, ws), out in zip(tasks, outs):
        ref = fedavg_torch.aggregate_modules([copy.deepcopy(m).cpu() for m in ms], ws)
        for p, q in zip(out.parameters(), ref.parameters()):
            assert orc.same_bits(p.detach().cpu().numpy().reshape(-1), q.detach().numpy().reshape(-1))
