"""Host-side logic of the drop-in boundary that needs no GPU: weight rules
and exception order (fedavg.py:14-17, 20), parameter layouts, arena
detection, the no-CPU-fallback rule, the task-function contract."""
from __future__ import annotations

import numpy as np
import pytest
import torch
from torch import nn

from dasklearn_amd import _native, arena, functions
from dasklearn_amd.gradient_aggregation import GradientAggregation, GradientAggregationMethod
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg
from dasklearn_amd.model_manager import ModelManager


def test_enum_matches_reference_value():
    # session_settings.py:40 default / gradient_aggregation/__init__.py:9
    assert GradientAggregationMethod.FEDAVG == 1
    assert issubclass(FedAvg, GradientAggregation)


def test_fp32_weight_rounding_is_rne_from_double():
    ws = [0.1, 1 / 3, 1e-40, 3.4e38, -0.7, 1.0000000596046448]
    got = _native.fp32_weights(ws)
    exp = torch.tensor(ws, dtype=torch.float64).to(torch.float32).numpy()
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


def test_empty_model_list_raises_index_error():
    with pytest.raises(IndexError):
        FedAvg.aggregate([], None)


def test_weight_count_mismatch_raises_assertion():
    m = [nn.Linear(2, 2), nn.Linear(2, 2)]
    with pytest.raises(AssertionError):
        FedAvg.aggregate(m, [1.0])


def test_no_cpu_fallback_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    m = [nn.Linear(2, 2), nn.Linear(2, 2)]
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        FedAvg.aggregate(m, None)


def test_unsupported_param_dtype_raises():
    m = nn.Linear(3, 3).to(torch.float16)
    with pytest.raises(TypeError):
        arena.ParamLayout(m)


def test_layout_groups_by_dtype_in_parameters_order():
    class Mixed(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Parameter(torch.zeros(5))
            self.b = nn.Parameter(torch.zeros(3, dtype=torch.bfloat16))
            self.c = nn.Parameter(torch.zeros(2, 2))

    lay = arena.ParamLayout(Mixed())
    assert list(lay.groups) == [torch.float32, torch.bfloat16]
    assert lay.groups[torch.float32] == [0, 2]
    assert lay.offsets[0] == 0 and lay.offsets[2] == 5 and lay.offsets[1] == 0
    assert lay.totals[torch.float32] == 9 and lay.totals[torch.bfloat16] == 3


def test_arena_view_detects_flat_backed_modules():
    m = nn.Sequential(nn.Linear(4, 3), nn.Linear(3, 2))
    lay = arena.ParamLayout(m)
    assert lay.arena_view(list(m.parameters()), torch.float32) is None  # separate storages
    flat = torch.arange(lay.totals[torch.float32], dtype=torch.float32)
    out = arena.module_from_arenas(m, lay, {torch.float32: flat})
    v = lay.arena_view(list(out.parameters()), torch.float32)
    assert v is not None and v.data_ptr() == flat.data_ptr() and torch.equal(v, flat)


def test_module_from_arenas_has_deepcopy_semantics():
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(4, 3), nn.BatchNorm1d(3))
    m[1].running_mean.fill_(7.0)
    m.extra_attribute = {"k": [1, 2]}
    m[0].bias.requires_grad_(False)
    lay = arena.ParamLayout(m)
    flat = torch.full((lay.totals[torch.float32],), 2.0)
    out = arena.module_from_arenas(m, lay, {torch.float32: flat})
    assert type(out) is type(m) and out is not m
    assert torch.equal(out[1].running_mean, m[1].running_mean)
    assert out[1].running_mean.data_ptr() != m[1].running_mean.data_ptr()
    assert out.extra_attribute == m.extra_attribute and out.extra_attribute is not m.extra_attribute
    assert [p.requires_grad for p in out.parameters()] == [p.requires_grad for p in m.parameters()]
    assert all(torch.all(p == 2.0) for p in out.parameters())
    assert all(torch.all(p != 2.0) for p in m.parameters())  # original untouched


def test_model_manager_first_model_per_peer_wins():
    mm = ModelManager(None, object(), 0)
    a, b = nn.Linear(1, 1), nn.Linear(1, 1)
    mm.process_incoming_trained_model(3, a)
    mm.process_incoming_trained_model(3, b)
    assert list(mm.incoming_trained_models.values()) == [a]
    mm.reset_incoming_trained_models()
    assert mm.incoming_trained_models == {}


def test_model_manager_method_selection():
    class S:
        gradient_aggregation = GradientAggregationMethod.FEDAVG

    assert ModelManager(None, S(), 0).get_aggregation_method() is FedAvg

    class T:
        gradient_aggregation = 99

    assert ModelManager(None, T(), 0).get_aggregation_method() is None


def test_task_function_is_star_exported():
    ns = {}
    exec("from dasklearn_amd.functions import *", ns)
    assert ns["aggregate"] is functions.aggregate


@pytest.mark.parametrize("numel,esz,expect", [
    (11_181_642, 4, 11_181_696),        # ResNet-18 fp32: 256 B padding only
    (125_000_000, 2, 125_000_064),      # cfg4 bf16: 256 B padding, not a 64 KiB multiple
    (1 << 20, 4, (1 << 20) + 1024),     # 4 MiB stride -> +4 KiB
    (1 << 23, 2, (1 << 23) + 2048),
    (85_354, 4, 85_376),
    (1, 4, 64),
])
def test_staging_row_stride(numel, esz, expect):
    s = arena.row_stride(numel, esz)
    assert s == expect
    assert (s * esz) % 256 == 0 and s >= numel
    assert (s * esz) % 65536 != 0
