"""Which host tasks the one-pass zero-copy path takes (round 6,
arena._host_zc_task; the GPU side: tests/test_gpu_dropin.py::
test_small_host_task_fast_path). Host-only decisions, no device call: a
model class whose layout is known, one dtype group (not fp64), at most
ZC_MAX_BYTES of rows, the zero-copy switch on, no device cache, every model
of models[0]'s signature with its parameters on the host."""
from __future__ import annotations

import pytest
import torch
from torch import nn

from dasklearn_amd import arena, device_cache


class Net(nn.Module):
    def __init__(self, dt=torch.float32, width=8):
        super().__init__()
        self.a = nn.Linear(width, 4)
        self.b = nn.Linear(4, 3)
        self.to(dt)


@pytest.fixture()
def known(monkeypatch):
    monkeypatch.setattr(arena, "_CLASS_LAYOUTS", {})
    monkeypatch.setattr(arena, "ZERO_COPY", True)
    monkeypatch.setattr(arena, "pinned_result", lambda nbytes: True)
    monkeypatch.setattr(device_cache, "_CACHE", None)

    def learn(m):
        arena.layout_of(m)  # what the general path's first task of the class does
    return learn


def test_known_class_of_one_signature_is_taken(known):
    ms = [Net() for _ in range(3)]
    assert arena._host_zc_task(ms) is None  # the class layout is not known yet
    known(ms[0])
    layout, dt, idx, params = arena._host_zc_task(ms)
    assert dt is torch.float32 and idx == [0, 1, 2, 3] and len(params) == 3
    assert all(p is q for p, q in zip(params[1], ms[1].parameters()))


def test_each_refusal(known, monkeypatch):
    ms = [Net() for _ in range(3)]
    known(ms[0])
    assert arena._host_zc_task(ms) is not None
    assert arena._host_zc_task([ms[0], Net(width=9)]) is None  # another signature (the zip path decides)
    monkeypatch.setattr(arena, "ZC_MAX_BYTES", 3 * 51 * 4 - 1)  # 51 params per model
    assert arena._host_zc_task(ms) is None
    monkeypatch.setattr(arena, "ZC_MAX_BYTES", 4 << 20)
    monkeypatch.setattr(arena, "ZERO_COPY", False)
    assert arena._host_zc_task(ms) is None
    monkeypatch.setattr(arena, "ZERO_COPY", True)
    monkeypatch.setattr(device_cache, "_CACHE", object())
    assert arena._host_zc_task(ms) is None
    monkeypatch.setattr(device_cache, "_CACHE", None)
    monkeypatch.setattr(arena, "pinned_result", lambda nbytes: False)  # the page-locked budget is spent
    assert arena._host_zc_task(ms) is None


def test_fp64_and_mixed_dtypes_go_to_the_general_path(known):
    d = [Net(torch.float64) for _ in range(2)]
    known(d[0])
    assert arena._host_zc_task(d) is None
    mixed = Net()
    mixed.b.bias.data = mixed.b.bias.data.to(torch.bfloat16)
    known(mixed)
    assert arena._host_zc_task([mixed, mixed]) is None  # two dtype groups
