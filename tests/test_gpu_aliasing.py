"""Aliasing and fan-in contract of the C ABI (GPU).

The reference never aliases (fedavg.py:20-25 accumulates into a deepcopy of
models[0]), so every aliasing form the ABI accepts must stay bit-exact, and
the forms it cannot honour must raise:

* dlsim_wreduce: d_out may BE any input (in-place update), for every fan-in —
  including n > DLSIM_MAX_FUSED_INPUTS, where the pointer table lives in device
  memory and the reduce is still a single pass;
* dlsim_wreduce_batched / dlsim_mean_batched / dlsim_chunk_mean_batched:
  results equal b separate calls made in task order, also when one task reads
  or overwrites another task's buffers;
* the descriptor-table batch runs all tasks concurrently: cross-task overlap is
  rejected (DlsimError).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

from dasklearn_amd import _native  # noqa: E402
from test_gpu_parity import dev, from_dev, make_rows, to_dev  # noqa: E402


def dirichlet(n, seed=0):
    return orc.reference_weights(n, list(np.random.default_rng(seed).dirichlet(np.ones(n))))


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("n,k", [(130, 129), (200, 150), (200, 0), (129, 128)])
def test_out_aliases_an_input_past_the_kernarg_slots(n, k, dtype):
    """n > 128 with d_out == d_inputs[k], k beyond the first 128: exact (one
    pass; round 1 split n > 128 into passes and overwrote in[k] first)."""
    p = 10_007
    rows = make_rows(n, p, 300 + n + k, dtype)
    w = dirichlet(n, k)
    xs = to_dev(list(rows), dtype)
    _native.wreduce(xs, w, xs[k])
    assert orc.same_bits(from_dev(xs[k]), orc.wreduce(list(rows), w, dtype))


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_out_aliases_an_input_scalar_path_large_fan_in(dtype):
    """Misaligned views (scalar kernel) with n = 200 and an in-place output."""
    n, p = 200, 3001
    rows = make_rows(n, p + 1, 11, dtype)
    xs = [t[1:] for t in to_dev(list(rows), dtype)]
    w = dirichlet(n, 3)
    _native.wreduce(xs, w, xs[177])
    assert orc.same_bits(from_dev(xs[177]), orc.wreduce([r[1:] for r in rows], w, dtype))


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_fast_mode_large_fan_in_rounds_once(dtype):
    """FAST bf16/f16 at n = 200: one fma chain in fp32, one final rounding (no
    intermediate rounding between passes)."""
    n, p = 200, 20_001
    rows = make_rows(n, p, 21, dtype)
    w = dirichlet(n, 4)
    xs = to_dev(list(rows), dtype)
    out = torch.empty_like(xs[0])
    _native.wreduce(xs, w, out, _native.DLSIM_FAST)
    assert orc.same_bits(from_dev(out), orc.wreduce(list(rows), w, dtype, mode="fast"))


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("n", [3, 200])
def test_mean_large_fan_in_rounds_once(n, dtype):
    """dlsim_mean: input-order fp32 sum, one division, one rounding, any n."""
    p = 20_003
    rows = make_rows(n, p, 31 + n, dtype)
    xs = to_dev(list(rows), dtype)
    out = torch.empty_like(xs[0])
    _native.mean(xs, out)
    assert orc.same_bits(from_dev(out), orc.mean(list(rows), dtype))


def _oracle_replay(bufs, tasks, dtype):
    """Sequential semantics: run tasks in order on host copies of the buffers.
    tasks: (input buffer ids, weights, output buffer id)."""
    host = {k: v.copy() for k, v in bufs.items()}
    for ins, w, o in tasks:
        host[o] = orc.wreduce([host[i] for i in ins], w, dtype)
    return host


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_batched_chain_matches_sequential_calls(dtype):
    """Task 1 reads task 0's output (RAW), task 2 overwrites an input of task 1
    (WAR), task 3 is independent: bit-identical to four calls in order."""
    p = 40_003
    names = ["a", "b", "c", "d", "e", "f", "g"]
    rows = make_rows(len(names), p, 5, dtype)
    bufs = {k: np.ascontiguousarray(r) for k, r in zip(names, rows)}
    dbufs = {k: t for k, t in zip(names, to_dev([bufs[k] for k in names], dtype))}
    tasks = [(["a", "b"], dirichlet(2, 1), "c"),
             (["c", "d", "a"], dirichlet(3, 2), "e"),
             (["e", "f"], dirichlet(2, 3), "d"),
             (["f", "g"], dirichlet(2, 4), "b")]
    exp = _oracle_replay(bufs, tasks, dtype)
    _native.wreduce_batched([([dbufs[i] for i in ins], w, dbufs[o]) for ins, w, o in tasks])
    for k in names:
        assert orc.same_bits(from_dev(dbufs[k]), exp[k]), k


def test_batched_in_place_tasks_stay_batched_and_exact():
    """Each task updating its own input 0 in place (no cross-task overlap)."""
    p = 9_001
    rows = make_rows(12, p, 8, "f32")
    xs = to_dev(list(rows), "f32")
    tasks = [([xs[3 * t], xs[3 * t + 1], xs[3 * t + 2]], dirichlet(3, t), xs[3 * t]) for t in range(4)]
    exps = [orc.wreduce(list(rows[3 * t:3 * t + 3]), dirichlet(3, t), "f32") for t in range(4)]
    _native.wreduce_batched(tasks)
    for t in range(4):
        assert orc.same_bits(from_dev(xs[3 * t]), exps[t])


def test_table_batch_rejects_cross_task_overlap():
    p = 4096
    xs = to_dev(list(make_rows(4, p, 9, "f32")), "f32")
    out = torch.empty(p, device=dev())
    tasks = [([xs[0], xs[1]], dirichlet(2, 1), out),
             ([out, xs[2]], dirichlet(2, 2), xs[3])]
    with pytest.raises(_native.DlsimError, match="overlaps another task"):
        _native.BatchPlan(tasks)
    # the same tasks without the dependency are accepted
    out2 = torch.empty(p, device=dev())
    _native.BatchPlan([([xs[0], xs[1]], dirichlet(2, 1), out),
                       ([xs[2], xs[1]], dirichlet(2, 2), out2)]).launch()


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_mean_batched_chain_matches_sequential_calls(dtype):
    p = 7_777
    rows = make_rows(5, p, 12, dtype)
    xs = to_dev(list(rows), dtype)
    # task 0: mean(x0, x1) -> x2; task 1: mean(x2, x3, x4) -> x0
    e2 = orc.mean([rows[0], rows[1]], dtype)
    e0 = orc.mean([e2, rows[3], rows[4]], dtype)
    _native.mean_batched([([xs[0], xs[1]], xs[2]), ([xs[2], xs[3], xs[4]], xs[0])])
    assert orc.same_bits(from_dev(xs[2]), e2)
    assert orc.same_bits(from_dev(xs[0]), e0)


def test_chunk_mean_batched_chain_matches_sequential_calls():
    p = 70_001
    rows = make_rows(6, p, 13, "f32")
    xs = to_dev(list(rows), "f32")
    e3 = orc.chunk_mean([rows[0], rows[1], rows[2]], "f32", 4)
    e5 = orc.chunk_mean([e3, rows[4]], "f32", 4)
    _native.chunk_mean_batched([([xs[0], xs[1], xs[2]], xs[3]), ([xs[3], xs[4]], xs[5])], threads=4)
    assert orc.same_bits(from_dev(xs[3]), e3)
    assert orc.same_bits(from_dev(xs[5]), e5)
