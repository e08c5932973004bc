"""bench.py's workload on the GPU (round 6): step k reduces input set k mod S
into output k mod O, bit-exact against the oracle, and the decoy set
(ReduceWorkload._prime) is read before anything timed and
is never one of the rotating sets."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import bench  # noqa: E402
from oracle import oracle as orc  # noqa: E402

pytestmark = pytest.mark.gpu


def _workload(n, p, monkeypatch, prime="1"):
    from dasklearn_amd import _native
    monkeypatch.setenv("DLSIM_BENCH_PRIME", prime)
    dev = torch.device("cuda", 0)
    w32 = _native.fp32_weights(bench.weights_for("dirichlet", n))
    wl = bench.ReduceWorkload(n, p, "f32", w32, _native.DLSIM_EXACT, 1, dev, 5, torch.cuda.current_stream(dev))
    return wl, w32


def _rows_of(plan):
    return np.stack([t.cpu().numpy() for t in plan._keep[0]])


def test_steps_rotate_sets_and_outputs_bit_exact(monkeypatch):
    n, p = 8, 1_397_760  # the 8-rank slice's shape
    wl, w32 = _workload(n, p, monkeypatch)
    assert wl.sets == 22 and wl.out_sets % wl.sets == 0 and wl.out_sets * p * 4 >= bench.MIN_OUT_FOOTPRINT
    for k in (0, 1, wl.sets - 1, wl.sets, wl.out_sets - 1):
        wl.launch(k)
        torch.cuda.synchronize()
        plan = wl.plans[k % wl.out_sets]
        assert plan._keep[0][0].data_ptr() == wl.plans[k % wl.sets]._keep[0][0].data_ptr()
        want = orc.wreduce_rows_f32(_rows_of(plan), w32)
        assert orc.same_bits(wl.outs[k % wl.out_sets].cpu().numpy(), want), k


def test_decoy_is_read_first_and_is_not_a_rotating_set(monkeypatch):
    n, p = 8, 1_397_760
    wl, w32 = _workload(n, p, monkeypatch)
    decoys = [x for x in wl._keep if isinstance(x, tuple) and len(x) == 3]
    assert len(decoys) == 1
    rows, out, plan = decoys[0]
    # the prime launches ran (synchronised in __init__): the decoy's output is its aggregate
    assert orc.same_bits(out.cpu().numpy(), orc.wreduce_rows_f32(_rows_of(plan), w32))
    lo, hi = rows.data_ptr(), rows.data_ptr() + rows.numel() * 4
    for pl in wl.plans:
        for t in pl._keep[0]:
            assert not lo <= t.data_ptr() < hi
    wl2, _ = _workload(n, p, monkeypatch, prime="0")
    assert not [x for x in wl2._keep if isinstance(x, tuple) and len(x) == 3]


def test_batched_workload_with_ragged_rows_builds_and_runs(monkeypatch):
    # p * 4 bytes not a multiple of 16: every task's rows and outputs must still
    # be 16-B aligned for the table batch (the decoy's included)
    from dasklearn_amd import _native
    monkeypatch.setenv("DLSIM_BENCH_PRIME", "1")
    dev = torch.device("cuda", 0)
    n, p = 4, 100_003
    w32 = _native.fp32_weights(bench.weights_for("dirichlet", n))
    wl = bench.ReduceWorkload(n, p, "f32", w32, _native.DLSIM_EXACT, 3, dev, 9, torch.cuda.current_stream(dev))
    for k in range(3):
        wl.launch(k)
    torch.cuda.synchronize()
    assert wl.kernel == "dlsim::k_wreduce_batch_table"
    assert all(torch.isfinite(o).all().item() for o in wl.outs[:3])
