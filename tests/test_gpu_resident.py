"""dlsim_host_wreduce_resident (include/dlsim.h; the device cache's library
call, dasklearn_amd/device_cache.py) against the oracle on MI355X.

Random tasks: fan-in 1-17, 1-5 tensors per model (empty ones included), fp32,
bf16 and fp16, a random subset of the models already resident in device rows
(read in place), the others packed into pinned staging and sent to their
rows — some of those rows back to back one staging stride apart (sent in one
DMA run), some in separate allocations. The result (device and host) must be
bit-identical to the reference's fold (fedavg.py:20-25, oracle.wreduce) and
every sent row must hold its model afterwards (the cache reads it in later
tasks)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}


def _bits(t: torch.Tensor) -> np.ndarray:
    t = t.detach().cpu().reshape(-1)
    return t.numpy() if t.dtype == torch.float32 else t.view(torch.int16).numpy().view(np.uint16)


def _case(rng, dt, h2d_kb, monkeypatch, all_resident=False, none_resident=False):
    from dasklearn_amd import _native
    from dasklearn_amd.arena import row_stride
    monkeypatch.setenv("DLSIM_AB", "1")  # A/B switches are read only under DLSIM_AB=1
    monkeypatch.setenv("DLSIM_H2D_MIN_KB", str(h2d_kb))
    dev = torch.device("cuda", 0)
    tdt = DT[dt]
    esz = torch.empty((), dtype=tdt).element_size()
    n = int(rng.integers(1, 18))
    t = int(rng.integers(1, 6))
    numels = [int(rng.choice([0, int(rng.integers(1, 70_000))], p=[0.15, 0.85])) for _ in range(t)]
    if sum(numels) == 0:
        numels[0] = 1000
    total = sum(numels)
    stride = row_stride(total, esz)
    models = [[(torch.randn(k) * 0.05).to(tdt) for k in numels] for _ in range(n)]
    flat = [torch.cat([x.reshape(-1) for x in m]) for m in models]
    resident = [bool(rng.random() < 0.5) for _ in range(n)]
    if all_resident:
        resident = [True] * n
    if none_resident:
        resident = [False] * n
    miss = [i for i in range(n) if not resident[i]]
    keep, rows = [], [0] * n
    for i in range(n):
        if resident[i]:  # already on the device, in a row of its own
            r = torch.empty(stride, dtype=tdt, device=dev)
            r[:total].copy_(flat[i])
            keep.append(r)
            rows[i] = r.data_ptr()
    # misses: the first half back to back in one block (one DMA run), the
    # rest in rows of their own
    block_n = len(miss) // 2 + (len(miss) % 2)
    if block_n:
        blk = torch.full((block_n * stride,), float("nan"), dtype=tdt, device=dev)
        keep.append(blk)
        for j, i in enumerate(miss[:block_n]):
            rows[i] = blk.data_ptr() + j * stride * esz
    for i in miss[block_n:]:
        r = torch.full((stride,), float("nan"), dtype=tdt, device=dev)
        keep.append(r)
        rows[i] = r.data_ptr()
    staging = torch.empty((max(1, len(miss)), stride), dtype=tdt, pin_memory=True) if miss else None
    src = []
    for i in range(n):
        src += [0 if resident[i] else x.data_ptr() for x in models[i]]
    w = list(rng.dirichlet(np.ones(n))) if rng.random() < 0.7 else None
    w32 = orc.reference_weights(n, w)
    out = torch.empty(total, dtype=tdt, device=dev)
    host = torch.empty(total, dtype=tdt, pin_memory=True)
    stream = torch.cuda.current_stream(dev)
    _native.host_wreduce_resident_raw(src, n, numels, w32, resident, rows, staging, out, host,
                                      _native.dtype_code(tdt), _native.DLSIM_EXACT, 4, stream.cuda_stream)
    stream.synchronize()
    exp = orc.wreduce([_bits(f) for f in flat], w32, dt)
    assert orc.same_bits(_bits(host), exp), (dt, n, numels, resident)
    assert orc.same_bits(_bits(out), exp)
    for i in miss:  # every sent row holds its model
        got = torch.empty(total, dtype=tdt)
        view = next(k for k in keep if k.data_ptr() <= rows[i] < k.data_ptr() + k.numel() * esz)
        off = (rows[i] - view.data_ptr()) // esz
        got.copy_(view[off:off + total])
        assert torch.equal(got.view(torch.int16 if esz == 2 else torch.int32),
                           flat[i].view(torch.int16 if esz == 2 else torch.int32)), (dt, i)


@pytest.mark.parametrize("dt", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_resident_random(dt, seed, monkeypatch):
    rng = np.random.default_rng(1000 * seed + len(dt))
    _case(rng, dt, int(rng.choice([0, 64, 1024])), monkeypatch)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_resident_all_and_none(dt, monkeypatch):
    rng = np.random.default_rng(7)
    _case(rng, dt, 1024, monkeypatch, all_resident=True)
    _case(rng, dt, 1024, monkeypatch, none_resident=True)


def test_resident_rejects_overlapping_written_rows():
    """A row the call writes (a model not resident) must not overlap another
    row; resident rows may alias each other (the same model twice)."""
    from dasklearn_amd import _native
    dev = torch.device("cuda", 0)
    total, n = 1000, 3
    models = [[torch.randn(total)] for _ in range(n)]
    rows = torch.zeros(4 * 1024, device=dev)
    w32 = orc.reference_weights(n, None)
    out = torch.empty(total, device=dev)
    staging = torch.empty((n, 1024), pin_memory=True)
    src = [m[0].data_ptr() for m in models]
    stream = torch.cuda.current_stream(dev).cuda_stream
    base = rows.data_ptr()
    # rows 0 and 1 overlap by half a row; row 1 is written
    bad = [base, base + 500 * 4, base + 2048 * 4]
    with pytest.raises(_native.DlsimError, match="overlap"):
        _native.host_wreduce_resident_raw(src, n, [total], w32, [True, False, True], bad, staging, out, None,
                                          _native.dtype_code(torch.float32), _native.DLSIM_EXACT, 1, stream)
    # two resident rows that alias: allowed, and exact
    r0 = rows[:total]
    r0.copy_(models[0][0].to(dev))
    same = [base, base, base + 2048 * 4]
    _native.host_wreduce_resident_raw(src, n, [total], w32, [True, True, False], same, staging, out, None,
                                      _native.dtype_code(torch.float32), _native.DLSIM_EXACT, 1, stream)
    torch.cuda.synchronize()
    exp = orc.wreduce([models[0][0].numpy(), models[0][0].numpy(), models[2][0].numpy()], w32, "f32")
    assert orc.same_bits(out.cpu().numpy(), exp)
