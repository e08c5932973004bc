"""Chunked-model path (Conflux/Shatter), CPU side: the oracle's sequential
mean and the chunking data movement against fixtures produced by the
reference's own ChunkManager (tests/golden/make_golden_chunks.py;
dasklearn/simulation/conflux/chunk_manager.py:13-53)."""
from __future__ import annotations

import glob
import json
import os

import numpy as np
import pytest
import torch
from torch import nn

from conftest import GOLDEN
from oracle import oracle as orc
from dasklearn_amd.chunk_manager import ChunkManager

CHUNK_FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "chunks", "*.npz")))


def load(path):
    with np.load(path, allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    return d


class Net(nn.Module):
    def __init__(self, shapes):
        super().__init__()
        self.ps = nn.ParameterList([nn.Parameter(torch.zeros(*s)) for s in shapes])


def model_from_flat(shapes, flat):
    m = Net(shapes)
    off = 0
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.from_numpy(flat[off:off + p.numel()].copy()).view_as(p))
            off += p.numel()
    return m


@pytest.mark.parametrize("path", CHUNK_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_chunking_matches_reference(path):
    d = load(path)
    k, counts = d["meta"]["num_chunks"], d["meta"]["counts"]
    for p in range(max(counts)):
        chunks = ChunkManager.chunk_model(model_from_flat(d["meta"]["shapes"], d[f"flat_{p}"]), k)
        assert len(chunks) == k
        for c in range(k):
            if p < counts[c]:
                assert np.array_equal(chunks[c].numpy(), d[f"chunks_{c}"][p])


@pytest.mark.parametrize("path", CHUNK_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_mean_vs_reference(path):
    """Bit-exact where PyTorch's dim-0 sum is sequential (<= 4 contributors);
    within m * 2^-23 of mean|x| otherwise."""
    d = load(path)
    k, counts = d["meta"]["num_chunks"], d["meta"]["counts"]
    got = np.concatenate([orc.mean(list(d[f"chunks_{c}"])) for c in range(k)])
    off = 0
    for c in range(k):
        L = d[f"chunks_{c}"].shape[1]
        g, e = got[off:off + L], d["expected"][off:off + L]
        if counts[c] <= 4:
            assert orc.same_bits(g, e), (c, counts[c])
        else:
            scale = np.abs(d[f"chunks_{c}"]).mean(axis=0)
            assert np.all(np.abs(g - e) <= counts[c] * 2.0 ** -23 * scale + 1e-30), (c, counts[c])
        off += L


def test_reconstruct_asserts_on_empty_chunk_index():
    with pytest.raises(AssertionError, match="No chunks received at index 1"):
        ChunkManager.reconstruct_model([[torch.zeros(3)], []], Net([[6]]))


def test_chunk_remainder_goes_to_last_chunk():
    m = Net([[10], [3]])
    chunks = ChunkManager.chunk_model(m, 4)  # 13 = 3+3+3+4
    assert [c.numel() for c in chunks] == [3, 3, 3, 4]


def test_span_is_a_cat_only_for_back_to_back_views():
    """reconstruct_model skips torch.cat when the chunk means already lie back
    to back in one buffer (chunk_manager._span); anything else still cats."""
    from dasklearn_amd.chunk_manager import _span
    buf = torch.arange(20.0)
    views = [buf[0:4], buf[4:12], buf[12:19]]
    s = _span(views)
    assert s is not None and torch.equal(s, torch.cat(views)) and s.data_ptr() == buf.data_ptr()
    assert _span([buf[0:4], buf[5:8]]) is None  # gap
    assert _span([buf[4:8], buf[0:4]]) is None  # out of order
    assert _span([buf[0:4], torch.arange(4.0)]) is None  # other storage
    assert _span([buf[0:8:2]]) is None  # strided
    assert _span([buf.view(4, 5)]) is None  # not flat


@pytest.mark.parametrize("path", CHUNK_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_chunk_mean_oracle_bit_exact_vs_reference(path):
    """The order-exact restatement (oracle.chunk_mean: ATen's cascade_sum
    column order at the fixture's torch_threads) reproduces every chunk mean
    the reference's ChunkManager produced, for every contributor count."""
    d = load(path)
    k, counts = d["meta"]["num_chunks"], d["meta"]["counts"]
    got = np.concatenate([orc.chunk_mean(list(d[f"chunks_{c}"]), "f32", d["meta"]["torch_threads"])
                          for c in range(k)])
    assert orc.same_bits(got, d["expected"])


@pytest.mark.parametrize("path", CHUNK_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_fixtures_record_the_build_their_order_is_pinned_to(path):
    """Every chunk fixture says which torch build and CPU dispatch produced it,
    and that is the scope ChunkManager.order_scope() accepts."""
    from dasklearn_amd import chunk_manager as cm
    meta = load(path)["meta"]
    assert cm.order_scope(meta["torch_version"], meta["cpu_capability"]) is None
    assert meta["torch_version"].startswith(cm.ORDER_PINNED_TORCH + ".")


def test_order_scope_names_another_build():
    from dasklearn_amd import chunk_manager as cm
    assert cm.order_scope("2.10.0+rocm7.0", "AVX512") is None
    assert cm.order_scope("2.10.1", "AVX2") is None
    msg = cm.order_scope("2.1.2+cpu", "AVX2")
    assert msg and "torch 2.1.2+cpu" in msg
    msg = cm.order_scope("2.10.0", "DEFAULT")
    assert msg and "CPU capability DEFAULT" in msg


def test_reconstruction_warns_once_outside_the_pinned_build(monkeypatch):
    from dasklearn_amd import chunk_manager as cm
    monkeypatch.setattr(cm, "_SCOPE_CHECKED", False)
    monkeypatch.setattr(cm.torch, "__version__", "2.1.2+cpu")
    with pytest.warns(cm.ParityScopeWarning, match="2.1.2"):
        cm._check_order_scope()
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        cm._check_order_scope()  # once per process


# ---- fp64 chunks ---------------------------------------
CHUNK_FIXTURES_F64 = sorted(glob.glob(os.path.join(GOLDEN, "chunks_f64", "*.npz")))


def net64(shapes):
    return Net(shapes).double()


def test_f64_fixtures_exist():
    assert len(CHUNK_FIXTURES_F64) >= 6


@pytest.mark.parametrize("path", CHUNK_FIXTURES_F64, ids=lambda p: os.path.basename(p)[:-4])
def test_f64_chunking_matches_reference(path):
    d = load(path)
    assert d["meta"]["dtype"] == "f64" and d["expected"].dtype == np.float64
    k, counts = d["meta"]["num_chunks"], d["meta"]["counts"]
    for p in range(max(counts)):
        m = net64(d["meta"]["shapes"])
        off = 0
        with torch.no_grad():
            for q in m.parameters():
                q.copy_(torch.from_numpy(d[f"flat_{p}"][off:off + q.numel()].copy()).view_as(q))
                off += q.numel()
        chunks = ChunkManager.chunk_model(m, k)
        for c in range(k):
            if p < counts[c]:
                assert np.array_equal(chunks[c].numpy(), d[f"chunks_{c}"][p])


@pytest.mark.parametrize("path", CHUNK_FIXTURES_F64, ids=lambda p: os.path.basename(p)[:-4])
def test_f64_chunk_mean_oracle_bit_exact_vs_reference(path):
    """oracle.chunk_mean(..., "f64"): PyTorch's double order (4-lane vectors,
    16-column blocks and rounding) reproduces every mean the reference's
    ChunkManager produced on double models."""
    d = load(path)
    k = d["meta"]["num_chunks"]
    got = np.concatenate([orc.chunk_mean(list(d[f"chunks_{c}"]), "f64", d["meta"]["torch_threads"])
                          for c in range(k)])
    assert np.array_equal(got.view(np.int64), d["expected"].view(np.int64))


@pytest.mark.parametrize("threads", [1, 2, 3, 4, 8])
def test_f64_chunk_mean_oracle_matches_torch(threads):
    """The double order against torch.mean itself across the branches: the
    vectorized (>= 4 columns) and scalar paths, 16-column blocks, the row_sum
    tail, the 4-lane inner reduction, the thread split, multi-level cascades."""
    rng = np.random.default_rng(threads + 64)
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        for m in (1, 2, 3, 4, 5, 7, 8, 16, 17, 33, 300):
            for n in (1, 2, 3, 4, 5, 15, 16, 17, 31, 33, 100, 8193, 40001):
                x = rng.standard_normal((m, n)) * np.exp(rng.standard_normal((m, n)) * 2)
                exp = torch.mean(torch.stack(list(torch.from_numpy(x))), 0).numpy()
                got = orc.chunk_mean(list(x), "f64", threads)
                assert np.array_equal(got.view(np.int64), exp.view(np.int64)), (m, n)
    finally:
        torch.set_num_threads(prev)


def test_chunk_scan_classifies_and_validates():
    """_pyhost.chunk_scan, the one-pass check ahead of the fast chunk-mean path
    (chunk_manager._fast_means): torch.stack's error for unequal contributors,
    the place code, per-index sizes and fan-in, the pointers in order, and None
    pointers when a chunk is not contiguous."""
    from dasklearn_amd.arena import _pyhost
    a = [torch.randn(5) for _ in range(3)]
    b = [torch.randn(7) for _ in range(2)]
    same, place, dix, numels, fans, ptrs = _pyhost.chunk_scan([a, b])
    assert (same, place, dix, numels, fans) == (True, 1, -1, [5, 7], [3, 2])
    assert ptrs == [t.data_ptr() for t in a + b]
    assert _pyhost.chunk_scan([a, [torch.randn(6, 2).t()]])[5] is None  # non-contiguous
    assert _pyhost.chunk_scan([a, [torch.randn(7, dtype=torch.float64)]])[0] is False  # two dtypes
    with pytest.raises(RuntimeError, match="stack expects each tensor to be equal size"):
        _pyhost.chunk_scan([[torch.randn(5), torch.randn(4)]])
    with pytest.raises(RuntimeError, match="stack expects each tensor to be equal size"):
        _pyhost.chunk_scan([[torch.randn(5), torch.randn(5, dtype=torch.float64)]])
    with pytest.raises(RuntimeError):
        _pyhost.chunk_scan([[]])
    assert _pyhost.chunk_scan([])[1] == 0
