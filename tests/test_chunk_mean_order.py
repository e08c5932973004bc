"""The chunk mean's summation order, pinned against PyTorch itself.

The reference's `reconstruct_model` computes torch.mean(torch.stack(chunks),
dim=0) on the worker's CPU (simulation/conflux/chunk_manager.py:40) at
settings.torch_threads intra-op threads (broker.py:31). The arithmetic is
PyTorch's, and this image's PyTorch is the one the reference runs on here, so
the order-exact restatement (oracle.chunk_mean, oracle/fedavg_oracle.c) is
checked bit for bit against torch.mean across thread counts, contributor
counts and chunk lengths that exercise every branch: the serial and the
thread-split column ranges, the 32-column cascade blocks, the row_sum (ILP)
tail, the scalar path below 8 columns, the one-element inner reduction, and
the multi-level cascade above 16 / 256 contributors.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as orc


def _torch_mean(x: np.ndarray, threads: int, dtype: str) -> np.ndarray:
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        half = {"bf16": torch.bfloat16, "f16": torch.float16}.get(dtype)
        t = torch.from_numpy(x.view(np.int16)).view(half) if half else torch.from_numpy(x)
        r = torch.mean(torch.stack(list(t)), dim=0)
        return r.view(torch.int16).numpy().view(np.uint16) if half == torch.bfloat16 else r.numpy()
    finally:
        torch.set_num_threads(prev)


def _rows(rng, m, n, dtype):
    x = (rng.standard_normal((m, n)) * np.exp(rng.standard_normal((m, n)) * 2)).astype(np.float32)
    if dtype == "f16":
        return orc.f32_to_f16_bits(np.clip(x, -6e4, 6e4))
    return orc.f32_to_bf16_bits(x) if dtype == "bf16" else x


CASES = [(m, n) for m in (1, 2, 3, 4, 5, 7, 8, 9, 16, 17, 18, 33, 64)
         for n in (1, 2, 3, 4, 5, 7, 8, 9, 31, 32, 33, 63, 65, 1000, 2047)]


@pytest.mark.parametrize("threads", [1, 4])
def test_small_grid_matches_torch(threads):
    rng = np.random.default_rng(threads)
    for m, n in CASES:
        x = _rows(rng, m, n, "f32")
        assert orc.same_bits(orc.chunk_mean(list(x), "f32", threads), _torch_mean(x, threads, "f32")), (m, n)


@pytest.mark.parametrize("threads", [2, 3, 4, 8])
@pytest.mark.parametrize("m,n", [(5, 9001), (10, 40001), (20, 8535), (33, 4001), (4, 8193), (1000, 37),
                                 (2000, 70)])
def test_thread_split_matches_torch(threads, m, n):
    """m * n >= 32768: columns split over the threads (32-column rounding);
    at (1000, 37) and (2000, 70) most ranges round to nothing."""
    rng = np.random.default_rng(m * 7 + n)
    x = _rows(rng, m, n, "f32")
    assert orc.same_bits(orc.chunk_mean(list(x), "f32", threads), _torch_mean(x, threads, "f32"))


@pytest.mark.parametrize("m", [255, 256, 257, 300])
def test_multilevel_cascade_matches_torch(m):
    rng = np.random.default_rng(m)
    for n in (1, 5, 40):
        x = _rows(rng, m, n, "f32")
        assert orc.same_bits(orc.chunk_mean(list(x), "f32", 4), _torch_mean(x, 4, "f32")), n


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("m", [2, 3, 5, 17, 20])
def test_half_types_match_torch(m, dtype):
    """bf16 and fp16 chunks: summed in fp32 in the same order, divided,
    rounded once."""
    rng = np.random.default_rng(100 + m)
    for n in (1, 7, 1000, 9001):
        x = _rows(rng, m, n, dtype)
        assert orc.same_bits(orc.chunk_mean(list(x), dtype, 4), _torch_mean(x, 4, dtype)), n


def test_ilp_begin_rule():
    # serial: the last n mod 32 columns (n >= 8), groups of 4 below 8 columns
    assert orc.chunk_mean_ilp_begin(4, 1000, 4) == 992
    assert orc.chunk_mean_ilp_begin(4, 7, 4) == 4
    assert orc.chunk_mean_ilp_begin(4, 1, 4) == 0
    # split over 4 threads: internal ranges are 32-multiples, so the same rule
    assert orc.chunk_mean_ilp_begin(10, 1118164, 4) == 1118144
    # ranges that round to nothing fold into the last one
    assert orc.chunk_mean_ilp_begin(1000, 37, 4) == 32
    # a final range of 5 columns (< 8 wide): groups of 4 columns there
    assert orc.chunk_mean_ilp_begin(400, 101, 20) == 100


def test_short_final_range_matches_torch():
    """20 threads over 101 columns: the final range is [96, 101), narrower
    than the 8-wide vector, so scalar_outer_sum's groups of 4 apply."""
    rng = np.random.default_rng(11)
    x = _rows(rng, 400, 101, "f32")
    assert orc.same_bits(orc.chunk_mean(list(x), "f32", 20), _torch_mean(x, 20, "f32"))


def test_abi_ilp_begin_matches_oracle():
    """The product's host rule (dlsim_chunk_mean_ilp_begin, csrc/dlsim_abi.hip)
    and the oracle's agree everywhere the column split can land."""
    from dasklearn_amd import _native
    rng = np.random.default_rng(0)
    cases = [(m, n, t) for m in (1, 4, 17, 400, 1000) for n in (0, 1, 2, 7, 8, 31, 32, 33, 37, 101, 1000, 40001)
             for t in (1, 2, 3, 4, 8, 20)]
    cases += [(int(rng.integers(1, 3000)), int(rng.integers(1, 200000)), int(rng.integers(1, 64)))
              for _ in range(300)]
    for m, n, t in cases:
        assert _native.chunk_mean_ilp_begin(m, n, t) == orc.chunk_mean_ilp_begin(m, n, t), (m, n, t)
