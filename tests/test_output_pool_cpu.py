"""Host logic of arena.OUTPUT_POOL (the contiguous-block cache for large
aggregate outputs) on the CPU: the library's device blocks
are replaced by host tensors, the stream handle by a counter. Reuse only
when no tensor views a block, only on the stream it was made for, release(),
the retry after an allocation failure, a forked child's fresh pool."""
from __future__ import annotations

import os

import pytest
import torch

from dasklearn_amd import _native, arena


class FakeBlock:
    made = 0
    fail_next = 0

    def __init__(self, nbytes, device, contiguous=True):
        if FakeBlock.fail_next:
            FakeBlock.fail_next -= 1
            raise _native.DlsimError("dlsim_device_alloc", -102, "out of memory")
        FakeBlock.made += 1
        self.nbytes, self.contiguous = nbytes, True
        self._t = torch.empty(nbytes, dtype=torch.uint8)

    def tensor(self):
        # like the real block: the storage keeps the memory, the block object
        # holds no tensor of its own
        t, self._t = self._t, None
        return t


@pytest.fixture()
def pool(monkeypatch):
    stream = {"h": 0}
    monkeypatch.setattr(_native, "DeviceBlock", FakeBlock)
    monkeypatch.setattr(torch._C, "_cuda_getCurrentRawStream", lambda idx: stream["h"], raising=False)
    monkeypatch.setattr(torch.cuda, "empty_cache", lambda: None)
    monkeypatch.delenv("DLSIM_CONTIGUOUS", raising=False)
    FakeBlock.made = FakeBlock.fail_next = 0
    p = arena._OutputPool()
    p.stream = stream
    return p


N = (6 << 20) // 4  # a 6 MiB fp32 output


def test_reuse_only_when_no_view_remains(pool):
    a = pool.take(N, torch.float32, "cuda:0")
    assert a.dtype == torch.float32 and a.numel() == N
    pa = a.data_ptr()
    b = pool.take(N, torch.float32, "cuda:0")
    assert b.data_ptr() != pa and FakeBlock.made == 2
    view = a[10:20]
    del a
    c = pool.take(N, torch.float32, "cuda:0")
    assert c.data_ptr() != pa and FakeBlock.made == 3
    del view
    d = pool.take(N - 1000, torch.float32, "cuda:0")  # same 2 MiB size class
    assert d.data_ptr() == pa and FakeBlock.made == 3
    p = torch.nn.Parameter(d[:100])  # a parameter view keeps the block busy
    del d
    e = pool.take(N, torch.float32, "cuda:0")
    assert e.data_ptr() != pa
    del p, b, c, e
    assert pool.release() == 4 and pool.cached_bytes() == 0


def test_blocks_are_per_stream_and_per_size(pool):
    a = pool.take(N, torch.float32, "cuda:0")
    pa = a.data_ptr()
    del a
    pool.stream["h"] = 7
    b = pool.take(N, torch.float32, "cuda:0")
    assert b.data_ptr() != pa  # made for stream 0, not reused on stream 7
    pool.stream["h"] = 0
    c = pool.take(3 * N, torch.float32, "cuda:0")
    assert c.data_ptr() != pa  # another size class
    d = pool.take(N, torch.bfloat16, "cuda:0")  # 3 MiB of bf16: a 4 MiB class
    assert d.data_ptr() != pa
    e = pool.take(2 * N, torch.bfloat16, "cuda:0")  # 6 MiB: the first block's class
    assert e.data_ptr() == pa and e.dtype == torch.bfloat16


def test_allocation_failure_releases_and_retries(pool):
    a = pool.take(N, torch.float32, "cuda:0")
    del a  # one idle block to give back
    FakeBlock.fail_next = 1
    b = pool.take(5 * N, torch.float32, "cuda:0")
    assert b.numel() == 5 * N
    assert pool.cached_bytes() == (5 * N * 4 + arena.ROW_ALIGN - 1) // arena.ROW_ALIGN * arena.ROW_ALIGN
    FakeBlock.fail_next = 2
    with pytest.raises(_native.DlsimError):
        pool.take(9 * N, torch.float32, "cuda:0")


def test_off_switch_and_fork(pool, monkeypatch):
    monkeypatch.setenv("DLSIM_CONTIGUOUS", "0")
    assert pool.take(N, torch.float32, "cuda:0") is None
    monkeypatch.delenv("DLSIM_CONTIGUOUS")
    a = pool.take(N, torch.float32, "cuda:0")
    assert pool.cached_bytes() > 0
    pool.pid = os.getpid() + 1  # as seen from a forked child
    b = pool.take(N, torch.float32, "cuda:0")
    assert pool.pid == os.getpid() and len(sum(pool.blocks.values(), [])) == 1
    assert b.data_ptr() != a.data_ptr()


def test_arena_empty_routes_by_size_and_device():
    small = arena.arena_empty(1000, torch.float32, "cpu")
    big = arena.arena_empty(N, torch.float32, "cpu")  # host arenas never use the pool
    assert small.numel() == 1000 and big.numel() == N and not big.is_cuda
    assert arena.OUT_POOL_MIN == 4 << 20 or os.environ.get("DLSIM_OUT_POOL_MIN_MB")
