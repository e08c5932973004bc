"""Host logic of arena.OUTPUT_POOL (large aggregate outputs allocated inside a
torch.cuda.MemPool over the library's contiguous blocks) on
the CPU: the MemPool and the allocation inside it are replaced by fakes.
Size classes, the dtype view, the 2 MiB alignment (and the re-alignment of a
block that an outside allocation split), one allocation context at a time
across threads, release(), the off switch and a forked child's fresh pools.
What torch's caching allocator does with the blocks (per-stream reuse,
record_stream, statistics) is tested on the GPU (test_gpu_resident_alloc.py)."""
from __future__ import annotations

import os
import threading
import time
import warnings

import pytest
import torch

from dasklearn_amd import arena

MIB2 = arena.ROW_ALIGN


class FakeDevice:
    """Host memory standing in for the pool: a 2 MiB-aligned bump allocator
    that can be told to hand out a misaligned block next."""

    def __init__(self):
        self.raw = torch.empty(512 << 20, dtype=torch.uint8)
        self.base = (-self.raw.data_ptr()) % MIB2
        self.off = 0
        self.misalign_next = 0
        self.calls = []  # (idx, nbytes)
        self.active = 0  # allocation contexts open at once
        self.max_active = 0

    def empty_in(self, mp, idx, nbytes):
        self.active += 1
        self.max_active = max(self.max_active, self.active)
        try:
            time.sleep(0.001)  # widen the window a concurrent caller would hit
            self.calls.append((idx, nbytes))
            skew = 0
            if self.misalign_next:
                self.misalign_next -= 1
                skew = 4096
            start = self.base + self.off + skew
            self.off += (nbytes + skew + MIB2 - 1) // MIB2 * MIB2
            return self.raw[start:start + nbytes]
        finally:
            self.active -= 1


class IdleMemPool:
    """A MemPool stand-in whose segments are all gone."""
    id = (0, 1)

    def snapshot(self):
        return []


@pytest.fixture()
def pool(monkeypatch):
    fake = FakeDevice()
    p = arena._OutputPool()
    monkeypatch.setattr(p, "_mempool", lambda idx: p.pools.setdefault(idx, IdleMemPool()))
    monkeypatch.setattr(p, "_empty_in", fake.empty_in)
    emptied = []
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    monkeypatch.setattr(torch.cuda, "empty_cache", lambda: emptied.append(1))
    monkeypatch.setattr(torch.cuda, "memory_snapshot", lambda pid=None: [])
    monkeypatch.delenv("DLSIM_CONTIGUOUS", raising=False)
    p.fake, p.emptied = fake, emptied
    return p


N = (6 << 20) // 4  # a 6 MiB fp32 output


def test_sizes_round_to_2mib_and_view_the_dtype(pool):
    a = pool.take(N, torch.float32, "cuda:0")
    assert a.dtype == torch.float32 and a.numel() == N and a.data_ptr() % MIB2 == 0
    b = pool.take(N - 1000, torch.bfloat16, "cuda:1")
    assert b.dtype == torch.bfloat16 and b.numel() == N - 1000 and b.data_ptr() % MIB2 == 0
    assert pool.fake.calls == [(0, 6 << 20), (1, 4 << 20)]  # (N - 1000) * 2 B rounds up to 4 MiB
    assert set(pool.pools) == {0, 1} and pool.made == 2


def test_a_misaligned_block_is_realigned(pool):
    pool.fake.misalign_next = 1
    a = pool.take(N, torch.float32, "cuda:0")
    assert a.data_ptr() % MIB2 == 0 and a.numel() == N
    assert pool.fake.calls == [(0, 6 << 20), (0, (6 << 20) + MIB2)]


def test_one_allocation_context_at_a_time(pool):
    outs, errs = [], []

    def worker():
        try:
            for _ in range(5):
                outs.append(pool.take(N, torch.float32, "cuda:0"))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)
    ts = [threading.Thread(target=worker) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs and len(outs) == 20
    assert pool.fake.max_active == 1
    assert len({o.data_ptr() for o in outs}) == 20


def test_release_retires_the_pools_and_empties_the_cache(pool):
    pool.take(N, torch.float32, "cuda:0")
    pool.take(N, torch.float32, "cuda:1")
    first = pool.pools[0]
    assert pool.release() == 2 and pool.pools == {} and pool.emptied == [1]
    assert pool.release() == 0 and pool.emptied == [1]  # nothing to retire: no device-wide sync
    pool.take(N, torch.float32, "cuda:0")
    assert pool.pools[0] is not first  # a fresh pool


def test_off_switch_and_fork(pool, monkeypatch):
    monkeypatch.setenv("DLSIM_CONTIGUOUS", "0")
    monkeypatch.delenv("DLSIM_AB", raising=False)
    assert pool.take(N, torch.float32, "cuda:0") is not None  # A/B switches are read only under DLSIM_AB=1
    monkeypatch.setenv("DLSIM_AB", "1")
    assert pool.take(N, torch.float32, "cuda:0") is None
    monkeypatch.delenv("DLSIM_CONTIGUOUS")
    pool.take(N, torch.float32, "cuda:0")
    parents = pool.pools
    pool.pid = os.getpid() + 1  # as seen from a forked child
    # (the fakes are instance attributes: the child's __init__ keeps them)
    pool.take(N, torch.float32, "cuda:0")
    assert pool.pid == os.getpid()
    assert pool.pools is not parents and pool.pools[0] is not parents[0]
    assert any(p is parents for p in arena._OutputPool._inherited)  # never released in the child
    arena._OutputPool._inherited.remove(parents)


def test_arena_empty_routes_by_size_and_device():
    small = arena.arena_empty(1000, torch.float32, "cpu")
    big = arena.arena_empty(N, torch.float32, "cpu")  # host arenas never use the pool
    assert small.numel() == 1000 and big.numel() == N and not big.is_cuda
    assert arena.OUT_POOL_MIN == 4 << 20 or os.environ.get("DLSIM_OUT_POOL_MIN_MB")


def test_pinned_result_budget(monkeypatch):
    """small host results are page-locked until torch's caching
    host allocator holds more than PINNED_RESULT_BUDGET; the statistics are
    read every CHECK_EVERY small results; large results stay page-locked."""
    b = arena._PinnedBudget()
    reserved = {"v": 0}
    monkeypatch.setattr(arena._PinnedBudget, "reserved", staticmethod(lambda: reserved["v"]))
    monkeypatch.setattr(arena, "PINNED_BUDGET", b)
    monkeypatch.setattr(arena, "PINNED_RESULT_BUDGET", 100)
    monkeypatch.setattr(arena, "HOST_RESULT_PINNED", True)
    assert arena.pinned_result(1000)
    reserved["v"] = 101
    for _ in range(b.CHECK_EVERY - 1):  # not re-read yet
        assert arena.pinned_result(1000)
    assert not arena.pinned_result(1000)  # re-read: over the budget
    assert arena.pinned_result(arena.PAGEABLE_RESULT_BYTES)  # large: always
    monkeypatch.setattr(arena, "HOST_RESULT_PINNED", False)
    reserved["v"] = 0
    b.calls = 0
    assert not arena.pinned_result(1000)  # DLSIM_HOST_RESULT=pageable


@pytest.mark.parametrize("missing", ["MemPool", "CUDAPluggableAllocator", *arena._OutputPool._TORCH_C_CALLS])
def test_pool_falls_back_when_torch_lacks_a_feature(monkeypatch, missing):
    """on a torch without one of the pool's features the
    pool turns itself off with ONE warning and arena_empty hands out outputs
    from torch's allocator (aligned_empty), instead of raising."""
    owner = {"MemPool": torch.cuda, "CUDAPluggableAllocator": torch.cuda.memory}.get(missing, torch._C)
    monkeypatch.delattr(owner, missing, raising=False)
    p = arena._OutputPool()
    monkeypatch.setattr(arena, "OUTPUT_POOL", p)
    made = []

    def fake_aligned(numel, dtype, device, align):
        made.append((numel, dtype, str(device), align))
        return torch.empty(numel, dtype=dtype)
    monkeypatch.setattr(arena, "aligned_empty", fake_aligned)
    monkeypatch.delenv("DLSIM_CONTIGUOUS", raising=False)
    with pytest.warns(RuntimeWarning, match="torch's allocator"):
        a = arena.arena_empty(N, torch.float32, "cuda:0")
    assert a.numel() == N and p.disabled and missing in p.disabled
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # no second warning
        b = arena.arena_empty(N, torch.float32, "cuda:0")
    assert b.numel() == N and p.made == 0 and not p.pools
    al = arena.base_align(N * 4, 4)  # aligned as arena_empty aligns any torch-allocated output
    assert made == [(N, torch.float32, "cuda:0", al)] * 2


def test_pool_falls_back_when_a_pool_call_raises(pool, monkeypatch):
    """A torch whose pool calls exist but fail (changed signature or
    behaviour): off, with the error recorded; out-of-memory still raises."""
    def broken(mp, idx, nbytes):
        raise TypeError("_cuda_beginAllocateCurrentThreadToPool(): incompatible function arguments")
    monkeypatch.setattr(pool, "_empty_in", broken)
    with pytest.warns(RuntimeWarning, match="TypeError"):
        assert pool.take(N, torch.float32, "cuda:0") is None
    assert pool.take(N, torch.float32, "cuda:0") is None and pool.made == 0
    q = arena._OutputPool()
    monkeypatch.setattr(q, "_mempool", lambda idx: q.pools.setdefault(idx, object()))

    def oom(mp, idx, nbytes):
        raise torch.OutOfMemoryError("HIP out of memory")
    monkeypatch.setattr(q, "_empty_in", oom)
    with pytest.raises(torch.OutOfMemoryError):
        q.take(N, torch.float32, "cuda:0")
    assert q.disabled is None


def test_released_pools_stay_counted_until_empty(pool, monkeypatch):
    """release() keeps the retired pools' ids (not the pools: a
    live MemPool would keep torch from freeing its idle segments) and counts
    their segments in retired_bytes() until torch's snapshot shows none."""
    class FakeMemPool:
        id = (0, 7)

        def snapshot(self):
            return segs.get(self.id, [])
    segs = {(0, 7): [{"total_size": 6 << 20}]}
    mp = FakeMemPool()
    monkeypatch.setattr(torch.cuda, "memory_snapshot", lambda pid=None: segs.get(pid, []))
    monkeypatch.setattr(pool, "_mempool", lambda idx: pool.pools.setdefault(idx, mp))
    pool.take(N, torch.float32, "cuda:0")
    assert pool.cached_bytes() == 6 << 20 and pool.retired_bytes() == 0
    assert pool.release() == 1
    assert pool.cached_bytes() == 0 and pool.retired_bytes() == 6 << 20 and pool.retired == [(0, 7)]
    segs.clear()  # the output died and the cache was emptied
    assert pool.retired_bytes() == 0 and pool.retired == []
