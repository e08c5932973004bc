"""Long-lived device buffers from the library (dlsim_device_alloc /
dlsim_device_free, DLSIM_ALLOC_CONTIGUOUS): the torch view, alignment,
freeing, and the staging rows of a large host aggregate (arena.resident_empty)."""
from __future__ import annotations

import gc

import numpy as np
import pytest
import torch
from torch import nn

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

from dasklearn_amd import _native, arena  # noqa: E402
from dasklearn_amd.gradient_aggregation.fedavg import FedAvg  # noqa: E402


def test_device_block_is_wrapped_not_copied():
    blk = _native.DeviceBlock(3 << 20, "cuda")
    t = blk.tensor()
    assert t.is_cuda and t.dtype == torch.uint8 and t.numel() == 3 << 20
    assert t.data_ptr() == blk.ptr
    t.fill_(7)
    assert int(t.sum().item()) == 7 * (3 << 20)
    del blk  # the tensor keeps the block alive
    gc.collect()
    t[5] = 1
    assert int(t[:8].sum().item()) == 7 * 7 + 1
    del t
    gc.collect()
    torch.cuda.synchronize()


def test_device_alloc_rejects_bad_arguments():
    lib = _native.load()
    import ctypes
    p, c = ctypes.c_void_p(), ctypes.c_int(0)
    assert lib.dlsim_device_alloc(0, 1, ctypes.byref(p), ctypes.byref(c)) == -1
    assert lib.dlsim_device_alloc(256, 8, ctypes.byref(p), ctypes.byref(c)) == -1
    assert lib.dlsim_device_alloc(256, 1, None, ctypes.byref(c)) == -1
    assert lib.dlsim_device_free(None) == 0


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float64])
def test_resident_empty_large_is_a_library_block(dt):
    before = dict(arena.RESIDENT_BLOCKS)
    esz = torch.tensor([], dtype=dt).element_size()
    numel = (80 << 20) // esz + 3
    x = arena.resident_empty(numel, dt, "cuda", 2 << 20)
    assert sum(arena.RESIDENT_BLOCKS.values()) == sum(before.values()) + 1
    assert x.dtype == dt and x.numel() == numel and x.data_ptr() % (2 << 20) == 0
    x.fill_(1.5)
    assert float(x[-1].item()) == 1.5
    small = arena.resident_empty(1000, dt, "cuda", 256)
    assert sum(arena.RESIDENT_BLOCKS.values()) == sum(before.values()) + 1  # torch's allocator
    del x, small
    gc.collect()
    torch.cuda.synchronize()


def test_reduce_reads_resident_rows_bit_exact():
    n, p = 8, 3_000_001
    rows = arena.resident_empty(n * arena.row_stride(p, 4), torch.float32, "cuda", 2 << 20)
    stride = arena.row_stride(p, 4)
    x = np.random.default_rng(5).standard_normal((n, p)).astype(np.float32) * np.float32(0.05)
    views = []
    for i in range(n):
        v = rows[i * stride:i * stride + p]
        v.copy_(torch.from_numpy(x[i]))
        views.append(v)
    w = orc.reference_weights(n, [float(a) for a in np.random.default_rng(6).dirichlet(np.ones(n))])
    out = arena.arena_empty(p, torch.float32, "cuda")
    _native.wreduce(views, w, out)
    assert orc.same_bits(out.cpu().numpy(), orc.wreduce_rows_f32(x, w))


class Big(nn.Module):
    def __init__(self, k):
        super().__init__()
        self.a = nn.Parameter(torch.randn(k) * 0.05)
        self.b = nn.Parameter(torch.randn(1000) * 0.05)


def test_large_host_aggregate_stages_through_a_resident_block():
    torch.manual_seed(11)
    models = [Big(9_000_000) for _ in range(3)]  # 3 rows of 36 MB: staging >= 64 MiB
    arena.STAGING.clear()
    before = sum(arena.RESIDENT_BLOCKS.values())
    out = FedAvg.aggregate(models, [0.2, 0.3, 0.5])
    assert sum(arena.RESIDENT_BLOCKS.values()) >= before + 1
    assert not out.a.is_cuda
    xs = [np.concatenate([m.a.detach().numpy(), m.b.detach().numpy()]) for m in models]
    ref = orc.wreduce(xs, orc.reference_weights(3, [0.2, 0.3, 0.5]))
    got = np.concatenate([out.a.detach().numpy(), out.b.detach().numpy()])
    assert orc.same_bits(got, ref)
    arena.STAGING.clear()
    gc.collect()
    torch.cuda.synchronize()


BIG = (20 << 20) // 4  # fp32 elements of a 20 MiB arena: pooled


def _fresh_pool():
    gc.collect()
    torch.cuda.synchronize()
    arena.OUTPUT_POOL.release()  # only this test's blocks from here on


def test_output_pool_reuses_a_block_only_when_unused():
    _fresh_pool()
    a = arena.arena_empty(BIG, torch.float32, "cuda")
    pa = a.data_ptr()
    assert pa % (2 << 20) == 0
    b = arena.arena_empty(BIG, torch.float32, "cuda")
    assert b.data_ptr() != pa  # a is alive
    view = a[100:200]
    del a
    c = arena.arena_empty(BIG, torch.float32, "cuda")
    assert c.data_ptr() != pa  # a view of a is still alive
    del view
    d = arena.arena_empty(BIG, torch.float32, "cuda")
    assert d.data_ptr() == pa  # no tensor uses a's block any more
    e = arena.arena_empty(BIG - 1000, torch.float32, "cuda")  # same 2 MiB size class
    assert e.data_ptr() not in (pa, b.data_ptr(), c.data_ptr()) and e.data_ptr() % (2 << 20) == 0
    del b, c, d, e
    assert arena.OUTPUT_POOL.release() == 1
    torch.cuda.synchronize()


def test_output_pool_is_per_stream():
    _fresh_pool()
    a = arena.arena_empty(BIG, torch.float32, "cuda")
    pa = a.data_ptr()
    del a
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        b = arena.arena_empty(BIG, torch.float32, "cuda")
    assert b.data_ptr() != pa  # a block freed on the default stream is not reused on another
    c = arena.arena_empty(BIG, torch.float32, "cuda")
    assert c.data_ptr() == pa
    del b, c
    torch.cuda.synchronize()
    arena.OUTPUT_POOL.release()


def test_output_pool_off_switch(monkeypatch):
    monkeypatch.setenv("DLSIM_AB", "1")
    monkeypatch.setenv("DLSIM_CONTIGUOUS", "0")
    made = arena.OUTPUT_POOL.made
    a = arena.arena_empty(BIG, torch.float32, "cuda")
    assert arena.OUTPUT_POOL.made == made and a.data_ptr() % (2 << 20) == 0


def test_output_pool_blocks_are_torch_allocations():
    """The pool's blocks are torch's: memory_allocated / memory_reserved count
    them, they come from the library's contiguous allocator, and release()
    gives their segments back."""
    _fresh_pool()
    a0 = torch.cuda.memory_allocated()
    r0 = torch.cuda.memory_reserved()
    segs0 = _native.pool_stats()
    x = arena.arena_empty(BIG, torch.float32, "cuda")
    assert torch.cuda.memory_allocated() == a0 + BIG * 4
    assert torch.cuda.memory_reserved() >= r0 + BIG * 4
    segs = _native.pool_stats()
    assert segs["contiguous"] + segs["fallback"] == segs0["contiguous"] + segs0["fallback"] + 1
    assert segs["live_bytes"] >= BIG * 4
    assert arena.OUTPUT_POOL.cached_bytes() >= BIG * 4
    x.fill_(1.0)
    del x
    assert torch.cuda.memory_allocated() == a0
    torch.cuda.synchronize()
    arena.OUTPUT_POOL.release()
    assert torch.cuda.memory_reserved() <= r0
    assert _native.pool_stats()["live_bytes"] == segs0["live_bytes"]


def test_release_with_a_live_output_counts_it_as_retired():
    """an output alive across release() keeps its segment; the
    pool counts it in retired_bytes() (not in cached_bytes()) until the output
    is gone and the cache emptied, and then the library's block is freed."""
    _fresh_pool()
    segs0 = _native.pool_stats()
    x = arena.arena_empty(BIG, torch.float32, "cuda")
    x.fill_(2.0)
    assert arena.OUTPUT_POOL.release() == 1
    assert arena.OUTPUT_POOL.cached_bytes() == 0 and arena.OUTPUT_POOL.retired_bytes() >= BIG * 4
    assert float(x[-1]) == 2.0  # still a valid allocation
    del x
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    assert arena.OUTPUT_POOL.retired_bytes() == 0 and arena.OUTPUT_POOL.retired == []
    assert _native.pool_stats()["live_bytes"] == segs0["live_bytes"]


def test_record_stream_keeps_a_side_stream_reader_safe():
    """an aggregate output read on a side stream (a long
    kernel queued first), record_stream'ed and dropped, then new aggregates on
    the main stream. The side stream's copy must be the first aggregate's
    exact result: the block is not recycled under its reads."""
    _fresh_pool()
    torch.manual_seed(3)
    models = [arena.to_device_arena(Wide().cuda()) for _ in range(4)]
    host = [np.concatenate([m.w.detach().cpu().numpy().ravel(), m.b.detach().cpu().numpy()]) for m in models]
    w1 = [float(v) for v in np.random.default_rng(31).dirichlet(np.ones(4))]
    w2 = [float(v) for v in np.random.default_rng(32).dirichlet(np.ones(4))]
    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    out = FedAvg.aggregate(models, w1)
    ptr = out.w.data_ptr()
    side.wait_stream(main)
    with torch.cuda.stream(side):
        torch.cuda._sleep(200_000_000)  # the side stream is busy for ~0.1 s
        copy_w = out.w.detach().clone()
        copy_b = out.b.detach().clone()
    out.w.record_stream(side)  # the torch rule for a tensor used on another stream
    del out
    later = []
    for k in range(3):
        nxt = FedAvg.aggregate(models[::-1], w2 if k % 2 == 0 else w1)
        assert nxt.w.data_ptr() != ptr  # the block waits for the side stream
        later.append(nxt)
    torch.cuda.synchronize()
    ref1 = orc.wreduce(host, orc.reference_weights(4, w1))
    got = np.concatenate([copy_w.cpu().numpy().ravel(), copy_b.cpu().numpy()])
    assert orc.same_bits(got, ref1)
    for k, nxt in enumerate(later):
        ref = orc.wreduce(host[::-1], orc.reference_weights(4, w2 if k % 2 == 0 else w1))
        got = np.concatenate([nxt.w.detach().cpu().numpy().ravel(), nxt.b.detach().cpu().numpy()])
        assert orc.same_bits(got, ref)
    del later, copy_w, copy_b
    torch.cuda.synchronize()
    arena.OUTPUT_POOL.release()


class Wide(nn.Module):
    def __init__(self):
        super().__init__()
        self.w = nn.Parameter(torch.randn(2048, 3000) * 0.05)
        self.b = nn.Parameter(torch.randn(3000) * 0.05)


def test_aggregate_outputs_from_the_pool_bit_exact_and_recycled():
    """Module outputs (parameters are views of a pooled arena): the block is
    busy while the module lives and returns when it is gone; results stay
    bit-exact while blocks are recycled under queued kernels."""
    torch.manual_seed(2)
    models = [arena.to_device_arena(Wide().cuda()) for _ in range(4)]
    host = [np.concatenate([m.w.detach().cpu().numpy().ravel(), m.b.detach().cpu().numpy()]) for m in models]
    for trial in range(6):
        w = [float(v) for v in np.random.default_rng(trial).dirichlet(np.ones(4))]
        out = FedAvg.aggregate(models, w)
        ptr = out.w.data_ptr()
        again = FedAvg.aggregate(models, w)
        assert again.w.data_ptr() != ptr  # out still holds its block
        ref = orc.wreduce(host, orc.reference_weights(4, w))
        got = np.concatenate([out.w.detach().cpu().numpy().ravel(), out.b.detach().cpu().numpy()])
        assert orc.same_bits(got, ref)
        got2 = np.concatenate([again.w.detach().cpu().numpy().ravel(), again.b.detach().cpu().numpy()])
        assert orc.same_bits(got2, ref)
        del out, again
    torch.cuda.synchronize()
    arena.OUTPUT_POOL.release()


def test_output_pool_soak_recycles_under_queued_kernels():
    """Random large aggregates whose outputs are kept or dropped at random,
    so pooled blocks are recycled while earlier kernels are still queued on
    the stream; every kept result is checked bit for bit at the end."""
    rng = np.random.default_rng(2024)
    sizes = [1_100_003, 1_500_000, 2_750_011]  # 4.4-11 MB fp32 outputs: pooled
    inputs = {p: [torch.from_numpy(rng.standard_normal(p).astype(np.float32) * np.float32(0.05)).cuda()
                  for _ in range(6)] for p in sizes}
    kept = []
    for it in range(40):
        p = sizes[int(rng.integers(len(sizes)))]
        n = int(rng.integers(2, 7))
        idx = rng.choice(6, size=n, replace=False)
        w = [float(v) for v in rng.dirichlet(np.ones(n))]
        out = arena.arena_empty(p, torch.float32, "cuda")
        _native.wreduce([inputs[p][i] for i in idx], orc.reference_weights(n, w), out)
        if rng.random() < 0.4:
            kept.append((p, idx, w, out))
        # else: dropped at once; its block returns to the pool with the kernel still queued
    torch.cuda.synchronize()
    host = {p: [x.cpu().numpy() for x in xs] for p, xs in inputs.items()}
    assert kept
    ptrs = [o.data_ptr() for *_, o in kept]
    assert len(set(ptrs)) == len(ptrs)  # no two live outputs share a block
    for p, idx, w, out in kept:
        ref = orc.wreduce([host[p][i] for i in idx], orc.reference_weights(len(idx), w))
        assert orc.same_bits(out.cpu().numpy(), ref)
    del kept
    arena.OUTPUT_POOL.release()
