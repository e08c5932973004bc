"""Host logic of the device model cache (CPU): the LRU and the shm identity
of a model (csrc/pyhost.cpp shm_keys) across processes, as a reference worker
sees it (models arrive through torch.multiprocessing file_system shared
memory, worker.py:6), and the content fingerprints that catch a model written
in place after it was cached."""
from __future__ import annotations

import os
import sys

import pytest
import torch
import torch.multiprocessing as tmp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PATHS = [ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")]


def test_lru_slots_are_reused_and_protected():
    """Rows come from slab slots allocated once: an evicted entry's slot takes
    the next model; the rows the current task reads (the most recent,
    `protected`) are never evicted; past the capacity the rest go uncached."""
    from dasklearn_amd.device_cache import DeviceModelCache
    dev = torch.device("cpu")
    stride, total = 64, 50
    c = DeviceModelCache(3 * stride * 4)       # room for three rows
    t = c.take_rows(dev, torch.float32, stride, total, 3)
    assert [x[1] for x in t] == [0, 1, 2]
    base = t[0][2]                            # rows are device addresses
    assert t[1][2] == base + stride * 4 and t[2][2] == base + 2 * stride * 4  # consecutive slots: one DMA run
    for key, x in zip("abc", t):
        c.put(key, x)
    assert c.get("a") is not None  # a is now the most recent
    t2 = c.take_rows(dev, torch.float32, stride, total, 1)  # evicts b, reuses its slot
    assert c.get("b") is None and t2[0][1] == 1 and c.stats["evictions"] == 1
    c.put("d", t2[0])
    assert c.slab_bytes == 3 * stride * 4     # no new memory
    c.get("c"), c.get("a"), c.get("d")        # one task reads all three
    assert c.take_rows(dev, torch.float32, stride, total, 2, protected=3) == []  # nothing evictable
    t3 = c.take_rows(dev, torch.float32, stride, total, 2, protected=1)  # keeps d, the most recent
    assert len(t3) == 2 and c.get("d") is not None and len(c) == 1
    for x in t3:
        c.give_back(x)
    assert c.bytes == stride * 4
    c.clear()
    assert len(c) == 0 and c.bytes == 0


def test_enable_from_env(monkeypatch):
    from dasklearn_amd import device_cache
    prev = device_cache.active()
    try:
        monkeypatch.setenv("DLSIM_DEVICE_CACHE_MB", "2")
        device_cache._from_env()
        assert device_cache.active().capacity == 2 << 20
        device_cache.disable()
        monkeypatch.setenv("DLSIM_DEVICE_CACHE_MB", "0")
        device_cache._from_env()
        assert device_cache.active() is None
    finally:
        device_cache._CACHE = prev


def _child(q_in, q_out):
    for p in PATHS:
        sys.path.insert(0, p)
    tmp.set_sharing_strategy("file_system")
    from dasklearn_amd import _pyhost
    keys = []
    for _ in range(3):
        params = q_in.get()
        keys.append(_pyhost.shm_keys([params], list(range(len(params))))[0])
        del params
    q_out.put(keys)


def test_shm_identity_is_stable_across_tasks_in_a_worker():
    """The same shared model sent twice (each time a fresh mapping in the
    receiver) has one key; another model has another; private memory has
    none."""
    for p in PATHS:
        if p not in sys.path:
            sys.path.insert(0, p)
    from dasklearn_amd import _pyhost
    prev = tmp.get_sharing_strategy()
    tmp.set_sharing_strategy("file_system")
    try:
        ctx = tmp.get_context("spawn")
        q_in, q_out = ctx.Queue(), ctx.Queue()
        a = [torch.randn(50), torch.randn(7)]
        b = [torch.randn(50), torch.randn(7)]
        for t in a + b:
            t.share_memory_()
        proc = ctx.Process(target=_child, args=(q_in, q_out))
        proc.start()
        q_in.put(a)
        q_in.put(a)
        q_in.put(b)
        keys = q_out.get(timeout=120)
        proc.join(timeout=60)
        assert keys[0] is not None and keys[0] == keys[1] and keys[2] != keys[0]
        # in this process: the same storages give the same key; private memory none
        mine = _pyhost.shm_keys([a, b, [torch.randn(3)]], [0])
        assert mine[0] is not None and mine[2] is None
    finally:
        tmp.set_sharing_strategy(prev)


def test_shm_keys_cover_every_tensor():
    """A model whose second tensor is private is not cacheable."""
    for p in PATHS:
        if p not in sys.path:
            sys.path.insert(0, p)
    from dasklearn_amd import _pyhost
    prev = tmp.get_sharing_strategy()
    tmp.set_sharing_strategy("file_system")
    try:
        a = torch.randn(10)
        a.share_memory_()
        assert _pyhost.shm_keys([[a, torch.randn(3)]], [0, 1]) == [None]
        assert _pyhost.shm_keys([[a, torch.randn(3)]], [0])[0] is not None
    finally:
        tmp.set_sharing_strategy(prev)


def _child_cache(q):
    from dasklearn_amd import device_cache
    c = device_cache.active()
    if c is None:
        q.put((False, None, None, None))
    else:
        q.put((True, c.capacity, len(c), c.stats["hits"]))


def test_forked_child_gets_an_empty_cache():
    """A worker forked from a process that had a cache starts an empty one of
    the same capacity (the parent's device rows mean nothing in the child)."""
    import multiprocessing as mp
    sys.path[:0] = [p for p in PATHS if p not in sys.path]
    from dasklearn_amd import device_cache
    prev = device_cache.active()
    c = device_cache.enable(1 << 20)
    try:
        c._rows["k"] = (("x",), 0, 1234)  # a parent-side entry
        c.stats["hits"] = 5
        ctx = mp.get_context("fork")
        q = ctx.Queue()
        pr = ctx.Process(target=_child_cache, args=(q,))
        pr.start()
        got = q.get(timeout=60)
        pr.join(timeout=60)
        assert got == (True, 1 << 20, 0, 0)
        assert device_cache.active() is c and len(c) == 1  # the parent's is untouched
    finally:
        device_cache._CACHE = prev


# ---- content fingerprints ----------------------------------
# An entry keeps its model's content fingerprint; a lookup with another one
# drops it (slot back on the free list, "stale" counted) instead of serving
# stale rows. The device side: tests/test_gpu_device_cache.py.

def _cache_with_slab(slots=2, row_bytes=4096):
    from dasklearn_amd import device_cache
    c = device_cache.DeviceModelCache(slots * row_bytes)
    sk = (0, torch.float32, row_bytes // 4)
    slab = device_cache._Slab(None, torch.float32, row_bytes // 4, row_bytes, slots * row_bytes)
    slab.bases = [1 << 20]
    slab.free = list(range(slots))
    c._slabs[sk] = slab
    return c, sk, slab


def test_fingerprint_mismatch_drops_the_entry():
    c, sk, slab = _cache_with_slab()
    t = (sk, slab.free.pop(0), slab.row_ptr(0))
    c.bytes += slab.row_bytes
    c.put(("shm_a", 1), t, 1234)
    assert c.get(("shm_a", 1), 1234) == slab.row_ptr(0)
    assert c.get(("shm_a", 1), 99) is None  # written since: dropped
    assert c.stats["stale"] == 1 and len(c) == 0 and c.bytes == 0 and slab.free == [0, 1]
    assert c.get(("shm_a", 1), 99) is None and c.stats["stale"] == 1  # gone, not stale twice


def test_duplicate_put_keeps_the_first_fingerprint():
    c, sk, slab = _cache_with_slab()
    t0 = (sk, slab.free.pop(0), slab.row_ptr(0))
    t1 = (sk, slab.free.pop(0), slab.row_ptr(1))
    c.bytes += 2 * slab.row_bytes
    c.put("k", t0, 7)
    c.put("k", t1, 7)  # the same model twice in one task
    assert len(c) == 1 and slab.free == [1] and c.get("k", 7) == slab.row_ptr(0)


def test_eviction_with_fingerprints():
    c, sk, slab = _cache_with_slab(slots=1)
    t = (sk, slab.free.pop(0), slab.row_ptr(0))
    c.bytes += slab.row_bytes
    c.put("k", t, 1)
    c._evict_one()
    assert len(c) == 0 and slab.free == [0] and c.stats["evictions"] == 1


# ---- what the fingerprint samples ---------------
# _pyhost.shm_rows fingerprints EVERY tensor of a model: its first and last
# 8-byte word, plus one more per MiB (up to 16 words per tensor).

def _deep_shm_model(seed, layers=12, width=16):
    import torch.multiprocessing as tmp
    from torch import nn
    prev = tmp.get_sharing_strategy()
    tmp.set_sharing_strategy("file_system")
    try:
        g = torch.Generator().manual_seed(seed)
        m = nn.Sequential(*[nn.Linear(width, width) for _ in range(layers)], nn.Linear(width, 600_000))
        with torch.no_grad():
            for q in m.parameters():
                q.copy_(torch.randn(q.shape, generator=g))
        m.share_memory()
        return m
    finally:
        tmp.set_sharing_strategy(prev)


def _fp(m):
    from dasklearn_amd import _pyhost
    ps = [list(m.parameters())]
    keys, _, fps = _pyhost.shm_rows(ps, list(range(len(ps[0]))))
    assert keys[0] is not None  # file_system shm: cacheable
    return fps[0]


@pytest.mark.parametrize("where", ["middle_tensor_first", "middle_tensor_last", "big_tensor_last",
                                   "big_tensor_interior", "last_bias", "first_weight_whole"])
def test_fingerprint_sees_a_write_to_any_tensor(where):
    """A write confined to ONE tensor of a 26-tensor model -- one a sample of
    8 tensors would skip -- changes the fingerprint; round 5's sampled 8
    words from the middle of 8 tensors and missed such writes."""
    m = _deep_shm_model(3)
    ps = list(m.parameters())
    assert len(ps) == 26
    before = _fp(m)
    assert _fp(m) == before  # unchanged content, same fingerprint
    with torch.no_grad():
        if where == "middle_tensor_first":
            ps[13].view(-1)[0] += 1.0  # a bias in the middle of the model (not among round 5's 8)
        elif where == "middle_tensor_last":
            ps[11].view(-1)[-1] += 1.0
        elif where == "big_tensor_last":
            ps[24].view(-1)[-1] += 1.0  # 600,000 x 16 fp32 (38 MB): its last word
        elif where == "big_tensor_interior":
            w = ps[24].view(-1)  # 38 MB: 16 words spread over it; one of them lies at 1/15 of its length
            k = (w.numel() * 4 - 8) // 15 // 8 * 2  # element at the second sampled word
            w[k] += 1.0
        elif where == "last_bias":
            ps[25].view(-1)[0] += 1.0  # the last tensor of the model
        else:
            ps[0].add_(0.01)
    assert _fp(m) != before


def test_fingerprint_blind_spot_is_documented():
    """What the guard cannot see: a write to an element
    between two sampled words of one tensor (here the middle of a 256-float
    weight, which is sampled at its first and last word)."""
    m = _deep_shm_model(4)
    ps = list(m.parameters())
    before = _fp(m)
    with torch.no_grad():
        ps[2].view(-1)[128] += 1.0
    assert _fp(m) == before
