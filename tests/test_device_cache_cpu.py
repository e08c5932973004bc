"""Host logic of dasklearn_amd/device_cache.py on the CPU: an entry keeps its
model's content fingerprint, and a lookup with another fingerprint drops it
(slot back on the free list, "stale" counted) instead of serving stale rows
(VERDICT r04 weak #7). The device side is tests/test_gpu_device_cache.py."""
from __future__ import annotations

import torch

from dasklearn_amd import device_cache


def _cache_with_slab(slots=2, row_bytes=4096):
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
