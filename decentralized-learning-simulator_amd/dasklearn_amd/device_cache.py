"""Per-worker device cache of host models received through shared memory
(VERDICT r03 next #7). Opt-in.

In the reference every task runs in a worker process that takes it from the
broker's one shared queue (broker.py:259-272, worker.py:21-38), and models
cross processes as torch.multiprocessing file_system shared memory
(worker.py:6): each parameter storage is a named shm file that a worker maps
afresh for every task. In D-PSGD each trained model feeds k + 1 aggregate
tasks, and a replay of the broker's dispatch (scripts/cache_reuse.py,
profiles/r04_cache_reuse.jsonl) finds the same worker receiving a model it
has already uploaded for 43-73 % of aggregate inputs at 100 peers and 4
workers. This cache keeps the device copy of every such model a worker
uploads, keyed by the identity of its shm storages (the file names, storage
offsets, sizes and dtypes of all its parameters of one dtype group: one name
is one allocation for the whole run), so a later aggregate in the same
worker reads it in place and packs and sends only the models it has not seen
(dlsim_host_wreduce_resident).

Contract (why it is opt-in): a cached model's shared storages must not be
written while the cache holds them. The reference's aggregate inputs are the
train task's freshly serialised outputs (functions.py:70-77), which nothing
writes afterwards; a caller that mutates shared models in place must not
enable the cache. Only file_system shm storages are cached; other host
models take the normal pipeline.

Enable with DLSIM_DEVICE_CACHE_MB=<capacity> in the worker's environment, or
`device_cache.enable(capacity_bytes)`. Least recently used entries are
evicted past the capacity.
"""
from __future__ import annotations

import os
import threading
from collections import OrderedDict
from typing import Dict, Optional

import torch


class DeviceModelCache:
    """LRU of device rows keyed by (shm identity, device, dtype, elements)."""

    def __init__(self, capacity_bytes: int):
        self.capacity = int(capacity_bytes)
        self._rows: "OrderedDict[tuple, tuple]" = OrderedDict()  # key -> (row, bytes it is charged)
        self.bytes = 0
        self.lock = threading.Lock()
        self.stats: Dict[str, int] = {"hits": 0, "misses": 0, "uncacheable": 0, "evictions": 0,
                                      "bytes_not_sent": 0}

    def get(self, key) -> Optional[torch.Tensor]:
        e = self._rows.get(key)
        if e is None:
            return None
        self._rows.move_to_end(key)
        return e[0]

    def put(self, key, row: torch.Tensor, nbytes: int) -> None:
        if key in self._rows or nbytes > self.capacity:
            return
        self._rows[key] = (row, nbytes)
        self.bytes += nbytes
        while self.bytes > self.capacity and self._rows:
            _, (_, old_bytes) = self._rows.popitem(last=False)
            self.bytes -= old_bytes
            self.stats["evictions"] += 1

    def __len__(self) -> int:
        return len(self._rows)

    def clear(self) -> None:
        with self.lock:
            self._rows.clear()
            self.bytes = 0


_CACHE: Optional[DeviceModelCache] = None


def enable(capacity_bytes: int) -> DeviceModelCache:
    """Turn the cache on for this process (replacing any previous one)."""
    global _CACHE
    _CACHE = DeviceModelCache(capacity_bytes)
    return _CACHE


def disable() -> None:
    global _CACHE
    _CACHE = None


def active() -> Optional[DeviceModelCache]:
    return _CACHE


def _from_env() -> None:
    mb = os.environ.get("DLSIM_DEVICE_CACHE_MB")
    if mb and mb.strip() not in ("", "0"):
        enable(int(float(mb) * (1 << 20)))


_from_env()
