"""Parameter arenas: nn.Module parameters <-> flat device buffers.

The reference folds parameters tensor by tensor, model by model
(dasklearn/gradient_aggregation/fedavg.py:23-25: N x T Python iterations).
Here a model's parameters() are one flat arena (concatenated in parameters()
order, one arena per dtype), so one kernel launch reduces every tensor of
every model. Three ways in:

* device arena   — every parameter of a CUDA model is a view into one flat
                   buffer in parameters() order (what `aggregate_modules`
                   returns for device inputs): zero copies, one launch;
* device tensors — CUDA parameters in separate storages: the tensor-list ABI
                   entry (`dlsim_wreduce_tensors`) reads them in place;
* host models    — CPU parameters (the reference's case: models reach the
                   worker through torch-mp shared memory, model_trainer.py:129):
                   packed into pinned staging, copied H2D per model on the
                   current stream, reduced, copied back.

The result is a fresh module with `copy.deepcopy(models[0])` semantics
(fedavg.py:20): buffers and attributes copied from models[0]; parameters
replaced — through the deepcopy memo, so they are never copied — by views of
the reduced arena, keeping each original's requires_grad.
"""
from __future__ import annotations

import copy
import os
import threading
import time
import weakref
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch import nn

from . import _native, device_cache
from . import _pyhost  # csrc/pyhost.cpp (built with the library by __graft_entry__.build())


def check_pyhost_build(built: str, running: str) -> None:
    """_pyhost reads at::Tensor fields and restates copy.deepcopy against the
    internals of the torch it was compiled with: under any other torch it
    could mis-clone silently, so it must fail loudly instead (VERDICT r02
    next #8)."""
    if built != running:
        raise ImportError(f"dasklearn_amd/_pyhost was built for torch {built}, this process runs torch {running}: "
                          "rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")


check_pyhost_build(getattr(_pyhost, "BUILT_FOR_TORCH", "unknown"), torch.__version__)


def module_params(module: nn.Module) -> List[nn.Parameter]:
    """list(module.parameters()): the modules in named_modules() pre-order
    (each once), then each module's _parameters in order, skipping None and
    parameters already seen (by identity) — walked in C (csrc/pyhost.cpp),
    the per-task path visits every parameter of every model."""
    return _pyhost.module_params(module)


def module_params_py(module: nn.Module) -> List[nn.Parameter]:
    """The same list in Python (tests compare the two)."""
    out: List[nn.Parameter] = []
    seen = set()  # ids of modules and parameters visited

    def visit(m):
        for p in m._parameters.values():
            if p is not None and id(p) not in seen:
                seen.add(id(p))
                out.append(p)
        for c in m._modules.values():
            if c is not None and id(c) not in seen:
                seen.add(id(c))
                visit(c)

    seen.add(id(module))
    visit(module)
    return out


class ZipMismatch(ValueError):
    """A model's parameter list differs from models[0]'s (count, shape or
    dtype): it cannot share models[0]'s arena layout."""


def _contiguous_strides(shape) -> Tuple[int, ...]:
    strides, acc = [], 1
    for d in reversed(tuple(shape)):
        strides.append(acc)
        acc *= max(int(d), 1)
    return tuple(reversed(strides))


class ParamLayout:
    """parameters() of a module grouped by dtype, with flat offsets."""

    def __init__(self, module: nn.Module, params: Optional[List[nn.Parameter]] = None):
        self.params: List[nn.Parameter] = module_params(module) if params is None else params
        self.shapes = [tuple(p.shape) for p in self.params]
        self.groups: "OrderedDict[torch.dtype, List[int]]" = OrderedDict()
        for k, p in enumerate(self.params):
            self.groups.setdefault(p.dtype, []).append(k)
        self.offsets: Dict[int, int] = {}
        self.totals: Dict[torch.dtype, int] = {}
        self._group_offsets: Dict[torch.dtype, List[int]] = {}
        for dt, idx in self.groups.items():
            _native.dtype_code(dt, single_task=True)  # raises TypeError for unsupported dtypes
            off = 0
            offs = []
            for k in idx:
                self.offsets[k] = off
                offs.append(off)
                off += self.params[k].numel()
            self.totals[dt] = off
            self._group_offsets[dt] = offs
        self._signature = tuple((p.shape, p.dtype) for p in self.params)
        # per dtype group: each tensor's byte offset in the arena
        self.byte_offsets = {dt: tuple(o * self.params[idx[0]].element_size() for o in self._group_offsets[dt])
                             for dt, idx in self.groups.items()}
        # per dtype group: element counts and shapes for splitting an arena
        self.split_sizes = {dt: [self.params[k].numel() for k in idx] for dt, idx in self.groups.items()}
        self.split_shapes = {dt: [None if self.params[k].dim() == 1 else self.params[k].shape for k in idx]
                             for dt, idx in self.groups.items()}
        # per dtype group: (shape, contiguous strides, element offset) of each
        # tensor's view into an arena (one as_strided per parameter)
        self.view_specs = {dt: [(tuple(self.params[k].shape), _contiguous_strides(self.params[k].shape), o)
                                for k, o in zip(idx, self._group_offsets[dt])]
                           for dt, idx in self.groups.items()}
        # per parameter, in parameters() order: (dtype, byte offset in its
        # dtype's arena, shape) -- what a registered arena's views must match
        self.param_slots = [None] * len(self.params)
        for dt, idx in self.groups.items():
            for k, bo in zip(idx, self.byte_offsets[dt]):
                self.param_slots[k] = (dt, bo, self.params[k].shape)

    def rebind(self, params: List[nn.Parameter]) -> "ParamLayout":
        """The same layout over another module's parameters (same signature,
        which the caller guarantees): no recomputation. A shallow copy of the
        attribute dict (what copy.copy does, without its reduce protocol:
        this runs several times per task)."""
        other = ParamLayout.__new__(ParamLayout)
        d = self.__dict__.copy()
        d["params"] = params
        other.__dict__ = d
        return other

    def matches(self, ps: Sequence[torch.Tensor]) -> bool:
        """ps has this layout's signature (count, shapes, dtypes); in C."""
        return _pyhost.matches(ps, self._signature)

    def check_compatible(self, module: nn.Module) -> List[nn.Parameter]:
        ps = _pyhost.checked_params(module, self._signature)  # walk + signature check in C
        if ps is not None:
            return ps
        ps = module_params(module)
        # Not the arena's signature: the reference zips parameters()
        # (fedavg.py:23-24), which aggregate_modules restates per parameter
        # (_aggregate_zip); the one-launch paths refuse such a model.
        if not self.matches(ps):
            if len(ps) != len(self.params):
                raise ZipMismatch("models have different numbers of parameters")
            for k, (a, (shape, dt)) in enumerate(zip(ps, self._signature)):
                if a.dtype is not dt or a.shape != shape:
                    raise ZipMismatch(f"parameter {k}: shape/dtype differs from models[0]")
        return ps

    def arena_view(self, params: Sequence[torch.Tensor], dt: torch.dtype) -> Optional[torch.Tensor]:
        """If the dtype group of `params` already is one contiguous flat buffer
        (in layout order), return a flat view of it, else None."""
        idx = self.groups[dt]
        total = self.totals[dt]
        # every tensor contiguous (a transposed view could start at the right
        # place) and at its offset in the layout, and the whole run inside the
        # first tensor's storage: adjacent separate allocations are not an
        # arena (read from the tensors in C++, csrc/pyhost.cpp)
        if not _pyhost.flat_run(params, idx, self.byte_offsets[dt], total):
            return None
        first = params[idx[0]]
        return torch.as_strided(first.detach(), (total,), (1,), first.storage_offset())


# One ParamLayout per model class, reused for every model of that class whose
# parameter signature matches (a new layout replaces it otherwise): the
# per-task path then builds no layout for the models of a simulation.
_CLASS_LAYOUTS: Dict[type, ParamLayout] = {}


def layout_of(module: nn.Module, params: Optional[List[nn.Parameter]] = None) -> ParamLayout:
    """ParamLayout over `module`'s parameters, from the per-class cache."""
    ps = module_params(module) if params is None else params
    known = _CLASS_LAYOUTS.get(type(module))
    if known is not None and known.matches(ps):
        return known.rebind(ps)
    layout = ParamLayout(module, ps)
    _CLASS_LAYOUTS[type(module)] = layout
    return layout


_ELEM_SIZE: Dict[torch.dtype, int] = {}


def _elem_size(dt: torch.dtype) -> int:
    esz = _ELEM_SIZE.get(dt)
    if esz is None:
        esz = _ELEM_SIZE[dt] = torch.empty((), dtype=dt).element_size()
    return esz


# Arena rows of 4- and 8-byte elements of at least ROW_ALIGN_MIN bytes start
# ROW_ALIGN-aligned (round 3; profiles/r03_layout*/, r03_rowrule/).
ROW_ALIGN = 2 << 20
ROW_ALIGN_MIN = 16 << 20


def row_stride(numel: int, elem_bytes: int) -> int:
    """Elements between consecutive model rows of an arena of rows (staging,
    a round's uploads, bench inputs).

    * 4/8-byte rows of >= 16 MiB: a whole number k of 2 MiB units, with
      k + 1 when k is a multiple of 4 (rows 8 MiB apart share HBM channels);
      the buffer's base is 2 MiB-aligned (aligned_empty). Measured for the
      fixed and grouped launch shapes with >= 1 GiB rotating: the north
      star's 8 x 11.2 M fp32 63.2 -> 61.7 us, 1.5-2.5 % at 6-25 M x 8, n = 4,
      17 and 100 at 11.2 M; n = 2 fp32 and bf16 rows: neutral (+-0.6 %), so
      2-byte rows keep the rule below (profiles/r03_rowrule/).
    * otherwise `numel` rounded up to 256 B (every row 16-byte aligned for the
      vector kernel), plus 4 KiB when that leaves a stride that is a multiple
      of 64 KiB: 8 x 8 M fp32 rows ran at 0.75 of peak at a 32 MiB stride and
      0.80 with 4 KiB added (profiles/r01_tune_pow2.log). Below 16 MiB 2 MiB
      alignment measured neutral to 2.4 % slower (2.8 M x 8 fp32,
      profiles/r03_layout_sweep/)."""
    nbytes = numel * elem_bytes
    if elem_bytes >= 4 and nbytes >= ROW_ALIGN_MIN:
        k = (nbytes + ROW_ALIGN - 1) // ROW_ALIGN
        if k % 4 == 0:
            k += 1
        return k * ROW_ALIGN // elem_bytes
    per256 = 256 // elem_bytes
    padded = (numel + per256 - 1) // per256 * per256
    if (padded * elem_bytes) % 65536 == 0:
        padded += 4096 // elem_bytes
    return padded


def base_align(nbytes: int, elem_bytes: int) -> int:
    """Alignment (bytes) of a device buffer that holds rows of `nbytes` each
    (row_stride) or one arena of `nbytes`: ROW_ALIGN under row_stride's
    2 MiB rule, else 256."""
    return ROW_ALIGN if elem_bytes >= 4 and nbytes >= ROW_ALIGN_MIN else 256


def aligned_empty(numel: int, dtype: torch.dtype, device, align: int) -> torch.Tensor:
    """torch.empty(numel) on `device` starting at an `align`-byte boundary
    (over-allocates align bytes; the view keeps the storage alive)."""
    if align <= 256:
        return torch.empty(numel, dtype=dtype, device=device)
    esz = _elem_size(dtype)
    raw = torch.empty(numel + align // esz, dtype=dtype, device=device)
    skip = (-raw.data_ptr()) % align // esz
    return raw[skip:skip + numel]


def arena_empty(numel: int, dtype: torch.dtype, device) -> torch.Tensor:
    """A fresh aggregate output (one dtype arena of a model), aligned like a
    row of its size (base_align). From OUT_POOL_MIN (4 MiB) on it comes from
    OUTPUT_POOL (physically contiguous blocks); below, torch's
    allocator."""
    esz = _elem_size(dtype)
    al = base_align(numel * esz, esz)
    if numel * esz >= OUT_POOL_MIN and torch.device(device).type == "cuda":
        t = OUTPUT_POOL.take(numel, dtype, device)
        if t is not None:
            return t
    return aligned_empty(numel, dtype, device, al)


# 4 MiB: the 8-rank slice of the north star (5.6 MB outputs) ran 9.55-9.60 us
# with pooled outputs against 9.71-9.97 us in torch's allocator; cfg2's 4 MB
# outputs measured neutral (profiles/r04s2_small/)
OUT_POOL_MIN = int(float(_native.ab_env("DLSIM_OUT_POOL_MIN_MB", "4")) * (1 << 20))  # bytes


class _OutputPool:
    """Physically contiguous device memory for large aggregate outputs, owned
    by torch's caching allocator.

    The output arena's placement sets the rate of the whole reduce: with the
    north star's rows fixed, outputs on the pages torch's allocator happened
    to get ran at 61.2-62.5 us per launch, outputs in a contiguous block at
    60.9-61.3 us in every process (profiles/r04s2_contig2/).
    Round 4 cached such blocks in lists of its own, outside torch: a returned
    output handed to a side stream with Tensor.record_stream could be
    recycled under that stream's reads, and torch's memory statistics,
    empty_cache and out-of-memory path did not see the blocks (VERDICT r04
    weak #2). Now the blocks come from the library's pluggable
    allocator (dlsim_pool_alloc / dlsim_pool_free: hipExtMallocWithFlags with
    hipDeviceMallocContiguous, 2 MiB-aligned) through one torch.cuda.MemPool
    per device, and outputs are plain torch.empty tensors allocated inside
    it: torch's caching allocator splits, caches and reuses the blocks per
    stream, record_stream defers a block's reuse until the recorded streams
    are done, memory_allocated / memory_reserved count them, and
    `use_on_oom` lets torch's other allocations take idle pool blocks before
    raising OutOfMemoryError. Sizes are rounded up to 2 MiB, so every block
    the pool hands out starts 2 MiB-aligned (base_align's rule).
    `release()` retires the pools: torch.cuda.empty_cache() then returns
    their idle segments to the driver (and those still in use once their
    tensors are gone and the cache is emptied again); later outputs start a
    fresh pool. A forked child starts without pools (the parent's are left
    alone: the child must not touch the parent's device state). The ids of
    retired pools are kept (`retired`, not the pools: a live MemPool keeps
    torch from freeing its idle segments) until torch's snapshot of them
    shows no segment left, so outputs still alive from them stay counted
    (retired_bytes()).
    The pool rests on torch.cuda.MemPool, CUDAPluggableAllocator and three
    private torch._C calls (_cuda_beginAllocateCurrentThreadToPool,
    _cuda_endAllocateToPool, _cuda_releasePool): they are feature-detected on
    first use, and if any is missing or the pool cannot be made, the pool turns
    itself off with one warning and outputs come from torch's allocator
    (aligned_empty: the same alignment, torch's placement) -- a different
    torch changes where outputs live, never whether an aggregate runs.
    DLSIM_AB=1 DLSIM_CONTIGUOUS=0 turns the pool off (A/B)."""

    # torch internals the pool needs (feature-detected by usable())
    _TORCH_C_CALLS = ("_cuda_beginAllocateCurrentThreadToPool", "_cuda_endAllocateToPool", "_cuda_releasePool")

    _inherited: List[dict] = []  # a forked child's copy of the parent's pools, never released

    def __init__(self):
        self.pid = os.getpid()
        self.pools: Dict[int, object] = {}  # device index -> torch.cuda.MemPool
        self.lock = threading.Lock()
        self.made = 0  # outputs handed out of the pool
        self._allocator = None
        self.retired: List[tuple] = []  # ids of released pools whose segments may still be held
        self.disabled: Optional[str] = None  # why the pool turned itself off (None: usable)

    @classmethod
    def missing_features(cls) -> List[str]:
        """The torch features the pool needs that this torch lacks."""
        miss = []
        if not hasattr(torch.cuda, "MemPool"):
            miss.append("torch.cuda.MemPool")
        if not hasattr(getattr(torch.cuda, "memory", None), "CUDAPluggableAllocator"):
            miss.append("torch.cuda.memory.CUDAPluggableAllocator")
        miss += [f"torch._C.{c}" for c in cls._TORCH_C_CALLS if not hasattr(torch._C, c)]
        return miss

    def _disable(self, why: str) -> None:
        """Turn the pool off for this process (one warning)."""
        if self.disabled is None:
            self.disabled = why
            import warnings
            warnings.warn(f"dasklearn_amd: aggregate outputs come from torch's allocator ({why})",
                          RuntimeWarning, stacklevel=3)

    def _mempool(self, idx: int):
        mp = self.pools.get(idx)
        if mp is None:
            if self._allocator is None:
                _native.load()  # the library must be built (no fallback)
                self._allocator = torch.cuda.memory.CUDAPluggableAllocator(
                    _native.LIB_PATH, "dlsim_pool_alloc", "dlsim_pool_free")
            with torch.cuda.device(idx):
                mp = torch.cuda.MemPool(self._allocator.allocator(), use_on_oom=True)
            self.pools[idx] = mp
        return mp

    @staticmethod
    def _empty_in(mp, idx: int, nbytes: int) -> torch.Tensor:
        """torch.empty(nbytes) on device idx, allocated inside MemPool `mp`
        (torch.cuda.use_mem_pool without the generator: this runs per call)."""
        torch._C._cuda_beginAllocateCurrentThreadToPool(idx, mp.id)
        try:
            return torch.empty(nbytes, dtype=torch.uint8, device=torch.device("cuda", idx))
        finally:
            torch._C._cuda_endAllocateToPool(idx, mp.id)
            torch._C._cuda_releasePool(idx, mp.id)

    def take(self, numel: int, dtype: torch.dtype, device) -> Optional[torch.Tensor]:
        """An output of `numel` elements from the pool, or None (the caller
        then allocates from torch): the pool is off, or turned itself off."""
        if self.disabled is not None or _native.ab_env("DLSIM_CONTIGUOUS", "1") == "0":
            return None
        if self._allocator is None and not self.pools:
            miss = self.missing_features()
            if miss:
                self._disable("this torch lacks " + ", ".join(miss))
                return None
        try:
            return self._take(numel, dtype, device)
        except torch.OutOfMemoryError:
            raise
        except (AttributeError, TypeError, RuntimeError) as e:
            # a torch whose pool calls changed behaviour: off, not broken
            self._disable(f"{type(e).__name__}: {e}"[:200])
            return None

    def _take(self, numel: int, dtype: torch.dtype, device) -> torch.Tensor:
        dev = torch.device(device)
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        nbytes = numel * _elem_size(dtype)
        size = (nbytes + ROW_ALIGN - 1) // ROW_ALIGN * ROW_ALIGN
        # one thread at a time: torch refuses a second concurrent
        # allocation-to-pool context on the same pool
        with self.lock:
            if self.pid != os.getpid():
                _OutputPool._inherited.append(self.pools)
                self.__init__()
            mp = self._mempool(idx)
            raw = self._empty_in(mp, idx, size)
            if raw.data_ptr() % ROW_ALIGN:
                # the rest of a block that an allocation outside the pool
                # split (use_on_oom): take 2 MiB more and align inside it
                raw = self._empty_in(mp, idx, size + ROW_ALIGN)
                skip = (-raw.data_ptr()) % ROW_ALIGN
                raw = raw[skip:skip + size]
            self.made += 1
        return raw[:nbytes].view(dtype)

    def cached_bytes(self) -> int:
        """Bytes of the live pools' segments (in use or cached)."""
        with self.lock:
            pools = list(self.pools.values())
        return sum(seg["total_size"] for mp in pools for seg in mp.snapshot())

    def retired_bytes(self) -> int:
        """Bytes of released pools' segments that are still held (outputs
        alive since before release(), or cached until the next
        torch.cuda.empty_cache()). Pools with no segment left are dropped."""
        with self.lock:
            keep, total = [], 0
            for pid in self.retired:
                b = sum(seg["total_size"] for seg in torch.cuda.memory_snapshot(pid))
                if b:
                    keep.append(pid)
                    total += b
            self.retired = keep
        return total

    def release(self) -> int:
        """Retire every pool and empty torch's cache (a device-wide
        synchronisation, like torch.cuda.empty_cache itself); returns the
        number of pools retired. Their segments still in use stay counted
        by retired_bytes() until they are gone."""
        with self.lock:
            n = len(self.pools)
            self.retired.extend(mp.id for mp in self.pools.values())
            self.pools = {}
        if n and torch.cuda.is_initialized():
            torch.cuda.empty_cache()
        if self.retired:
            self.retired_bytes()  # drop the pools the empty_cache emptied
        return n


OUTPUT_POOL = _OutputPool()


RESIDENT_CONTIG_MIN = 64 << 20  # bytes
RESIDENT_BLOCKS = {"contiguous": 0, "fallback": 0}  # library blocks made, by kind


def resident_empty(numel: int, dtype: torch.dtype, device, align: int) -> torch.Tensor:
    """A LONG-LIVED device buffer (the grow-only staging rows, the device
    cache's model blocks) starting at an `align`-byte boundary. From
    RESIDENT_CONTIG_MIN bytes on it is physically contiguous memory from the
    library (dlsim_device_alloc, DLSIM_ALLOC_CONTIGUOUS; hipMalloc if the
    driver has none): rows in torch's allocator land on whatever physical
    pages the driver hands out, and the north star's 8 rows ran 1-2 % apart
    between two such allocations of one process, where contiguous blocks ran
    at the fast end every time (profiles/r04s2_contig/).
    Freeing such a block synchronises the device, so per-call buffers
    (aggregate outputs, a wave's uploads) stay in torch's caching allocator.
    DLSIM_AB=1 DLSIM_CONTIGUOUS=0 turns it off (A/B)."""
    esz = _elem_size(dtype)
    nbytes = numel * esz
    if nbytes < RESIDENT_CONTIG_MIN or _native.ab_env("DLSIM_CONTIGUOUS", "1") == "0" \
            or torch.device(device).type != "cuda":
        return aligned_empty(numel, dtype, device, align)
    align = max(align, 256)
    blk = _native.DeviceBlock(nbytes + align, device)
    RESIDENT_BLOCKS["contiguous" if blk.contiguous else "fallback"] += 1
    raw = blk.tensor()
    skip = (-raw.data_ptr()) % align
    return raw[skip:skip + nbytes].view(dtype)


class _Staging:
    """Reusable staging rows: ONE grow-only device buffer per (device, dtype)
    and one grow-only pinned buffer per (device, dtype), carved into rows for
    each call (`rows[i, :numel]`, rows 16-byte aligned at row_stride). Memory
    is bounded by the largest request seen, not by the number of distinct
    (fan-in, size) shapes: gossip and D-PSGD vary the fan-in per peer.

    acquire() takes the key's lock and waits for the previous user's event
    (its H2D copies and kernel may still be queued when it returns);
    release() records the new event and drops the lock. Callers pair them
    with try/finally, so a failing call cannot leave the rows reusable while
    copies into them are still in flight, and two threads cannot pack into
    the same rows at once."""

    def __init__(self):
        self.dev: Dict[Tuple, torch.Tensor] = {}
        self.host: Dict[Tuple, torch.Tensor] = {}
        self.last_use: Dict[Tuple, torch.cuda.Event] = {}  # pending: the last user's work
        self._events: Dict[Tuple, torch.cuda.Event] = {}    # one reusable event per key
        self._views: Dict[Tuple, Tuple] = {}                # last (n, numel, bufs, rows, host) per key
        self._locks: Dict[Tuple, threading.Lock] = {}
        self._locks_guard = threading.Lock()

    @staticmethod
    def _key(device, dt):
        if isinstance(device, torch.device):
            return (device.type, device.index, dt)
        d = torch.device(device)
        return (d.type, d.index, dt)

    def _lock(self, key) -> threading.Lock:
        with self._locks_guard:
            lk = self._locks.get(key)
            if lk is None:
                lk = self._locks[key] = threading.Lock()
            return lk

    @staticmethod
    def _grow(pool: Dict[Tuple, torch.Tensor], key, need: int, make, align: int = 0) -> torch.Tensor:
        buf = pool.get(key)
        if buf is None or buf.numel() < need or (align and buf.data_ptr() % align):
            pool.pop(key, None)  # drop the old one first (device memory returns to torch's cache)
            buf = pool[key] = make(need)
        return buf

    def acquire(self, device, dt, n, numel, stream, pinned: bool = True, device_rows: bool = True):
        """(device rows or None, pinned rows or None) as [n, numel] views.
        device_rows=False: pinned rows only, under their own key (the device
        cache's misses go H2D straight into cache rows)."""
        key = self._key(device, dt) if device_rows else self._key(device, dt) + ("host",)
        self._lock(key).acquire()
        try:
            ev = self.last_use.pop(key, None)
            if ev is not None:
                ev.synchronize()
            esz = _elem_size(dt)
            stride = row_stride(numel, esz)
            need = max(1, n * stride)
            al = base_align(numel * esz, esz)
            # aligned as this call needs (a later call that needs 2 MiB rows regrows the buffer)
            flat = self._grow(self.dev, key, need, lambda k: resident_empty(k, dt, device, al), align=al) \
                if device_rows else None
            hflat = self._grow(self.host, key, need, lambda k: torch.empty(k, dtype=dt, pin_memory=True)) \
                if pinned else None
            last = self._views.get(key)
            if last is not None and last[0] == n and last[1] == numel and last[2] is flat and last[3] is hflat:
                return last[4], last[5]  # the same rows as the previous call
            rows = flat[:n * stride].view(n, stride)[:, :numel] if device_rows else None
            host = hflat[:n * stride].view(n, stride)[:, :numel] if pinned else None
            self._views[key] = (n, numel, flat, hflat, rows, host)
            return rows, host
        except BaseException:
            self._lock(key).release()
            raise

    def release(self, device, dt, stream, synced: bool = False, device_rows: bool = True):
        """synced: the caller has synchronised `stream` after its last use of
        the rows, so the next user need not wait (no event). device_rows as
        given to acquire()."""
        key = self._key(device, dt) if device_rows else self._key(device, dt) + ("host",)
        if not synced:
            ev = self._events.get(key)
            if ev is None:
                ev = self._events[key] = torch.cuda.Event()
            ev.record(stream)  # re-recording moves the event to this call's work
            self.last_use[key] = ev
        self._lock(key).release()

    def clear(self):
        for ev in self.last_use.values():
            ev.synchronize()
        self.last_use.clear()
        self._views.clear()
        self.dev.clear()
        self.host.clear()


STAGING = _Staging()


def _target_device(params0: Sequence[torch.Tensor], device) -> torch.device:
    if device is not None:
        dev = torch.device(device)
        if dev.type == "cuda" and dev.index is None:
            # 'cuda' means the current device: without the index every
            # `t.device == dev` check would fail and each task would take the
            # copy paths
            if not torch.cuda.is_available():
                raise RuntimeError("dasklearn_amd aggregation runs on an AMD GPU; none is visible "
                                   "(there is no CPU fallback)")
            dev = torch.device("cuda", torch.cuda.current_device())
        return dev
    for p in params0:
        if p.is_cuda:
            return p.device
    if not torch.cuda.is_available():
        raise RuntimeError("dasklearn_amd aggregation runs on an AMD GPU; none is visible "
                           "(there is no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


class _Stages:
    """Optional wall-clock stage breakdown (scripts/bench_host.py). When on,
    the stream is synchronised at every stage boundary, so only use it to
    measure."""

    def __init__(self, sink: Optional[dict], stream):
        self.sink, self.stream = sink, stream
        self.t = time.perf_counter() if sink is not None else 0.0

    def mark(self, name: str):
        if self.sink is None:
            return
        self.stream.synchronize()
        now = time.perf_counter()
        self.sink[name] = self.sink.get(name, 0.0) + (now - self.t)
        self.t = now


_SIDE_STREAMS: Dict[torch.device, Tuple[torch.cuda.Stream, torch.cuda.Stream]] = {}


def _side_streams(dev: torch.device):
    """(H2D stream, D2H stream) of a device: copies in both directions run
    beside the reduce kernels on the caller's stream (PCIe is full duplex and
    each direction has its own DMA engine)."""
    ss = _SIDE_STREAMS.get(dev)
    if ss is None:
        ss = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
        _SIDE_STREAMS[dev] = ss
    return ss


# Host pipeline chunking: about this many bytes of each model per chunk, at
# most this many chunks (dlsim_host_wreduce rounds the chunk to 1024 elements,
# which keeps every chunk of a 256-B aligned staging row 16-B aligned).
PIPELINE_CHUNK_BYTES = 8 << 20
PIPELINE_MAX_CHUNKS = 32


def pipeline_chunk_elems(total: int, esz: int) -> int:
    """Chunk length of the host pipeline for a total-element arena (0 = one chunk)."""
    k = max(1, min(PIPELINE_MAX_CHUNKS, round(total * esz / PIPELINE_CHUNK_BYTES)))
    return 0 if k == 1 else -(-total // k)


# Host results come back into page-locked memory from torch's caching host
# allocator: the D2H is then asynchronous, so the output module is built while
# the pipeline still runs (round 4), and once the simulation's results turn
# over, a result reuses a freed block (a fresh hipHostMalloc costs ~0.2 ms,
# scripts/probes/probe_result_alloc.py). DLSIM_AB=1 DLSIM_HOST_RESULT=pageable restores
# round 3's rule for A/B runs: results below PAGEABLE_RESULT_BYTES in pageable
# memory (the runtime stages that copy, and the library call waits for it).
PAGEABLE_RESULT_BYTES = 4 << 20
HOST_RESULT_PINNED = _native.ab_env("DLSIM_HOST_RESULT", "pinned") != "pageable"
# torch's caching host allocator never gives page-locked memory back to the
# OS and rounds blocks up to powers of two, so a caller that keeps many small
# results alive (an in-process simulation holding one model per peer) would
# pin up to twice their bytes. Once the allocator holds more than
# this many page-locked bytes, small results come back in pageable memory
# (round 3's rule: a synchronous D2H); large ones stay page-locked.
# DLSIM_PINNED_RESULT_BUDGET_MB overrides the 2 GiB.
PINNED_RESULT_BUDGET = int(float(os.environ.get("DLSIM_PINNED_RESULT_BUDGET_MB", "2048")) * (1 << 20))


class _PinnedBudget:
    """Whether small host results may still be page-locked: the caching host
    allocator's reserved bytes against PINNED_RESULT_BUDGET, read every
    CHECK_EVERY small results (reading the statistics costs microseconds)."""
    CHECK_EVERY = 32

    def __init__(self):
        self.calls = 0
        self.over = False

    @staticmethod
    def reserved() -> int:
        st = torch.cuda.memory.host_memory_stats()  # flat: "reserved_bytes.current", ...
        return int(st.get("reserved_bytes.current", st.get("allocated_bytes.current", 0)))

    def allow(self) -> bool:
        if self.calls % self.CHECK_EVERY == 0:
            try:
                self.over = self.reserved() > PINNED_RESULT_BUDGET
            except (AttributeError, RuntimeError, TypeError, ValueError):
                self.over = False
        self.calls += 1
        return not self.over


PINNED_BUDGET = _PinnedBudget()


def pinned_result(nbytes: int) -> bool:
    """Whether a host result of nbytes comes back page-locked (see above)."""
    if nbytes >= PAGEABLE_RESULT_BYTES:
        return True
    return HOST_RESULT_PINNED and PINNED_BUDGET.allow()


# Zero-copy host tasks (round 5): host
# models of at most ZC_MAX_BYTES of staged rows whose result goes back to the
# host are packed into page-locked rows that the reduce kernel reads in place
# over PCIe, and the kernel writes the page-locked result: no H2D and no D2H
# DMA (dlsim_host_wreduce_zc). 2 x GNLeNet: the library call with its wait
# 81 -> 63 us (profiles/r05d/zero_copy.json). Under DLSIM_AB=1 (the A/B
# switches, _native.ab_env), DLSIM_ZERO_COPY=0 turns it off and
# DLSIM_ZC_MAX_KB moves the 4 MiB.
ZERO_COPY = _native.ab_env("DLSIM_ZERO_COPY", "1") != "0"
ZC_MAX_BYTES = int(float(_native.ab_env("DLSIM_ZC_MAX_KB", "4096")) * 1024)
ZC_CALLS = [0]  # zero-copy dtype groups reduced (tests and probes)


def _host_pipeline(all_params, idx, layout, dt, dev, out, weights_f32, mode, stream, want_host, defer=False):
    """Host models -> device reduce (-> host result) in one dlsim_host_wreduce
    call: the parameters are packed into pinned staging rows by the library's
    thread pool (torch's intra-op thread count), chunk by chunk of the
    parameter axis; each model's share of a chunk goes H2D on the H2D stream as
    soon as it is packed, each chunk is reduced on the caller's stream once all
    its shares are on the device, and its result comes back on the D2H
    stream (PCIe is full duplex). Bytes and results are those of the
    unchunked reduce (elements are independent). One-chunk models use the
    caller's stream for everything (the side-stream events cost more than
    they hide there). Returns (the host result (want_host; complete once
    `stream` is) or None (the result is in `out`, queued on `stream`),
    whether a non-contiguous tensor was copied, whether the caller must still
    wait for `stream` before reading the host result: defer and a page-locked
    result; otherwise this call has waited)."""
    n = len(all_params)
    total = layout.totals[dt]
    esz = _elem_size(dt)
    host = None
    pinned_out = want_host and pinned_result(total * esz)
    if want_host:
        host = torch.empty(total, dtype=dt, pin_memory=pinned_out)
    # the layout checked every tensor's shape and dtype against models[0];
    # the library reads data pointers, so only non-contiguous ones are copied
    keep, ptrs = _data_ptrs(all_params, idx)
    if out is None:  # the zero-copy form (reduce_modules_to_arenas chose it)
        if pinned_out:
            ZC_CALLS[0] += 1
            _, rows = STAGING.acquire(dev, dt, n, total, stream, device_rows=False)
            synced = False
            try:
                _native.host_wreduce_zc_raw(ptrs, n, layout.split_sizes[dt], weights_f32, rows, host,
                                            _native.dtype_code(dt), mode, torch.get_num_threads(),
                                            stream.cuda_stream)
                if not defer:
                    stream.synchronize()
                    synced = True
            finally:
                STAGING.release(dev, dt, stream, synced, device_rows=False)
            return host, bool(keep), not synced
        out = arena_empty(total, dt, dev)  # past the page-locked budget: the DMA pipeline
    chunk = pipeline_chunk_elems(total, esz)
    h2d, d2h = _side_streams(dev) if chunk else (None, None)
    dev_rows, pinned = STAGING.acquire(dev, dt, n, total, stream)
    synced = False
    try:
        _native.host_wreduce_raw(ptrs, n, layout.split_sizes[dt], weights_f32, pinned, dev_rows, out, host,
                                 _native.dtype_code(dt), mode, chunk, torch.get_num_threads(), stream.cuda_stream,
                                 h2d, d2h)
        if want_host and not (defer and pinned_out):
            # the host result is complete once `stream` is: wait here, and
            # hand the rows back free
            stream.synchronize()
            synced = True
    finally:
        STAGING.release(dev, dt, stream, synced)
    return host, bool(keep), want_host and not synced


def _cached_host_reduce(cache, all_params, idx, layout, dt, dev, out, weights_f32, mode, stream, defer):
    """Host models with a device cache (device_cache.py): the models whose
    file_system shm storages this process uploaded before are read from their
    cached device rows; the others are packed and sent to free cache slots
    (or to transient rows past the capacity, or for models not in shared
    memory) and cached; then the reduce and the D2H, one
    dlsim_host_wreduce_resident call. None when no model is in shared memory
    (the normal pipeline then runs). Returns as _host_pipeline."""
    keys, ptrs, fps = _pyhost.shm_rows(all_params, idx)
    if all(k is None for k in keys):
        return None
    n = len(all_params)
    total = layout.totals[dt]
    esz = _elem_size(dt)
    stride = row_stride(total, esz)
    full = [None if k is None else (k, dev.index, dt, total) for k in keys]
    with cache.lock:
        cache.order(stream)
        # device addresses of resident rows (a stale entry drops out here)
        rows = [None if k is None else cache.get(k, fps[i]) for i, k in enumerate(full)]
        resident = [r is not None for r in rows]
        miss = [i for i in range(n) if rows[i] is None]
        # cache slots for the keyed misses (one per distinct key), never
        # evicting the rows this task reads; the rest get transient rows
        want, seen = [], set()
        for i in miss:
            if full[i] is not None and full[i] not in seen:
                seen.add(full[i])
                want.append(i)
        taken = cache.take_rows(dev, dt, stride, total, len(want), protected=n - len(miss)) if want else []
        slot_of = dict(zip(want, taken))
        staged = synced = False
        try:  # from here every failure hands the taken slots back
            for i, t in slot_of.items():
                rows[i] = t[2]
            rest = [i for i in miss if i not in slot_of]
            block = None
            if rest:
                block = aligned_empty(len(rest) * stride, dt, dev, base_align(total * esz, esz))
                b0 = block.data_ptr()
                for j, i in enumerate(rest):
                    rows[i] = b0 + j * stride * esz
            keep, src = [], ptrs  # resident models' pointers go unread
            if ptrs is None:  # a non-contiguous tensor somewhere: the misses' copies
                t = len(idx)
                src = [0] * (n * t)
                if miss:
                    keep, mp = _data_ptrs([all_params[i] for i in miss], idx)
                    for j, i in enumerate(miss):
                        src[i * t:(i + 1) * t] = mp[j * t:(j + 1) * t]
            pinned_out = pinned_result(total * esz)
            host = torch.empty(total, dtype=dt, pin_memory=pinned_out)
            pinned = None
            if miss:
                # pinned rows for all n models, of which the misses use the
                # first ones: the same shape every task, so acquire() reuses
                # its views (a shape per miss count rebuilt them, ~30 us a
                # task); no device rows: misses go straight to their cache
                # or transient rows
                _, pinned = STAGING.acquire(dev, dt, n, total, stream, device_rows=False)
                staged = True
            _native.host_wreduce_resident_raw(src, n, layout.split_sizes[dt], weights_f32, resident,
                                              rows, pinned, out, host,
                                              _native.dtype_code(dt), mode, torch.get_num_threads(),
                                              stream.cuda_stream)
            if not (defer and pinned_out):
                stream.synchronize()
                synced = True
        except BaseException:
            for t in slot_of.values():
                cache.give_back(t)
            raise
        finally:
            if staged:
                STAGING.release(dev, dt, stream, synced, device_rows=False)
        for i, t in slot_of.items():
            cache.put(full[i], t, fps[i])
        st = cache.stats
        st["hits"] += n - len(miss)
        st["misses"] += sum(1 for i in miss if full[i] is not None)
        st["uncacheable"] += sum(1 for i in miss if full[i] is None)
        st["bytes_not_sent"] += (n - len(miss)) * total * esz
    return host, bool(keep), not synced


def _data_ptrs(all_params, idx):
    """(keep-alive list, data pointers of tensor k of every model for k in
    idx, model-major). Non-contiguous tensors are copied (and kept alive until
    the stream-ordered work that reads them is queued)."""
    ptrs = _pyhost.data_ptrs(all_params, idx)
    if ptrs is not None:
        return [], ptrs
    keep, ptrs = [], []
    for ps in all_params:
        for k in idx:
            q = ps[k]
            if not q.is_contiguous():
                q = q.detach().contiguous()
                keep.append(q)
            ptrs.append(q.data_ptr())
    return keep, ptrs


def _staged_reduce(all_params, idx, dt, dev, out, weights, mode, stream):
    """Models whose parameters are neither one device arena nor host tensors
    the native pipeline takes (another GPU; separate fp64 tensors): each
    model's parameters are concatenated into a device staging row, then one
    reduce over the rows."""
    n = len(all_params)
    dev_rows, _ = STAGING.acquire(dev, dt, n, out.numel(), stream, pinned=False)
    try:
        for i, ps in enumerate(all_params):
            torch.cat([ps[k].detach().reshape(-1).to(dev) for k in idx], out=dev_rows[i])
        _native.wreduce([dev_rows[i] for i in range(n)], weights, out, mode)
    finally:
        STAGING.release(dev, dt, stream)


def reduce_modules_to_arenas(models: List[nn.Module], weights_f32: np.ndarray, mode: int,
                             device=None, timing: Optional[dict] = None, host_out: Optional[bool] = False,
                             weights_f64: Optional[np.ndarray] = None, defer_host_sync: bool = False
                             ) -> Tuple[ParamLayout, Dict[torch.dtype, torch.Tensor], torch.device, bool, bool,
                                        bool, bool]:
    """Reduce the parameters of `models` into one fresh arena per dtype.

    weights_f32: the fp32-rounded weights (fp32/bf16/fp16 groups);
    weights_f64: the Python-float weights, kept exact as doubles for an fp64
    group (fedavg.py:25 keeps the Python float exact for a double tensor);
    default: widened fp32.
    host_out None: as the reference's output, iff models[0]'s parameters are on
    the host. Returns (layout, arenas, device, on_host, host_out, staged,
    pending): staged = some group went through a path that also takes
    non-contiguous tensors (the caller then gives such parameters models[0]'s
    strides). With host_out, host models take the chunked pipeline and come
    back in host memory (on_host True): complete, or with defer_host_sync
    still in flight on the device's current stream (pending True: the caller
    waits for that stream before reading them). Otherwise the arenas are on
    the device."""
    layout, all_params, in_views = input_arenas(models)
    if host_out is None:
        host_out = not any(p.is_cuda for p in layout.params)
    dev = _target_device(all_params[0], device)
    n = len(models)
    outs: Dict[torch.dtype, torch.Tensor] = {}
    # the raw handle from C (torch.cuda.current_stream costs a few us of
    # Python per call); the Stream object only where a path needs it
    raw_stream = torch._C._cuda_getCurrentRawStream(dev.index)
    _stream = []

    def get_stream():
        if not _stream:
            _stream.append(torch.cuda.current_stream(dev))
        return _stream[0]
    st = _Stages(timing, get_stream() if timing is not None else None)
    host_models = all(not all_params[i][idx[0]].is_cuda
                      for idx in layout.groups.values() for i in range(n))
    piped = host_out and host_models and len(layout.groups) > 0
    staged = pending = False
    with torch.no_grad():
        for dt, idx in layout.groups.items():
            total = layout.totals[dt]
            f64 = dt == torch.float64
            w = (_native.f64_weights(weights_f64) if weights_f64 is not None else weights_f32.astype(np.float64)) \
                if f64 else weights_f32
            # small host models whose result goes back to the host: no device
            # output (dlsim_host_wreduce_zc writes the page-locked result)
            zc = piped and not f64 and ZERO_COPY and n * total * _elem_size(dt) <= ZC_MAX_BYTES \
                and device_cache.active() is None
            out = None if zc and total else arena_empty(total, dt, dev)
            outs[dt] = out
            if total == 0:
                if piped:
                    outs[dt] = torch.empty(0, dtype=dt)
                continue
            dix = dev.index
            on_dev = all(all_params[i][idx[0]].get_device() == dix for i in range(n))
            if on_dev:
                views = in_views[dt]
                st.mark("layout")
                if views is not None:
                    _native.wreduce(views, w, out, mode)
                    st.mark("kernel")
                    continue
                if f64:  # one task through dlsim_wreduce_f64
                    _staged_reduce(all_params, idx, dt, dev, out, w, mode, get_stream())
                    staged = True
                    st.mark("kernel")
                    continue
                # separate device tensors, read in place: the layout checked
                # shapes and dtypes, so only pointers go to the library, read
                # in C (no detach() objects, no output slices)
                if not _native.wreduce_rows(all_params, idx, layout.split_sizes[dt], weights_f32, out.data_ptr(),
                                            layout.byte_offsets[dt], _native.dtype_code(dt), mode,
                                            raw_stream, dix):
                    # a tensor is not contiguous, or (in a model whose first
                    # tensor is here) on another device: stage them all
                    _staged_reduce(all_params, idx, dt, dev, out, w, mode, get_stream())
                    staged = True
                st.mark("kernel")
                continue
            if not f64 and not any(all_params[i][idx[0]].is_cuda for i in range(n)):
                # host models (the reference's case): chunked pack / H2D /
                # reduce (/ D2H) pipeline, or with a device cache the models
                # this process has uploaded before are read in place
                st.mark("layout")
                cache = device_cache.active()
                r = _cached_host_reduce(cache, all_params, idx, layout, dt, dev, out, weights_f32, mode,
                                        get_stream(), defer_host_sync) if cache is not None and piped else None
                h, copied, waits = r if r is not None else _host_pipeline(
                    all_params, idx, layout, dt, dev, out, weights_f32, mode, get_stream(), piped, defer_host_sync)
                staged = staged or copied
                pending = pending or waits
                if h is not None:
                    outs[dt] = h
                st.mark("pipeline")
                continue
            # models on another GPU (or fp64 host models): gather onto this
            # one, then reduce
            st.mark("layout")
            _staged_reduce(all_params, idx, dt, dev, out, w, mode, get_stream())
            staged = True
            st.mark("kernel")
    if piped:
        left = {dt: a for dt, a in outs.items() if a.is_cuda}
        if left:  # single-chunk groups: their D2H now (and the wait)
            outs.update(arenas_to_host(left, get_stream()))
            pending = False
            st.mark("d2h")
        elif not pending:
            get_stream().synchronize()
    return layout, outs, dev, piped, host_out, staged, pending


def arenas_to_host(arenas: Dict[torch.dtype, torch.Tensor], stream) -> Dict[torch.dtype, torch.Tensor]:
    """D2H into page-locked memory from torch's caching host allocator (the
    block returns to the cache when the returned module is freed; small
    results in pageable memory past PINNED_RESULT_BUDGET), then wait for the
    copies: the output module may be used as soon as this returns."""
    host = {}
    with torch.cuda.stream(stream):
        for dt, a in arenas.items():
            h = torch.empty(a.numel(), dtype=dt, pin_memory=pinned_result(a.numel() * a.element_size()))
            h.copy_(a, non_blocking=True)
            host[dt] = h
    stream.synchronize()
    return host


# Atomic attribute types a module clone may share (deepcopy returns them as is).
_ATOMIC = frozenset((type(None), bool, int, float, complex, str, bytes, torch.dtype, torch.device, torch.layout,
                     torch.memory_format))

_PLAIN_CLASSES: Dict[type, int] = {}


def _plain_module_class(cls) -> int:
    """How copy.deepcopy copies an instance of module class `cls`, which
    _clone_module restates without the generic __reduce_ex__ machinery
    (cached per class):
      0 — its own reduce/deepcopy/getstate: copy.deepcopy itself;
      1 — nn.Module's default reduce/getstate/setstate round trip;
      2 — the same with the class's own __setstate__ (e.g. _ConvNd's), which
          the clone calls with the copied state, as copy.deepcopy does."""
    kind = _PLAIN_CLASSES.get(cls)
    if kind is None:
        default = (cls.__reduce_ex__ is object.__reduce_ex__ and cls.__reduce__ is object.__reduce__
                   and getattr(cls, "__deepcopy__", None) is None and cls.__getstate__ is nn.Module.__getstate__)
        kind = _PLAIN_CLASSES[cls] = 0 if not default else (1 if cls.__setstate__ is nn.Module.__setstate__ else 2)
    return kind


# Attributes nn.Module.__setstate__ adds when an (old) state lacks them; with
# all of them present it is exactly __dict__.update(state).
_SETSTATE_KEYS = frozenset(("_forward_pre_hooks", "_forward_pre_hooks_with_kwargs", "_forward_hooks_with_kwargs",
                            "_forward_hooks_always_called", "_state_dict_hooks", "_state_dict_pre_hooks",
                            "_load_state_dict_pre_hooks", "_load_state_dict_post_hooks",
                            "_non_persistent_buffers_set", "_is_full_backward_hook", "_backward_pre_hooks"))


def _all_atomic(v) -> bool:
    for x in v:
        if type(x) not in _ATOMIC:
            return False
    return True


def _clone_module_py(m: nn.Module, memo: dict) -> nn.Module:
    """copy.deepcopy(m, memo) for a module tree, several times faster for plain
    modules. The product path runs the same walk in C (`_clone_module`,
    csrc/pyhost.cpp); this is its specification, and tests compare the two.

    deepcopy of an nn.Module is: state = Module.__getstate__() (the __dict__
    minus _compiled_call_impl), deep-copied with the shared memo, then
    cls.__new__(cls).__setstate__(state). That is what this does, taking
    parameters from the memo (the arena views module_from_arenas installs),
    recursing into `_modules` directly, and keeping what deepcopy would return
    unchanged without a round trip: atomic values and tuples of atomic values
    (deepcopy returns those very objects), lists of atomic values (a shallow
    copy, entered in the memo like deepcopy does) and fresh empty hook
    containers. Anything else (buffers, non-empty containers, custom
    attributes) goes through copy.deepcopy with the same memo; classes with
    their own reduce/deepcopy/getstate take copy.deepcopy whole."""
    got = memo.get(id(m))
    if got is not None:
        return got
    cls = type(m)
    kind = _plain_module_class(cls)
    if not kind:
        return copy.deepcopy(m, memo)
    new = cls.__new__(cls)
    memo[id(m)] = new
    d = m.__dict__
    state = d.copy()
    for k, v in d.items():
        tv = type(v)
        if tv in _ATOMIC:
            continue
        if k == "_modules":
            state[k] = tv((name, None if c is None else _clone_module_py(c, memo)) for name, c in v.items())
        elif k == "_parameters":
            state[k] = tv((name, None if q is None else (memo[id(q)] if id(q) in memo else copy.deepcopy(q, memo)))
                          for name, q in v.items())
        elif k == "_compiled_call_impl":
            del state[k]
        elif tv is tuple and _all_atomic(v):
            continue
        elif (tv is dict or tv is OrderedDict or tv is set) and not v:
            state[k] = tv()
        elif tv is list and _all_atomic(v):
            c = memo.get(id(v))
            if c is None:
                c = memo[id(v)] = list(v)
            state[k] = c
        else:
            state[k] = copy.deepcopy(v, memo)
    if kind == 1 and _SETSTATE_KEYS.issubset(state):
        new.__dict__.update(state)  # what Module.__setstate__ does with a complete state
    else:
        new.__setstate__(state)
    return new


_pyhost.clone_init(_PLAIN_CLASSES, _plain_module_class, _ATOMIC, _SETSTATE_KEYS, copy.deepcopy, OrderedDict)
_clone_module = _pyhost.clone_module


_make_param = torch.Tensor._make_subclass


class _ArenaEntry:
    __slots__ = ("layout", "arenas", "bases")

    def __init__(self, layout, arenas, bases):
        self.layout, self.arenas, self.bases = layout, arenas, bases


# Modules whose parameters this package installed as views of flat arenas
# (module_from_arenas): their layout and arenas, so later aggregates skip the
# layout/contiguity checks. Weak keys: an entry lives as long as its module.
_ARENAS: Dict[int, Tuple["weakref.ref", _ArenaEntry]] = {}  # id(module) -> (weak ref, entry)


def _arena_entry(module) -> Optional[_ArenaEntry]:
    """The entry of `module` (one dict lookup by id; the weak reference
    proves the id still belongs to it)."""
    e = _ARENAS.get(id(module))
    if e is None or e[0]() is not module:
        return None
    return e[1]


def _register_arenas(module: nn.Module, entry: _ArenaEntry) -> None:
    key = id(module)

    def gone(ref, key=key):  # runs when the module is freed, before its id can be reused
        cur = _ARENAS.get(key)
        if cur is not None and cur[0] is ref:
            del _ARENAS[key]
    _ARENAS[key] = (weakref.ref(module, gone), entry)


def registered_arenas(module: nn.Module, params: Optional[List[nn.Parameter]] = None):
    """(layout over `module`'s parameters, {dtype: flat arena}) if `module` was
    built by module_from_arenas and its parameters still are those views
    (same count, shapes and addresses, and contiguous: a parameter
    re-assigned or re-pointed since, e.g. `p.data = t`, or re-viewed with
    other strides at the same address, e.g. `p.data = p.data.t()` on a square
    weight, invalidates the entry); else None."""
    e = _arena_entry(module)
    if e is None:
        return None
    ps = module_params(module) if params is None else params
    slots, bases = e.layout.param_slots, e.bases
    if len(ps) != len(slots):
        return None
    for q, (dt, bo, shape) in zip(ps, slots):
        if q.data_ptr() != bases[dt] + bo or q.shape != shape or not q.is_contiguous():
            return None
    return e.layout.rebind(ps), e.arenas


def module_from_arenas(model0: nn.Module, layout: ParamLayout,
                       arenas: Dict[torch.dtype, torch.Tensor]) -> nn.Module:
    """`copy.deepcopy(model0)` whose parameters are views of `arenas`
    (registered, so a later aggregate reads the arenas without checks)."""
    memo = {}
    params = layout.params
    for dt, idx in layout.groups.items():
        # memo[id(p)] = nn.Parameter(view of the arena, p.requires_grad) for
        # every p of the group, built in C++ (_param_views_py restates it)
        _pyhost.fill_param_views(memo, arenas[dt], layout.view_specs[dt], params, idx)
    out = _clone_module(model0, memo)
    # The clone maps every parameter of model0 to its view one to one and keeps
    # the module/parameter order, so parameters() of `out` are those views.
    _register_arenas(out, _ArenaEntry(layout.rebind([]), dict(arenas),
                                      {dt: a.data_ptr() for dt, a in arenas.items()}))
    return out


def _param_views_py(memo: dict, arena: torch.Tensor, specs, params, idx) -> None:
    """Specification of csrc/pyhost.cpp fill_param_views (tests compare them)."""
    base = arena.storage_offset()
    for k, (shape, strides, off) in zip(idx, specs):
        p = params[k]
        memo[id(p)] = _make_param(nn.Parameter, arena.as_strided(shape, strides, base + off), p.requires_grad)


def input_arenas(models: Sequence[nn.Module]):
    """Layout of models[0], every model's parameter list, and per dtype the
    flat arena view of every model — or None for a dtype where some model is
    not an arena (separate storages, host memory, ...). Registered arenas
    (module_from_arenas outputs) skip the layout and contiguity checks."""
    reg0 = registered_arenas(models[0])
    layout = reg0[0] if reg0 is not None else layout_of(models[0])
    all_params, views = [], {dt: [] for dt in layout.groups}
    for i, m in enumerate(models):
        reg = reg0 if i == 0 else registered_arenas(m)
        if reg is not None and (reg[0]._signature is layout._signature or reg[0]._signature == layout._signature):
            ps = reg[0].params
            all_params.append(ps)
            for dt in layout.groups:
                if views[dt] is not None:
                    views[dt].append(reg[1][dt])
            continue
        ps = layout.check_compatible(m)
        all_params.append(ps)
        for dt in layout.groups:
            if views[dt] is not None:
                v = layout.arena_view(ps, dt)
                views[dt] = None if v is None else views[dt] + [v]
    return layout, all_params, views


# the current stream's torch object per raw handle (torch.cuda.current_stream
# costs a few us of Python per call; the raw handle is one C call)
_STREAM_OBJS: Dict[int, torch.cuda.Stream] = {}
_DEVICES: Dict[int, torch.device] = {}


def _current_stream(idx: int, raw: int) -> torch.cuda.Stream:
    s = _STREAM_OBJS.get(raw)
    if s is None or s.cuda_stream != raw or s.device_index != idx:
        s = torch.cuda.current_stream(idx)
        if len(_STREAM_OBJS) > 64:
            _STREAM_OBJS.clear()
        _STREAM_OBJS[raw] = s
    return s


def _host_zc_task(models: List[nn.Module]):
    """(class layout, dtype, parameter indices, every model's parameters) when
    `models` is a task _host_zc_aggregate runs, else None (host-side checks
    only; no device call)."""
    if not ZERO_COPY or device_cache._CACHE is not None:
        return None
    known = _CLASS_LAYOUTS.get(type(models[0]))
    if known is None or len(known.groups) != 1:
        return None
    (dt, idx), = known.groups.items()
    total = known.totals[dt]
    esz = _elem_size(dt)
    if dt is torch.float64 or total == 0 or len(models) * total * esz > ZC_MAX_BYTES:
        return None
    sig = known._signature
    k0 = idx[0]
    all_params = []
    for m in models:
        ps = _pyhost.checked_params(m, sig)
        if ps is None or ps[k0].is_cuda:
            return None
        all_params.append(ps)
    if not pinned_result(total * esz):
        return None
    return known, dt, idx, all_params


def _host_zc_aggregate(models: List[nn.Module], w32: np.ndarray, mode: int) -> Optional[nn.Module]:
    """The small host task in one pass (round 6): the
    reference's default deployment (host GNLeNets, worker.py:24-33 ->
    functions.py:89-106) with the zero-copy reduce. What
    reduce_modules_to_arenas + _host_pipeline(out=None) + module_from_arenas
    do for such a task, minus their generic machinery: the models' class
    layout (one dtype group), each model's parameters walked and checked
    against it in C, one _pyhost call that hands the data pointers to
    dlsim_host_wreduce_zc (pack, then the reduce reading the page-locked rows
    and writing the page-locked result over PCIe), the output module built
    while the kernel runs, one wait. None when the task is not such a task
    (the general path then runs it): another signature or layout class, a
    device model, a non-contiguous parameter, more than ZC_MAX_BYTES of rows,
    fp64, the device cache on, or the page-locked result budget spent."""
    task = _host_zc_task(models)
    if task is None:
        return None
    known, dt, idx, all_params = task
    n = len(models)
    total = known.totals[dt]
    m0 = models[0]
    di = torch.cuda.current_device()
    dev = _DEVICES.get(di)
    if dev is None:
        dev = _DEVICES[di] = torch.device("cuda", di)
    raw = torch._C._cuda_getCurrentRawStream(di)
    host = torch.empty(total, dtype=dt, pin_memory=True)
    _, rows = STAGING.acquire(dev, dt, n, total, None, device_rows=False)
    done = False  # the rows are free: nothing launched, or the kernel waited for
    try:
        if not _native.host_zc(all_params, idx, known.split_sizes[dt], w32, rows, host, _native.dtype_code(dt),
                               mode, torch.get_num_threads(), raw):
            done = True  # a non-contiguous or device tensor, refused before any launch: the general path
            return None
        ZC_CALLS[0] += 1
        layout = known.rebind(all_params[0])
        out = module_from_arenas(m0, layout, {dt: host})  # while the kernel runs
        _current_stream(di, raw).synchronize()
        done = True
        return out
    finally:
        if not done:  # an error after (or during) the library call: some chunks may be queued
            _current_stream(di, raw).synchronize()
        STAGING.release(dev, dt, None, True, device_rows=False)


def aggregate_modules(models: List[nn.Module], weights: Optional[Sequence[float]], mode: int,
                      device=None, to_host: Optional[bool] = None,
                      timing: Optional[dict] = None) -> nn.Module:
    """FedAvg.aggregate semantics on the GPU (see module docstring).

    to_host: copy the result back to host memory (default: iff models[0]'s
    parameters are on the host, like the reference's output).
    timing: if a dict, filled with a wall-clock stage breakdown (synchronising)."""
    # fedavg.py:14-17, same order of checks => same exceptions
    if not weights:
        weights = [float(1. / len(models)) for _ in range(len(models))]
    else:
        assert len(weights) == len(models)
    model0 = models[0]  # IndexError for an empty list, as the reference
    w32 = _native.fp32_weights(weights)
    if timing is None and device is None and to_host is not False:
        out = _host_zc_aggregate(models, w32, mode)
        if out is not None:
            return out
    try:
        layout, arenas, dev, on_host, host_out, staged, pending = reduce_modules_to_arenas(
            models, w32, mode, device, timing, to_host, weights_f64=weights, defer_host_sync=timing is None)
    except ZipMismatch:  # raised by the layout check, before any device work
        return _aggregate_zip(models, weights, mode, device, to_host)
    if timing is None and not (host_out and not on_host):
        # the output module is built while a host result's copies may still
        # run (pending); it only makes views of the result
        out = module_from_arenas(model0, layout, arenas)
        if pending:
            torch.cuda.current_stream(dev).synchronize()
        return _restride(out, layout) if staged else out
    stream = torch.cuda.current_stream(dev)
    st = _Stages(timing, stream)
    if host_out and not on_host:
        arenas = arenas_to_host(arenas, stream)
        st.mark("d2h")
    out = module_from_arenas(model0, layout, arenas)
    if staged:
        _restride(out, layout)
    st.mark("module")
    return out


def _aggregate_zip(models: List[nn.Module], weights: Sequence[float], mode: int,
                   device=None, to_host: Optional[bool] = None) -> nn.Module:
    """The reference's pairing for models whose parameter lists differ from
    models[0]'s (fedavg.py:23-24): `zip(center.parameters(), m.parameters())`
    stops at the shorter list, so output parameter t sums, in model order,
    w_i * p_i[t] over the models that have a t-th parameter (models[0]
    always does; a model's extra parameters are ignored), starting from
    models[0][t] * 0; `c1.add_(w * p1)` broadcasts a p1 whose shape
    broadcasts to c1's and raises RuntimeError otherwise, as torch does.
    A p1 of another dtype follows torch's type promotion: the product in
    p1's dtype, the add in the promoted dtype, rounded into c1's
    (dlsim_wreduce_mixed; pinned by tests/golden/mixed_*.npz, made by running
    the reference). One reduce launch per parameter, on the GPU; a host
    model's tensors are copied in first. A rare path: simulations aggregate
    one architecture and take the one-launch paths above."""
    weights = [float(w) for w in weights]
    n = len(models)
    plists = [module_params(m) for m in models]
    p0 = plists[0]
    layout = ParamLayout(models[0], p0)
    dev = _target_device(p0, device)
    host_out = (not any(p.is_cuda for p in p0)) if to_host is None else to_host
    with torch.no_grad():
        arenas = {dt: arena_empty(layout.totals[dt], dt, dev) for dt in layout.groups}
        for t, c in enumerate(p0):
            rows, ws = [], []
            for i in range(n):
                if len(plists[i]) <= t:
                    continue
                q = plists[i][t].detach()
                if q.shape != c.shape:
                    if torch.broadcast_shapes(q.shape, c.shape) != c.shape:
                        raise RuntimeError(f"output with shape {list(c.shape)} doesn't match the broadcast "
                                           f"shape {list(torch.broadcast_shapes(q.shape, c.shape))}")
                    q = q.expand(c.shape)
                rows.append(q.to(dev).contiguous().reshape(-1))
                ws.append(weights[i])
            if c.numel() == 0:
                continue
            off = layout.offsets[t]
            out = arenas[c.dtype][off:off + c.numel()]
            if any(r.dtype != c.dtype for r in rows):
                _native.wreduce_mixed(rows, ws, out)  # exact: torch's promotion, step by step
                continue
            w = _native.weights_for_dtype(ws, c.dtype)
            _native.wreduce(rows, w, out, mode)
        if host_out:
            arenas = arenas_to_host(arenas, torch.cuda.current_stream(dev))
    out = module_from_arenas(models[0], layout, arenas)
    return _restride(out, layout)


def _restride(out: nn.Module, layout: ParamLayout) -> nn.Module:
    """Give every output parameter whose models[0] counterpart is not
    contiguous the layout deepcopy(models[0]) gives it (fedavg.py:20:
    Parameter.__deepcopy__ clones with preserve_format, e.g. a transposed
    weight stays transposed); the values are the reduce's, element for
    element. Such parameters leave the result arena (the next aggregate reads
    them as separate tensors)."""
    with torch.no_grad():
        for q, p0 in zip(module_params(out), layout.params):
            if not p0.is_contiguous():
                fresh = torch.empty_like(p0, memory_format=torch.preserve_format, device=q.device)
                fresh.copy_(q.detach())
                q.data = fresh
    return out


def to_device_arena(model: nn.Module, device=None) -> nn.Module:
    """A copy of `model` (deepcopy semantics) whose parameters are views of one
    device arena per dtype — the form the aggregate reads in place. A plain
    copy (not a 1-way reduce: x*0 + 1*x is not the identity for inf/NaN)."""
    layout = ParamLayout(model)
    dev = _target_device(layout.params, device)
    arenas = {}
    with torch.no_grad():
        for dt, idx in layout.groups.items():
            flat = arena_empty(layout.totals[dt], dt, dev)
            for k in idx:
                off = layout.offsets[k]
                p = layout.params[k]
                flat[off:off + p.numel()].copy_(p.detach().reshape(-1), non_blocking=True)
            arenas[dt] = flat
    return module_from_arenas(model, layout, arenas)
