"""Round executor: the broker's task scheduling (broker.py:261-290) for a DAG
of simulator tasks, with every ready `aggregate` task of a wave batched into
one GPU launch and models kept resident on the device (SURVEY.md §8f rows 1
and 4).

The reference runs one task at a time on a worker (worker.py:21-38): the
broker resolves `(task_name, output_index)` placeholders when producers finish
(Task.set_data, tasks/task.py:26-51) and schedules tasks whose inputs are all
present. Here the same resolution happens in topological *waves*: every task
whose inputs are ready runs in the wave; the aggregate tasks of a wave go to
`aggregate_batch` together (descriptor-table launches), other tasks (train,
test, ...) are called through the function table like the worker does.

Models that reach an aggregate are resolved once per wave: aggregate outputs
are registered arenas (read in place), other device arenas are read in place,
models that keep their parameters in separate contiguous tensors on the
device (a device train task's deepcopy) are read in place tensor by tensor,
anything else (host models, other devices) is copied once into a fresh arena
(one concatenation, no module built). So an aggregate -> train ->
aggregate chain never crosses PCIe when the train function works on the
device. Results are bit-identical to running the same tasks one by one with
FedAvg.aggregate.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
from torch import nn

from . import _native
from .arena import (ParamLayout, ZipMismatch, _target_device, aggregate_modules, aligned_empty, arena_empty, base_align,
                    layout_of, module_params, registered_arenas, row_stride)
from .batch import _device_views, _resolve, aggregate_arena_tasks

Task = Tuple[str, str, dict]  # (task_name, func_name, data with placeholders)

# Host-trained models of a wave go to the device in groups of at most this
# many bytes (RoundExecutor._upload_host_models).
UPLOAD_GROUP_BYTES = 256 << 20


def _is_ref(v) -> bool:
    return isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], str) and isinstance(v[1], int)


def _refs(v, out):
    if _is_ref(v):
        out.append(v[0])
    elif isinstance(v, (list, tuple)):
        for x in v:
            _refs(x, out)
    elif isinstance(v, dict):
        for x in v.values():
            _refs(x, out)
    return out


class RoundExecutor:

    def __init__(self, funcs: Dict[str, Callable], settings, device=None,
                 mode: int = _native.DLSIM_EXACT, timing: bool = False, keep_all: bool = False,
                 tensors_in_place: bool = True, release_early: bool = True, foreign_streams: bool = False):
        """timing: accumulate wall seconds per kind of wave work in
        `self.stats` ("aggregate", "other"); the stream is synchronised after
        every batched aggregate so its kernels count (measurement only).
        keep_all: keep every task's result; by default a result is dropped
        once every task that reads it has run, as the broker clears a
        completed task's data (broker.py:221), so memory is bounded by the
        DAG's frontier, not by the number of rounds.
        tensors_in_place: read models whose parameters are separate device
        tensors where they are (False: copy each into an arena first, the
        session-1 behaviour, kept for comparison).
        release_early: drop the results no later task reads as soon as a
        wave's launches are queued, before its output modules are built
        (the default: a wave's inputs and outputs never coexist, and the
        inputs' deallocations offset the outputs' allocations, so the cyclic
        collector runs far less inside the wave; 100 GNLeNet peers on one
        box: 96 against 217 µs per task, collector passes 87/6/0 against
        468/45/3 by generation, profiles/r02_release_ab/). False drops them
        after the wave, as the broker drops a task's inputs after the task
        returns (broker.py:221).
        foreign_streams: results are dropped while the wave's kernels may
        still be queued; the caching allocator keeps that safe for tensors
        allocated on the stream the reduce runs on (torch's current stream,
        where train functions allocate unless they switch streams). A train
        function that allocates its outputs under another stream must set
        foreign_streams=True: every released device parameter is then
        recorded on the current stream (Tensor.record_stream), so its block
        is not reused before the reduce has read it."""
        self.timing = timing
        self.keep_all = keep_all
        self.tensors_in_place = tensors_in_place
        self.release_early = release_early
        self.foreign_streams = foreign_streams
        self.stats: Dict[str, float] = {"aggregate": 0.0, "other": 0.0, "aggregate_tasks": 0}
        self.funcs = dict(funcs)
        self.settings = settings
        self.device = device
        self.mode = mode
        self.results: Dict[str, list] = {}
        self.waves: List[List[str]] = []
        self._stages: List[Optional[torch.Tensor]] = [None, None]  # pinned upload buffers
        self._stage_events: List[Optional[torch.cuda.Event]] = [None, None]

    def _resolve(self, v):
        if _is_ref(v):
            return self.results[v[0]][v[1]]
        if isinstance(v, list):
            return [self._resolve(x) for x in v]
        if isinstance(v, dict):
            return {k: self._resolve(x) for k, x in v.items()}
        return v

    def _layout_for(self, m: nn.Module, params=None) -> ParamLayout:
        """m's ParamLayout; a model of a class seen before reuses that layout
        when the parameter signature matches (arena.layout_of)."""
        return layout_of(m, params)

    def _arena_of(self, m: nn.Module, cache: dict, walked: Optional[dict] = None):
        """(layout over m's parameters, {dtype: flat device arena}) for one
        model, once per wave (`cache` keeps the model alive, so its id cannot
        be reused while the entry exists). walked: {id(m): (m, parameters)}
        from this wave's upload scan, so the parameters are walked once."""
        hit = cache.get(id(m))
        if hit is not None and hit[0] is m:
            return hit[1], hit[2]
        w = walked.get(id(m)) if walked is not None else None
        ps = w[1] if w is not None and w[0] is m else None
        reg = registered_arenas(m, ps)
        if reg is not None:  # an aggregate output: its arenas as they are
            layout, ar = reg
            views = {dt: [ar[dt]] for dt in layout.groups}
        else:
            layout = self._layout_for(m, ps)
            views = {dt: None if (v := layout.arena_view(layout.params, dt)) is None else [v]
                     for dt in layout.groups}
        params = [layout.params]
        dev = _device_views(views)
        if dev is not None and (self.device is None or dev == _target_device((), self.device)):
            arenas = {dt: vs[0] for dt, vs in views.items()}
        else:
            dev = _target_device(params[0], self.device)
            arenas = {}
            with torch.no_grad():
                for dt, idx in layout.groups.items():
                    ts = [params[0][k] for k in idx]
                    if self.tensors_in_place and dt != torch.float64 and \
                            all(t.device == dev and t.is_contiguous() for t in ts):
                        # separate tensors on the target device (a device
                        # train task's deepcopy): read in place by the wave's
                        # reduce (None = "use the parameter tensors"), no copy
                        arenas[dt] = None
                    elif all(t.device == dev for t in ts):
                        # one C++ call (torch's flatten, as DDP buckets use)
                        # instead of a reshape per tensor and a cat
                        arenas[dt] = torch._C._nn.flatten_dense_tensors(ts)
                    else:
                        arenas[dt] = torch.cat([t.detach().reshape(-1).to(dev, non_blocking=True) for t in ts])
        cache[id(m)] = (m, layout, arenas)
        return layout, arenas

    def _stage(self, k: int, nbytes: int) -> torch.Tensor:
        """Pinned staging buffer k of 2 (grow-only, reused across waves), once
        the H2D copy that last read it has completed."""
        ev = self._stage_events[k]
        if ev is not None:
            ev.synchronize()
        buf = self._stages[k]
        if buf is None or buf.numel() < nbytes:
            self._stages[k] = None  # back to torch's pinned cache before growing
            buf = self._stages[k] = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        return buf

    def _upload_host_models(self, models, cache: dict, walked: Optional[dict] = None) -> None:
        """Every host model of a wave (the reference's CPU-trained models) to
        the device in bounded groups: the library's threads pack a group's
        parameters into a persistent pinned buffer (dlsim_host_pack; one arena
        per model and dtype at 256-B aligned offsets), then one H2D per group.
        Groups hold at most UPLOAD_GROUP_BYTES (a larger model is a group of
        its own) and alternate between two pinned buffers, so the pack of
        group g+1 overlaps the copy of group g and pinned memory stays bounded
        by two groups, however many models a wave has. Fills `cache` as
        _arena_of would (instead of one small H2D per parameter tensor).
        walked: filled with {id(m): (m, parameters)} for the models it walks
        and leaves to _arena_of."""
        pending, seen = [], set()
        for m in models:
            if id(m) in seen or (id(m) in cache and cache[id(m)][0] is m):
                continue
            seen.add(id(m))
            ps = module_params(m)
            if walked is not None:
                walked[id(m)] = (m, ps)
            if registered_arenas(m, ps) is not None:
                continue
            if not ps or any(p.get_device() != -1 for p in ps):
                continue
            pending.append((m, self._layout_for(m, ps)))
        if not pending:
            return
        dev = _target_device(pending[0][1].params, self.device)
        stream = torch.cuda.current_stream(dev)
        groups, cur, cur_bytes = [], [], 0
        def span_bytes(layout, dt, idx):  # one dtype arena, at the row rule's stride
            esz = layout.params[idx[0]].element_size()
            return row_stride(layout.totals[dt], esz) * esz

        for m, layout in pending:
            nb = sum(span_bytes(layout, dt, idx) for dt, idx in layout.groups.items())
            if cur and cur_bytes + nb > UPLOAD_GROUP_BYTES:
                groups.append(cur)
                cur, cur_bytes = [], 0
            cur.append((m, layout))
            cur_bytes += nb
        groups.append(cur)
        for g, group in enumerate(groups):
            srcs, offs, spans, off = [], [], [], 0
            align = 256
            for m, layout in group:
                span = {}
                for dt, idx in layout.groups.items():
                    esz = layout.params[idx[0]].element_size()
                    span[dt] = (off, layout.totals[dt], esz)
                    start = off
                    for k in idx:
                        p = layout.params[k]
                        srcs.append(p.detach() if p.is_contiguous() else p.detach().contiguous())
                        offs.append(off)
                        off += p.numel() * esz
                    # the next arena one row stride on (arena.row_stride: large
                    # 4/8-byte arenas 2 MiB-aligned in a 2 MiB-aligned buffer)
                    off = start + span_bytes(layout, dt, idx)
                    align = max(align, base_align(layout.totals[dt] * esz, esz))
                spans.append(span)
            size = max(off, 1)
            stage = self._stage(g % 2, size)
            _native.host_pack(srcs, offs, stage[:size])
            # from 4 MiB the output pool's physically contiguous blocks (a
            # torch MemPool: freed after the wave, reused by the next), as for
            # single calls' staging rows; 2 MiB-aligned
            buf = arena_empty(size, torch.uint8, dev)
            if buf.data_ptr() % align:
                buf = aligned_empty(size, torch.uint8, dev, align)
            buf.copy_(stage[:size], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
            self._stage_events[g % 2] = ev
            for (m, layout), span in zip(group, spans):
                arenas = {dt: buf[o:o + n * esz].view(dt) for dt, (o, n, esz) in span.items()}
                cache[id(m)] = (m, layout, arenas)

    def _aggregate_wave(self, aggs, on_launched=None) -> List[nn.Module]:
        """One batched aggregate per dtype over the wave's tasks. on_launched:
        see batch.aggregate_arena_tasks (the executor releases the results
        no later task reads there, so the input modules are freed while the
        output modules are built)."""
        cache: dict = {}
        prepared = []
        resolved = []
        for name, _, data in aggs:
            d = self._resolve(data)
            models = d["models"]
            ws = _resolve(models, d.get("weights"))  # fedavg.py:14-17 rules and exceptions
            resolved.append((models, ws))
        walked: dict = {}
        self._upload_host_models([m for models, _ in resolved for m in models], cache, walked)
        single = {}  # task position -> result of the per-parameter zip path
        for j, (models, ws) in enumerate(resolved):
            ents = [self._arena_of(m, cache, walked) for m in models]
            layout0 = ents[0][0]
            sig = layout0._signature
            try:
                for i in range(1, len(ents)):
                    lay = ents[i][0]
                    if lay._signature is not sig and lay._signature != sig:
                        layout0.check_compatible(models[i])
            except ZipMismatch:  # parameter lists differ (fedavg.py:23-24 zip)
                single[j] = aggregate_modules(models, ws, self.mode, to_host=False)
                continue
            views = {dt: [a[dt] for _, a in ents] for dt in layout0.groups}
            prepared.append((models[0], layout0, views, ws, [lay.params for lay, _ in ents]))
        n_tasks = len(resolved)
        resolved.clear()
        cache.clear()
        walked.clear()
        outs = aggregate_arena_tasks(prepared, self.mode, on_launched)
        if not single:
            return outs
        it = iter(outs)
        return [single[j] if j in single else next(it) for j in range(n_tasks)]

    def run(self, tasks: Sequence[Task], seed: Optional[Dict[str, list]] = None) -> Dict[str, list]:
        """Execute `tasks`; `seed` pre-populates results (e.g. initial models).
        Returns {task_name: result list}: every result (keep_all), else the
        results no task of `tasks` reads (the DAG's sinks, e.g. the last
        round's aggregates) and the seeds none of them reads."""
        if seed:
            self.results.update(seed)
        pending = list(tasks)
        names = {t[0] for t in pending}
        readers: Dict[str, int] = {}
        for t in pending:
            for r in set(_refs(t[2], [])):
                readers[r] = readers.get(r, 0) + 1
        while pending:
            ready = [t for t in pending
                     if all(r in self.results for r in _refs(t[2], []))]
            if not ready:
                missing = sorted({r for t in pending for r in _refs(t[2], [])
                                  if r not in self.results and r not in names})
                raise RuntimeError(f"unresolvable task inputs: {missing[:5]}")
            aggs = [t for t in ready if t[1] == "aggregate"]
            dying: List[str] = []  # results no task after this wave reads
            if not self.keep_all:
                for t in ready:
                    for r in set(_refs(t[2], [])):
                        readers[r] -= 1
                        if readers[r] == 0:
                            dying.append(r)

            def release():
                for r in dying:
                    res = self.results.pop(r, None)
                    if self.foreign_streams and res is not None:
                        _record_on_current_stream(res)
                dying.clear()
            t0 = time.perf_counter()
            for name, func, data in ready:
                if func == "aggregate":
                    continue
                res = self.funcs[func](self.settings, self._resolve(data))
                assert isinstance(res, (list, tuple))  # broker.py:282-283
                self.results[name] = list(res)
            if self.timing and torch.cuda.is_available():
                torch.cuda.synchronize()
            t1 = time.perf_counter()
            if aggs:
                outs = self._aggregate_wave(aggs, release if self.release_early else None)
                for (name, _, _), out in zip(aggs, outs):
                    self.results[name] = [out]
                if self.timing:
                    torch.cuda.synchronize()
            if self.timing:
                t2 = time.perf_counter()
                self.stats["other"] += t1 - t0
                self.stats["aggregate"] += t2 - t1
                self.stats["aggregate_tasks"] += len(aggs)
            done = {t[0] for t in ready}
            self.waves.append(sorted(done))
            release()
            pending = [t for t in pending if t[0] not in done]
        return self.results


def _record_on_current_stream(objs) -> None:
    """Tensor.record_stream(current stream) on every device parameter of the
    modules (and device tensors) in `objs` (RoundExecutor foreign_streams)."""
    for o in objs:
        ts = module_params(o) if isinstance(o, nn.Module) else [o] if isinstance(o, torch.Tensor) else []
        for t in ts:
            if t.is_cuda:
                t.record_stream(torch.cuda.current_stream(t.device))
