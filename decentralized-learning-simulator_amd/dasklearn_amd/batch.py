"""Batched aggregation: many independent `aggregate` tasks in few launches.

In a simulated round every peer aggregates its neighbours' models
(dasklearn/simulation/dpsgd/client.py:142-151); the broker schedules those
tasks one by one (broker.py:261-275), so each is one call of
functions.aggregate (functions.py:89-106). For small models (GNLeNet: 3 MB
per 8-way task) one launch per task is launch-bound; `aggregate_batch` runs
the tasks that are ready together through `dlsim_wreduce_batched` (up to 32
tasks / 192 inputs per launch). Results are bit-identical to calling
FedAvg.aggregate on each task.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
from torch import nn

from . import _native
from .arena import ZipMismatch, aggregate_modules, arena_empty, input_arenas, module_from_arenas


def _resolve(models, weights) -> List[float]:
    # fedavg.py:14-17 rules, same exceptions; the Python floats (each dtype
    # group rounds them as the reference's op does: _native.weights_for_dtype)
    if not weights:
        weights = [float(1. / len(models)) for _ in range(len(models))]
    else:
        assert len(weights) == len(models)
    return [float(w) for w in weights]


def aggregate_batch(tasks: Sequence[Tuple[List[nn.Module], Optional[Sequence[float]]]],
                    mode: int = _native.DLSIM_EXACT) -> List[nn.Module]:
    """tasks: [(models, weights)] -> one aggregated module per task.

    Tasks whose models are device-resident arenas (what this package returns
    for device inputs) are reduced together in batched launches; any other
    task goes through the single-task path. Output placement follows
    FedAvg.aggregate (where models[0] lives)."""
    results: List[Optional[nn.Module]] = [None] * len(tasks)
    prepared, where = [], []
    for ti, (models, weights) in enumerate(tasks):
        ws = _resolve(models, weights)
        model0 = models[0]  # IndexError for an empty task, as the reference
        try:
            layout, _, views = input_arenas(models)
        except ZipMismatch:  # parameter lists differ: the per-parameter zip path
            layout, views = None, None
        if _device_views(views) is None:
            results[ti] = aggregate_modules(models, weights, mode)
            continue
        prepared.append((model0, layout, views, ws))
        where.append(ti)
    for ti, out in zip(where, aggregate_arena_tasks(prepared, mode)):
        results[ti] = out
    return results


def _device_views(views) -> Optional[torch.device]:
    """The one CUDA device every flat view lives on, or None."""
    dev = None
    if not views:
        return None
    for vs in views.values():
        if vs is None:
            return None
        for v in vs:
            if not v.is_cuda or (dev is not None and v.device != dev):
                return None
            dev = v.device
    return dev


def _row_on(params, view, idx, sizes, dev):
    """Model i's tensors of a dtype group as the rows path reads them: its
    parameters when they are on `dev` (read in place; a registered arena's
    parameters are views of it), else the pieces of its flat view (an arena
    uploaded or copied to `dev`, e.g. a host model of the wave)."""
    if view is None or params[idx[0]].device == dev:
        return params
    row = [None] * len(params)
    for k, piece in zip(idx, view.split(sizes)):
        row[k] = piece
    return row


def _rows_device(vs, rows, layout, dt) -> torch.device:
    """The task's device: that of its flat views, or (none) of the first
    model read in place (its tensors are on the target device by
    construction, RoundExecutor._arena_of)."""
    for v in vs:
        if v is not None:
            return v.device
    t = rows[0][layout.groups[dt][0]]
    if not t.is_cuda:
        raise ValueError("rows input: tensors must be on a CUDA device")
    return t.device


def aggregate_arena_tasks(prepared, mode: int = _native.DLSIM_EXACT,
                          on_launched: Optional[Callable[[], None]] = None) -> List[nn.Module]:
    """prepared: [(model0, layout of model0, {dtype: [flat arena per model]},
    weights as Python floats[, rows])] with every arena on one device -> one
    module per task (deepcopy(model0) semantics, parameters views of a fresh
    output arena), all tasks of a dtype and device in batched launches (fp64
    groups: one dlsim_wreduce_f64 per task).

    rows (optional): every model's parameter list. A dtype group whose arena
    list holds None (a model that keeps its parameters in separate device
    tensors, e.g. a device train task's deepcopy) is read from those tensors
    in place: every such task's tensors in one dlsim_wreduce_batched call per
    dtype and device (one sub-task per tensor, pointers collected in C),
    instead of copying each such model into an arena first.

    on_launched: called once every launch is queued, before the output
    modules are built; the list `prepared` is consumed while they are (each
    entry set to None once its module exists). A caller that drops its own
    references to the input modules there lets them go as the outputs are
    made: the arenas stay alive through the launch views, and the stream
    orders any reuse of their memory after the kernels."""
    by_dtype = {}
    by_rows = {}
    outs = []
    for entry in prepared:
        model0, layout, views, ws = entry[:4]
        o = {}
        for dt, vs in views.items():
            if any(v is None for v in vs):
                rows = entry[4]
                dev = _rows_device(vs, rows, layout, dt)
                out = arena_empty(layout.totals[dt], dt, dev)
                o[dt] = out
                idx = layout.groups[dt]
                rows = [_row_on(rows[i], v, idx, layout.split_sizes[dt], dev) for i, v in enumerate(vs)]
                by_rows.setdefault((dt, dev), []).append(
                    ((rows, idx, layout.split_sizes[dt], _native.weights_for_dtype(ws, dt), out.data_ptr(),
                      layout.byte_offsets[dt]), vs, out))
                continue
            dev = vs[0].device
            out = arena_empty(layout.totals[dt], dt, dev)
            o[dt] = out
            by_dtype.setdefault((dt, dev), []).append((vs, _native.weights_for_dtype(ws, dt), out))
        outs.append(o)
    for (dt, dev), group in by_rows.items():
        # every task read from separate tensors: one library call for all
        stream = torch.cuda.current_stream(dev)
        code = _native.dtype_code(dt)
        if _native.wreduce_rows_multi([g[0] for g in group], code, mode, stream.cuda_stream, dev.index):
            continue
        for (rows, idx, sizes, w, out_ptr, offs), vs, out in group:
            if not _native.wreduce_rows(rows, idx, sizes, w, out_ptr, offs, code, mode, stream.cuda_stream, dev.index):
                # a model's tensors are elsewhere (its arena was copied
                # here): flatten the in-place ones too, one reduce
                with torch.no_grad():
                    flat = [v if v is not None else
                            torch._C._nn.flatten_dense_tensors([rows[i][k] for k in idx]).to(dev)
                            for i, v in enumerate(vs)]
                _native.wreduce(flat, w, out, mode, stream)
    by_rows.clear()
    for (dt, dev), group in by_dtype.items():
        stream = torch.cuda.current_stream(dev)
        if dt == torch.float64:
            for vs, w, out in group:
                _native.wreduce(vs, w, out, mode, stream)
            continue
        _native.wreduce_batched(group, mode, stream)
    by_dtype.clear()
    if on_launched is not None:
        on_launched()
    mods = []
    for i, o in enumerate(outs):
        model0, layout = prepared[i][:2]
        prepared[i] = None
        mods.append(module_from_arenas(model0, layout, o))
    return mods
