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

Models that reach an aggregate are uploaded once each into a device arena
(`to_device_arena`), so an aggregate -> train -> aggregate chain never
crosses PCIe when the train function works on the device. Results are
bit-identical to running the same tasks one by one with FedAvg.aggregate.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
from torch import nn

from . import _native
from .arena import ParamLayout, to_device_arena
from .batch import aggregate_batch

Task = Tuple[str, str, dict]  # (task_name, func_name, data with placeholders)


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
                 mode: int = _native.DLSIM_EXACT):
        self.funcs = dict(funcs)
        self.settings = settings
        self.device = device
        self.mode = mode
        self.results: Dict[str, list] = {}
        self.waves: List[List[str]] = []
        self._resident: Dict[int, nn.Module] = {}

    def _resolve(self, v):
        if _is_ref(v):
            return self.results[v[0]][v[1]]
        if isinstance(v, list):
            return [self._resolve(x) for x in v]
        if isinstance(v, dict):
            return {k: self._resolve(x) for k, x in v.items()}
        return v

    def _resident_model(self, m: nn.Module) -> nn.Module:
        """Device-arena form of `m` (uploaded once per object)."""
        layout = ParamLayout(m)
        params = layout.params
        if params and all(p.is_cuda for p in params) and all(
                layout.arena_view(params, dt) is not None for dt in layout.groups):
            return m
        key = id(m)
        if key not in self._resident:
            self._resident[key] = to_device_arena(m, self.device)
        return self._resident[key]

    def run(self, tasks: Sequence[Task], seed: Optional[Dict[str, list]] = None) -> Dict[str, list]:
        """Execute `tasks`; `seed` pre-populates results (e.g. initial models).
        Returns {task_name: result list}."""
        if seed:
            self.results.update(seed)
        pending = list(tasks)
        names = {t[0] for t in pending}
        while pending:
            ready = [t for t in pending
                     if all(r in self.results for r in _refs(t[2], []))]
            if not ready:
                missing = sorted({r for t in pending for r in _refs(t[2], [])
                                  if r not in self.results and r not in names})
                raise RuntimeError(f"unresolvable task inputs: {missing[:5]}")
            aggs = [t for t in ready if t[1] == "aggregate"]
            for name, func, data in ready:
                if func == "aggregate":
                    continue
                res = self.funcs[func](self.settings, self._resolve(data))
                assert isinstance(res, (list, tuple))  # broker.py:282-283
                self.results[name] = list(res)
            if aggs:
                batch = []
                for name, _, data in aggs:
                    d = self._resolve(data)
                    models = [self._resident_model(m) for m in d["models"]]
                    batch.append((models, d.get("weights")))
                outs = aggregate_batch(batch, self.mode)
                for (name, _, _), out in zip(aggs, outs):
                    self.results[name] = [out]
            done = {t[0] for t in ready}
            self.waves.append(sorted(done))
            pending = [t for t in pending if t[0] not in done]
        return self.results
