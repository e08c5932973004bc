"""The per-worker device model cache (dasklearn_amd/device_cache.py; SURVEY.md
§8f row 1) on MI355X.

Host models whose parameters live in torch.multiprocessing file_system shared
memory (what a reference worker receives, worker.py:6) are uploaded once per
process and read from the device on later aggregates; every result stays
bit-identical to the oracle's fold (fedavg.py:20-25), hits or not. In one
process here, and through the reference's broker/worker process model
(tests/_broker_child.py in cache mode: a forked worker that receives the same
models in several tasks)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as tmp
from torch import nn

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


class Net(nn.Module):
    def __init__(self, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.conv = nn.Conv2d(3, 16, 5)
        self.fc = nn.Linear(400, 10)
        with torch.no_grad():
            for q in self.parameters():
                q.copy_(torch.randn(q.shape, generator=g) * 0.05)


def flat(m):
    return torch.cat([q.detach().reshape(-1) for q in m.parameters()]).numpy()


@pytest.fixture()
def shm_models():
    prev = tmp.get_sharing_strategy()
    tmp.set_sharing_strategy("file_system")
    try:
        ms = [Net(s) for s in range(9)]
        for m in ms:
            m.share_memory()
        yield ms
    finally:
        tmp.set_sharing_strategy(prev)


@pytest.fixture()
def cache():
    from dasklearn_amd import device_cache
    prev = device_cache.active()
    c = device_cache.enable(64 << 20)
    yield c
    if prev is None:
        device_cache.disable()
    else:
        device_cache._CACHE = prev


def _check(models, weights):
    from dasklearn_amd.gradient_aggregation.fedavg import FedAvg
    out = FedAvg.aggregate(models, weights)
    assert not any(q.is_cuda for q in out.parameters())
    exp = orc.wreduce([flat(m) for m in models], orc.reference_weights(len(models), weights), "f32")
    assert orc.same_bits(flat(out), exp)


def test_cache_hits_are_bit_exact(shm_models, cache):
    ms = shm_models
    _check(ms[:7], None)
    assert cache.stats["misses"] == 7 and cache.stats["hits"] == 0 and len(cache) == 7
    _check(ms[:7], [0.1, 0.2, 0.1, 0.2, 0.1, 0.2, 0.1])
    assert cache.stats["hits"] == 7
    _check([ms[8], ms[0], ms[7], ms[3]], None)  # two new, two resident, in another order
    assert cache.stats["hits"] == 9 and cache.stats["misses"] == 9
    row_bytes = sum(q.numel() for q in ms[0].parameters()) * 4
    assert cache.stats["bytes_not_sent"] == 9 * row_bytes


def test_non_shared_models_take_the_normal_pipeline(cache):
    ms = [Net(s) for s in range(3)]  # private host memory: no identity across tasks
    _check(ms, None)
    _check(ms, None)
    assert cache.stats["hits"] == 0 and len(cache) == 0


def test_eviction_keeps_results_exact(shm_models):
    """A cache with room for three rows: the first task caches three of five
    models (the rest take transient rows), the next reads them and cannot
    evict them, a task of new models evicts and reuses their slots; every
    result exact."""
    from dasklearn_amd import arena, device_cache
    ms = shm_models
    row = arena.row_stride(sum(q.numel() for q in ms[0].parameters()), 4) * 4
    c = device_cache.enable(3 * row)  # room for three models
    try:
        _check(ms[:5], None)
        assert len(c) == 3 and c.stats["misses"] == 5 and c.slab_bytes == 3 * row
        _check(ms[:5], None)  # three resident, two sent again (no slot may be taken from this task)
        assert c.stats["hits"] == 3 and c.stats["evictions"] == 0
        _check(ms[4:9], [0.3, 0.2, 0.2, 0.2, 0.1])
        assert c.stats["evictions"] == 3 and c.slab_bytes == 3 * row
    finally:
        device_cache.disable()


@pytest.mark.parametrize("method", ["fork", "spawn"])
def test_worker_process_cache(method):
    """The broker/worker process model with the cache on in the worker: the
    second worker's three tasks send 7 models and read 5 from its cache, all
    results exact."""
    r = subprocess.run([sys.executable, os.path.join(HERE, "_broker_child.py"), method, "cache"],
                       capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-3000:]
    out = json.loads(lines[-1])
    assert all(out["checks"].values()), out
    assert out["cache_stats"]["hits"] == 5 and out["cache_stats"]["misses"] == 7, out["cache_stats"]
    assert out["ok"] and r.returncode == 0, out


def test_calls_on_two_streams_stay_ordered(shm_models):
    """Two threads' streams taking turns on one cache: each call waits for the
    other stream's reads and fills of the rows (DeviceModelCache.order); a
    slot evicted on one stream is refilled on the other only after the first
    stream's reads, so every result stays exact."""
    from dasklearn_amd import arena, device_cache
    ms = shm_models
    row = arena.row_stride(sum(q.numel() for q in ms[0].parameters()), 4) * 4
    c = device_cache.enable(4 * row)  # room for four rows: the alternation evicts
    try:
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        sets = [ms[0:4], ms[4:8], ms[2:6], ms[5:9], ms[0:3] + [ms[8]]]
        for k, group in enumerate(sets * 2):
            with torch.cuda.stream(streams[k % 2]):
                _check(group, None)
        assert c.stats["evictions"] > 0 and c.stats["hits"] > 0
    finally:
        device_cache.disable()


def test_non_contiguous_shared_parameters(cache):
    """A shm model with a transposed parameter: misses are copied to a
    contiguous row first; a task whose models are all resident needs no
    pointers at all (fuzz_parity 'cached' found this case); exact."""
    prev = tmp.get_sharing_strategy()
    tmp.set_sharing_strategy("file_system")
    try:
        ms = []
        for s in range(3):
            m = Net(s)
            m.fc.weight = nn.Parameter(m.fc.weight.detach().t().contiguous().t())  # same shape, transposed layout
            assert not m.fc.weight.is_contiguous()
            m.share_memory()
            ms.append(m)
        _check(ms, None)
        _check(ms, [0.5, 0.25, 0.25])  # every model resident
        _check([ms[2], ms[2], ms[0]], None)  # a duplicate, all resident
        assert cache.stats["hits"] == 6 and cache.stats["misses"] == 3
    finally:
        tmp.set_sharing_strategy(prev)


def test_a_model_written_in_place_is_not_served_stale(shm_models, cache):
    """a cached model trained in place afterwards (the
    reference trains its input model in place, functions.py:57) no longer
    matches its entry's content fingerprint: the entry is dropped, the model
    sent again, and the result is the new model's, exact."""
    ms = shm_models
    _check(ms[:4], None)
    assert cache.stats["misses"] == 4
    with torch.no_grad():
        for q in ms[1].parameters():
            q.add_(0.01)  # an SGD-like update of every element, same shm storage
    _check(ms[:4], None)
    assert cache.stats["stale"] == 1 and cache.stats["hits"] == 3 and cache.stats["misses"] == 5
    _check(ms[:4], [0.4, 0.3, 0.2, 0.1])  # the re-sent row is cached again
    assert cache.stats["hits"] == 7 and cache.stats["stale"] == 1


class DeepNet(nn.Module):
    """26 parameter tensors: more than round 5's fingerprint sampled (8)."""

    def __init__(self, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.body = nn.Sequential(*[nn.Linear(32, 32) for _ in range(12)], nn.Linear(32, 1000))
        with torch.no_grad():
            for q in self.parameters():
                q.copy_(torch.randn(q.shape, generator=g) * 0.05)


def test_a_rewritten_middle_tensor_is_not_served_stale(cache):
    """a cached model one of whose MIDDLE tensors alone is
    rewritten in place (a partial fine-tune; round 5's guard sampled 8 of 26
    tensors and not this one) is caught by the fingerprint of every tensor:
    the entry is dropped ("stale"), the model re-sent, the result exact."""
    prev = tmp.get_sharing_strategy()
    tmp.set_sharing_strategy("file_system")
    try:
        ms = [DeepNet(s) for s in range(4)]
        for m in ms:
            m.share_memory()
        assert len(list(ms[0].parameters())) == 26
        _check(ms, None)
        assert cache.stats["misses"] == 4 and cache.stats["stale"] == 0
        _check(ms, None)
        assert cache.stats["hits"] == 4
        with torch.no_grad():
            list(ms[2].parameters())[13].mul_(0.5)  # layer 6's bias only, same shm storage
        _check(ms, [0.1, 0.2, 0.3, 0.4])
        assert cache.stats["stale"] == 1 and cache.stats["hits"] == 7 and cache.stats["misses"] == 5
    finally:
        tmp.set_sharing_strategy(prev)
