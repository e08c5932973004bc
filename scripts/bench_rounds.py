"""Wall time of the aggregate work of simulated D-PSGD rounds (SURVEY.md §8f
row 4): the reference's DAG shape (every peer trains, then aggregates its k
ring neighbours' models and its own, dasklearn/simulation/dpsgd/client.py:
142-151; fan-in k+1 with k = floor(log2 n)), GNLeNet-shaped models.

Three ways of running the same aggregate tasks:
  batched     RoundExecutor: each wave's aggregates in batched launches over
              device-resident arenas (dasklearn_amd/rounds.py)
  sequential  one functions.aggregate call per task, as the reference worker
              does (worker.py:27-31), models on the device
  cpu_ref     the reference's FedAvg.aggregate op sequence (oracle restatement)
              per task on host models at the worker's 4 threads (broker.py:31)
The train task is a synthetic device-side perturbation (the real one needs
network datasets; out of scope) and is not counted. With --host it returns a
host model instead (the reference's CPU training, model_trainer.py:129), so
every aggregate reads host models: the executor uploads each wave's models
once, the sequential worker loop stages them per task.

    python scripts/bench_rounds.py [--peers 100] [--rounds 4] [--host] [--model gnlenet|flat|resnet18]

BASELINE.json configs[0] (cfg1: the 2-peer D-PSGD average of the default
CIFAR-10 model, tests/test_dpsgd.py:26-35) is `--peers 2 --host`: every
aggregate is functions.aggregate of 2 host GNLeNet modules, the reference's
own worker path (functions.py:89-106), against its op sequence at 4 threads.
"""
from __future__ import annotations

import argparse
import copy
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
from torch import nn  # noqa: E402

GNLENET = [(32, 3, 5, 5), (32,), (32,), (32,), (32, 32, 5, 5), (32,), (32,), (32,), (64, 32, 5, 5),
           (64,), (64,), (64,), (10, 576), (10,)]


class Shaped(nn.Module):
    def __init__(self, shapes):
        super().__init__()
        self.ps = nn.ParameterList([nn.Parameter(torch.randn(*s) * 0.05) for s in shapes])


class GNLeNetTree(nn.Module):
    """The module tree of the reference's default model (GNLeNet,
    dasklearn/models/cifar10.py:103-136, on models/Model.py's attributes):
    16 modules, 14 parameters in GNLENET's order. The per-task host cost of
    both the reference (deepcopy of models[0]) and this package (its clone)
    grows with the module count, so the round is timed on this tree."""

    def __init__(self):
        super().__init__()
        self.model_change = self._param_count_ot = self._param_count_total = None
        self.accumulated_changes = self.shared_parameters_counter = self.gradient = None
        self.input_channel, self.output, self.model_input, self.classifier_input = 3, 10, (24, 24), 576
        self.features = nn.Sequential(
            nn.Conv2d(3, 32, 5, 1, 2), nn.MaxPool2d(3, 2), nn.GroupNorm(2, 32), nn.ReLU(True),
            nn.Conv2d(32, 32, 5, 1, 2), nn.GroupNorm(2, 32), nn.MaxPool2d(3, 2), nn.ReLU(True),
            nn.Conv2d(32, 64, 5, 1, 2), nn.GroupNorm(2, 64), nn.MaxPool2d(3, 2), nn.ReLU(True))
        self.classifier = nn.Sequential(nn.Linear(576, 10))


def resnet18_shapes():
    from bench import resnet18_shapes as shapes
    return shapes()


def model_shapes(kind):
    return resnet18_shapes() if kind == "resnet18" else GNLENET


def make_model(kind):
    if kind == "gnlenet":
        return GNLeNetTree()
    return Shaped(model_shapes(kind))


class Settings:
    from dasklearn_amd.gradient_aggregation import GradientAggregationMethod
    gradient_aggregation = GradientAggregationMethod.FEDAVG


def ring(n, k):
    nb = {}
    for p in range(n):
        s = set()
        for d in range(1, k // 2 + 1):
            s.add((p + d) % n)
            s.add((p - d) % n)
        if k % 2:
            s.add((p + k // 2 + 1) % n)
        s.discard(p)
        nb[p] = sorted(s)
    return nb


def dag(n, rounds):
    k = min(max(1, math.floor(math.log2(n))), n - 1)
    nb = ring(n, k)
    tasks = []
    for r in range(1, rounds + 1):
        for p in range(n):
            model = ("init", 0) if r == 1 else (f"agg_{p}_{r - 1}", 0)
            tasks.append((f"train_{p}_{r}", "train", {"model": model, "round": r, "peer": p}))
        for p in range(n):
            models = [(f"train_{q}_{r}", 0) for q in nb[p]] + [(f"train_{p}_{r}", 0)]
            tasks.append((f"agg_{p}_{r}", "aggregate", {"models": models, "round": r, "peer": p}))
    return tasks, k + 1


def train(settings, params):
    out = copy.deepcopy(params["model"])
    with torch.no_grad():
        for p in out.parameters():
            p.add_(1e-3 * (params["peer"] + 1))
    return [out]


def train_host(settings, params):
    out = copy.deepcopy(params["model"]).cpu()
    with torch.no_grad():
        for p in out.parameters():
            p.add_(1e-3 * (params["peer"] + 1))
    if SHM:  # as the worker's result crosses to the broker: file_system shared memory (worker.py:6)
        out.share_memory()
    return [out]


SHM = False


def resolve(results, v):
    if isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], str):
        return results[v[0]][v[1]]
    if isinstance(v, list):
        return [resolve(results, x) for x in v]
    return v


class GCMeter:
    """Python's cyclic collector inside the timed regions (gc.callbacks): its
    pauses are charged to whatever code allocates when a threshold trips, and
    their length grows with every container object the process keeps alive,
    so the lines report them beside the per-task time."""

    def __init__(self):
        self.active = False
        self.seconds = 0.0
        self.collections = [0, 0, 0]
        self._t0 = None

    def __call__(self, phase, info):
        if phase == "start":
            self._t0 = time.perf_counter()
        elif self._t0 is not None:
            if self.active:
                self.seconds += time.perf_counter() - self._t0
                self.collections[info["generation"]] += 1
            self._t0 = None

    def reset(self):
        self.seconds, self.collections = 0.0, [0, 0, 0]


GC = GCMeter()


def _reads(v, out):
    if isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], str):
        out.add(v[0])
    elif isinstance(v, list):
        for x in v:
            _reads(x, out)
    return out


def sequential(tasks, agg_fn, init, sync, train_fn=None):
    """The worker's one-task-at-a-time loop; only aggregate calls are timed.
    A result is dropped once every task reading it has run (the broker
    clears a completed task's data, broker.py:221), so the process holds the
    DAG's frontier, like the reference's broker and workers, not every model
    of the run."""
    train_fn = train_fn or train
    results = {"init": [init]}
    reads = [_reads(list(data.values()), set()) for _, _, data in tasks]
    left = {}
    for rs in reads:
        for r in rs:
            left[r] = left.get(r, 0) + 1
    t_agg, n_agg = 0.0, 0
    for (name, f, data), rs in zip(tasks, reads):
        d = {k: resolve(results, v) for k, v in data.items()}
        if f == "aggregate":
            sync()
            GC.active = True
            t0 = time.perf_counter()
            results[name] = agg_fn(Settings(), d)
            sync()
            t_agg += time.perf_counter() - t0
            GC.active = False
            n_agg += 1
        else:
            results[name] = train_fn(Settings(), d)
        del d
        for r in rs:
            left[r] -= 1
            if left[r] == 0:
                del results[r]
    return t_agg, n_agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--cpu-rounds", type=int, default=2)
    ap.add_argument("--host", action="store_true", help="train returns host models (CPU training)")
    ap.add_argument("--model", choices=("gnlenet", "flat", "resnet18"), default="gnlenet",
                    help="gnlenet: the reference's module tree; flat: the same 14 tensors in one ParameterList; "
                         "resnet18: the north star's 62 ResNet-18 parameter tensors in one ParameterList")
    ap.add_argument("--release-late", action="store_true",
                    help="RoundExecutor drops a wave's inputs after the wave (release_early=False)")
    ap.add_argument("--flatten", action="store_true",
                    help="RoundExecutor copies device-trained models into arenas first (tensors_in_place=False)")
    ap.add_argument("--shm", action="store_true",
                    help="with --host: trained models move to torch.multiprocessing file_system shared memory, as a "
                         "reference worker's results do (the device model cache keys on it; DLSIM_DEVICE_CACHE_MB)")
    ap.add_argument("--profile", default=None, help="cProfile the batched run into this file")
    ap.add_argument("--profile-seq", default=None, help="cProfile the sequential run into this file")
    ap.add_argument("--reps", type=int, default=3,
                    help="repetitions of each way, interleaved; the line reports the median and the best "
                         "(Python's collector runs at times set by the objects the whole run keeps alive)")
    a = ap.parse_args()
    global SHM
    SHM = a.shm
    if a.shm:
        torch.multiprocessing.set_sharing_strategy("file_system")
    from dasklearn_amd.functions import aggregate
    from dasklearn_amd.rounds import RoundExecutor
    from oracle import fedavg_torch

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    init_h = make_model(a.model)
    shapes = model_shapes(a.model)
    assert [tuple(q.shape) for q in init_h.parameters()] == [tuple(s) for s in shapes]
    init_d = copy.deepcopy(init_h).to(dev)
    tasks, fan = dag(a.peers, a.rounds)
    p = sum(int(torch.Size(s).numel()) for s in shapes)
    task_bytes = (fan + 1) * p * 4
    sync = torch.cuda.synchronize

    tr = train_host if a.host else train
    init_x = init_h if a.host else init_d
    # warm-up at full size (library load, kernels, and the device and pinned
    # allocator caches for a wave's buffers, so the timed rounds are steady state)
    wt, _ = dag(a.peers, 1)
    RoundExecutor({"train": tr}, Settings(), device=dev, tensors_in_place=not a.flatten,
                  release_early=not a.release_late).run(
        wt, seed={"init": [init_x]})
    sequential(wt, aggregate, init_x, sync, tr)

    def run_batched(profile=None):
        ex = RoundExecutor({"train": tr}, Settings(), device=dev, timing=True, tensors_in_place=not a.flatten,
                           release_early=not a.release_late)
        wave = ex._aggregate_wave

        def metered(aggs, *rest):  # the executor times the wave plus a sync
            GC.active = True
            try:
                return wave(aggs, *rest)
            finally:
                GC.active = False
        ex._aggregate_wave = metered
        if profile:
            import cProfile
            import pstats
            prof = cProfile.Profile()
            prof.enable()
            ex.run(tasks, seed={"init": [init_x]})
            prof.disable()
            with open(profile, "w") as f:
                pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(45)
        else:
            ex.run(tasks, seed={"init": [init_x]})
        return ex.stats["aggregate"], ex.stats["aggregate_tasks"]

    def run_sequential(profile=None):
        if profile:
            import cProfile
            import pstats
            prof = cProfile.Profile()
            prof.enable()
            r = sequential(tasks, aggregate, init_x, sync, tr)
            prof.disable()
            with open(profile, "w") as f:
                pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(45)
            return r
        return sequential(tasks, aggregate, init_x, sync, tr)

    def cpu_agg(settings, d):
        return [fedavg_torch.aggregate_modules(d["models"], d.get("weights"))]

    ctasks, _ = dag(a.peers, a.cpu_rounds)

    def run_cpu():
        prev = torch.get_num_threads()
        torch.set_num_threads(4)
        try:
            return sequential(ctasks, cpu_agg, init_h, lambda: None)
        finally:
            torch.set_num_threads(prev)

    import gc
    import statistics
    if a.profile:  # profiled passes are not timed
        run_batched(a.profile)
    if a.profile_seq:
        run_sequential(a.profile_seq)
    samples = {"batched": [], "sequential": [], "cpu_ref_4threads": []}
    gc_s = {k: [] for k in samples}
    gc_n = {k: [0, 0, 0] for k in samples}
    gc.callbacks.append(GC)
    for _ in range(max(1, a.reps)):
        for kind, fn in (("batched", run_batched), ("sequential", run_sequential), ("cpu_ref_4threads", run_cpu)):
            gc.collect()
            GC.reset()
            t, n = fn()
            samples[kind].append(t / n)
            gc_s[kind].append(GC.seconds / n)
            gc_n[kind] = [x + y for x, y in zip(gc_n[kind], GC.collections)]
    gc.callbacks.remove(GC)

    def line(kind):
        per = statistics.median(samples[kind])
        return {"kind": kind + ("_host_models" if a.host and not kind.startswith("cpu") else "")
                + ("_flatten" if a.flatten and kind == "batched" else "")
                + ("_release_late" if a.release_late and kind == "batched" else ""), "model": a.model,
                "peers": a.peers,
                "fan_in": fan, "reps": len(samples[kind]), "params": p,
                "ms_per_round": round(per * a.peers * 1e3, 3), "us_per_task": round(per * 1e6, 1),
                "us_per_task_best": round(min(samples[kind]) * 1e6, 1),
                "us_per_task_all": [round(x * 1e6, 1) for x in samples[kind]],
                "GBps_algorithmic": round(task_bytes / per / 1e9, 2),
                "gc_us_per_task": round(statistics.median(gc_s[kind]) * 1e6, 1),
                "us_per_task_excl_gc": round(statistics.median([t - g for t, g in zip(samples[kind], gc_s[kind])])
                                             * 1e6, 1),
                "gc_collections_by_generation": gc_n[kind]}

    from bench import box_info
    from dasklearn_amd import device_cache
    box = box_info()
    extra = {"shm_models": a.shm}
    if device_cache.active() is not None:
        extra["device_cache"] = dict(device_cache.active().stats, capacity=device_cache.active().capacity)
    for kind in samples:
        print(json.dumps(dict(line(kind), box=box, **extra)), flush=True)


if __name__ == "__main__":
    main()
