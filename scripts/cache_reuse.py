"""How often would a per-worker device model cache hit? (VERDICT r03 next #7;
SURVEY.md §8f row 1.) CPU-only replay of the broker's dispatch.

The reference broker puts every ready task on ONE shared multiprocessing
queue (broker.py:259-272 put_in_worker_queue / schedule_task) and each of W
worker processes takes the next task when it is free (worker.py:21-38); a
task becomes ready when its last input arrives (broker.py:277-290,
task.py:26-51). Results travel as host modules through torch's file_system
shared memory (worker.py:6): a worker that receives model M for an aggregate
maps M's storages afresh, and a device cache keyed by the storage handle
would skip M's pack and H2D if this worker had uploaded M before.

The replay: the D-PSGD DAG of scripts/bench_rounds.py (the reference's
shape: every peer trains, then aggregates its k ring neighbours' models and
its own, k = floor(log2 n); dpsgd/client.py:142-151), an event simulation
of W workers on a FIFO queue with train and aggregate durations drawn around
the given means (seeded jitter), and per aggregate input the question "has
this worker held this model before":
  hit_upload   an earlier aggregate on this worker uploaded it
  hit_producer this worker trained it (only a cache filled by the train task
               would have it: the reference's trainer returns a host model,
               model_trainer.py:129)
Prints one JSON line per (n, W, duration ratio) case: the fraction of input
models (= of H2D bytes, all models being the same size) each kind of hit saves.

    python scripts/cache_reuse.py [--peers 100] [--workers 4] [--rounds 6]
"""
from __future__ import annotations

import argparse
import heapq
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from bench_rounds import dag  # noqa: E402  (the reference's D-PSGD DAG shape)


def replay(n, workers, rounds, train_ms, agg_ms, jitter, seed):
    tasks, fan = dag(n, rounds)
    rng = random.Random(seed)
    by_name = {name: (f, data) for name, f, data in tasks}
    inputs = {}
    consumers = {}
    for name, f, data in tasks:
        deps = [m[0] for m in data["models"]] if f == "aggregate" else \
            ([data["model"][0]] if data["model"][0] != "init" else [])
        inputs[name] = deps
        for d in deps:
            consumers.setdefault(d, []).append(name)
    waiting = {name: len(deps) for name, deps in inputs.items()}
    queue = [name for name, _, _ in tasks if waiting[name] == 0]  # FIFO of ready tasks
    qpos = 0
    free = list(range(workers))
    events = []  # (finish time, seq, worker, task)
    seq = 0
    now = 0.0
    producer = {}
    held = [set() for _ in range(workers)]  # models each worker has uploaded
    n_in = hit_up = hit_prod = hit_any = 0
    while qpos < len(queue) or events:
        while free and qpos < len(queue):
            w = free.pop(0)
            t = queue[qpos]
            qpos += 1
            f, data = by_name[t]
            if f == "aggregate":
                for m in inputs[t]:
                    n_in += 1
                    up = m in held[w]
                    pr = producer.get(m) == w
                    hit_up += up
                    hit_prod += pr
                    hit_any += up or pr
                    held[w].add(m)
            mean = train_ms if f == "train" else agg_ms
            dur = mean * (1.0 + jitter * (2 * rng.random() - 1))
            heapq.heappush(events, (now + dur, seq, w, t))
            seq += 1
        now, _, w, t = heapq.heappop(events)
        if by_name[t][0] == "train":
            producer[t] = w
        free.append(w)
        for c in consumers.get(t, []):
            waiting[c] -= 1
            if waiting[c] == 0:
                queue.append(c)
    return {"peers": n, "workers": workers, "rounds": rounds, "fan_in": fan, "train_ms": train_ms, "agg_ms": agg_ms,
            "jitter": jitter, "seed": seed, "aggregate_inputs": n_in,
            "hit_upload": round(hit_up / n_in, 4), "hit_producer": round(hit_prod / n_in, 4),
            "hit_either": round(hit_any / n_in, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, nargs="+", default=[10, 100])
    ap.add_argument("--workers", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--rounds", type=int, default=6)
    a = ap.parse_args()
    # train/aggregate duration ratios: the reference's CPU trainer takes far
    # longer than an aggregate; 1 is the other extreme
    for n in a.peers:
        for w in a.workers:
            for train_ms, agg_ms in ((100.0, 1.0), (10.0, 1.0), (1.0, 1.0)):
                rows = [replay(n, w, a.rounds, train_ms, agg_ms, 0.3, s) for s in range(5)]
                mean = {k: round(sum(r[k] for r in rows) / len(rows), 4) for k in ("hit_upload", "hit_producer",
                                                                                     "hit_either")}
                print(json.dumps(dict(rows[0], seed="0-4 (mean)", **mean)), flush=True)


if __name__ == "__main__":
    main()
