"""Probe (round 4): how much do the north star's rotating input sets differ?

bench.py rotates over >= 1 GiB of input sets (3 for the north star) carved
from one allocation, and fresh bench processes land anywhere in 0.795-0.827
(profiles/r04_final/, DESIGN.md §5b: the physical pages). Here one process
builds SETS sets in one allocation (bench.ReduceWorkload with
DLSIM_BENCH_MIN_SETS), times K launches of each set alone, then K launches
rotating over the first 3 sets (the bench's rotation) and over all SETS.
If the sets' rates spread independently, a longer rotation averages the page
lottery instead of sampling three draws of it.

    python scripts/probes/probe_set_spread.py [SETS] [K]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "decentralized-learning-simulator_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import bench  # noqa: E402
from dasklearn_amd import _native  # noqa: E402

N, P = 8, bench.RESNET18_P
dev = torch.device("cuda", 0)


def timed(launch, k_steps):
    for k in range(10):
        launch(k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(k_steps):
        launch(k)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k_steps


def frac(us):
    return round(9 * P * 4 / (us * 1e-6) / 8e12, 4)


def main():
    sets = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    k_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    os.environ["DLSIM_BENCH_MIN_SETS"] = str(sets)
    stream = torch.cuda.current_stream(dev)
    w32 = _native.fp32_weights(bench.weights_for("dirichlet", N))
    wl = bench.ReduceWorkload(N, P, "f32", w32, _native.DLSIM_EXACT, 1, dev, 1234, stream)
    assert wl.sets == sets
    per_set = []
    for rnd in range(2):
        for s in range(sets):
            us = timed(lambda k, s=s: wl.plans[s].launch(stream), k_steps)
            per_set.append((rnd, s, us))
            print(json.dumps({"round": rnd, "set": s, "us_per_launch": round(us, 3), "frac": frac(us)}), flush=True)
    rot3 = [timed(lambda k: wl.plans[k % 3].launch(stream), k_steps) for _ in range(3)]
    rot_all = [timed(lambda k: wl.plans[k % sets].launch(stream), k_steps) for _ in range(3)]
    means = [statistics.mean(us for r, s2, us in per_set if s2 == s) for s in range(sets)]
    print(json.dumps({"summary": True, "sets": sets, "K": k_steps,
                      "per_set_mean_us": [round(x, 3) for x in means],
                      "per_set_min_us": round(min(means), 3), "per_set_max_us": round(max(means), 3),
                      "per_set_sd_us": round(statistics.pstdev(means), 3),
                      "first3_mean_us": round(statistics.mean(means[:3]), 3),
                      "rotate3_us": [round(x, 3) for x in rot3], "rotate_all_us": [round(x, 3) for x in rot_all],
                      "rotate3_frac": frac(statistics.mean(rot3)), "rotate_all_frac": frac(statistics.mean(rot_all))}),
          flush=True)


if __name__ == "__main__":
    main()
