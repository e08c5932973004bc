"""Per-dispatch times of bench.py's reduce kernel from a rocprofv3 kernel
trace, bucketed by rotating input set and by position in the timed burst
(does the spread of the small slices follow the set —
placement, translation — or the position — launch jitter, clocks?).

bench.py launches step k on set k mod S: (from round 6) P launches on a
decoy set first (bench.PRIME_LAUNCHES; --prime P skips them), W warm-up launches (k = 0..W-1),
then the K timed ones (k = 0..K-1), then launch_floor's backlog (k = 0..B-1);
the pattern probe and the floor's tiny launches are other kernels.

usage: python scripts/dispatch_buckets.py <run_kernel_trace.csv> --sets S --warmup W --steps K
       [--kernel SUBSTRING] [--out summary.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics as st


def load(path, kernel):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            if kernel in name and "XorProbe" not in name:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    return rows


def summ(xs):
    xs = sorted(xs)
    if not xs:
        return None
    return {"n": len(xs), "mean": round(st.fmean(xs), 3), "min": round(xs[0], 3),
            "p50": round(xs[len(xs) // 2], 3), "max": round(xs[-1], 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--sets", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--prime", type=int, default=0)
    ap.add_argument("--kernel", default="k_wreduce_tiles")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = load(a.trace, a.kernel)[a.prime:]
    names = sorted({r[2] for r in rows})
    if len(names) != 1:
        raise SystemExit(f"expected one reduce kernel, found {names}")
    W, K, S = a.warmup, a.steps, a.sets
    if len(rows) < W + K:
        raise SystemExit(f"{len(rows)} dispatches, expected >= {W + K}")
    dur = [(e - s) / 1e3 for s, e, _ in rows]  # us
    gap = [(rows[i + 1][0] - rows[i][1]) / 1e3 for i in range(len(rows) - 1)]
    timed = list(range(W, W + K))
    by_set = {s: [] for s in range(S)}
    for i in timed:
        by_set[(i - W) % S].append(dur[i])
    by_pos = {"first": [dur[W]], "2-10": [dur[i] for i in range(W + 1, W + 10)],
              "11-50": [dur[i] for i in range(W + 10, min(W + 50, W + K))],
              "51+": [dur[i] for i in range(W + 50, W + K)]}
    backlog = list(range(W + K, len(rows)))
    set_means = {s: st.fmean(v) for s, v in by_set.items() if v}
    res = {
        "kernel": names[0], "dispatches": len(rows),
        "timed": summ([dur[i] for i in timed]),
        "timed_gaps_us": summ([gap[i] for i in range(W, W + K - 1)]),
        "by_set_mean_us": {str(s): round(m, 3) for s, m in set_means.items()},
        "set_means": summ(list(set_means.values())),
        "within_set_spread_us": summ([max(v) - min(v) for v in by_set.values() if len(v) > 1]),
        "by_position": {k: summ(v) for k, v in by_pos.items()},
        "warmup": summ([dur[i] for i in range(W)]),
        "backlog": summ([dur[i] for i in backlog]),
        "backlog_by_set_mean_us": {str(s): round(st.fmean([dur[i] for i in backlog if (i - W - K) % S == s]), 3)
                                   for s in range(S) if any((i - W - K) % S == s for i in backlog)},
        "timed_sequence_us": [round(dur[i], 2) for i in timed],
    }
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    print(json.dumps({k: res[k] for k in ("timed", "timed_gaps_us", "set_means", "within_set_spread_us",
                                         "by_position", "backlog")}, indent=1))


if __name__ == "__main__":
    main()
