"""Per-leg kernel durations from a rocprofv3 kernel trace of a probe that
runs its legs one after another (round 6: probe_chunk_vs_reduce.py, whose
chunk legs are host-bound on the events clock when a call's Python costs
more than its kernel). Dispatches are sorted by start time and cut into runs
of one kernel name; each run prints its count, mean, median and min duration
(us) and the mean gap between its dispatches (a gap near zero: the GPU was
kept busy; a large gap: the host could not enqueue fast enough).

    python scripts/probes/trace_legs.py <run_kernel_trace.csv> [--min-run 50] [--out legs.json]
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics as st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-run", type=int, default=50)
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    runs, cur = [], []
    for r in rows:
        if cur and r[2] != cur[-1][2]:
            runs.append(cur)
            cur = []
        cur.append(r)
    if cur:
        runs.append(cur)
    out = []
    for run in runs:
        if len(run) < a.min_run:
            continue
        d = [(e - s) / 1e3 for s, e, _ in run]
        gaps = [(run[i + 1][0] - run[i][1]) / 1e3 for i in range(len(run) - 1)]
        name = run[0][2]
        short = name.split("(")[0].replace("void ", "")[:110]
        out.append({"kernel": short, "n": len(run), "mean_us": round(st.fmean(d), 3),
                    "median_us": round(st.median(d), 3), "min_us": round(min(d), 3),
                    "mean_gap_us": round(st.fmean(gaps), 3) if gaps else None})
        print(json.dumps(out[-1]))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
