"""Per-group means of rocprofv3 counters (round 6): the dispatches of one kernel,
in dispatch order, cut into consecutive groups of G (a probe that runs G
launches per leg, e.g. probe_slice_sets.py --offsets: 10 warm-up + 200 timed);
prints one JSON line per group with each counter's mean per dispatch, and
with --trace the mean duration from the same run's kernel trace.

    python scripts/probes/pmc_groups.py <counter_collection.csv> --kernel k_wreduce_tiles \
        --group 210 [--trace <kernel_trace.csv>]
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("counters")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--group", type=int, required=True)
    ap.add_argument("--trace")
    a = ap.parse_args()
    per = defaultdict(dict)
    with open(a.counters) as f:
        for r in csv.DictReader(f):
            if a.kernel in r["Kernel_Name"]:
                d = per[int(r["Dispatch_Id"])]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur = {}
    if a.trace:
        with open(a.trace) as f:
            for r in csv.DictReader(f):
                if a.kernel in r["Kernel_Name"]:
                    dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ids = sorted(per)
    for g in range(0, len(ids), a.group):
        chunk = ids[g:g + a.group]
        names = sorted({k for i in chunk for k in per[i]})
        row = {"group": g // a.group, "dispatches": len(chunk)}
        for k in names:
            row[k] = round(sum(per[i].get(k, 0.0) for i in chunk) / len(chunk), 1)
        ds = [dur[i] for i in chunk if i in dur]
        if ds:
            row["mean_us"] = round(sum(ds) / len(ds), 3)
        print(json.dumps(row))


if __name__ == "__main__":
    main()
