"""Summarise rocprofv3 output for the reduce kernel (or another, --kernel).

    python scripts/pmc_summary.py --trace DIR --fetch DIR --write DIR \
        --config north_star --mode exact --bytes-per-launch B --out profiles/r01_pmc_traffic.json

--trace : a `rocprofv3 --kernel-trace --stats -f csv` output directory
--fetch : a `rocprofv3 --pmc FETCH_SIZE -f csv` output directory
--write : a `rocprofv3 --pmc WRITE_SIZE -f csv` output directory

HBM bytes per launch follow MI355X_MICROARCH.md §HBM for gfx950:
FETCH_SIZE (KiB) reports exactly half of a wide coalesced streaming read, so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024. Counters come from separate
passes (FETCH_SIZE and WRITE_SIZE do not fit one pass), each with only
--pmc, never combined with the sys/runtime trace domains.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics

KERNEL_RE = "k_wreduce"
PROBE_RE = "XorProbe"  # bench.py's pattern probe runs the same kernel template: not the reduce


def is_reduce(name: str) -> bool:
    return KERNEL_RE in name and PROBE_RE not in name


def rows(dirpath, suffix):
    out = []
    for path in glob.glob(os.path.join(dirpath, "**", "*" + suffix), recursive=True):
        with open(path, newline="") as f:
            out.extend(csv.DictReader(f))
    return out


def counter_avg(dirpath, counter):
    vals = []
    for r in rows(dirpath, "counter_collection.csv"):
        name = r.get("Kernel_Name", "")
        if is_reduce(name) and r.get("Counter_Name") == counter:
            vals.append(float(r["Counter_Value"]))
    if not vals:
        return None, 0
    # skip the first dispatches (warm-up) when there are enough
    body = vals[5:] if len(vals) > 10 else vals
    return statistics.mean(body), len(vals)


def trace_avg_ns(dirpath):
    durs = []
    for r in rows(dirpath, "kernel_trace.csv"):
        if is_reduce(r.get("Kernel_Name", "")):
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    if not durs:
        return None, 0
    return statistics.mean(durs), len(durs)


def main():
    global KERNEL_RE
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--config", required=True)
    ap.add_argument("--mode", default="exact")
    ap.add_argument("--bytes-per-launch", type=float, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--kernel", default=KERNEL_RE,
                    help="substring of the kernel to summarise (k_chunk_mean_batch for bench_chunks.py)")
    a = ap.parse_args()
    KERNEL_RE = a.kernel

    ent = {"algorithmic_bytes_per_launch": a.bytes_per_launch, "kernel": a.kernel}
    if a.trace:
        avg, cnt = trace_avg_ns(a.trace)
        if avg:
            ent["rocprof_kernel_avg_us"] = round(avg / 1e3, 3)
            ent["rocprof_dispatches"] = cnt
            ent["rocprof_achieved_GBps"] = round(a.bytes_per_launch / (avg * 1e-9) / 1e9, 1)
    fetch = write = None
    if a.fetch:
        fetch, nf = counter_avg(a.fetch, "FETCH_SIZE")
        ent["FETCH_SIZE_KiB_avg"] = fetch
    if a.write:
        write, nw = counter_avg(a.write, "WRITE_SIZE")
        ent["WRITE_SIZE_KiB_avg"] = write
    if fetch is not None and write is not None:
        hbm = (2.0 * fetch + write) * 1024.0
        ent["hbm_bytes_per_launch"] = round(hbm)
        ent["hbm_over_algorithmic"] = round(hbm / a.bytes_per_launch, 4)
        ent["correction"] = "gfx950: FETCH_SIZE doubled (reports half of wide streaming reads)"

    data = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            data = json.load(f)
    data.setdefault(a.config, {})[a.mode] = ent
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(json.dumps({a.config: {a.mode: ent}}, indent=1))


if __name__ == "__main__":
    main()
