"""Per-dispatch means of rocprofv3 --pmc counters for one kernel, across
several runs (round 5, VERDICT r04 next #4: translation counters at 3 and 12
rotating sets).

Each run directory holds one or more passes (subdirectories with a
run_counter_collection.csv, one counter group each). For every counter, the
mean over the dispatches of the kernel whose name contains --kernel (the
bench's reduce, not its probes) is reported, per run, with derived ratios.

usage: python scripts/pmc_table.py --kernel k_wreduce_tiles --out table.json \
           name1=gpurun_out/x/sets3 name2=gpurun_out/x/sets12
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics


def run_means(root: str, kernel: str) -> dict:
    vals = {}
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", "")
                if kernel not in name or "XorProbe" in name:
                    continue
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: {"mean": statistics.fmean(v), "n": len(v)} for k, v in sorted(vals.items())}


def ratios(m: dict) -> dict:
    g = lambda k: m.get(k, {}).get("mean")  # noqa: E731
    out = {}
    req, hit, miss = g("TCP_UTCL1_REQUEST_sum"), g("TCP_UTCL1_TRANSLATION_HIT_sum"), g("TCP_UTCL1_TRANSLATION_MISS_sum")
    if req and miss is not None:
        out["utcl1_miss_per_request"] = miss / req
    if hit is not None and miss is not None and hit + miss:
        out["utcl1_miss_rate"] = miss / (hit + miss)
    lat, rr = g("TCP_TCC_READ_REQ_LATENCY_sum"), g("TCP_TCC_READ_REQ_sum")
    if lat and rr:
        out["tcp_tcc_read_latency_cycles"] = lat / rr
    fetch = g("FETCH_SIZE")
    if fetch is not None:
        out["fetch_bytes_x2"] = fetch * 1024 * 2  # FETCH_SIZE is in KB; gfx950 correction x2
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="k_wreduce_tiles")
    ap.add_argument("--out")
    ap.add_argument("runs", nargs="+", help="name=directory")
    a = ap.parse_args()
    res = {}
    for spec in a.runs:
        name, root = spec.split("=", 1)
        m = run_means(root, a.kernel)
        res[name] = {"counters": m, "derived": ratios(m)}
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    for name, r in res.items():
        print(name, json.dumps({k: round(v["mean"], 1) for k, v in r["counters"].items()}),
              json.dumps({k: round(v, 4) for k, v in r["derived"].items()}))


if __name__ == "__main__":
    main()
