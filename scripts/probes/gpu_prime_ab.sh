#!/bin/bash
# Round 6: the decoy-set priming in bench.py (ReduceWorkload._prime), A/B.
# For the 8-rank slice and the north star: bench lines with and without the
# decoy (DLSIM_BENCH_PRIME=0), each under a rocprofv3 kernel trace bucketed by
# rotating set (scripts/dispatch_buckets.py).
#   bash scripts/probes/gpu_prime_ab.sh [outdir]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/r06_prime}
mkdir -p "$OUT"
for leg in on off; do
  for cfg in s8 ns; do
    if [ $cfg = s8 ]; then extra="--slice-of 8"; sets=22; else extra=""; sets=3; fi
    if [ $leg = off ]; then export DLSIM_BENCH_PRIME=0; prime=0; else unset DLSIM_BENCH_PRIME; prime=8; fi
    timeout -k 10 240 rocprofv3 --kernel-trace -d "$OUT/${cfg}_${leg}" -o run --output-format csv -- \
      python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline $extra > "$OUT/${cfg}_${leg}.json" 2> "$OUT/${cfg}_${leg}.err"
    python3 scripts/dispatch_buckets.py "$(find "$OUT/${cfg}_${leg}" -name '*kernel_trace.csv')" --sets $sets \
      --warmup 20 --steps 200 --prime $prime --kernel k_wreduce --out "$OUT/${cfg}_${leg}_buckets.json" > /dev/null
    python3 - "$OUT/${cfg}_${leg}" <<'PY'
import json, sys
b = json.load(open(sys.argv[1] + "_buckets.json"))
l = json.loads(open(sys.argv[1] + ".json").read().strip().splitlines()[-1])
print(json.dumps({"leg": sys.argv[1].rsplit("/", 1)[1], "value": l["value"], "ms_per_step": l["ms_per_step"],
                  "host_enqueue_us": (l.get("launch_floor") or {}).get("host_enqueue_us_per_launch"),
                  "timed": b["timed"], "set_means": b["set_means"], "by_set": b["by_set_mean_us"]}))
PY
  done
done
