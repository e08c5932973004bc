#!/bin/bash
# Round 4 (j): the cache path after the row-address change, with a profile.
set -o pipefail
mkdir -p gpurun_out/r04j

timeout -k 10 300 python -u scripts/probes/probe_cache_path.py 200 > gpurun_out/r04j/probe_cache_path.txt 2>&1 &&
timeout -k 10 400 python -u scripts/bench_workers.py --ways hip hip_cache --rounds 12 > gpurun_out/r04j/bench_workers.jsonl 2>&1
