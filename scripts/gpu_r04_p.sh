#!/bin/bash
# Round 4 (p): pack helpers for small (cold) packs in the worker deployment:
# DLSIM_PACK_HELPERS_MIN_KB 1024 (round-4 default) vs 64, way hip_cache and hip.
set -o pipefail
mkdir -p gpurun_out/r04p
timeout -k 10 300 python -u scripts/bench_workers.py --ways hip hip_cache > gpurun_out/r04p/workers_1024.jsonl 2> gpurun_out/r04p/workers_1024.err &&
DLSIM_PACK_HELPERS_MIN_KB=64 timeout -k 10 300 python -u scripts/bench_workers.py --ways hip hip_cache > gpurun_out/r04p/workers_64.jsonl 2> gpurun_out/r04p/workers_64.err &&
timeout -k 10 300 python -u scripts/bench_workers.py --ways hip_cache > gpurun_out/r04p/workers_1024b.jsonl 2> gpurun_out/r04p/workers_1024b.err &&
DLSIM_PACK_HELPERS_MIN_KB=64 timeout -k 10 300 python -u scripts/bench_workers.py --ways hip_cache > gpurun_out/r04p/workers_64b.jsonl 2> gpurun_out/r04p/workers_64b.err
