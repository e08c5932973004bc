#!/bin/bash
# Chunk reconstruction bench with >= 1 GiB of rotating inputs, and its
# rocprofv3 kernel stats. Output under gpurun_out/$1.
set -o pipefail
out=gpurun_out/${1:-ch}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/bench_chunks.py > "$out/bench_chunks.jsonl" 2> "$out/bench_chunks.err" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$out/trace" -o run -- python3 scripts/bench_chunks.py > "$out/trace.log" 2>&1
