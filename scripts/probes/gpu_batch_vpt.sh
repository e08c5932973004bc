#!/bin/bash
# Batched-kernel VPT experiment: batch parity, the batched GNLeNet bench line,
# and the batched rounds. Output under gpurun_out/$1.
set -o pipefail
out=gpurun_out/${1:-bv}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_rounds.py tests/test_gpu_aliasing.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1 &&
timeout -k 10 200 python -u bench.py --config cfg2_gnlenet --batch 100 --no-cpu-baseline > "$out/bench_gnl_b100.json" 2> "$out/bench_gnl_b100.err" &&
timeout -k 10 200 python -u bench.py --config cfg2 --batch 8 --no-cpu-baseline > "$out/bench_cfg2_b8.json" 2> "$out/bench_cfg2_b8.err" &&
timeout -k 10 400 python -u scripts/bench_rounds.py --model flat --reps 3 > "$out/rounds_flat.jsonl" 2> "$out/rounds_flat.err"
