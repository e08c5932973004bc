#!/bin/bash
# cfg2 lines (single 1 M task, GNLeNet task, and GNLeNet batched x100) with
# rocprofv3 kernel stats, plus the per-task probes on the final code. Output
# under gpurun_out/$1.
set -o pipefail
out=gpurun_out/${1:-c2}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --config cfg2 --no-cpu-baseline > "$out/bench_cfg2.json" 2> "$out/bench_cfg2.err" &&
timeout -k 10 200 python -u bench.py --config cfg2_gnlenet --no-cpu-baseline > "$out/bench_cfg2_gnlenet.json" 2> "$out/bench_cfg2_gnlenet.err" &&
timeout -k 10 200 python -u bench.py --config cfg2_gnlenet --batch 100 --no-cpu-baseline > "$out/bench_cfg2_gnlenet_b100.json" 2> "$out/bench_cfg2_gnlenet_b100.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_cfg2" -o run -- python3 bench.py --config cfg2 --no-cpu-baseline > "$out/prof_cfg2.log" 2>&1 &&
timeout -k 10 300 python -u scripts/probes/probe_task_parts.py > "$out/parts.jsonl" 2> "$out/parts.err" &&
timeout -k 10 300 python -u scripts/probes/probe_device_task.py > "$out/dev_task.jsonl" 2> "$out/dev_task.err"
