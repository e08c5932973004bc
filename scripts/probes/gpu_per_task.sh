#!/bin/bash
# Per-task path on one MI355X: drop-in/round/DAG parity, then bench_rounds on
# the reference's GNLeNet module tree and the flat 14-tensor model (device and
# host models), then the single host-task probe. Results in gpurun_out/$1.
set -o pipefail
out=gpurun_out/${1:-pt}
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_rounds.py tests/test_gpu_dag_replay.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1 &&
for model in gnlenet flat; do
  timeout -k 10 400 python -u scripts/bench_rounds.py --model $model > "$out/rounds_$model.jsonl" 2> "$out/rounds_$model.err" &&
  timeout -k 10 400 python -u scripts/bench_rounds.py --model $model --host > "$out/rounds_${model}_host.jsonl" 2> "$out/rounds_${model}_host.err" || exit $?
done &&
timeout -k 10 300 python -u scripts/probes/probe_host_task.py > "$out/host_task.jsonl" 2> "$out/host_task.err"
