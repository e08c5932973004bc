# Per-task path and slice evidence after the host-walk / parameter-view changes:
# drop-in + rounds GPU tests, device-task probes, bench_rounds (GNLeNet device and
# host), and bench lines with the launch floor for the north star and its slices.
# usage: bash scripts/probes/gpu_task_r02s2.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-task}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_rounds.py tests/test_gpu_dag_replay.py \
    tests/test_gpu_staging.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
step device_task
timeout -k 10 300 python3 -u scripts/probes/probe_device_task.py > $O/device_task.jsonl 2> $O/device_task.err || exit $?
step task_parts
timeout -k 10 300 python3 -u scripts/probes/probe_task_parts.py > $O/task_parts.jsonl 2> $O/task_parts.err || exit $?
step rounds
timeout -k 10 400 python3 -u scripts/bench_rounds.py --model gnlenet > $O/rounds_gnlenet.jsonl 2> $O/rounds_gnlenet.err || exit $?
timeout -k 10 400 python3 -u scripts/bench_rounds.py --model gnlenet --host > $O/rounds_gnlenet_host.jsonl 2> $O/rounds_gnlenet_host.err || exit $?
step bench
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_ns.json 2>> $O/bench.err || exit $?
for s in 2 4 8; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --slice-of $s > $O/bench_ns_s$s.json 2>> $O/bench.err || exit $?
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --config cfg3 --slice-of 8 > $O/bench_cfg3_s8.json 2>> $O/bench.err || exit $?
step done
