# After the host-pipeline stream change: the full GPU suite, smoke, the host
# task probe, the GNLeNet round with host models, and the 2-rank rehearsal
# (its stdout must be the one JSON line).
# usage: bash scripts/probes/gpu_host_r02s2.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-host2}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
tail -1 $O/pytest_gpu.log
step smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
step host task
timeout -k 10 300 python3 -u scripts/probes/probe_host_task.py > $O/host_task.jsonl 2> $O/host_task.err || exit $?
step rounds host
timeout -k 10 400 python3 -u scripts/bench_rounds.py --model gnlenet --host > $O/rounds_gnlenet_host.jsonl 2> $O/rounds_gnlenet_host.err || exit $?
step rehearse
timeout -k 10 300 python3 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo > $O/bench_2rank_spawn.json 2> $O/bench_2rank_spawn.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_2rank_spawn.json')); print(d['n_gpus'], d['scaling'], d['value'])" || exit $?
step done
