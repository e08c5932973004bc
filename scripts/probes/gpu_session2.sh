# Round 2, session 2 evidence: the default bench line (as the driver runs it),
# the multi-rank flow rehearsed on one GPU (self-spawned and torchrun, 2 ranks,
# gloo control plane), and rocprofv3 kernel stats + PMC traffic for the north
# star and its 8-rank slice with this bench (launch floor on the probe entry).
# usage: bash scripts/probes/gpu_session2.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-s2}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step bench default
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
step rehearse self-spawn
timeout -k 10 300 python3 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo > $O/bench_2rank_spawn.json 2> $O/bench_2rank_spawn.err || exit $?
step rehearse torchrun
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29613 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo > $O/bench_2rank_torchrun.json 2> $O/bench_2rank_torchrun.err || exit $?
step device task
timeout -k 10 300 python3 -u scripts/probes/probe_device_task.py > $O/device_task.jsonl 2> $O/device_task.err || exit $?
timeout -k 10 300 python3 -u scripts/probes/probe_task_parts.py > $O/task_parts.jsonl 2> $O/task_parts.err || exit $?
step rounds
timeout -k 10 400 python3 -u scripts/bench_rounds.py --model gnlenet > $O/rounds_gnlenet.jsonl 2> $O/rounds_gnlenet.err || exit $?
step profile
bash scripts/probes/gpu_profile_r02.sh ${1:-s2}/prof "ns:north_star:1 ns_s8:north_star:8" || exit $?
step done
