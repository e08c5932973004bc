# Rehearse bench.py's multi-process flow on a one-GPU box: torchrun with 2
# ranks sharing the GPU, gloo control plane (RCCL runs only on the driver's
# 8-GPU node). Weak and strong scaling.
# usage: bash scripts/probes/gpu_rehearse_multi.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-multi}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step weak
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo > $O/bench_2rank_weak.json 2> $O/bench_2rank.err || exit $?
cat $O/bench_2rank_weak.json
step strong
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29612 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo --strong > $O/bench_2rank_strong.json 2>> $O/bench_2rank.err || exit $?
cat $O/bench_2rank_strong.json
step done
