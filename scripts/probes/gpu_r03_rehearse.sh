# Rehearse the driver's multi-GPU bench invocations at HEAD on a one-GPU box
# (ranks share the card, gloo control plane; RCCL with several ranks runs only
# on the driver's 8-GPU node): torchrun with 2 and 4 ranks (the driver's form)
# and the self-spawned form, strong scaling (the default).
# usage: bash scripts/probes/gpu_r03_rehearse.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-rehearse}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
for N in 2 4; do
  step "torchrun $N ranks"
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
    --master-port 2961$N bench.py --gpus $N --steps 50 --warmup 5 --backend gloo > $O/torchrun_$N.json 2> $O/torchrun_$N.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/torchrun_$N.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['scaling'], d['timing']['kernel_avg_us_per_rank'], d.get('single_gpu_reference', {}).get('speedup'))" || exit 1
done
step "self-spawn 2 ranks"
timeout -k 10 300 python3 bench.py --gpus 2 --steps 50 --warmup 5 --backend gloo > $O/spawn_2.json 2> $O/spawn_2.err || exit $?
python3 -c "import json; d=json.loads(open('$O/spawn_2.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['scaling'])" || exit 1
wc -l $O/*.json
step done
