# Rehearse the driver's N > 1 bench at HEAD on a one-GPU box: every rank is
# its own process (gloo control plane, all ranks on cuda:0), so the
# multi-process flow, each rank's allocations and its slice's kernel run as
# they will on an 8-GPU node; the timings are contended (8 ranks share one
# GPU) and only the line's shape and the per-rank kernels are evidence.
# Then a rocprofv3 kernel trace of rank 0's 8-rank slice alone (the per-rank
# work of the north star at N = 8), bucketed over the timed dispatches only.
# usage: bash scripts/gpu_rehearse.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06_rehearse}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
run() {  # name, bench.py arguments
  local NAME=$1; shift
  step "$NAME: bench.py $*"
  timeout -k 10 400 python3 bench.py "$@" > $O/$NAME.json 2> $O/$NAME.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc for $NAME"; tail -30 $O/$NAME.err; exit $rc; fi
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['n_gpus'], d['value'], d['timing']['kernel_avg_us_per_rank'])" $O/$NAME.json || exit 1
}
run g8_north_star --gpus 8 --backend gloo --steps 20 --warmup 5
run g4_cfg4 --gpus 4 --backend gloo --config cfg4 --steps 20 --warmup 5
run g8_cfg5 --gpus 8 --backend gloo --config cfg5 --steps 20 --warmup 5
run g2_north_star --gpus 2 --backend gloo --steps 20 --warmup 5
run g4_north_star --gpus 4 --backend gloo --steps 20 --warmup 5
# the driver's own launcher (torchrun sets RANK/WORLD_SIZE; bench.py does not spawn)
step "torchrun g4"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 4 --backend gloo --steps 20 --warmup 5 > $O/torchrun_g4.json 2> $O/torchrun_g4.err \
  || { echo "torchrun rc=$?"; tail -30 $O/torchrun_g4.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['n_gpus'], d['value'])" $O/torchrun_g4.json || exit 1
# rank 0's 8-rank slice alone, traced: K = 200 timed launches after 20 warm-ups
ARGS="--slice-of 8 --no-cpu-baseline --steps 200 --warmup 20"
step "slice-8 bench"
timeout -k 10 300 python3 bench.py $ARGS > $O/ns_s8.json 2> $O/ns_s8.err || exit 1
step "slice-8 trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_ns_s8 -o run -- python3 $R/bench.py $ARGS \
  > $O/trace_ns_s8.log 2>&1 || exit 1
SETS=$(python3 -c "import json; print(json.load(open('$O/ns_s8.json'))['data'].split(' rotating input')[0].split()[-1])")
TRACE=$(find $O/trace_ns_s8 -name '*kernel_trace.csv' | head -1)
python3 scripts/dispatch_buckets.py "$TRACE" --sets $SETS --warmup 20 --steps 200 --prime 8 --kernel k_wreduce --out $O/ns_s8_buckets.json || exit 1
step done
