# Multi-rank flow of bench.py on the one-GPU box (gloo control plane, ranks
# sharing the card), the N=1 line, and rank 0's slice alone at 2/4/8 ranks
# (the per-rank work of the strong split) with a rocprofv3 kernel trace of
# the 8-rank slice: per-dispatch durations next to the event time.
# usage: bash scripts/probes/gpu_bench_multi.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-multi}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step "N=1"
timeout -k 10 200 python3 bench.py --cpu-seconds 6 > $O/n1.json 2> $O/n1.err || exit $?
step "N=2 gloo rehearsal (self-spawned ranks)"
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --steps 50 > $O/n2_gloo.json 2> $O/n2_gloo.err || exit $?
for s in 2 4 8; do
  step "slice of $s"
  timeout -k 10 200 python3 bench.py --slice-of $s --no-cpu-baseline --steps 400 --warmup 40 >> $O/slices.jsonl 2>> $O/slices.err || exit $?
done
step "rocprof slice of 8"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_slice8 -o run -- python3 $R/bench.py --slice-of 8 --no-cpu-baseline --steps 400 --warmup 40 > $O/prof_slice8.json 2> $O/prof_slice8.err || exit $?
step done
