# rocprofv3 evidence for the round-3 bench lines: for the north star at N=1
# and rank 0's slice of the 2/4/8-rank strong split (the per-rank work of the
# driver's multi-GPU run), plus cfg3/cfg4/cfg5: a kernel trace with --stats,
# then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (no trace domains),
# summarised per config by scripts/pmc_summary.py (gfx950 FETCH_SIZE x2).
# usage: bash scripts/gpu_profile.sh <outdir> ["name:config:slice ..."]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-prof_r03}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
run() {  # name config slice
  local NAME=$1 C=$2 S=$3
  local KEY=$C; [ "$S" -gt 1 ] && KEY="$C@slice$S"
  local BYTES=$(python3 -c "
import sys; sys.path.insert(0, '.'); sys.path.insert(0, 'decentralized-learning-simulator_amd')
import bench
from dasklearn_amd import _native
n, p, dt, _, _ = bench.CONFIGS['$C']
b, e = _native.shard_range(p, $S, 0, 64)
print((n + 1) * (e - b) * bench.ELEM_BYTES[dt])")
  local ARGS="--config $C --slice-of $S --no-cpu-baseline"
  step "$NAME bench";  timeout -k 10 300 python3 bench.py $ARGS > $O/bench_$NAME.json 2> $O/bench_$NAME.err || return 1
  step "$NAME trace";  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_$NAME -o run -- python3 $R/bench.py $ARGS --steps 200 --warmup 20 > $O/trace_$NAME.log 2>&1 || return 1
  step "$NAME fetch";  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch_$NAME -o run -- python3 $R/bench.py $ARGS --steps 50 --warmup 5 > $O/fetch_$NAME.log 2>&1 || return 1
  step "$NAME write";  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write_$NAME -o run -- python3 $R/bench.py $ARGS --steps 50 --warmup 5 > $O/write_$NAME.log 2>&1 || return 1
  python3 scripts/pmc_summary.py --trace $O/trace_$NAME --fetch $O/fetch_$NAME --write $O/write_$NAME \
    --config $KEY --mode exact --bytes-per-launch $BYTES --out $O/${PMC_NAME:-r03_pmc_traffic.json} > /dev/null || return 1
}
if [ $# -ge 2 ]; then  # a chosen list: "name:config:slice ..."
  for spec in $2; do
    IFS=: read -r NAME C S <<< "$spec"
    run $NAME $C $S || exit 1
  done
else
  run ns north_star 1 && run ns_s2 north_star 2 && run ns_s4 north_star 4 && run ns_s8 north_star 8 \
    && run cfg4 cfg4 1 && run cfg5 cfg5 1 && run cfg3 cfg3 1 || exit 1
fi
step done
