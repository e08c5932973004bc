# Address-translation counters for the large-footprint loss (round 5, VERDICT
# r04 next #4): the north star at 3 rotating sets (1.2 GB, the bench) and at
# 12 (4.8 GB, a 100-peer round's distinct models), a kernel trace each, then
# one rocprofv3 --pmc pass per counter group (no trace domains; at most 4 TCP
# and 2 GRBM counters a pass), summarised by scripts/pmc_table.py.
# usage: bash scripts/gpu_translation_pmc.sh <outdir-name> [extra bench args]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-translation_pmc}
shift
EXTRA="$*"
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
PASSES=(
  "TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_PERMISSION_MISS_sum"
  "TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
for S in 3 12; do
  export DLSIM_BENCH_MIN_SETS=$S
  ARGS="--no-cpu-baseline --steps 60 --warmup 6 $EXTRA"
  step "sets=$S bench"
  timeout -k 10 120 python3 bench.py --no-cpu-baseline $EXTRA > $O/bench_sets$S.json 2> $O/bench_sets$S.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_sets$S.json')); print('sets=$S', d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['data'])"
  step "sets=$S trace"
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/sets$S/trace -o run -- python3 $R/bench.py $ARGS > $O/sets$S.trace.log 2>&1 || exit $?
  k=0
  for P in "${PASSES[@]}"; do
    k=$((k + 1))
    step "sets=$S pass $k: $P"
    timeout -s KILL 90 rocprofv3 --pmc $P -f csv -d $O/sets$S/pass$k -o run -- python3 $R/bench.py $ARGS > $O/sets$S.pass$k.log 2>&1 || exit $?
  done
done
unset DLSIM_BENCH_MIN_SETS
python3 scripts/pmc_table.py --out $O/translation_table.json sets3=$O/sets3 sets12=$O/sets12
step done
