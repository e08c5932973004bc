# rocprofv3 evidence for one bench config: kernel trace + stats, then PMC
# FETCH_SIZE and WRITE_SIZE in separate passes (never combined with trace
# domains), summarised by scripts/pmc_summary.py.
# usage: bash scripts/probes/gpu_profile.sh <outdir> [config] [extra bench args...]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-profile}
C=${2:-north_star}
shift 2 2>/dev/null || shift $#
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
BYTES=$(python3 -c "
import sys; sys.path.insert(0, '.')
import bench; n, p, dt, _, _ = bench.CONFIGS['$C']; print((n + 1) * p * bench.ELEM_BYTES[dt])")
step bench;  timeout -k 10 300 python3 bench.py --config $C "$@" > $O/bench_$C.json 2> $O/bench.err || exit $?
cat $O/bench_$C.json
step trace;  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_$C -- python3 bench.py --config $C --no-cpu-baseline --steps 200 --warmup 20 "$@" > $O/trace.log 2>&1 || exit $?
step fetch;  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch_$C -- python3 bench.py --config $C --no-cpu-baseline --steps 50 --warmup 5 "$@" > $O/fetch.log 2>&1 || exit $?
step write;  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write_$C -- python3 bench.py --config $C --no-cpu-baseline --steps 50 --warmup 5 "$@" > $O/write.log 2>&1 || exit $?
python3 scripts/pmc_summary.py --trace $O/trace_$C --fetch $O/fetch_$C --write $O/write_$C \
  --config $C --mode exact --bytes-per-launch $BYTES --out $O/pmc_traffic.json
step done
