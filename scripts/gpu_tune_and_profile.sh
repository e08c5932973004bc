# GPU session: kernel-shape sweep, default bench line, rocprofv3 kernel trace
# and PMC (FETCH_SIZE / WRITE_SIZE in separate passes). Every GPU step has its
# own time limit; a crash/timeout stops the script.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
step() { echo "[$(date +%T)] $*"; }
step tune n8;   timeout -k 10 300 $T 8 11181642 f32 exact 40 > $O/tune2_n8_f32.log 2>&1 || exit $?
step tune n17;  timeout -k 10 300 $T 17 11181642 f32 exact 30 > $O/tune2_n17_f32.log 2>&1 || exit $?
step tune bf16; timeout -k 10 300 $T 2 125000000 bf16 exact 30 > $O/tune2_n2_bf16.log 2>&1 || exit $?
step tune n2f32; timeout -k 10 300 $T 2 11181642 f32 exact 40 > $O/tune2_n2_f32.log 2>&1 || exit $?
step bench;     timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
cat $O/bench_default.json
step trace;     timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/r01_trace -- python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 > $O/r01_trace.log 2>&1 || exit $?
step fetch;     timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/r01_fetch -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > $O/r01_fetch.log 2>&1 || exit $?
step write;     timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/r01_write -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > $O/r01_write.log 2>&1 || exit $?
python3 scripts/pmc_summary.py --trace $O/r01_trace --fetch $O/r01_fetch --write $O/r01_write \
  --config north_star --mode exact --bytes-per-launch $((9*11181642*4)) --out $O/r01_pmc_traffic.json
find $O/r01_trace -name "*stats*" | head
step done
