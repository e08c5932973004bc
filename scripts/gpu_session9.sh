# ragged end on block 0: tests, smoke, bench (north star), rocprof trace + PMC, host stages.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s9
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke;  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
step bench;  timeout -k 10 300 python3 bench.py > $O/bench_north_star.json 2> $O/bench.err || exit $?
cat $O/bench_north_star.json
step bench2; timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_north_star_2.json 2>> $O/bench.err || exit $?
cat $O/bench_north_star_2.json
step tune;   timeout -k 10 300 $T 8 11182080 f32 exact 60 > $O/tune_n8.log 2>&1 || exit $?
step trace;  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -- python3 bench.py --no-cpu-baseline --steps 200 --warmup 20 > $O/trace.log 2>&1 || exit $?
step fetch;  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > $O/fetch.log 2>&1 || exit $?
step write;  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > $O/write.log 2>&1 || exit $?
python3 scripts/pmc_summary.py --trace $O/trace --fetch $O/fetch --write $O/write \
  --config north_star --mode exact --bytes-per-launch $((9*11181642*4)) --out $O/pmc_traffic.json
step host;   timeout -k 10 600 python3 scripts/bench_host.py > $O/bench_host.jsonl 2> $O/bench_host.err || exit $?
cat $O/bench_host.jsonl
step done
