# Round 4, session 2 (fresh container, libraries rebuilt from the same sources):
# the whole -m gpu suite, smoke(), the default bench line and the driver's shape,
# then rocprofv3 kernel stats of the default bench.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04s2_check}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
step smoke;  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
step bench;  timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['cpu_baseline']['value'])"
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_driver.json')); print('driver shape', d['ms_per_step'], d['roofline']['frac'])"
step rocprof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || exit $?
step done
