# Targeted GPU check after a change: the named test files (or -k expression),
# then the default bench line and the driver's shape twice.
# usage: bash scripts/gpu_targeted.sh <outdir-name> <pytest args...>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-targeted}
shift
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest "$@"
timeout -k 10 900 python3 -u -m pytest -p no:cacheprovider -x -v --timeout 180 --timeout-method thread "$@" > $O/pytest.log 2>&1
rc=$?; tail -40 $O/pytest.log | grep -E "passed|failed|error|Error|FAIL" | tail -12
if [ $rc -ne 0 ]; then exit $rc; fi
step bench; timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('default', d['ms_per_step'], d['roofline']['frac'], d['config']['outputs_alloc'])"
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_driver_$i.json')); print('driver shape', $i, d['ms_per_step'], d['roofline']['frac'])"
done
step done
