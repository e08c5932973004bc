# After a kernel change: GPU tests, smoke, bench lines for the configs
# (no CPU leg) and the fan-in sweep.
# usage: bash scripts/gpu_quick.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-quick}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke;  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for c in north_star cfg2 cfg3 cfg4 cfg5; do
  step bench $c; timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err || exit $?
  python3 -c "import json,sys; d=json.load(open('$O/bench_$c.json')); print('  ', '$c', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'])"
done
step sweep;  timeout -k 10 600 python3 scripts/sweep_fanin.py > $O/sweep.jsonl 2> $O/sweep.err || exit $?
step done
