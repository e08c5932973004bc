# Full evidence run: tests, smoke, fan-in sweep, every config's bench line,
# batched lines, host/wire rates, rocprofv3 + PMC for the north star and cfg4.
# usage: bash scripts/probes/gpu_evidence.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-evidence}
O=$R/gpurun_out/$N
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke;  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
step sweep;  timeout -k 10 600 python3 scripts/sweep_fanin.py > $O/sweep.jsonl 2> $O/sweep.err || exit $?
for c in cfg2 cfg2_gnlenet cfg3 cfg4 cfg5; do
  step bench $c; timeout -k 10 300 python3 bench.py --config $c --cpu-seconds 8 > $O/bench_$c.json 2>> $O/bench.err || exit $?
done
step bench b; timeout -k 10 300 python3 bench.py --config cfg2_gnlenet --batch 100 --no-cpu-baseline > $O/bench_cfg2_gnlenet_b100.json 2>> $O/bench.err || exit $?
timeout -k 10 300 python3 bench.py --config cfg2 --batch 16 --no-cpu-baseline > $O/bench_cfg2_b16.json 2>> $O/bench.err || exit $?
step host;   timeout -k 10 600 python3 scripts/bench_host.py > $O/bench_host.jsonl 2> $O/bench_host.err || exit $?
bash scripts/probes/gpu_profile.sh $N/ns north_star || exit $?
bash scripts/probes/gpu_profile.sh $N/c4 cfg4 || exit $?
step done
