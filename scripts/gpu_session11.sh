# Batched launches: tests + batched bench lines for the launch-bound configs.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s11
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for b in 1 8 32; do
  step gnlenet b$b; timeout -k 10 300 python3 bench.py --config cfg2_gnlenet --batch $b --no-cpu-baseline > $O/bench_gnlenet_b$b.json 2>> $O/bench.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_gnlenet_b$b.json')); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'])"
done
for b in 1 4 16; do
  step cfg2 b$b; timeout -k 10 300 python3 bench.py --config cfg2 --batch $b --no-cpu-baseline > $O/bench_cfg2_b$b.json 2>> $O/bench.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_cfg2_b$b.json')); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'])"
done
step trace; timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_gnlenet_b32 -- python3 bench.py --config cfg2_gnlenet --batch 32 --no-cpu-baseline --steps 200 > $O/trace.log 2>&1 || exit $?
step done
