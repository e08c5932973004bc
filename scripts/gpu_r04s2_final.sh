# Round 4 session 2 evidence with the contiguous blocks: the whole -m gpu
# suite, smoke(), the default bench line, the driver's shape three times, then
# rocprofv3 kernel stats + PMC traffic (r04s2_pmc_traffic.json) per config.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04s2_final
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
step smoke;  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
step bench;  timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print(d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_us'], d['pattern_ceiling']['frac'], d['cpu_baseline']['value'])"
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_driver_$i.json')); print('driver shape', $i, d['ms_per_step'], d['roofline']['frac'])"
done
step profile
PMC_NAME=r04s2_pmc_traffic.json bash scripts/gpu_profile_r03.sh r04s2_final/prof \
  "ns:north_star:1 ns_s8:north_star:8 cfg2:cfg2:1 cfg3:cfg3:1 cfg4:cfg4:1 cfg5:cfg5:1" || exit 1
step done
