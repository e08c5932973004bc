# Every bench line of the round at HEAD (no rocprof): the default line, the
# driver's shape twice, each BASELINE config and the north star's 2/4/8-rank
# slices, then a summary table. Optionally the -m gpu suite and smoke() first.
# usage: bash scripts/gpu_lines.sh <outdir-name> [--suite]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-lines}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
if [ "${2:-}" = "--suite" ]; then
  step pytest
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -25 $O/pytest_gpu.log | grep -E "passed|failed|error" | tail -3
  if [ $rc -ne 0 ]; then exit $rc; fi
  step smoke; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -1 $O/smoke.log
fi
step bench default; timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || exit $?
done
for spec in cfg2:1 cfg3:1 cfg4:1 cfg5:1 north_star:2 north_star:4 north_star:8 cfg3:8 cfg5:8 cfg4:4; do
  IFS=: read -r C S <<< "$spec"
  step "bench $C slice $S"
  timeout -k 10 300 python3 bench.py --config $C --slice-of $S --no-cpu-baseline > $O/bench_${C}_s$S.json 2> $O/bench_${C}_s$S.err || exit $?
done
python3 - "$O" <<'PY'
import glob, json, os, sys
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "bench_*.json"))):
    d = json.load(open(f))
    r = d["roofline"]
    print(f"{os.path.basename(f):28s} {r['kernel_avg_us']:9.3f} us  frac {r['frac']:.4f}  {d['data'][:90]}")
PY
step done
