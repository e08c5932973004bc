# Quick GPU validation: full -m gpu suite, smoke(), default bench line.
# usage: bash scripts/gpu_check.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-check}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke;  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
step bench;  timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
step done
