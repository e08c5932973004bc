# Round-level aggregate wall time (scripts/bench_rounds.py) plus the GPU tests
# of the round executor / batch / drop-in paths.
# usage: bash scripts/probes/gpu_rounds.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-rounds}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step rounds; timeout -k 10 300 python3 scripts/bench_rounds.py > $O/rounds.jsonl 2> $O/rounds.err || exit $?
cat $O/rounds.jsonl
step profile; timeout -k 10 300 python3 scripts/bench_rounds.py --rounds 2 --cpu-rounds 1 --profile $O/prof.txt > $O/prof.jsonl 2>&1 || exit $?
step done
