# Chunked-model path: GPU tests, then the reconstruction bench.
# usage: bash scripts/probes/gpu_chunks.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-chunks}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -8
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step chunks; timeout -k 10 300 python3 scripts/bench_chunks.py > $O/bench_chunks.jsonl 2> $O/bench_chunks.err || exit $?
cat $O/bench_chunks.jsonl
step done
