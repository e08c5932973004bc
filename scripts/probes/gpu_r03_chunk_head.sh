# After the chunk-mean head peel: the chunk GPU tests, then the kernel-only
# chunk bench with rocprofv3 stats and PMC, and the parity soak
# (scripts/probes/gpu_r03_chunk_pmc.sh).
# usage: bash scripts/probes/gpu_r03_chunk_head.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03_chunk_head}
mkdir -p $O
echo "[$(date +%T)] chunk tests"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_f64.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_chunks.log 2>&1
rc=$?; tail -5 $O/pytest_chunks.log
[ $rc -ne 0 ] && exit $rc
bash scripts/probes/gpu_r03_chunk_pmc.sh ${1:-r03_chunk_head}
