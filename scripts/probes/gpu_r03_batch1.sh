# Round 3, call batch: the GPU tests touched this session, the small host
# chunk probe (one-DMA path), then the row-alignment size sweep.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_batch1
mkdir -p $O
echo "[$(date +%T)] pytest"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chunks.py tests/test_gpu_rounds.py tests/test_gpu_sharded_stub.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo "[$(date +%T)] small parts"
timeout -k 10 300 python3 scripts/probes/probe_small_parts.py > $O/small_parts.json 2> $O/small_parts.err || { tail -20 $O/small_parts.err; exit 1; }
cat $O/small_parts.json
echo "[$(date +%T)] sizes"
bash scripts/probes/gpu_r03_layout_sizes.sh r03_layout_sizes
