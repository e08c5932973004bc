# Round 3: the chunk-mean kernel against its own
# memory-only probe at ResNet-18 chunk sizes (k = 10 indices of 1.1 M fp32,
# m = 4 and 10 contributors, plus m = 16), every chunk index in one launch;
# then the chunk benches (device and host chunks, the reference's GNLeNet).
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_chunks
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for m in 4 10 16; do
  echo "[$(date +%T)] m=$m"
  DLSIM_TUNE_CHUNK=1 timeout -k 10 180 $T $m 1118164 10 100 > $O/cm_m$m.log 2>&1 || { cat $O/cm_m$m.log; exit 1; }
  grep -E "^variant" $O/cm_m$m.log | awk '{print $1, $5, $7, $8}'
done
echo "[$(date +%T)] bench_chunks"
timeout -k 10 300 python3 scripts/bench_chunks.py > $O/bench_chunks.jsonl 2> $O/bench_chunks.err || { tail -5 $O/bench_chunks.err; exit 1; }
cat $O/bench_chunks.jsonl
timeout -k 10 300 python3 scripts/bench_chunks.py --models > $O/bench_chunks_models.jsonl 2> $O/bench_chunks_models.err || { tail -5 $O/bench_chunks_models.err; exit 1; }
cat $O/bench_chunks_models.jsonl
echo "[$(date +%T)] done"
