# Zero-copy small host tasks with the pack and the PCIe-reading reduce
# pipelined over chunks of the element axis (DLSIM_ZC_CHUNK_KB, default 128)
# against one chunk (0): cfg1 and the 100-peer fan-in-7 round, fresh
# processes, alternating (round 5).
# usage: bash scripts/gpu_zc_chunks_ab.sh <outdir-name> "<chunk KB list>"
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-zc_chunks_ab}
mkdir -p $O
for i in 1 2; do for kb in ${2:-0 128 64}; do
  export DLSIM_ZC_CHUNK_KB=$kb
  timeout -k 10 300 python3 scripts/bench_rounds.py --peers 2 --host --rounds 40 > $O/cfg1_kb${kb}_$i.jsonl 2> $O/cfg1_kb${kb}_$i.err || exit $?
  timeout -k 10 300 python3 scripts/bench_rounds.py --peers 100 --host --rounds 4 > $O/r100_kb${kb}_$i.jsonl 2> $O/r100_kb${kb}_$i.err || exit $?
  echo "chunk_kb=$kb run=$i"; tail -n 1 $O/cfg1_kb${kb}_$i.jsonl | cut -c1-300; tail -n 1 $O/r100_kb${kb}_$i.jsonl | cut -c1-300
done; done
