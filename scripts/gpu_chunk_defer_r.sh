# Chunk-mean deferred kernel: rows per block (DLSIM_DEFER_R) against the
# tiled kernel, ResNet-18 chunks k = 10 (round 5). R "d": the shipped rule.
# usage: bash scripts/gpu_chunk_defer_r.sh <outdir-name> "<m list>" "<R list>"
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-chunk_defer_r}
mkdir -p $O
for m in ${2:-4 10}; do
  for r in 0 ${3:-8 12 16 20 24}; do
    if [ $r = 0 ]; then v="DLSIM_CHUNK_DEFER=0"; elif [ $r = d ]; then v="DLSIM_CHUNK_DEFER=1"; else v="DLSIM_DEFER_R=$r"; fi
    env $v timeout -k 10 180 python3 scripts/bench_chunks.py --kernel-only --m $m --reps 200 > $O/m${m}_r$r.json 2> $O/m${m}_r$r.err || exit $?
    python3 -c "import json; d=json.load(open('$O/m${m}_r$r.json')); print('m=$m $v', d['kernel_us'], d['kernel_frac_of_8TBps'])"
  done
done
