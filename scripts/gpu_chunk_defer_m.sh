# Chunk means: the deferred-store chunk kernel (compiled for its R) at every
# contributor count (DLSIM_CHUNK_DEFER_MIN_M=2) against the tiled kernel
# (DLSIM_CHUNK_DEFER=0), ResNet-18 chunks k = 10, fresh processes (round 5).
# usage: bash scripts/gpu_chunk_defer_m.sh <outdir-name> "<m list>"
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-chunk_defer_m}
mkdir -p $O
for i in 1 2; do
  for m in ${2:-4 10 16}; do
    for v in DLSIM_CHUNK_DEFER=0 DLSIM_CHUNK_DEFER_MIN_M=2; do
      env $v timeout -k 10 180 python3 scripts/bench_chunks.py --kernel-only --m $m --reps 200 > $O/m${m}_${v%%=*}_$i.json 2> $O/m${m}_${v%%=*}_$i.err || exit $?
      python3 -c "import json; d=json.load(open('$O/m${m}_${v%%=*}_$i.json')); print('m=$m $v run $i', d['kernel_us'], d['kernel_frac_of_8TBps'])"
    done
  done
done
