# Chunk means (ResNet-18 chunks, k = 10, m = 4 / 10 / 16) with the deferred
# -store kernel (default) and without (DLSIM_CHUNK_DEFER=0), fresh processes,
# alternating, outputs rotating beyond the Infinity Cache (round 5).
# usage: bash scripts/gpu_chunk_defer_ab.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-chunk_defer_ab}
mkdir -p $O
for i in 1 2; do
  for m in 4 10 16; do
    for v in 0 1; do
      DLSIM_CHUNK_DEFER=$v timeout -k 10 180 python3 scripts/bench_chunks.py --kernel-only --m $m --reps 200 > $O/m${m}_d${v}_$i.json 2> $O/m${m}_d${v}_$i.err || exit $?
      python3 -c "import json; d=json.load(open('$O/m${m}_d${v}_$i.json')); print('m=$m defer=$v run $i', d['kernel_us'], d['kernel_frac_of_8TBps'])"
    done
  done
done
