# Deferred-store kernel: one round of blocks (R = ceil(rows / CUs), even; the
# shipped rule) against two rounds (R = ceil(rows / 2 CUs), even) and the
# tiled kernel, per fan-in and size, in fresh bench processes (round 5).
# usage: bash scripts/gpu_defer_rounds.sh <outdir-name> ["n:P ..."]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-defer_rounds}
mkdir -p $O
SHAPES=${2:-"4:11181642 4:16000000 6:8400000 6:11181642 8:5600000 8:8400000 8:11181642 8:16000000 10:11181642 10:16000000"}
for sh in $SHAPES; do
  n=${sh%%:*}; P=${sh##*:}
  rows=$(( (P / 4 + 511) / 512 ))
  one=$(( ((rows + 255) / 256 + 1) / 2 * 2 )); two=$(( ((rows + 511) / 512 + 1) / 2 * 2 ))
  for v in "DLSIM_DEFER=0" "DLSIM_DEFER_R=$one,DLSIM_DEFER_MAX_FAN_IN=14" "DLSIM_DEFER_R=$two,DLSIM_DEFER_MAX_FAN_IN=14"; do
    tag=$(echo "$v" | tr ',=' '__')
    env ${v//,/ } timeout -k 10 120 python3 bench.py --shape $n:$P --no-cpu-baseline > $O/n${n}_P${P}_$tag.json 2> $O/n${n}_P${P}_$tag.err || exit $?
    python3 -c "import json; d=json.load(open('$O/n${n}_P${P}_$tag.json')); r=d['roofline']; print('n=$n P=$P $v', r['kernel'], r['kernel_avg_us'], r['frac'])"
  done
done
