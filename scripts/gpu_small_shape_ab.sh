# A/B of round 5's small-row shape rule (dispatch.hpp size_class) against
# round 4's (DLSIM_SMALL_SHAPE_R04=1) in fresh bench processes, alternating.
# usage: bash scripts/gpu_small_shape_ab.sh <outdir-name> "<bench args>"
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-small_shape_ab}
mkdir -p $O
ARGS=${2:---config cfg2}
for i in 1 2 3; do
  for v in r05 r04; do
    if [ $v = r04 ]; then export DLSIM_SMALL_SHAPE_R04=1; else unset DLSIM_SMALL_SHAPE_R04; fi
    timeout -k 10 120 python3 bench.py $ARGS --no-cpu-baseline > $O/${v}_$i.json 2> $O/${v}_$i.err || exit $?
    python3 -c "import json; d=json.load(open('$O/${v}_$i.json')); print('$v', $i, d['roofline']['kernel_avg_us'], d['roofline']['frac'])"
  done
done
