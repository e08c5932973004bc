# Physically contiguous output blocks and staging rows on/off (DLSIM_CONTIGUOUS)
# in fresh bench processes, alternating, with the outputs rotating beyond the
# Infinity Cache (round 5: does round 4's placement gain survive there?).
# usage: bash scripts/gpu_contig_ab.sh <outdir-name> "<bench args>"
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-contig_ab}
mkdir -p $O
ARGS=${2:-}
for i in 1 2 3; do
  for v in 1 0; do
    DLSIM_CONTIGUOUS=$v timeout -k 10 120 python3 bench.py $ARGS --no-cpu-baseline > $O/c${v}_$i.json 2> $O/c${v}_$i.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c${v}_$i.json')); print('contig=$v', $i, d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['config']['rows_alloc'][:30])"
  done
done
