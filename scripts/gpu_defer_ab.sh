# Deferred-store kernel variants in fresh bench processes, round-robin,
# outputs rotating beyond the Infinity Cache (round 5). A variant is a
# comma-separated env list ("DLSIM_DEFER=0", "DLSIM_DEFER_R=16,DLSIM_DEFER_LDS_KB=0").
# usage: bash scripts/gpu_defer_ab.sh <outdir-name> "<bench args>" [runs] [variant ...]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-defer_ab}
mkdir -p $O
ARGS=${2:-}
N=${3:-3}
shift 3 2>/dev/null || shift $#
VARIANTS=("$@")
[ ${#VARIANTS[@]} -eq 0 ] && VARIANTS=("DLSIM_DEFER=1" "DLSIM_DEFER=0")
for i in $(seq 1 $N); do
  k=0
  for v in "${VARIANTS[@]}"; do
    k=$((k+1))
    env ${v//,/ } timeout -k 10 120 python3 bench.py $ARGS --no-cpu-baseline > $O/v${k}_$i.json 2> $O/v${k}_$i.err || exit $?
    python3 -c "import json; d=json.load(open('$O/v${k}_$i.json')); r=d['roofline']; print('$v', $i, r['kernel'], r['kernel_avg_us'], r['frac'])"
  done
done
