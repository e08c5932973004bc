# Per-rank work of the strong-scaling split on one GPU: rank 0's slice of the
# north star (and cfg5) over 1, 2, 4, 8 ranks, each alone on the card. With no
# data-path collective the N-rank strong-scaling time is the slowest rank's,
# so these per-slice times bound the speed-up.
# usage: bash scripts/probes/gpu_strong_slices.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-strong}
mkdir -p $O
for c in north_star cfg5; do
  for n in 1 2 4 8; do
    echo "[$(date +%T)] $c slice of $n"
    timeout -k 10 200 python3 bench.py --config $c --slice-of $n --no-cpu-baseline --steps 400 --warmup 40 \
      >> $O/slices.jsonl 2>> $O/slices.err || exit $?
  done
done
