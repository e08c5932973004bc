# Small-slice launch shapes in the tuning harness (round 5):
# the shipped one-tile-per-block shapes against software-pipelined persistent
# grids, n = 8 fp32 at the 8-, 4- and 2-rank slices and cfg2, contiguous rows
# and outputs (the bench's allocation), >= 1 GiB rotating.
# usage: bash scripts/gpu_tune_small.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tune_small}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for P in 1397760 1048576 2795456 5590848; do
  echo "[$(date +%T)] P=$P"
  DLSIM_TUNE_SMALL=1 DLSIM_TUNE_CONTIG=1 DLSIM_TUNE_ALIGN=256 timeout -k 10 240 $T 8 $P f32 exact 200 > $O/small_$P.log 2>&1 || exit $?
  grep variant $O/small_$P.log | awk '{print $1, $6, $9, $10, $12}'
done
