# A/B of the small-slice shapes in fresh harness processes (round 5): the
# shipped whole-tile grids against the balanced one-shot grids (k_bal).
# usage: bash scripts/gpu_tune_small_ab.sh <outdir-name> "<sizes>"
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-small_ab}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for P in ${2:-1048576 1397760 1800000 2795456}; do for k in 1 2 3; do
  DLSIM_TUNE_SMALL=1 DLSIM_TUNE_SMALL_BAL=1 DLSIM_TUNE_CONTIG=1 DLSIM_TUNE_ALIGN=256 \
    timeout -k 10 120 $T 8 $P f32 exact 400 > $O/s_${P}_$k.log 2>&1 || exit $?
  echo "P=$P run=$k $(grep variant $O/s_${P}_$k.log | sed -E 's/.*variant=(\S+).*batch_us=(\S+).*bfrac=(\S+) same=(\S).*/\1 \2 \3 \4/' | tr '\n' ' ')"
done; done
