# Deferred-store grids (k_defer: each block folds R tiles, keeps the results in
# registers and stores them at the end) against the shipped shape, outputs
# rotating over 24 buffers (beyond the Infinity Cache), round 5.
# usage: bash scripts/gpu_tune_defer.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tune_defer}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for k in 1 2; do
  env DLSIM_TUNE_R03=1 DLSIM_TUNE_DEFER=1 DLSIM_TUNE_CONTIG=1 DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_SETS=3 DLSIM_TUNE_OUT_SETS=24 \
    timeout -k 10 240 $T 8 11181642 f32 exact 100 > $O/defer_$k.log 2>&1 || exit $?
  echo "run $k: $(grep variant $O/defer_$k.log | sed -E 's/.*variant=NF8_(\S+).*batch_us=(\S+).*bfrac=(\S+) same=(\S) moved.*/\1 \2 \3 same=\4/' | tr '\n' '|')"
done
