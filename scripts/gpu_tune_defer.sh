# Deferred-store grids (k_defer: each block folds R tiles, keeps the results in
# registers and stores them at the end; R chosen from the size so the grid is
# about one block per CU) against the shipped shape, outputs rotating beyond
# the Infinity Cache, over fan-in and size, round 5.
# usage: bash scripts/gpu_tune_defer.sh <outdir-name> ["n:P n:P ..."]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tune_defer}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
CASES=${2:-"8:11181642 8:11181642 8:2795410 8:44726568 2:11181642 4:11181642 4:2795410"}
k=0
for c in $CASES; do
  n=${c%%:*}; P=${c##*:}; k=$((k+1))
  # outputs: >= 1 GiB of rotation (24 x 44.7 MB at the north-star size)
  os=$(( (1073741824 / (P * 4)) + 1 )); [ $os -lt 4 ] && os=4
  env DLSIM_TUNE_R03=1 DLSIM_TUNE_DEFER=1 DLSIM_TUNE_CONTIG=1 DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_OUT_SETS=$os \
    timeout -k 10 240 $T $n $P f32 exact 100 > $O/defer_${k}_n${n}_P${P}.log 2>&1 || exit $?
  echo "n=$n P=$P: $(grep variant $O/defer_${k}_n${n}_P${P}.log | sed -E 's/.*variant=NF[0-9]+_(\S+).*batch_us=(\S+).*bfrac=(\S+) same=(\S) moved.*/\1 \2 \3 same=\4/' | tr '\n' '|')"
done
