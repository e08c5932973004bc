# Every output store cache policy of the north star's shape with the outputs
# rotating over 3 buffers (they stay in the 256 MiB Infinity Cache) and over
# 24 (1.07 GB: every write reaches HBM), inputs over 3 and 12 sets (round 5).
# usage: bash scripts/gpu_tune_stpol.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tune_stpol}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for S in 3 12; do for OS in 3 24; do
  env DLSIM_TUNE_R03=1 DLSIM_TUNE_STPOL=1 DLSIM_TUNE_CONTIG=1 DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_SETS=$S DLSIM_TUNE_OUT_SETS=$OS \
    timeout -k 10 240 $T 8 11181642 f32 exact 100 > $O/in${S}_out${OS}.log 2>&1 || exit $?
  echo "in=$S out=$OS $(grep variant $O/in${S}_out${OS}.log | sed -E 's/.*variant=NF8_V4_(\S+).*batch_us=(\S+).*bfrac=(\S+) same=(\S).*/\1 \2 \3/' | tr '\n' ' ')"
done; done
