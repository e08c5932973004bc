# North star in the tuning harness with the input rotation and the output
# rotation set apart (round 5): inputs over 3 or 12 sets, outputs over 1, 3,
# 12 or 24 buffers; sc1 (shipped), nt and plain stores.
# usage: bash scripts/gpu_tune_outsets.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tune_outsets}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for S in 3 12; do for OS in 1 3 12 24; do
  env DLSIM_TUNE_R03=1 DLSIM_TUNE_STORES=1 DLSIM_TUNE_CONTIG=1 DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_SETS=$S DLSIM_TUNE_OUT_SETS=$OS \
    DLSIM_TUNE_ONLY=NF8_V4_sc1_wave,NF8_V4_nt_wave,NF8_V4_plain_wave \
    timeout -k 10 240 $T 8 11181642 f32 exact 100 > $O/in${S}_out${OS}.log 2>&1 || exit $?
  echo "in=$S out=$OS $(grep variant $O/in${S}_out${OS}.log | sed -E 's/.*variant=(\S+).*batch_us=(\S+).*bfrac=(\S+) same=(\S).*/\1 \2 \3/' | tr '\n' ' ')"
done; done
