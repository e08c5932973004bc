# Ragged end split over two blocks (RAGGED=2, shipped) vs block 0 alone
# (RAGGED=1, round-1 shape), bench-like arena layout.
# usage: bash scripts/probes/gpu_ragged.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ragged}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
export DLSIM_TUNE_STAGGER=0
step() { echo "[$(date +%T)] $*"; }
for rep in 1 2; do
  for p in 1048576 11181642; do
    step "f32 n8 P=$p rep $rep"
    DLSIM_TUNE_ONLY=NF8_V4_sc1_wave,NF8_V4_sc1_wave_r1,NF8_V4,NF8_V4_r1 timeout -k 10 120 $T 8 $p f32 exact 200 > $O/f32_n8_${p}_$rep.log 2>&1 || exit $?
  done
  step "f32 n17 rep $rep"
  DLSIM_TUNE_ONLY=NF17_V4_sc1_wave,NF17_V4_sc1_wave_r1 timeout -k 10 120 $T 17 11181642 f32 exact 100 > $O/f32_n17_11181642_$rep.log 2>&1 || exit $?
  for p in 11181642 125000000; do
    step "bf16 n2 P=$p rep $rep"
    DLSIM_TUNE_ONLY=NF2_V4,NF2_V4_r1,NF2_V4_sc1_wave,NF2_V4_sc1_wave_r1 timeout -k 10 120 $T 2 $p bf16 exact 100 > $O/bf16_n2_${p}_$rep.log 2>&1 || exit $?
  done
done
step done
