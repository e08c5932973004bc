# Launch-shape sweep at the strong-scaling per-rank slice sizes:
# the north star (8 x 11,181,642 fp32) split over 8/4/2 ranks, cfg5's 100-way
# at the 8-rank slice, and cfg4 (2 x 125 M bf16) over 4 ranks. The harness
# rotates >= 1 GiB of input sets, so slices cannot be served by the MALL.
# usage: bash scripts/probes/gpu_tune_slices.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-slices}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
step() { echo "[$(date +%T)] $*"; }
F8=NF8_V4_sc1,NF8_V4_sc1_wave,NF8_V2_sc1_wave,NF8_V1_sc1_wave,NF8_V2_sc1_blk,NF8_V1_sc1_g1,NF8_V1_sc1_g2,NF8_V1_sc1_g4,NF8_V2_sc1_g1,NF8_V2_sc1_g2,NF8_V4_sc1_g1,NF8_V1_nt,NF8_V2_nt_wave,NF8_V4_nt_wave,NF8_V1_plain,NF8_V1_sc1_ldplain,NF8_xorprobe
for p in 1397760 2795456 5590848 11181642; do
  step "f32 n8 P=$p"
  DLSIM_TUNE_ONLY=$F8 timeout -k 10 200 $T 8 $p f32 exact 200 > $O/f32_n8_${p}.log 2>&1 || exit $?
done
B2=NF2_V4,NF2_V4_sc1,NF2_V1_sc1_wave,NF2_V2_sc1_wave,NF2_V2_sc1_blk,NF2_V1_sc1_g2,NF2_V1_sc1_g4,NF2_V2_sc1_g2,NF2_V1_nt,NF2_V2_nt_wave,NF2_V4_nt_wave
for p in 31250000 62500000; do
  step "bf16 n2 P=$p"
  DLSIM_TUNE_ONLY=$B2 timeout -k 10 200 $T 2 $p bf16 exact 100 > $O/bf16_n2_${p}.log 2>&1 || exit $?
done
step "f32 n100 P=1397760"
DLSIM_TUNE_ONLY=T_G8_V2,T_G8_V4,T_G8_V4_sc1,T_G8_V4_sc1_wave timeout -k 10 200 $T 100 1397760 f32 exact 50 > $O/f32_n100_1397760.log 2>&1 || exit $?
step done
