# Size sweep of the launch shape per dtype: fp32 block vs wave lane map (n=8),
# bf16 V4 nt block map vs V1/V2 sc1 wave map (n=2, n=8); arena rows staggered
# by 4 KiB like arena.row_stride does at power-of-two strides.
# usage: bash scripts/probes/gpu_shape_sweep.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-shape}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
export DLSIM_TUNE_STAGGER=4096
step() { echo "[$(date +%T)] $*"; }
for p in 1048576 2097152 3145728 4194304 6291456 8388608 11182080; do
  step "f32 n8 P=$p"
  DLSIM_TUNE_ONLY=NF8_V4_sc1,NF8_V4_sc1_wave timeout -k 10 120 $T 8 $p f32 exact 200 > $O/f32_n8_${p}.log 2>&1 || exit $?
done
for p in 4194304 11182080 22364160 33546240 67092480 125001728; do
  step "bf16 n2 P=$p"
  DLSIM_TUNE_ONLY=NF2_V4,NF2_V4_sc1,NF2_V2_sc1_wave,NF2_V1_sc1_wave timeout -k 10 120 $T 2 $p bf16 exact 100 > $O/bf16_n2_${p}.log 2>&1 || exit $?
done
for p in 1048576 11182080 33546240; do
  step "bf16 n8 P=$p"
  DLSIM_TUNE_ONLY=NF8_V4,NF8_V4_sc1,NF8_V2_sc1_wave,NF8_V1_sc1_wave timeout -k 10 120 $T 8 $p bf16 exact 100 > $O/bf16_n8_${p}.log 2>&1 || exit $?
done
step done
