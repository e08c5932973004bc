# Row stride at power-of-two model sizes: does staggering arena rows help?
# usage: bash scripts/probes/gpu_pow2.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pow2}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
export DLSIM_TUNE_ONLY=NF8_V4,NF8_V4_sc1,NF8_V4_sc1_wave
step() { echo "[$(date +%T)] $*"; }
for p in 4194304 8388608 33554432; do
  step "P=$p separate"
  timeout -k 10 120 $T 8 $p f32 exact 100 > $O/f32_n8_${p}_sep.log 2>&1 || exit $?
  for s in 0 256 1024 4096 16384 65536; do
    step "P=$p stagger $s"
    DLSIM_TUNE_STAGGER=$s timeout -k 10 120 $T 8 $p f32 exact 100 > $O/f32_n8_${p}_s$s.log 2>&1 || exit $?
  done
done
export DLSIM_TUNE_ONLY=NF2_V4,NF2_V4_sc1,NF2_B512_V4
for p in 8388608 67108864; do
  for s in 0 256 4096; do
    step "bf16 P=$p stagger $s"
    DLSIM_TUNE_STAGGER=$s timeout -k 10 120 $T 2 $p bf16 exact 100 > $O/bf16_n2_${p}_s$s.log 2>&1 || exit $?
  done
done
step done
