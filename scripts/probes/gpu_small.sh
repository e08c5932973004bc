# Launch shapes for the small, launch-bound sizes (cfg2: 8 x 1,048,576 fp32;
# 2 x 11 M bf16), every variant of csrc/tune_wreduce.hip.
# usage: bash scripts/probes/gpu_small.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-small}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
step() { echo "[$(date +%T)] $*"; }
step cfg2;  DLSIM_TUNE_STAGGER=0 timeout -k 10 120 $T 8 1048576 f32 exact 200 > $O/n8_1M_f32.log 2>&1 || exit $?
step cfg2b; DLSIM_TUNE_STAGGER=0 timeout -k 10 120 $T 8 4194304 f32 exact 200 > $O/n8_4M_f32.log 2>&1 || exit $?
step bf16;  DLSIM_TUNE_STAGGER=0 timeout -k 10 120 $T 2 11181642 bf16 exact 200 > $O/n2_11M_bf16.log 2>&1 || exit $?
step done
