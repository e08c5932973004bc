# Kernel-shape sweep with the standalone harness (csrc/tune_wreduce.hip).
# usage: bash scripts/probes/gpu_tune.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tune}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
step() { echo "[$(date +%T)] $*"; }
# P multiple of the tile so the LDS-DMA experiment variants are exact
step n8;   timeout -k 10 300 $T 8 11182080 f32 exact 60 > $O/tune_n8_f32.log 2>&1 || exit $?
step n17;  timeout -k 10 300 $T 17 11182080 f32 exact 40 > $O/tune_n17_f32.log 2>&1 || exit $?
step n2;   timeout -k 10 300 $T 2 125001728 bf16 exact 30 > $O/tune_n2_bf16.log 2>&1 || exit $?
step done
