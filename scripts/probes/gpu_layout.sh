# Input-layout experiment: separate allocations vs one arena, with and
# without a per-row stagger (csrc/tune_wreduce.hip, DLSIM_TUNE_STAGGER).
# usage: bash scripts/probes/gpu_layout.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-layout}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
export DLSIM_TUNE_ONLY=NF8_V4_sc1_wave,NF8_V4_sc1,NF17_V4_sc1_wave,NF17_V4_sc1,NF2_V4,NF2_V4_sc1
step() { echo "[$(date +%T)] $*"; }
for rep in 1 2; do
  step "separate rep $rep"
  timeout -k 10 120 $T 8 11181642 f32 exact 60 > $O/n8_separate_$rep.log 2>&1 || exit $?
  for s in 0 256 1024 4096 12288 65536 2101248; do
    step "stagger $s rep $rep"
    DLSIM_TUNE_STAGGER=$s timeout -k 10 120 $T 8 11181642 f32 exact 60 > $O/n8_stagger${s}_$rep.log 2>&1 || exit $?
  done
done
step "n17"
timeout -k 10 120 $T 17 11181642 f32 exact 40 > $O/n17_separate.log 2>&1 || exit $?
for s in 0 4096; do
  DLSIM_TUNE_STAGGER=$s timeout -k 10 120 $T 17 11181642 f32 exact 40 > $O/n17_stagger$s.log 2>&1 || exit $?
done
step "n2 bf16"
timeout -k 10 120 $T 2 125000000 bf16 exact 30 > $O/n2_separate.log 2>&1 || exit $?
for s in 0 4096; do
  DLSIM_TUNE_STAGGER=$s timeout -k 10 120 $T 2 125000000 bf16 exact 30 > $O/n2_stagger$s.log 2>&1 || exit $?
done
step done
