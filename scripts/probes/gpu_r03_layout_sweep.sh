# Round 3: input/output alignment across the configs' sizes. For each
# (n, P, dtype) the fast harness (csrc/build/tune_f32, DLSIM_TUNE_LAYOUT)
# times every shipped launch shape with the inputs as arena rows aligned to
# 256 B (today's arena.row_stride), 4 KiB, 2 MiB, 2 MiB with the outputs
# 256 B off their 2 MiB alignment, and separate allocations.
# usage: bash scripts/probes/gpu_r03_layout_sweep.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03_layout_sweep}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
run() {  # tag n P dtype env...
  local TAG=$1 N=$2 P=$3 DT=$4; shift 4
  env DLSIM_TUNE_LAYOUT=1 "$@" timeout -k 10 120 $T $N $P $DT exact 200 > $O/$TAG.log 2>&1 || return 1
  echo "$TAG $(grep -E '^variant' $O/$TAG.log | awk '{print $1, $8}' | sed 's/variant=//; s/batch_us=//' | tr '\n' ' ')"
}
for cfg in "8 11181642 f32" "8 8388608 f32" "8 5590848 f32" "8 2795456 f32" "8 1397760 f32" \
           "17 11181642 f32" "17 1397760 f32" "100 1397760 f32" "2 125000000 bf16" "2 31250000 bf16"; do
  set -- $cfg
  K="n$1_p$2_$3"
  echo "[$(date +%T)] $K"
  run ${K}_a256 $1 $2 $3 DLSIM_TUNE_ALIGN=256 || exit 1
  run ${K}_a2m $1 $2 $3 DLSIM_TUNE_ALIGN=2097152 || exit 1
  run ${K}_a4k $1 $2 $3 DLSIM_TUNE_ALIGN=4096 || exit 1
  run ${K}_a2m_o256 $1 $2 $3 DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_OUT_OFFSET=256 || exit 1
  run ${K}_sep $1 $2 $3 || exit 1
  run ${K}_a2m_r $1 $2 $3 DLSIM_TUNE_ALIGN=2097152 || exit 1
  run ${K}_a256_r $1 $2 $3 DLSIM_TUNE_ALIGN=256 || exit 1
done
echo "[$(date +%T)] done"
