# Lane map (block vs wave-contiguous) and store policy across sizes, repeated
# (csrc/tune_wreduce.hip; arena layout as in bench.py).
# usage: bash scripts/probes/gpu_mapsize.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-mapsize}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
export DLSIM_TUNE_STAGGER=0
step() { echo "[$(date +%T)] $*"; }
for rep in 1 2 3; do
  for p in 1048576 2097152 4194304 8388608 11181642 33554432; do
    step "f32 n8 P=$p rep $rep"
    DLSIM_TUNE_ONLY=NF8_V4,NF8_V4_sc1,NF8_V4_sc1_wave timeout -k 10 120 $T 8 $p f32 exact 200 > $O/f32_n8_${p}_$rep.log 2>&1 || exit $?
  done
  for p in 11181642 125000000; do
    step "bf16 n2 P=$p rep $rep"
    DLSIM_TUNE_ONLY=NF2_V4,NF2_V4_sc1,NF2_V4_sc1_wave,NF2_B512_V4 timeout -k 10 120 $T 2 $p bf16 exact 100 > $O/bf16_n2_${p}_$rep.log 2>&1 || exit $?
  done
done
step done
