# sc1 against non-temporal output stores for every shipped launch shape with
# the outputs rotating over >= 1 GiB (none stays in the 256 MiB Infinity
# Cache; round 5), inputs >= 1 GiB as always. Contiguous rows, the product's
# row alignment.
# usage: bash scripts/gpu_tune_ntsweep.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tune_ntsweep}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
run() {  # dtype n P
  local DT=$1 N=$2 P=$3
  local ESZ=4; [ $DT = bf16 ] && ESZ=2
  local OS=$(python3 -c "import math; print(max(3, math.ceil((1 << 30) / ($P * $ESZ))))")
  local AL=256; [ $ESZ = 4 ] && [ $((P * ESZ)) -ge 16777216 ] && AL=2097152
  env DLSIM_TUNE_NTSWEEP=1 DLSIM_TUNE_CONTIG=1 DLSIM_TUNE_ALIGN=$AL DLSIM_TUNE_OUT_SETS=$OS \
    timeout -k 10 240 $T $N $P $DT exact 100 > $O/${DT}_n${N}_$P.log 2>&1 || return 1
  echo "$DT n=$N P=$P out_sets=$OS $(grep variant $O/${DT}_n${N}_$P.log | sed -E 's/.*variant=(\S+).*batch_us=(\S+).*bfrac=(\S+) same=(\S).*/\1 \2 \3/' | tr '\n' ' ')"
}
for P in 1048576 1397760 2795456 5590848 11181642; do run f32 8 $P || exit 1; done
for P in 1397760 11181642; do run f32 17 $P || exit 1; done
for P in 1397760 11181642; do run f32 100 $P || exit 1; done
for P in 31250048 62500000 125000000; do run bf16 2 $P || exit 1; done
run bf16 17 11181642 || exit 1
