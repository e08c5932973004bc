# Launch shapes of the north star at 3 and 12 rotating sets in the tuning
# harness (round 5, after the translation counters of gpu_translation_pmc.sh):
# does a shape with more bytes in flight, another store policy or a tile order
# recover the 12-set loss? Contiguous 2 MiB-aligned rows as the bench.
# usage: bash scripts/gpu_tune_footprint.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tune_footprint}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for mode in STORES TLB; do for S in 3 12; do
  env DLSIM_TUNE_R03=1 DLSIM_TUNE_$mode=1 DLSIM_TUNE_CONTIG=1 DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_SETS=$S \
    timeout -k 10 240 $T 8 11181642 f32 exact 100 > $O/${mode}_sets$S.log 2>&1 || exit $?
  echo "$mode sets=$S $(grep variant $O/${mode}_sets$S.log | sed -E 's/.*variant=(\S+).*batch_us=(\S+).*bfrac=(\S+) same=(\S).*/\1 \2 \3/' | tr '\n' ' ')"
done; done
