# The north star's shapes with non-temporal buffer stores, outputs rotating
# over 24 buffers (1.07 GB, none stays in the Infinity Cache), inputs over 3
# sets: register streaming (VPT 1-8, grid-stride grids), the software-
# pipelined grid, the LDS-DMA ring, and read-only / write-only probes of the
# same tiles (round 5).
# usage: bash scripts/gpu_tune_honest.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-tune_honest}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for k in 1 2; do
  env DLSIM_TUNE_R03=1 DLSIM_TUNE_HONEST=1 DLSIM_TUNE_CONTIG=1 DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_SETS=3 DLSIM_TUNE_OUT_SETS=24 \
    timeout -k 10 240 $T 8 11181642 f32 exact 100 > $O/honest_$k.log 2>&1 || exit $?
  echo "run $k: $(grep variant $O/honest_$k.log | sed -E 's/.*variant=NF8_(\S+).*batch_us=(\S+).*bfrac=(\S+) same=(\S) moved=\S+ moved_bfrac=(\S+).*/\1 \2 \3 \5/' | tr '\n' '|')"
done
