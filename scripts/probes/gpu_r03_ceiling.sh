# Round 3: the ceiling of the north star's 8:1
# read/write mix. The tuning harness (DLSIM_TUNE_R03) times the shipped large
# fp32 shape, the memory-only probe, read-only and write-only probes of the
# same tiles and pipelined LDS-DMA rings (nt / default policy), interleaved,
# >= 1 GiB rotating, at a wave-tile multiple of the north star's size, in the
# bench's arena layout and with separate allocations.
# usage: bash scripts/probes/gpu_r03_ceiling.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03_ceiling}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
echo "[$(date +%T)] arena"
DLSIM_TUNE_R03=1 DLSIM_TUNE_STAGGER=0 timeout -k 10 240 $T 8 11181568 f32 exact 100 > $O/ceiling_arena.log 2>&1 || exit $?
cat $O/ceiling_arena.log
echo "[$(date +%T)] separate"
DLSIM_TUNE_R03=1 timeout -k 10 240 $T 8 11181568 f32 exact 100 > $O/ceiling_separate.log 2>&1 || exit $?
cat $O/ceiling_separate.log
echo "[$(date +%T)] slice8"
DLSIM_TUNE_R03=1 DLSIM_TUNE_STAGGER=0 timeout -k 10 240 $T 8 1397760 f32 exact 200 > $O/ceiling_slice8.log 2>&1 || exit $?
cat $O/ceiling_slice8.log
echo "[$(date +%T)] done"
