# Kernel-shape sweep round 2 (LDS-DMA, store policy) + aligned bench line.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
step() { echo "[$(date +%T)] $*"; }
# P multiple of the tile (2048 vectors = 8192 floats) so LDS variants are exact
step tune n8;    timeout -k 10 300 $T 8 11182080 f32 exact 40 > $O/tune3_n8_f32.log 2>&1 || exit $?
step tune n8big; timeout -k 10 300 $T 8 44728320 f32 exact 20 > $O/tune3_n8_f32_big.log 2>&1 || exit $?
step tune n17;   timeout -k 10 300 $T 17 11182080 f32 exact 30 > $O/tune3_n17_f32.log 2>&1 || exit $?
step tune bf16;  timeout -k 10 300 $T 2 125001728 bf16 exact 30 > $O/tune3_n2_bf16.log 2>&1 || exit $?
step bench;      timeout -k 10 300 python3 bench.py > $O/bench2_default.json 2> $O/bench2_default.err || exit $?
cat $O/bench2_default.json
step done
