set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s8
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
step() { echo "[$(date +%T)] $*"; }
step n8;   timeout -k 10 300 $T 8 11182080 f32 exact 60 > $O/tune_n8.log 2>&1 || exit $?
step n8b;  timeout -k 10 300 $T 8 11182080 f32 exact 60 > $O/tune_n8_rep.log 2>&1 || exit $?
step n2;   timeout -k 10 300 $T 2 125001728 bf16 exact 30 > $O/tune_n2_bf16.log 2>&1 || exit $?
step done
