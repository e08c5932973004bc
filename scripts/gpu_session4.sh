# bf16 exact rounding variants + full GPU test suite on the new BF16Exact.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_wreduce
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -m pytest tests -m gpu -q -p no:cacheprovider -x > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in exact exactint exactold; do
  for n in 2 8; do
    step tune bf16 $m n$n; timeout -k 10 300 $T $n 11182080 bf16 $m 30 > $O/tune_bf16_${m}_n$n.log 2>&1 || exit $?
  done
done
step tune f32 n8; timeout -k 10 300 $T 8 11182080 f32 exact 30 > $O/tune_f32_n8.log 2>&1 || exit $?
step sweep; timeout -k 10 600 python3 scripts/sweep_fanin.py > $O/sweep.jsonl 2> $O/sweep.err || exit $?
step done
