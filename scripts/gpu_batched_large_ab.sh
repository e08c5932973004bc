# dlsim_wreduce_batched over ResNet-18-sized tasks: large tasks alone through
# the deferred-store kernel (default) against one kernel-argument batch
# (DLSIM_DEFER=0), fresh processes, alternating (round 5).
# usage: bash scripts/gpu_batched_large_ab.sh <outdir-name> [b]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-batched_large}
mkdir -p $O
for i in 1 2; do
  for v in 0 1; do
    DLSIM_DEFER=$v timeout -k 10 180 python3 scripts/probes/probe_batched_large.py ${2:-8} >> $O/ab.jsonl 2> $O/err_${v}_${i}.log || exit $?
    tail -1 $O/ab.jsonl
  done
done
