# Zero-copy small host tasks against the DMA pipeline (round 5): cfg1 (2-peer
# D-PSGD, host GNLeNet models, 40 rounds) and the 100-peer fan-in-7 round,
# DLSIM_ZERO_COPY=1 (shipped) and 0 alternating in fresh processes; then the
# library-level probe.
# usage: bash scripts/gpu_zc_ab.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-zc_ab}
mkdir -p $O
for i in 1 2; do for zc in 1 0; do
  export DLSIM_ZERO_COPY=$zc
  timeout -k 10 300 python3 scripts/bench_rounds.py --peers 2 --host --rounds 40 > $O/cfg1_zc${zc}_$i.jsonl 2> $O/cfg1_zc${zc}_$i.err || exit $?
  timeout -k 10 300 python3 scripts/bench_rounds.py --peers 100 --host --rounds 4 > $O/r100_zc${zc}_$i.jsonl 2> $O/r100_zc${zc}_$i.err || exit $?
  echo "zc=$zc run=$i"; tail -n 3 $O/cfg1_zc${zc}_$i.jsonl | cut -c1-400; tail -n 3 $O/r100_zc${zc}_$i.jsonl | cut -c1-400
done; done
unset DLSIM_ZERO_COPY
timeout -k 10 300 python3 scripts/probes/probe_zero_copy.py 400 > $O/zero_copy.json || exit $?
cat $O/zero_copy.json
