# rocprofv3 kernel stats and PMC traffic of k_chunk_mean_batch (Conflux's
# reconstruct, k = 10 ResNet-18-sized chunks, m = 4 and 10; >= 1 GiB rotating),
# then a parity soak of the whole product path at HEAD.
# usage: bash scripts/probes/gpu_r03_chunk_pmc.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03_chunk_pmc}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
P=11181642
for M in 4 10; do
  B=$(( (M + 1) * P * 4 ))
  A="scripts/bench_chunks.py --kernel-only --m $M"
  step "m=$M events"; timeout -k 10 300 python3 $A > $O/events_m$M.jsonl 2> $O/events_m$M.err || exit $?
  cat $O/events_m$M.jsonl
  step "m=$M trace";  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace_m$M -o run -- python3 $R/$A > $O/trace_m$M.log 2>&1 || exit $?
  step "m=$M fetch";  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch_m$M -o run -- python3 $R/$A --reps 50 > $O/fetch_m$M.log 2>&1 || exit $?
  step "m=$M write";  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write_m$M -o run -- python3 $R/$A --reps 50 > $O/write_m$M.log 2>&1 || exit $?
  python3 scripts/pmc_summary.py --trace $O/trace_m$M --fetch $O/fetch_m$M --write $O/write_m$M --kernel k_chunk_mean_batch \
    --config chunk_mean_k10_m$M --mode exact --bytes-per-launch $B --out $O/r03_chunk_pmc_traffic.json || exit 1
done
step soak; timeout -k 10 200 python3 scripts/fuzz_parity.py --seconds 150 --seed 313 > $O/fuzz.json 2> $O/fuzz.err || exit $?
tail -c 600 $O/fuzz.json
step done
