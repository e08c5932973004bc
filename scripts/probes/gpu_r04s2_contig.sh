# Round 4 session 2: physically contiguous rows vs torch's allocator (probe_contiguous.py),
# then the default bench under rocprofv3 kernel stats (csv).
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04s2_contig
mkdir -p $O
echo "[$(date +%T)] probe"
timeout -k 10 400 python3 -u scripts/probes/probe_contiguous.py 3 > $O/contig.jsonl 2> $O/contig.err || exit $?
tail -4 $O/contig.jsonl
echo "[$(date +%T)] rocprof"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || exit $?
echo "[$(date +%T)] done"
