# Round 4 session 2: which stream's placement matters (rows / outputs / both
# contiguous), three fresh processes of the probe.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04s2_contig2
mkdir -p $O
for i in 1 2 3; do
  echo "[$(date +%T)] probe $i"
  PROBE_NO12=1 timeout -k 10 300 python3 -u scripts/probes/probe_contiguous.py 3 > $O/contig_$i.jsonl 2> $O/contig_$i.err || exit $?
done
echo "[$(date +%T)] done"
