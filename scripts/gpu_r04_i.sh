# Round 4: the device cache's host path against the normal one, one process.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04i
mkdir -p $O
echo "[$(date +%T)] cache_path"
timeout -k 10 400 python3 -u scripts/probes/probe_cache_path.py 200 > $O/cache_path.json 2> $O/cache_path.err || exit $?
cat $O/cache_path.json
echo "[$(date +%T)] done"
