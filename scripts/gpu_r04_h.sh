# Round 4: the device cache in the 4-worker deployment, task time by hits.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04h
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step workers
timeout -k 10 600 python3 -u scripts/bench_workers.py --peers 100 --workers 4 --rounds 6 --ways hip hip_cache > $O/workers_gnlenet.jsonl 2> $O/workers_gnlenet.err || exit $?
timeout -k 10 600 python3 -u scripts/bench_workers.py --peers 100 --workers 1 --rounds 6 --ways hip hip_cache > $O/workers_gnlenet_w1.jsonl 2> $O/workers_gnlenet_w1.err || exit $?
python3 -c "
import json
for f in ['$O/workers_gnlenet.jsonl', '$O/workers_gnlenet_w1.jsonl']:
    for l in open(f):
        d=json.loads(l); print(d['way'], d['workers'], d['aggregate_us_median'], d['aggregate_us_mean'], d.get('aggregate_us_median_by_hits'), d.get('device_cache', {}).get('hit_fraction'))"
step done
