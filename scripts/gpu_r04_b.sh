# Round 4, second GPU call: the whole -m gpu suite after the host-path
# changes (pinned host results with the deferred wait, pack-pool prewarm and
# spin), then the host-task A/B: parts and the whole call by result memory
# and prewarm, with and without the pool's spin; the 100-peer host round and
# cfg1 with the new defaults and with round 3's behaviour.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04b
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
step host_parts
timeout -k 10 300 python3 -u scripts/probes/probe_host_task_parts.py 400 > $O/host_parts_spin.json 2> $O/host_parts_spin.err || exit $?
DLSIM_PACK_SPIN_US=0 timeout -k 10 300 python3 -u scripts/probes/probe_host_task_parts.py 400 > $O/host_parts_nospin.json 2> $O/host_parts_nospin.err || exit $?
step rounds_host
timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 100 --host > $O/rounds_host_100_new.jsonl 2> $O/rounds_host_100_new.err || exit $?
DLSIM_PACK_SPIN_US=0 DLSIM_HOST_PREWARM=0 DLSIM_HOST_RESULT=pageable timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 100 --host > $O/rounds_host_100_r03.jsonl 2> $O/rounds_host_100_r03.err || exit $?
step cfg1
timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 2 --host --rounds 300 --cpu-rounds 300 > $O/cfg1_new.jsonl 2> $O/cfg1_new.err || exit $?
for f in $O/rounds_host_100_new.jsonl $O/rounds_host_100_r03.jsonl $O/cfg1_new.jsonl; do
  python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); print('$(basename $f)', d['kind'], d['us_per_task'], d['us_per_task_excl_gc'])"
done
step done
