# Round 4, host-path GPU call (r04c; r04b ran the same steps on the prewarm /
# spin version, since removed): the whole -m gpu suite, then the host-task
# A/B: parts and the whole call by result memory (pinned with the deferred
# wait / pageable) and smallest H2D run (DLSIM_H2D_MIN_KB); the 100-peer host
# round and cfg1 with the new defaults and with round 3's behaviour.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04c
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -3
if [ $rc -ne 0 ]; then exit $rc; fi
step host_parts
timeout -k 10 300 python3 -u scripts/probes/probe_host_task_parts.py 400 > $O/host_parts.json 2> $O/host_parts.err || exit $?
step rounds_host
timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 100 --host > $O/rounds_host_100_new.jsonl 2> $O/rounds_host_100_new.err || exit $?
DLSIM_H2D_MIN_KB=0 DLSIM_HOST_RESULT=pageable timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 100 --host > $O/rounds_host_100_r03.jsonl 2> $O/rounds_host_100_r03.err || exit $?
step cfg1
timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 2 --host --rounds 300 --cpu-rounds 300 > $O/cfg1_new.jsonl 2> $O/cfg1_new.err || exit $?
DLSIM_H2D_MIN_KB=0 DLSIM_HOST_RESULT=pageable timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 2 --host --rounds 300 --cpu-rounds 300 > $O/cfg1_r03.jsonl 2> $O/cfg1_r03.err || exit $?
cat $O/host_parts.json
for f in $O/rounds_host_100_new.jsonl $O/rounds_host_100_r03.jsonl $O/cfg1_new.jsonl $O/cfg1_r03.jsonl; do
  python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); print('$(basename $f)', d['kind'], d['us_per_task'], d['us_per_task_excl_gc'])"
done
step done
