# Round 4: the per-worker device model cache (device_cache.py) on MI355X:
# its GPU tests (single process, eviction, the broker/worker fork and spawn
# models), the host-path tests, then host rounds whose trained models live in
# file_system shared memory, with and without the cache (GNLeNet, 100 peers;
# ResNet-18, 16 peers).
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04d
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 600 python3 -u -m pytest -p no:cacheprovider -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_device_cache.py tests/test_gpu_worker_process.py tests/test_gpu_dropin.py > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|error" $O/pytest.log | tail -4
if [ $rc -ne 0 ]; then exit $rc; fi
step rounds
for m in gnlenet:100 resnet18:16; do
  model=${m%%:*}; peers=${m##*:}
  timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers $peers --model $model --host --shm > $O/rounds_${model}_shm.jsonl 2> $O/rounds_${model}_shm.err || exit $?
  DLSIM_DEVICE_CACHE_MB=4096 timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers $peers --model $model --host --shm > $O/rounds_${model}_shm_cache.jsonl 2> $O/rounds_${model}_shm_cache.err || exit $?
done
for f in $O/rounds_*.jsonl; do
  python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); print('$(basename $f)', d['kind'], d['us_per_task'], d['us_per_task_excl_gc'], d.get('device_cache', {}).get('hits'), d.get('device_cache', {}).get('misses'))"
done
step done
