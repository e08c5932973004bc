# Round 4: the slab-backed device cache: its GPU tests, then the reference's
# broker/worker deployment timed (bench_workers.py: CPU reference, HIP, HIP +
# cache; GNLeNet 100 peers and ResNet-18 16 peers, 4 workers).
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04g
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 400 python3 -u -m pytest -p no:cacheprovider -x -q --timeout 240 --timeout-method thread \
  tests/test_gpu_device_cache.py tests/test_gpu_dropin.py tests/test_gpu_worker_process.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
step workers
timeout -k 10 600 python3 -u scripts/bench_workers.py --peers 100 --workers 4 --rounds 6 > $O/workers_gnlenet.jsonl 2> $O/workers_gnlenet.err || exit $?
cut -c1-460 $O/workers_gnlenet.jsonl
timeout -k 10 600 python3 -u scripts/bench_workers.py --peers 16 --workers 4 --rounds 4 --model resnet18 > $O/workers_resnet18.jsonl 2> $O/workers_resnet18.err || exit $?
cut -c1-460 $O/workers_resnet18.jsonl
step rounds_shm
DLSIM_DEVICE_CACHE_MB=4096 timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 100 --host --shm > $O/rounds_gnlenet_shm_cache.jsonl 2> $O/rounds_gnlenet_shm_cache.err || exit $?
cut -c1-200 $O/rounds_gnlenet_shm_cache.jsonl
step done
