# Round 4: row layouts of the north star averaged over physical placements
# (probe_layout_placements.py), then five fresh bench processes at the
# driver's shape; a cProfile of the 100-peer host round, one call per task.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04e
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 300 python3 -u -m pytest -p no:cacheprovider -x -q --timeout 180 --timeout-method thread \
  tests/test_gpu_sharded_stub.py tests/test_gpu_sharded_rccl.py tests/test_gpu_c_host.py tests/test_gpu_device_cache.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
step layouts
timeout -k 10 400 python3 -u scripts/probes/probe_layout_placements.py 4 200 > $O/layout_placements.jsonl 2> $O/layout_placements.err || exit $?
grep summary $O/layout_placements.jsonl
step bench
for i in 1 2 3 4 5; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
  DLSIM_BENCH_SET_ALLOC=per_set DLSIM_BENCH_MIN_SETS=6 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_perset6_$i.json 2> $O/bench_perset6_$i.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$i.json')); e=json.load(open('$O/bench_perset6_$i.json')); print($i, 'arena', d['ms_per_step'], d['roofline']['frac'], 'per_set x6', e['ms_per_step'], e['roofline']['frac'])"
done
step profile_seq_host
timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 100 --host --reps 1 --profile-seq $O/seq_host_prof.txt > $O/seq_host.jsonl 2> $O/seq_host.err || exit $?
head -60 $O/seq_host_prof.txt
step workers
timeout -k 10 500 python3 -u scripts/bench_workers.py --peers 100 --workers 4 --rounds 6 > $O/workers_gnlenet.jsonl 2> $O/workers_gnlenet.err || exit $?
timeout -k 10 500 python3 -u scripts/bench_workers.py --peers 16 --workers 4 --rounds 4 --model resnet18 > $O/workers_resnet18.jsonl 2> $O/workers_resnet18.err || exit $?
cut -c1-400 $O/workers_gnlenet.jsonl $O/workers_resnet18.jsonl
step c_host
timeout -k 10 120 ./tests/native/_build/c_host_check > $O/c_host.txt 2>&1 || exit $?
tail -4 $O/c_host.txt
step done
