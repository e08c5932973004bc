# Round 4: bench.py's input construction against outputs-first, several
# allocations each in one process (probe_bench_setup.py); the bench at the
# driver's shape and at K = 200 in fresh processes; the reference's
# broker/worker deployment timed (bench_workers.py, one broker per way).
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04f
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step setup_probe
timeout -k 10 400 python3 -u scripts/probes/probe_bench_setup.py 4 200 > $O/bench_setup.jsonl 2> $O/bench_setup.err || exit $?
grep summary $O/bench_setup.jsonl
step bench
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_k20_$i.json 2> $O/bench_k20_$i.err || exit $?
  DLSIM_BENCH_OUTS_FIRST=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_k20_of_$i.json 2> $O/bench_k20_of_$i.err || exit $?
  timeout -k 10 120 python3 bench.py --steps 200 --warmup 200 --no-cpu-baseline > $O/bench_k200_$i.json 2> $O/bench_k200_$i.err || exit $?
  python3 -c "
import json
a=json.load(open('$O/bench_k20_$i.json')); b=json.load(open('$O/bench_k20_of_$i.json')); c=json.load(open('$O/bench_k200_$i.json'))
print($i, 'k20', a['ms_per_step'], 'k20 outs_first', b['ms_per_step'], 'k200', c['ms_per_step'])"
done
step workers
timeout -k 10 600 python3 -u scripts/bench_workers.py --peers 100 --workers 4 --rounds 6 > $O/workers_gnlenet.jsonl 2> $O/workers_gnlenet.err || exit $?
cut -c1-420 $O/workers_gnlenet.jsonl
timeout -k 10 600 python3 -u scripts/bench_workers.py --peers 16 --workers 4 --rounds 4 --model resnet18 > $O/workers_resnet18.jsonl 2> $O/workers_resnet18.err || exit $?
cut -c1-420 $O/workers_resnet18.jsonl
step done
