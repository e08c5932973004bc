# Round 4, first GPU call: the new and changed GPU tests (sharded plans and the
# padded all-gather through the stub RCCL and world-1 RCCL, two processes with
# the HIP reduce on a gloo control plane, the small-job D2H layouts, cfg5 at
# full size), then the placement/data/window probe and the driver's bench
# shape (--steps 20 --warmup 5) with and without the timing gate, alternating
# in fresh processes.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04a
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 600 python3 -u -m pytest -p no:cacheprovider -x -v --timeout 180 --timeout-method thread \
  tests/test_gpu_sharded_stub.py tests/test_gpu_sharded_rccl.py tests/test_gpu_sharded_multiproc.py \
  "tests/test_gpu_chunks.py::test_host_chunk_mean_small_job_one_dma" \
  "tests/test_gpu_parity.py::test_cfg5_100way_11M_f32_bit_exact" -s > $O/pytest.log 2>&1
rc=$?; grep -E "PER_CALL_US|passed|failed|error" $O/pytest.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
step probe_placement
timeout -k 10 300 python3 -u scripts/probes/probe_placement.py 3 > $O/placement.jsonl 2> $O/placement.err || exit $?
step bench_ab
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_gate_$i.json 2> $O/bench_gate_$i.err || exit $?
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gate > $O/bench_nogate_$i.json 2> $O/bench_nogate_$i.err || exit $?
done
for f in $O/bench_*.json; do
  python3 -c "import json,sys; d=json.load(open('$f')); print('$(basename $f)', d['ms_per_step'], d['roofline']['frac'], d['pattern_ceiling']['frac'])"
done
step done
step host_task_parts
timeout -k 10 300 python3 -u scripts/probes/probe_host_task_parts.py 400 > $O/host_task_parts.json 2> $O/host_task_parts.err || exit $?
cat $O/host_task_parts.json
step cfg1
timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 2 --host --rounds 300 --cpu-rounds 300 > $O/cfg1.jsonl 2> $O/cfg1.err || exit $?
cut -c1-300 $O/cfg1.jsonl
step rounds_host_100
timeout -k 10 400 python3 -u scripts/bench_rounds.py --peers 100 --host > $O/rounds_host_100.jsonl 2> $O/rounds_host_100.err || exit $?
cut -c1-300 $O/rounds_host_100.jsonl
step done2
