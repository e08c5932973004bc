# Round 4 session 2: the whole -m gpu suite with the contiguous output pool,
# then fresh-process A/B of bench.py: DLSIM_CONTIGUOUS=1 (staging rows and
# aggregate outputs in physically contiguous blocks) vs 0 (torch's allocator),
# alternating, driver shape and default K.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04s2_pool}
mkdir -p $O
echo "[$(date +%T)] pytest"
timeout -k 10 900 python3 -u -m pytest ${PYTEST_TARGET:-tests} -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log | grep -vE "^\s*$" | tail -4
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3 4; do
  for c in 1 0; do
    DLSIM_CONTIGUOUS=$c timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_c${c}_$i.json 2> $O/drv_c${c}_$i.err || exit $?
    DLSIM_CONTIGUOUS=$c timeout -k 10 120 python3 bench.py --no-cpu-baseline > $O/def_c${c}_$i.json 2> $O/def_c${c}_$i.err || exit $?
    python3 -c "import json; a=json.load(open('$O/drv_c${c}_$i.json')); b=json.load(open('$O/def_c${c}_$i.json')); print('contig=$c run $i', a['roofline']['kernel_avg_us'], a['roofline']['frac'], b['roofline']['kernel_avg_us'], b['roofline']['frac'], b['config']['rows_alloc'])"
  done
done
echo "[$(date +%T)] done"
