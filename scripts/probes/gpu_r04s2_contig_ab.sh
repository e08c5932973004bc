# Round 4 session 2: the resident-block tests, then fresh-process A/B of the
# bench's rows allocated physically contiguous (default) vs torch's allocator
# (DLSIM_CONTIGUOUS=0), alternating, driver shape and default K.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r04s2_contig_ab}
mkdir -p $O
echo "[$(date +%T)] tests"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_resident_alloc.py tests/test_gpu_staging.py tests/test_gpu_device_cache.py tests/test_gpu_mismatch.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3 4; do
  for c in 1 0; do
    DLSIM_CONTIGUOUS=$c timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_c${c}_$i.json 2> $O/drv_c${c}_$i.err || exit $?
    DLSIM_CONTIGUOUS=$c timeout -k 10 120 python3 bench.py --no-cpu-baseline > $O/def_c${c}_$i.json 2> $O/def_c${c}_$i.err || exit $?
    python3 -c "import json; a=json.load(open('$O/drv_c${c}_$i.json')); b=json.load(open('$O/def_c${c}_$i.json')); print('contig=$c run $i', a['roofline']['kernel_avg_us'], a['roofline']['frac'], b['roofline']['kernel_avg_us'], b['roofline']['frac'], b['config']['rows_alloc'])"
  done
done
echo "[$(date +%T)] done"
