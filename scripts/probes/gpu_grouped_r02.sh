#!/bin/bash
# Grouped-kernel shapes (dispatch.hpp grouped_shape): parity, then the bench
# lines they change (cfg3 n = 17, cfg5 n = 100, at full size and at the
# 8-rank slice), the north star as a control. Output under gpurun_out/$1.
set -o pipefail
out=gpurun_out/${1:-gs}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_f64.py tests/test_gpu_aliasing.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
for spec in "cfg3 1" "cfg5 1" "cfg3 8" "cfg5 8" "north_star 1"; do
  set -- $spec
  timeout -k 10 300 python -u bench.py --config $1 --slice-of $2 --no-cpu-baseline > "$out/bench_$1_s$2.json" 2> "$out/bench_$1_s$2.err" || exit $?
done
