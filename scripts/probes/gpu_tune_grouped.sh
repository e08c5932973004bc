#!/bin/bash
# Grouped (runtime fan-in) kernel shapes at the fan-ins above the fixed
# specialisations: cfg3 (n = 17) and cfg5 (n = 100) at full size and at their
# 8-rank slices. Build first: DLSIM_BUILD_TUNE=1 python -c "import __graft_entry__ as g; g.build()"
set -o pipefail
out=gpurun_out/${1:-tg}
mkdir -p "$out"
T=decentralized-learning-simulator_amd/csrc/build/tune_wreduce
for spec in "17 11181642 40" "100 11181642 20" "17 1397760 100" "100 1397760 60"; do
  set -- $spec
  timeout -k 10 240 $T $1 $2 f32 exact $3 > "$out/f32_n$1_$2.log" 2>&1 || exit $?
done
