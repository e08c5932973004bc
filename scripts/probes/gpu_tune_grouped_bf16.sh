#!/bin/bash
# 2-byte grouped kernel shapes (fan-in above the fixed specialisations, 9):
# bf16 n = 17 at 11.2 M and 62.5 M and at 1.4 M. Output under gpurun_out/$1.
set -o pipefail
out=gpurun_out/${1:-tb}
mkdir -p "$out"
T=decentralized-learning-simulator_amd/csrc/build/tune_wreduce
for spec in "17 11181642 40" "17 1397760 100" "12 62500000 10"; do
  set -- $spec
  timeout -k 10 240 $T $1 $2 bf16 exact $3 > "$out/bf16_n$1_$2.log" 2>&1 || exit $?
done
