#!/bin/bash
# Round 4 (l): tile orders against translation reach, 3 vs 12 rotating sets.
set -o pipefail
mkdir -p gpurun_out/r04l
T=decentralized-learning-simulator_amd/csrc/build/tune_f32
for S in 3 12; do
  DLSIM_TUNE_R03=1 DLSIM_TUNE_TLB=1 DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_SETS=$S timeout -k 10 240 $T 8 11181642 f32 exact 50 > gpurun_out/r04l/tlb_sets$S.txt 2>&1 || exit $?
  grep variant= gpurun_out/r04l/tlb_sets$S.txt | awk '{print $1, $5, $7, $8, $10, $11}'
done
