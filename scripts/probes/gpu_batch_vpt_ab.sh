#!/bin/bash
# A/B of the batched kernels' VPT on one box: libraries built with a fixed
# batch VPT of 1, 2, 4 (before batch_vpt chose it per launch; copied by hand
# into dasklearn_amd/lib_exp/v*, not kept), swapped in turn, two rounds.
# Results: profiles/r02_batch_vpt/.
set -o pipefail
out=gpurun_out/${1:-bab}
mkdir -p "$out"
L=decentralized-learning-simulator_amd/dasklearn_amd/lib
X=decentralized-learning-simulator_amd/dasklearn_amd/lib_exp
cp $L/libdlsim_hip.so "$out/orig.so"
for r in 1 2; do
  for v in 4 2 1; do
    cp $X/v$v/libdlsim_hip.so $L/libdlsim_hip.so
    timeout -k 10 200 python -u bench.py --config cfg2_gnlenet --batch 100 --no-cpu-baseline > "$out/gnl_b100_v${v}_r$r.json" 2>/dev/null || exit 1
    timeout -k 10 200 python -u bench.py --config cfg2 --batch 8 --no-cpu-baseline > "$out/cfg2_b8_v${v}_r$r.json" 2>/dev/null || exit 1
  done
done
cp "$out/orig.so" $L/libdlsim_hip.so
