# Preloaded leading kernel arguments (round 6) against the kernels with every
# argument loaded (DLSIM_AB=1 DLSIM_PRELOAD=0), in fresh bench.py processes,
# two passes, for the north star, its 4- and 8-rank slices, cfg2 and cfg4.
# usage: bash scripts/gpu_preload_ab.sh <outdir-name>
set -u
O=${1:-preload_ab}
for spec in "ns:" "s8:--slice-of 8" "s4:--slice-of 4" "cfg2:--config cfg2" "cfg4:--config cfg4"; do
  name=${spec%%:*}; args=${spec#*:}
  bash scripts/gpu_ab.sh $O/$name 2 200 "old:DLSIM_PRELOAD=0" "pre:-" -- python3 bench.py --no-cpu-baseline $args > /dev/null || exit 1
  for f in gpurun_out/$O/$name/*.out; do
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-2:], d['roofline']['kernel'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])" $f || exit 1
  done
done
