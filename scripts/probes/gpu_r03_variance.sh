# Round 3: run-to-run spread of the north-star bench line (fresh process per
# run) against the harness's 2 MiB-row layout, alternating.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_variance
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for i in 1 2 3 4 5; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --steps 400 > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
  B=$(python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print(d['roofline']['kernel_avg_us'], d['roofline']['frac'])")
  DLSIM_TUNE_LAYOUT=1 DLSIM_TUNE_ONLY=NF8_V4_sc1_wave,NF8_V4_sc1_blk DLSIM_TUNE_ALIGN=2097152 timeout -k 10 120 $T 8 11181642 f32 exact 200 > $O/harness_$i.log 2>&1 || exit 1
  H=$(grep -E '^variant=NF8_V4_sc1_wave' $O/harness_$i.log | awk '{print $8}')
  echo "run $i bench $B harness $H"
done
