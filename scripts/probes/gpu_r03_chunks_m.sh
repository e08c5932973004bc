# Round 3: chunk-mean rows per load group (RF 4 vs 8) by contributor count.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03_chunks_m
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for m in 2 3 4 5 6 7 8 9 12; do
  for pass in 1 2; do
    DLSIM_TUNE_CHUNK=1 timeout -k 10 180 $T $m 1118164 10 100 > $O/cm_m${m}_$pass.log 2>&1 || { cat $O/cm_m${m}_$pass.log; exit 1; }
    echo "m=$m pass=$pass $(grep -E '^variant=cm_(V4_wave_RF8|V4_wave_RF4|V2_wave_RF8|V4_blk_RF8|xorprobe)' $O/cm_m${m}_$pass.log | awk '{print $1, $5}' | sed 's/variant=cm_//; s/batch_us=//' | tr '\n' ' ')"
  done
done
