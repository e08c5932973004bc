# The harness/bench gap by HIP runtime: the tuning harness (its shipped
# north-star variant and the library's Slots<16> carrier) under /opt/rocm's
# HIP 7.2 (its RUNPATH) and under the HIP 7.0.2 runtime PyTorch bundles (and
# every bench.py / product process loads), LD_LIBRARY_PATH=torch/lib;
# alternating processes, two each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03_runtime}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
for i in 1 2; do
  DLSIM_TUNE_R03=1 DLSIM_TUNE_ARGS=1 DLSIM_TUNE_ALIGN=2097152 timeout -k 10 240 $T 8 11181642 f32 exact 200 > $O/rocm72_$i.log 2>&1 || exit $?
  echo "rocm 7.2 run $i"; grep -E "variant=NF8_V4_sc1_wave( |_S16)" $O/rocm72_$i.log | sed 's/median_us.*batch_us=/batch_us=/'
  LD_LIBRARY_PATH=$TL DLSIM_TUNE_R03=1 DLSIM_TUNE_ARGS=1 DLSIM_TUNE_ALIGN=2097152 timeout -k 10 240 $T 8 11181642 f32 exact 200 > $O/torch702_$i.log 2>&1 || exit $?
  echo "torch's 7.0.2 run $i"; grep -E "variant=NF8_V4_sc1_wave( |_S16)" $O/torch702_$i.log | sed 's/median_us.*batch_us=/batch_us=/'
done
