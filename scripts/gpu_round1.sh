set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 ./decentralized-learning-simulator_amd/csrc/build/tune_wreduce 8 11181642 f32 exact 50 > gpurun_out/tune_n8_f32.log 2>&1 || exit $?
timeout -k 10 300 ./decentralized-learning-simulator_amd/csrc/build/tune_wreduce 17 11181642 f32 exact 50 > gpurun_out/tune_n17_f32.log 2>&1 || exit $?
timeout -k 10 300 ./decentralized-learning-simulator_amd/csrc/build/tune_wreduce 2 125000000 bf16 exact 30 > gpurun_out/tune_n2_bf16.log 2>&1 || exit $?
timeout -k 10 300 ./decentralized-learning-simulator_amd/csrc/build/tune_wreduce 100 11181642 f32 exact 20 > gpurun_out/tune_n100_f32.log 2>&1 || exit $?
echo done
