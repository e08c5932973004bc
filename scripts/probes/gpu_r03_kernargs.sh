# Is the harness/bench gap the kernel-argument carrier? The shipped north-star
# kernel with Slots<128> (the harness's), Slots<16> (the library's, n <= 16)
# and DevSlots (pointers and weights in device memory), 2 MiB rows as bench.py
# lays them out, and at the 8-rank slice; interleaved rounds in one process.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03_kernargs}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
DLSIM_TUNE_R03=1 DLSIM_TUNE_ARGS=1 DLSIM_TUNE_ALIGN=2097152 timeout -k 10 240 $T 8 11181642 f32 exact 200 > $O/ns.log 2>&1 || exit $?
grep variant $O/ns.log
DLSIM_TUNE_R03=1 DLSIM_TUNE_ARGS=1 DLSIM_TUNE_STAGGER=0 timeout -k 10 240 $T 8 1397760 f32 exact 400 > $O/s8.log 2>&1 || exit $?
grep variant $O/s8.log
