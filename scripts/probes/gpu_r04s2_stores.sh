# Round 4 session 2: store policies and launch shapes of the north star on
# contiguous blocks vs hipMalloc (csrc/tune_wreduce.hip, tune_f32 build,
# DLSIM_TUNE_STORES; rows 2 MiB-aligned as the product's row rule).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04s2_stores
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for i in 1 2; do
  echo "[$(date +%T)] contig $i"
  DLSIM_TUNE_R03=1 DLSIM_TUNE_STORES=1 DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_CONTIG=1 timeout -k 10 200 $T 8 11181642 f32 exact 100 > $O/contig_$i.log 2>&1 || exit $?
  echo "[$(date +%T)] hipMalloc $i"
  DLSIM_TUNE_R03=1 DLSIM_TUNE_STORES=1 DLSIM_TUNE_ALIGN=2097152 timeout -k 10 200 $T 8 11181642 f32 exact 100 > $O/plain_$i.log 2>&1 || exit $?
done
tail -12 $O/contig_1.log
