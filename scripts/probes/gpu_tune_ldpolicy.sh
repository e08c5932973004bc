# Load cache-policy bits on the north star's shipped shape (NF8, VPT 4, wave
# map, sc1 stores): global nt (shipped) against buffer loads with sc0/sc1/nt
# combinations, with >= 1 GiB of rotating inputs; then at the 8-rank slice.
# usage: bash scripts/probes/gpu_tune_ldpolicy.sh <outdir>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ldpolicy}
mkdir -p $O
C=$R/decentralized-learning-simulator_amd/csrc
T=$C/build/tune_wreduce
mkdir -p $C/build
# the harness is not shipped to the box (.gpurunignore): build it here
timeout -k 10 600 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I $R/include -I $C \
  $C/tune_wreduce.hip -o $T > $O/build.log 2>&1 || exit $?
V=NF8_V4_sc1_wave,NF8_V4w_ldb_nt,NF8_V4w_ldb_sc0nt,NF8_V4w_ldb_sc1nt,NF8_V4w_ldb_sc01nt,NF8_V4w_ldb_sc1,NF8_V4w_ldb_sc01,NF8_V4w_ldb_plain,NF8_xorprobe
for rep in 1 2; do
  DLSIM_TUNE_ONLY=$V timeout -k 10 200 $T 8 11181642 f32 exact 200 > $O/f32_n8_11181642_$rep.log 2>&1 || exit $?
done
DLSIM_TUNE_ONLY=$V timeout -k 10 200 $T 8 1397760 f32 exact 200 > $O/f32_n8_1397760.log 2>&1 || exit $?
