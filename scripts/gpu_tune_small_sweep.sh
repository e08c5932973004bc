# VPT 2 against VPT 4 (block map, sc1) for fp32 rows below 8 MB per stream,
# fan-in 2, 4 and 8 (round 5: does the whole-tile count per CU pick the shape?)
# usage: bash scripts/gpu_tune_small_sweep.sh <outdir-name>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-small_sweep}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
for n in 8 2 4; do for P in 524288 655360 786432 917504 1048576 1179648 1310720 1397760 1441792 1572864 1703936 1835008 1966080; do
  DLSIM_TUNE_SMALL=1 DLSIM_TUNE_CONTIG=1 DLSIM_TUNE_ALIGN=256 DLSIM_TUNE_ONLY=NF${n}_V2_sc1_blk,NF${n}_V4_sc1_blk,NF${n}_V1_sc1_blk \
    timeout -k 10 120 $T $n $P f32 exact 400 > $O/s_${n}_${P}.log 2>&1 || exit $?
  echo "n=$n P=$P $(grep variant $O/s_${n}_${P}.log | sed -E 's/.*variant=(\S+).*batch_us=(\S+).*bfrac=(\S+) same=(\S).*/\1 \2 \3 \4/' | tr '\n' ' ')"
done; done
