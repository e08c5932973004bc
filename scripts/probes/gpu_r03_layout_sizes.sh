# Round 3: is 2 MiB row alignment a rule or a quirk of one stride? n = 8 fp32
# at row sizes from 18 MiB to 120 MiB (a power of two included): arena rows
# aligned to 256 B, to 2 MiB, 2 MiB plus a 2 MiB stagger, 2 MiB plus 4 KiB;
# the two large-size fixed shapes (wave and block map, VPT 4).
# usage: bash scripts/probes/gpu_r03_layout_sizes.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03_layout_sizes}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
run() {  # tag n P env...
  local TAG=$1 N=$2 P=$3; shift 3
  env DLSIM_TUNE_LAYOUT=1 DLSIM_TUNE_ONLY=NF8_V4_sc1_wave,NF8_V4_sc1_blk "$@" timeout -k 10 120 $T $N $P f32 exact 200 > $O/$TAG.log 2>&1 || return 1
  echo "$TAG $(grep -E '^variant' $O/$TAG.log | awk '{print $1, $8}' | sed 's/variant=//; s/batch_us=//' | tr '\n' ' ')"
}
for P in 4718592 5590848 6291456 7000000 8388608 9437184 10000000 11181642 12582912 15000000 20000000 30000000; do
  echo "[$(date +%T)] P=$P"
  run p${P}_a256 8 $P DLSIM_TUNE_ALIGN=256 || exit 1
  run p${P}_a2m 8 $P DLSIM_TUNE_ALIGN=2097152 || exit 1
  run p${P}_a2m_s2m 8 $P DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_STAGGER=2097152 || exit 1
  run p${P}_a2m_s4k 8 $P DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_STAGGER=4096 || exit 1
  run p${P}_a256_s4k 8 $P DLSIM_TUNE_ALIGN=256 DLSIM_TUNE_STAGGER=4096 || exit 1
done
echo "[$(date +%T)] done"
