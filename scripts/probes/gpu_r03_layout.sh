# Round 3: does the input layout move the north star? The fp32 harness
# (csrc/build/tune_f32, DLSIM_TUNE_R03) times the shipped shape and its
# memory-only probe with the 8 inputs as separate hipMallocs or as arena rows
# whose starts are aligned to 256 B (bench.py / arena.row_stride today),
# 4 KiB, 64 KiB or 2 MiB; two passes in rotating order, then bench.py's line
# on the same box.
# usage: bash scripts/probes/gpu_r03_layout.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03_layout}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
P=${P:-11181642}
run() {  # name env...
  local NAME=$1; shift
  env DLSIM_TUNE_R03=1 DLSIM_TUNE_ONLY=NF8_V4_sc1_wave,NF8_xorprobe "$@" timeout -k 10 120 $T 8 $P f32 exact 200 > $O/$NAME.log 2>&1 || return 1
  echo "$NAME $(grep -E 'addr_mod' $O/$NAME.log) $(grep -E '^variant' $O/$NAME.log | awk '{print $1, $8, $9}' | tr '\n' ' ')"
}
for pass in 1 2; do
  echo "[$(date +%T)] pass $pass"
  run sep_$pass || exit 1
  run a256_$pass DLSIM_TUNE_ALIGN=256 || exit 1
  run a4k_$pass DLSIM_TUNE_ALIGN=4096 || exit 1
  run a64k_$pass DLSIM_TUNE_ALIGN=65536 || exit 1
  run a2m_$pass DLSIM_TUNE_ALIGN=2097152 || exit 1
  run a2m_s4k_$pass DLSIM_TUNE_ALIGN=2097152 DLSIM_TUNE_STAGGER=4096 || exit 1
done
echo "[$(date +%T)] bench"
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['roofline']['kernel_avg_us'], d['roofline']['frac'])"
echo "[$(date +%T)] done"
