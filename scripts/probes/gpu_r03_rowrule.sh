# Round 3: the candidate arena row rule against today's, across the configs'
# fan-ins, dtypes and sizes. old = 256-B rows (+4 KiB at 64 KiB multiples,
# round 1's rule); new = rows >= 16 MiB start 2 MiB-aligned, with one more
# 2 MiB unit when the stride would be a multiple of 8 MiB (the layout sweeps:
# profiles/r03_layout*/). Rotating order old/new/old/new.
# usage: bash scripts/probes/gpu_r03_rowrule.sh <outdir>
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r03_rowrule}
mkdir -p $O
T=$R/decentralized-learning-simulator_amd/csrc/build/tune_f32
envs() {  # rule n P dtype -> env assignments for the harness
  python3 - "$@" <<'PY'
import sys
rule, n, P, dt = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
esz = 2 if dt == "bf16" else 4
b = P * esz
r256 = (b + 255) // 256 * 256
if rule == "new" and b >= 16 << 20:
    k = (b + (2 << 20) - 1) // (2 << 20)
    print("DLSIM_TUNE_ALIGN=2097152", "DLSIM_TUNE_STAGGER=%d" % ((2 << 20) if k % 4 == 0 else 0))
else:
    print("DLSIM_TUNE_ALIGN=256", "DLSIM_TUNE_STAGGER=%d" % (4096 if r256 % 65536 == 0 else 0))
PY
}
for cfg in "8 11181642 f32" "8 5590848 f32" "8 6291456 f32" "8 8388608 f32" "8 12582912 f32" "8 16777216 f32" \
           "8 25000000 f32" "4 11181642 f32" "2 11181642 f32" "2 50000000 f32" "17 11181642 f32" "100 11181642 f32" \
           "2 125000000 bf16" "2 62500000 bf16" "2 31250000 bf16" "12 62500000 bf16"; do
  set -- $cfg
  for pass in 1 2; do
    for rule in old new; do
      TAG=n$1_p$2_$3_${rule}_$pass
      E=$(envs $rule $1 $2 $3)
      env DLSIM_TUNE_LAYOUT=1 $E timeout -k 10 180 $T $1 $2 $3 exact 100 > $O/$TAG.log 2>&1 || exit 1
      echo "$TAG [$E] $(grep -E '^variant' $O/$TAG.log | awk '{print $1, $8}' | sed 's/variant=//; s/batch_us=//' | tr '\n' ' ')"
    done
  done
done
echo "[$(date +%T)] done"
