# Round 3 evidence, part B: rocprofv3 kernel stats + PMC traffic and bench
# lines for every other BASELINE config at N=1 and its multi-GPU slice.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
echo "[$(date +%T)] profile"
bash scripts/gpu_profile_r03.sh r03_profB "cfg2:cfg2:1 cfg3:cfg3:1 cfg3_s8:cfg3:8 cfg4:cfg4:1 cfg4_s4:cfg4:4 cfg5:cfg5:1 cfg5_s8:cfg5:8" || exit 1
echo "[$(date +%T)] done"
