# Parametrised A/B driver (round 6; replaces round 5's one-off gpu_*_ab.sh
# launchers): runs one command under several sets of A/B switches, each leg in
# a fresh process, the legs interleaved over P passes so box drift hits every
# leg alike. Every leg runs with DLSIM_AB=1 (the library reads its tuning
# switches only then; csrc/ab_env.hpp). Output: <outdir>/<label>_p<pass>.out
# (stdout) and .err, plus a one-line summary per leg on stdout.
#
# usage: bash scripts/gpu_ab.sh <outdir-name> <passes> <seconds-per-leg> \
#            "<label>:<VAR=value,VAR=value|->" ... -- <command ...>
# e.g.   bash scripts/gpu_ab.sh chunk_ab 2 120 "tiled:DLSIM_CHUNK_DEFER_FIXED=0" "fixed:-" \
#            -- python3 scripts/bench_chunks.py --kernel-only --m 4
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
P=$2
LIMIT=$3
shift 3
LEGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LEGS+=("$1"); shift; done
[ "${1:-}" = "--" ] || { echo "usage: missing -- <command>"; exit 2; }
shift
mkdir -p $O
for p in $(seq 1 $P); do
  for leg in "${LEGS[@]}"; do
    label=${leg%%:*}
    spec=${leg#*:}
    envs=(DLSIM_AB=1)
    if [ "$spec" != "-" ]; then IFS=, read -r -a extra <<< "$spec"; envs+=("${extra[@]}"); fi
    echo "[$(date +%T)] pass $p $label: ${envs[*]} $*"
    env "${envs[@]}" timeout -k 10 $LIMIT "$@" > $O/${label}_p$p.out 2> $O/${label}_p$p.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc for $label pass $p"; tail -20 $O/${label}_p$p.err; exit $rc; fi
    tail -c 600 $O/${label}_p$p.out
  done
done
echo "[$(date +%T)] done"
