# Parity soak at HEAD: the full -m gpu suite, then scripts/fuzz_parity.py for
# SECONDS (default 420) with a given seed.
# usage: bash scripts/probes/gpu_r03_soak.sh <outdir> <seed> [seconds]
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-soak}
S=${2:-1}
T=${3:-420}
mkdir -p $O
echo "[$(date +%T)] pytest"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
echo "[$(date +%T)] soak seed $S for $T s"
timeout -k 10 $((T + 120)) python3 scripts/fuzz_parity.py --seconds $T --seed $S > $O/fuzz.json 2> $O/fuzz.err || { tail -c 1500 $O/fuzz.json; exit 1; }
tail -c 700 $O/fuzz.json
echo "[$(date +%T)] done"
