# cfg4 (2 x 125 M bf16) reduce against its memory-only probe in fresh
# processes: is the r03 reduce/probe 0.962 a property of the kernel or of
# the process's placement?
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-cfg4_var}
mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 200 python3 bench.py --config cfg4 --no-cpu-baseline > $O/cfg4_$i.json 2>> $O/err.log || exit $?
  python3 -c "import json; d=json.load(open('$O/cfg4_$i.json')); r=d['roofline']; p=d['pattern_ceiling']; print($i, r['kernel_avg_us'], r['frac'], p['us_per_launch'], p['frac'], p['reduce_over_probe'])"
done
