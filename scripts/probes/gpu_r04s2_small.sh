# Round 4 session 2: do contiguous outputs help the small launches? cfg2 and
# the north star's 8-rank slice with the output pool from 1 MiB, from 16 MiB
# (default: these outputs stay in torch's allocator) and off, fresh processes.
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04s2_small
mkdir -p $O
for i in 1 2 3; do
  for v in 1 16 off; do
    for c in "cfg2 1" "north_star 8"; do
      set -- $c
      if [ $v = off ]; then E="DLSIM_CONTIGUOUS=0"; else E="DLSIM_OUT_POOL_MIN_MB=$v"; fi
      env $E timeout -k 10 120 python3 bench.py --config $1 --slice-of $2 --no-cpu-baseline > $O/${1}_s$2_${v}_$i.json 2> $O/${1}_s$2_${v}_$i.err || exit $?
      python3 -c "import json; d=json.load(open('$O/${1}_s$2_${v}_$i.json')); print('$1 s$2 pool=$v run $i', d['roofline']['kernel_avg_us'], d['roofline']['frac'])"
    done
  done
done
