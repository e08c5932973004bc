#!/bin/bash
# Round 4 (k): the spread of the north star's rotating sets within one
# process, three fresh processes.
set -o pipefail
mkdir -p gpurun_out/r04k
for i in 1 2 3; do
  timeout -k 10 200 python -u scripts/probes/probe_set_spread.py 12 100 > gpurun_out/r04k/set_spread_$i.jsonl 2>&1 || exit $?
  tail -1 gpurun_out/r04k/set_spread_$i.jsonl | cut -c1-600
done
