#!/bin/bash
# Round 4 (x): the deployment's CPU budget. bench_workers' hip way (4 workers,
# GNLeNet) with the defaults, with OpenMP's passive wait policy, with 2 pack
# threads per worker, and with both; each in a fresh broker.
set -o pipefail
mkdir -p gpurun_out/r04x
O=gpurun_out/r04x
timeout -k 10 200 python -u scripts/bench_workers.py --ways hip cpu_ref > $O/default.jsonl 2> $O/default.err &&
OMP_WAIT_POLICY=PASSIVE timeout -k 10 200 python -u scripts/bench_workers.py --ways hip cpu_ref > $O/omp_passive.jsonl 2> $O/omp_passive.err &&
DLSIM_PACK_THREADS=2 timeout -k 10 200 python -u scripts/bench_workers.py --ways hip > $O/pack2.jsonl 2> $O/pack2.err &&
OMP_WAIT_POLICY=PASSIVE DLSIM_PACK_THREADS=2 timeout -k 10 200 python -u scripts/bench_workers.py --ways hip > $O/both.jsonl 2> $O/both.err &&
timeout -k 10 200 python -u scripts/bench_workers.py --ways hip > $O/default2.jsonl 2> $O/default2.err
