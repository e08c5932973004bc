#!/bin/bash
# Host cost of small launches (csrc/launch_probe.hip; built here, run on the box).
set -o pipefail
out=gpurun_out/${1:-lp}
mkdir -p "$out"
timeout -k 10 120 decentralized-learning-simulator_amd/csrc/build/launch_probe > "$out/launch_probe.json" 2> "$out/launch_probe.err"
