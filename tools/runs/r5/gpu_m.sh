#!/bin/bash
# Kernel stats of the headline step on ONE stream (no lane overlap: isolated kernel times).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5m
export MIPIPE_LANES=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5m/prof -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 3 --schedules none --ref-fp32 0 --no-supervise --no-bubble > gpurun_out/r5m/prof.log 2>&1
rc=$?; grep '^{' gpurun_out/r5m/prof.log | cut -c1-200; exit $rc
