#!/bin/bash
# Round 6: kernel-time profile of the headline step (GPT-2 small, 1 GPU) with the v2 attention.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6prof/trace -o run -- python3 bench.py --gpus 1 --steps 10 --warmup 3 --schedules none --ref-fp32 0 --no-supervise --no-bubble > gpurun_out/r6prof/prof.log 2>&1 || { tail -20 gpurun_out/r6prof/prof.log; exit 1; }
find gpurun_out/r6prof/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/r6prof/kernel_stats.csv \;
rm -rf gpurun_out/r6prof/trace
head -25 gpurun_out/r6prof/kernel_stats.csv | cut -c1-160
