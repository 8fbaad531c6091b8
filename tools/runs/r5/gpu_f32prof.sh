#!/bin/bash
# Kernel trace of the reference's fp32 workload (L8 H8, 32 x 128, m = 4) at P = 1: where the 22 ms go.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f32prof
timeout -k 10 300 python -u bench.py --phase ref --ref-p 1 --no-supervise --steps 20 --warmup 5 --no-bubble > gpurun_out/f32prof/plain.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/f32prof/trace -o run -- python -u bench.py --phase ref --ref-p 1 --no-supervise --steps 20 --warmup 5 --no-bubble > gpurun_out/f32prof/prof.log 2>&1
find gpurun_out/f32prof -name '*stats*' | head -5
