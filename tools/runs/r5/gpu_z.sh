#!/bin/bash
# Kernel trace of the reference fp32 config (L8 H8, 32 x 128, m = 4, P = 1) as the bench runs it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5z
export MIPIPE_BENCH_CHILD=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5z/prof -o run -- python3 bench.py --gpus 1 --phase ref --ref-p 1 --ref-grid l8h8 --steps 20 --warmup 5 > gpurun_out/r5z/ref.log 2>&1
rc=$?; grep '^{' gpurun_out/r5z/ref.log | cut -c1-300; exit $rc
